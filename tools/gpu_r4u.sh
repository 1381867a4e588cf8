#!/bin/bash
# One-XCD auction batches: parity (tests/test_auction.py), then C4 wall time at several thresholds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4u
rm -rf $O; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_auction.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for cfg in ${CFGS:-"0 32" "1024 32" "512 32" "2048 32" "1024 0" "4096 0" "0 32" "1024 32"}; do
  set -- $cfg
  SWARM_AUCTION_XCD=$1 SWARM_AUCTION_TAIL=$2 timeout -k 10 200 python3 -u tools/auction_probe.py > $O/ab_tmp.log 2>&1 \
      || { cat $O/ab_tmp.log; exit 1; }
  echo "xcd=$1 tail=$2 $(tail -1 $O/ab_tmp.log)" | tee -a $O/ab.log
done
