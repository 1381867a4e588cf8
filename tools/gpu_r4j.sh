#!/bin/bash
# Single-XCD tail: parity (forced and default thresholds, layout-boundary sizes), then the election
# wall time with the tail off / on at several switch points (tools/elect_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    tests/test_xcd_tail.py tests/test_elect_sizes.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for n in 10000000 1000000; do
  for cfg in "0 -1" "1 -1" "1 2000" "1 4000" "1 16000" "1 30000"; do
    set -- $cfg
    SWARM_XCD_TAIL=$1 SWARM_XCD_MIN_CHANGES=$2 timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so $n \
        > $O/ab_tmp.log 2>&1 || { cat $O/ab_tmp.log; exit 1; }
    echo "xcd=$1 min=$2 $(tail -1 $O/ab_tmp.log)" | tee -a $O/ab.log
  done
done
MINC=${MINC:-4000} bash tools/gpu_r4k.sh
