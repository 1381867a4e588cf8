#!/bin/bash
# Small-swarm one-XCD elections: parity (layout-boundary sizes, forced paths), then the election
# wall time with the one-XCD rounds off / on at several sizes (tools/elect_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4r
rm -rf $O; mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu \
    tests/test_elect_sizes.py tests/test_gpu_parity.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAIL|Error" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
for n in ${SIZES:-100000 30000 300000 1000000}; do
  for mx in 0 300000 2000000; do
    SWARM_XCD_MAX_N=$mx timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so $n > $O/ab_tmp.log 2>&1 \
        || { cat $O/ab_tmp.log; exit 1; }
    echo "xcd_max_n=$mx $(tail -1 $O/ab_tmp.log)" | tee -a $O/ab.log
  done
done
