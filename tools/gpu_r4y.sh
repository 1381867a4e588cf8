#!/bin/bash
# Tail chunk teams split over several workgroups: election parity, then wall time against the
# previous build and at several split factors (SWARM_TAIL_SPLIT; tools/elect_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4y
rm -rf $O; mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  SWARM_TAIL_SPLIT=${TEST_SPLIT:-2} timeout -k 10 800 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
      tests/test_elect_sizes.py tests/test_gpu_parity.py tests/test_scale.py tests/test_dist_gpu.py > $O/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
fi
for n in ${SIZES:-10000000 1000000}; do
  for cfg in "libswarm_head.so 1" "libswarm.so 1" "libswarm.so 2" "libswarm.so 4" "libswarm_head.so 1" "libswarm.so 1" "libswarm.so 2" "libswarm.so 4"; do
    set -- $cfg
    SWARM_TAIL_SPLIT=$2 timeout -k 10 200 python3 -u tools/elect_ab.py $1 $n > $O/ab_tmp.log 2>&1 || { cat $O/ab_tmp.log; exit 1; }
    echo "split=$2 $(tail -1 $O/ab_tmp.log)" | tee -a $O/ab.log
  done
done
