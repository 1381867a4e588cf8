#!/bin/bash
# Election A/B of two builds (libswarm_head.so = the committed tree, libswarm.so = the change),
# interleaved runs at 10M and 1M agents (tools/elect_ab.py), after the election parity suites.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4z
rm -rf $O; mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 800 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
      tests/test_elect_sizes.py tests/test_gpu_parity.py tests/test_scale.py tests/test_dist_gpu.py > $O/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
fi
for n in ${SIZES:-10000000 1000000}; do
  for lib in libswarm_head.so libswarm.so libswarm_head.so libswarm.so libswarm_head.so libswarm.so; do
    timeout -k 10 200 python3 -u tools/elect_ab.py $lib $n > $O/ab_tmp.log 2>&1 || { cat $O/ab_tmp.log; exit 1; }
    tail -1 $O/ab_tmp.log | tee -a $O/ab.log
  done
done
