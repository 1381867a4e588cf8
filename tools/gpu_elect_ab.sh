#!/bin/bash
# Election A/B on one MI355X: parity tests of the election paths on the current build, then the
# untimed wall-time probe (tools/elect_ab.py) for each library named in $LIBS at 10M and 100k agents.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab_${TAG:-x}
mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
      tests/test_gpu_parity.py tests/test_scale.py tests/test_protocol.py > $O/tests.log 2>&1 \
      || { tail -30 $O/tests.log; exit 1; }
  tail -1 $O/tests.log
fi
for lib in ${LIBS:-libswarm.so}; do
  for n in ${SIZES:-10000000 100000}; do
    timeout -k 10 200 python3 -u tools/elect_ab.py $lib $n >> $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
  done
done
cat $O/ab.log
