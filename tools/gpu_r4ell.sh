#!/bin/bash
# ELL rows for the sparse election rounds: parity suites, then wall time with and without them
# (SWARM_ELL=0: swarm_elect_ell falls back to row_ptr + 16-bit columns; tools/elect_ab.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4ell
rm -rf $O; mkdir -p $O
if [ "${TESTS:-1}" = "1" ]; then
  timeout -k 10 800 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread -m gpu \
      tests/test_ell.py tests/test_compact_cols.py tests/test_elect_sizes.py tests/test_gpu_parity.py tests/test_scale.py > $O/tests.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { tail -60 $O/tests.log; exit $rc; }
fi
for n in ${SIZES:-10000000 1000000}; do
  for e in ${ELLS:-1 0 1 0 1 0}; do
    SWARM_ELL=$e timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so $n > $O/ab_tmp.log 2>&1 \
        || { cat $O/ab_tmp.log; exit 1; }
    echo "ell=$e $(tail -1 $O/ab_tmp.log)" | tee -a $O/ab.log
  done
done
