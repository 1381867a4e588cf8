#!/bin/bash
# Balanced busy rounds: election parity tests, then the knob sweep of SWARM_BAL_MIN_FRAC at 10M.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/bal_${TAG:-a}; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_scale.py tests/test_elect_sizes.py tests/test_compact_cols.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for k in ${KNOBS:-SWARM_BAL_MIN_FRAC=0 SWARM_BAL_MIN_FRAC=0.01 SWARM_BAL_MIN_FRAC=0.003 SWARM_BAL_MIN_FRAC=0.03 SWARM_BAL_MIN_FRAC=0.001}; do
  echo "== $k" >> $O/ab.log
  env $k timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so 10000000 >> $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
done
grep -v amdgpu.ids $O/ab.log
