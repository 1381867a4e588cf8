#!/bin/bash
# An election change: the election parity tests, then tools/elect_ab.py at 10M for each env
# setting in $KNOBS, then the per-round-range kernel trace of the same settings (tools/trace_knobs.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/ab_${TAG:-a}; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
    ${TESTS:-tests/test_gpu_parity.py tests/test_scale.py tests/test_elect_sizes.py tests/test_compact_cols.py} > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for k in $KNOBS; do
  echo "== $k" >> $O/ab.log
  env $k timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so 10000000 >> $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
done
grep -v amdgpu.ids $O/ab.log
[ -n "${TRACE:-}" ] && TAG=${TAG:-a} bash tools/trace_knobs.sh
true
