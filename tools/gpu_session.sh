#!/bin/bash
# Round-6 GPU session: selected test files (-k filter), then optionally the default bench line.
# Stops at the first crash-like exit (fault / abort / timeout).
#   TESTS="tests/a.py tests/b.py" K="expr" TAG=x BENCH=1 bash tools/gpu_session.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r6}
crash() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 "${TTIME:-900}" python -u -m pytest $TESTS ${K:+-k "$K"} -m gpu -v --maxfail=10 --timeout 300 \
      --timeout-method thread > gpurun_out/t_$TAG.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/t_$TAG.log | tail -40
  crash $rc && exit $rc
fi
if [ "${BENCH:-0}" = "1" ]; then
  timeout -k 10 600 python -u bench.py ${BARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; cut -c1-1500 gpurun_out/bench_$TAG.json
  [ $rc -eq 0 ] || exit $rc
fi
exit 0
