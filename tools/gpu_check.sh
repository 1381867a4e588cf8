#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprof kernel stats.  Stops at the first
# crash-like exit (fault / abort / timeout); ordinary test failures still let the bench run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r1}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=30 --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/gpu_tests_$TAG.log | tail -3
ok $rc || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/smoke_$TAG.log
ok $rc || exit $rc
if [ "${BENCH:-1}" = "1" ]; then
  timeout -k 10 600 python -u bench.py --agents 1000000 --tasks 1000 --steps 3 --cpu-baseline 0 \
      > gpurun_out/bench_1m_$TAG.json 2> gpurun_out/bench_1m_$TAG.err
  rc=$?; echo "bench1m rc=$rc"; cat gpurun_out/bench_1m_$TAG.json
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python -u bench.py --steps 3 > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 600 python -u bench.py --steps 2 --elect-mode dense --cpu-baseline 0 \
      > gpurun_out/bench_dense_$TAG.json 2> gpurun_out/bench_dense_$TAG.err
  rc=$?; echo "bench dense rc=$rc"; cat gpurun_out/bench_dense_$TAG.json
  [ $rc -eq 0 ] || exit $rc
fi
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
      -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 gpurun_out/prof_$TAG.log
  find gpurun_out/prof_$TAG -name "*stats*" | head
fi
