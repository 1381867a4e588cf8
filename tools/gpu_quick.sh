#!/bin/bash
# Quick GPU iteration: election parity tests, then the C3 bench without the CPU leg.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-q}
# PYTEST_K: a pytest -k expression (quoted as one argument); BENCH=0 skips the bench
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gpu_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
[ "${BENCH:-1}" = "1" ] || exit 0
timeout -k 10 300 python -u bench.py --steps 3 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; tail -2 gpurun_out/bench_$TAG.err
exit $rc
