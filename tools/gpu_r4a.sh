#!/bin/bash
# Round 4: the native sharded loops over the shared-memory transport (2-3 processes on one GPU),
# and the device-wide synchronisation price (tools/barrier_bench.hip).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 tools/build/barrier_bench 2000 > gpurun_out/barrier_bench.json 2> gpurun_out/barrier_bench.err
rc=$?; echo "barrier rc=$rc"; cat gpurun_out/barrier_bench.json; cat gpurun_out/barrier_bench.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/dist_gpu_r4a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/dist_gpu_r4a.log
exit $rc
