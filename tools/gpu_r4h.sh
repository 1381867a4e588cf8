#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4h.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/gpu_tests_r4h.log
exit $rc
