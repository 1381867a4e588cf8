#!/bin/bash
# Round 4: sharded loop with the tail's agent-order layout -- multi-process SHM + single-rank RCCL tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_parity.py tests/test_scale.py -k "sharded or dist or native or long" -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_r4g.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -14 gpurun_out/gpu_tests_r4g.log
exit $rc
