#!/bin/bash
# Round 4: guard band (dense deferred chains), auction (sparse exchange, 1-rank RCCL), multi-process SHM loops.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r4c}
timeout -k 10 600 python -u -m pytest tests/test_guard_band.py tests/test_auction.py tests/test_dist_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/gpu_tests_$TAG.log
exit $rc
