#!/bin/bash
# Allocation changes: the allocation GPU tests, then its host/device cost at C3
# (tools/alloc_host_probe.py) and the bench's allocation window (tools/prof_alloc.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/alloc_${TAG:-a}; mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
    tests/test_alloc_index.py tests/test_guard_band.py tests/test_gpu_parity.py tests/test_scale.py tests/test_dist_gpu.py \
    > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/alloc_host_probe.py > $O/probe.log 2>&1 || { tail $O/probe.log; exit 1; }
head -3 $O/probe.log | grep allocate
TAG=${TAG:-a} bash tools/prof_alloc.sh
