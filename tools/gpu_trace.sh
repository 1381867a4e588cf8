#!/bin/bash
# Kernel trace of one bench step (rocprofv3 --kernel-trace --stats), for per-round analysis.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-trace}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
    -- python3 bench.py --steps 1 --warmup 1 --cpu-baseline 0 ${BENCH_ARGS:-} > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/prof_$TAG.log
exit $rc
