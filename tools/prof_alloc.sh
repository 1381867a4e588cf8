#!/bin/bash
# Kernel trace of a short bench run; the allocation call's kernels and gaps (tools/alloc_window.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pa_${TAG:-a}; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O -o run \
    -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 --rows 0 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
f=$(ls $O/*/run_kernel_trace.csv $O/run_kernel_trace.csv 2>/dev/null | head -1)
python3 tools/alloc_window.py "$f" > $O/alloc_window.txt && cat $O/alloc_window.txt
grep -o '"breakdown_ms": {[^}]*}' $O/bench.log
