#!/bin/bash
# rocprofv3 kernel trace of tools/elect_ab.py for each library in $LIBS at $N agents, summarised
# by round range (tools/trace_ranges.py).  Each profiled run has its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/trace_${TAG:-x}
mkdir -p $O
for lib in ${LIBS:-libswarm.so}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/$lib -o run \
      -- python3 tools/elect_ab.py $lib ${N:-10000000} > $O/$lib.log 2>&1 || { tail $O/$lib.log; exit 1; }
  grep "elect ms" $O/$lib.log
  python3 tools/trace_ranges.py $(find $O/$lib -name "run_kernel_trace.csv" | head -1) $lib
done
