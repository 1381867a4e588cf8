#!/bin/bash
# rocprofv3 kernel trace of tools/elect_ab.py at $N agents for each env setting in $KNOBS,
# summarised per round range by tools/trace_ranges.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/tk_${TAG:-a}; mkdir -p $O
i=0
for k in $KNOBS; do
  i=$((i+1))
  env $k timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/k$i -o run \
      -- python3 -u tools/elect_ab.py libswarm.so ${N:-10000000} > $O/k$i.log 2>&1 || { tail -5 $O/k$i.log; exit 1; }
  f=$(ls $O/k$i/*/run_kernel_trace.csv $O/k$i/run_kernel_trace.csv 2>/dev/null | head -1)
  python3 tools/trace_ranges.py "$f" "$k" >> $O/ranges.txt || exit 1
  rm -f "$f"
done
cat $O/ranges.txt
