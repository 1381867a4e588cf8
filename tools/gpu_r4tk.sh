#!/bin/bash
# Per-tick kernel times of the final protocol form (rocprofv3 kernel trace of tools/protocol_probe.py).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4tk
rm -rf $O; mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
    python3 -u tools/protocol_probe.py --modes hybrid:0.125 > $O/run.log 2>&1
rc=$?; echo "prof rc=$rc"; grep hybrid $O/run.log | cut -c1-100
python3 tools/trace_protocol.py $O/prof 200 ticks > $O/ticks.txt; head -3 $O/ticks.txt
rm -rf $O/prof
