#!/bin/bash
# C4 auction: wall time and kernel trace (per-kernel totals of the last call, gaps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4t
rm -rf $O; mkdir -p $O
timeout -k 10 200 python3 -u tools/auction_probe.py > $O/wall.log 2>&1; echo "wall rc=$?"; tail -1 $O/wall.log
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
    python3 -u tools/auction_probe.py > $O/run.log 2>&1
echo "prof rc=$?"
