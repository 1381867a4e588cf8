#!/bin/bash
# C4 auction kernel trace with the one-XCD batches on (SWARM_AUCTION_XCD=$XCD).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4v
rm -rf $O; mkdir -p $O
SWARM_AUCTION_XCD=${XCD:-512} timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
    python3 -u tools/auction_probe.py > $O/run.log 2>&1
echo "prof rc=$?"; tail -1 $O/run.log
