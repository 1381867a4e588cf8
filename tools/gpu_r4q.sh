#!/bin/bash
# C2-sized election (100k agents): wall time and its kernel trace (per-round kernels, gaps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4q
rm -rf $O; mkdir -p $O
timeout -k 10 120 python3 -u tools/elect_ab.py libswarm.so 100000 > $O/wall.log 2>&1; echo "wall rc=$?"; tail -1 $O/wall.log
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
    python3 -u tools/elect_ab.py libswarm.so 100000 > $O/run.log 2>&1
echo "prof rc=$?"
