#!/bin/bash
# Batch plan of a 10M election (SWARM_BATCH_LOG) next to its kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
SWARM_XCD_TAIL=${XT:-0} SWARM_BATCH_LOG=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
    python3 -u tools/elect_ab.py libswarm.so 10000000 > $O/run.log 2>&1
rc=$?; echo "rc=$rc"; grep "elect ms" $O/run.log
