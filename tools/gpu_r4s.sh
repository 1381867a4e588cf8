#!/bin/bash
# Per-round election log at 10M agents (tools/round_log.py: round, changes, marked, edges, kind, us).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4s
rm -rf $O; mkdir -p $O
timeout -k 10 300 python3 -u tools/round_log.py 10000000 libswarm.so $O/rounds.log > $O/run.log 2>&1
rc=$?; echo "rc=$rc"; tail -8 $O/run.log
