#!/bin/bash
# Round 4: kernel split of the protocol ticks (hybrid) under rocprofv3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_fsm
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fsm -o fsm -- python3 tools/protocol_probe.py --modes hybrid:0.125 > gpurun_out/prof_fsm/probe.log 2>&1
rc=$?; echo "rc=$rc"; find gpurun_out/prof_fsm -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof_fsm -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -c1-60,200-400 "$f" | head -12
exit $rc
