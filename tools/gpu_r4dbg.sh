#!/bin/bash
# DEBUG (results invalid when a role is skipped): k_tick per-tick durations with both roles, the
# receive role only (sweep skipped) and the sweep role only (receive skipped).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
for dbg in 0 1 2; do
  O=gpurun_out/r4dbg$dbg; rm -rf $O; mkdir -p $O
  SWARM_FSM_DEBUG_SKIP=$dbg timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- \
      python3 -u tools/protocol_probe.py --modes hybrid:0.125 --ticks 100 > $O/run.log 2>&1
  echo "dbg=$dbg rc=$?"; python3 tools/trace_protocol.py $O/prof 100 | head -3
done
