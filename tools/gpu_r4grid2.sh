#!/bin/bash
# One-launch ticks: sweep / receive-role grid re-sweep (SWARM_FSM_SWEEP_WGS / SWARM_FSM_RECV_WGS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4grid2
rm -rf $O; mkdir -p $O
for g in ${GRIDS:-"2048 1280" "2048 1024" "2048 1536" "3072 1536" "1536 1280" "2048 1280" "2560 1280" "2048 768"}; do
  set -- ${g/_/ }
  SWARM_FSM_SWEEP_WGS=$1 SWARM_FSM_RECV_WGS=$2 timeout -k 10 200 python3 -u tools/protocol_probe.py --modes hybrid:0.125 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "sweep=$1 recv=$2 $(grep -h hybrid $O/tmp.log | cut -c1-60)" | tee -a $O/ab.log
done
