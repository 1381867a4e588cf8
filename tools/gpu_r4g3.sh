#!/bin/bash
# Second grid A/B pass (pairs "sweep recv").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4g3
rm -rf $O; mkdir -p $O
for cfg in "4096 2048" "2048 1536" "2048 1280" "3072 1536" "4096 2048" "2048 1536" "2048 1280" "3072 1536"; do
  set -- $cfg
  SWARM_FSM_SWEEP_WGS=$1 SWARM_FSM_RECV_WGS=$2 timeout -k 10 200 python3 -u tools/protocol_probe.py --modes hybrid:0.125 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "sweep=$1 recv=$2 $(grep -h hybrid $O/tmp.log | cut -c1-60)" | tee -a $O/ab.log
done
