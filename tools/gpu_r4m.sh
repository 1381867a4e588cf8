#!/bin/bash
# Protocol ticks: GPU parity tests, then the previous build (4 launches per tick) against the
# role-split k_tick (2 launches) at bench scale, at several receive-role grid sizes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_protocol.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for cfg in "libswarm_oldfsm.so 0" "libswarm.so 0" "libswarm.so 0" "libswarm_oldfsm.so 0"; do
  set -- $cfg
  SWARM_FSM_RECV_WGS=$2 timeout -k 10 200 python3 -u tools/protocol_probe.py --lib $1 --modes hybrid:0.125 > $O/ab_tmp.log 2>&1 || { cat $O/ab_tmp.log; exit 1; }
  echo "recv_wgs=$2 $(grep -h hybrid $O/ab_tmp.log | cut -c1-80) $(tail -1 $O/ab_tmp.log | cut -c1-60)" | tee -a $O/ab.log
done
bash tools/gpu_r4n.sh
