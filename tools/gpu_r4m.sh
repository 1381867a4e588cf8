#!/bin/bash
# Protocol ticks: GPU parity tests, then A/B at bench scale (tools/protocol_probe.py, hybrid 0.125):
# the round-4 build (libswarm_oldfsm.so, 4 launches per tick) and the current one at several
# heavy-tick thresholds (SWARM_FSM_HEAVY), then the current build's per-tick kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4m
rm -rf $O; mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_protocol.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/tests.log; [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for cfg in ${CFGS:-"libswarm.so -1" "libswarm.so 0.005" "libswarm.so 0.01" "libswarm.so 0.02" "libswarm.so 0.05" "libswarm.so -1" "libswarm.so 0.01"}; do
  set -- $cfg
  SWARM_FSM_HEAVY=$2 timeout -k 10 200 python3 -u tools/protocol_probe.py --lib $1 --modes hybrid:0.125 > $O/ab_tmp.log 2>&1 || { cat $O/ab_tmp.log; exit 1; }
  echo "$1 heavy=$2 $(grep -h hybrid $O/ab_tmp.log | cut -c1-60)" | tee -a $O/ab.log
done
if [ "${PROF:-1}" = "1" ]; then bash tools/gpu_r4n.sh; fi
