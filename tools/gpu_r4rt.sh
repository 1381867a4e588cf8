#!/bin/bash
# k_tick row-walk chunk A/B: 4 CSR entries per chunk (libswarm.so, 63 VGPRs, 8 waves per SIMD) against
# 8 (_rt8, 75 VGPRs, 6 waves) and 5 (_rt5, 66, 7); then grid settings of the 4-entry build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4rt
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_protocol.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for lib in libswarm.so libswarm_rt8.so libswarm_rt5.so libswarm.so libswarm_rt8.so libswarm_rt5.so; do
  timeout -k 10 200 python3 -u tools/protocol_probe.py --lib $lib --modes hybrid:0.125 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "$lib $(grep -h hybrid $O/tmp.log | cut -c1-60) $(tail -1 $O/tmp.log | grep -o 'counts_sums.*')" | tee -a $O/ab.log
done
for g in "2048 1280" "1536 768" "2048 768" "1536 1024" "2048 1280"; do
  set -- $g
  SWARM_FSM_SWEEP_WGS=$1 SWARM_FSM_RECV_WGS=$2 timeout -k 10 200 python3 -u tools/protocol_probe.py --modes hybrid:0.125 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "sweep=$1 recv=$2 $(grep -h hybrid $O/tmp.log | cut -c1-60)" | tee -a $O/ab.log
done
