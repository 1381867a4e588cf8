#!/bin/bash
# Same-box A/B runs: each argument is "ENV=VAL ... -- command args"; every run is timed and logged
# to gpurun_out/ab_$TAG.log (stops at the first failing run).  Example:
#   TAG=x bash tools/gpu_ab.sh "SWARM_TICK_XCD_GROUP=0 -- python3 tools/protocol_probe.py --modes hybrid:0.125"
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
LOG=gpurun_out/ab_$TAG.log
: > $LOG
for spec in "$@"; do
  envs=${spec%% -- *}; cmd=${spec#* -- }
  echo "=== $envs :: $cmd" | tee -a $LOG
  env $envs timeout -k 10 ${LIMIT:-300} $cmd >> $LOG 2>&1
  rc=$?; echo "rc=$rc" | tee -a $LOG
  [ $rc -eq 0 ] || exit $rc
done
grep -v "^\[" $LOG | tail -40
