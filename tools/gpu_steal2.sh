#!/bin/bash
# Round 4: work stealing restricted to the busiest rounds (SWARM_STEAL_MIN), fewer donor tries.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/steal_ab2.log
: > $out
for cfg in "SWARM_STEAL=0" "SWARM_STEAL_MIN=300000" "SWARM_STEAL_MIN=1000000" "SWARM_STEAL_MIN=2000000" \
           "SWARM_STEAL_MIN=300000 SWARM_STEAL_TRIES=1" "SWARM_STEAL_MIN=300000 SWARM_STEAL_KEEP=4" \
           "SWARM_STEAL_MIN=100000 SWARM_STEAL_TRIES=1 SWARM_STEAL_KEEP=4" "SWARM_STEAL=0"; do
    echo "== $cfg" >> $out
    env $cfg timeout -k 10 120 python -u tools/elect_ab.py libswarm.so 10000000 >> $out 2>&1 || { echo "fail $cfg"; cat $out; exit 1; }
done
grep -v amdgpu.ids $out
