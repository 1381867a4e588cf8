#!/bin/bash
# Round 4: work stealing in busy sparse rounds -- A/B at 10M / 1M agents, then the election parity tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-steal}
out=gpurun_out/steal_ab_$TAG.log
: > $out
for cfg in "SWARM_STEAL=0" "SWARM_STEAL=1" "SWARM_STEAL=1 SWARM_STEAL_KEEP=1" "SWARM_STEAL=1 SWARM_STEAL_KEEP=3" \
           "SWARM_STEAL=1 SWARM_STEAL_TRIES=8" "SWARM_STEAL=0" "SWARM_STEAL=1"; do
    echo "== $cfg" >> $out
    env $cfg timeout -k 10 120 python -u tools/elect_ab.py libswarm.so 10000000 >> $out 2>&1 || { echo "fail $cfg"; cat $out; exit 1; }
done
for cfg in "SWARM_STEAL=0" "SWARM_STEAL=1"; do
    echo "== 1M $cfg" >> $out
    env $cfg timeout -k 10 120 python -u tools/elect_ab.py libswarm.so 1000000 >> $out 2>&1 || { echo "fail $cfg"; cat $out; exit 1; }
done
grep -v amdgpu.ids $out
timeout -k 10 900 python -u -m pytest tests/test_scale.py tests/test_elect_sizes.py tests/test_gpu_parity.py tests/test_compact_cols.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/steal_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/steal_tests_$TAG.log
exit $rc
