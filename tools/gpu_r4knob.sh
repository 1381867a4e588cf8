#!/bin/bash
# Election knob re-sweep on the round-4 tree (tools/elect_ab.py at 10M agents, same box): the
# interleaved -> agent-order switch, the stamp block size, the sparse grid and the dense rounds.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4knob
rm -rf $O; mkdir -p $O
run() {  # label, env assignments...
  local label=$1; shift
  env "$@" timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so 10000000 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "$label $(tail -1 $O/tmp.log)" | tee -a $O/ab.log
}
run base X=0
for v in 2000 4000 16000 32000; do run il=$v SWARM_IL_MIN_CHANGES=$v; done
run base X=0
for v in 3 4 6 7; do run bshift=$v SWARM_STAMP_BSHIFT=$v; done
run base X=0
for v in 1024 1536 3072; do run sparse=$v SWARM_SPARSE_BLOCKS=$v; done
run base X=0
for v in 8 10; do run dense=$v SWARM_DENSE_ROUNDS=$v; done
run base X=0
