#!/bin/bash
# Election knob sweep on one MI355X: tools/elect_ab.py at 10M agents, one process per setting
# (libswarm reads its SWARM_* tuning once per process).  KNOBS: space-separated "VAR=val,VAR=val".
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/knobs_${TAG:-a}; mkdir -p $O
for k in ${KNOBS:-none}; do
  env_args=$(echo "$k" | tr ',' ' ')
  [ "$k" = "none" ] && env_args=""
  echo "== $k" >> $O/ab.log
  env $env_args timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so ${N:-10000000} >> $O/ab.log 2>&1 || { tail $O/ab.log; exit 1; }
done
cat $O/ab.log
