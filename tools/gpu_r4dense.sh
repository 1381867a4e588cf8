#!/bin/bash
# Dense-round grid cap re-sweep (SWARM_DENSE_BLOCKS), 10M agents, tools/elect_ab.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4dense
rm -rf $O; mkdir -p $O
for v in ${VALS:-2048 1024 4096 8192 2048 1536 3072 2048}; do
  SWARM_DENSE_BLOCKS=$v timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so 10000000 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "dense_blocks=$v $(tail -1 $O/tmp.log)" | tee -a $O/ab.log
done
