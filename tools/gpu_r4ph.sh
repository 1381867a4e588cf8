#!/bin/bash
# Physics grid A/B (SWARM_PHYS_WGS; tools/physics_probe.py, 10M agents).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4ph
rm -rf $O; mkdir -p $O
for w in 8192 1536 2048 3072 4096 16384 8192 1536 2048 3072 4096 16384; do
  SWARM_PHYS_WGS=$w timeout -k 10 200 python3 -u tools/physics_probe.py 10000000 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "wgs=$w $(tail -1 $O/tmp.log)" | tee -a $O/ab.log
done
for w in 4096 1024 2048 8192 16384 4096 1024 2048 8192 16384; do
  SWARM_CODEC_WGS=$w timeout -k 10 200 python3 -u tools/codec_probe.py > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "codec_wgs=$w $(tail -1 $O/tmp.log)" | tee -a $O/ab.log
done
