#!/bin/bash
# Physics step A/B over libswarm builds ($LIBS; tools/physics_probe.py, 10M agents).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4x
rm -rf $O; mkdir -p $O
for lib in ${LIBS:-libswarm.so libswarm_ph2_8.so libswarm_ph6_8.so libswarm_ph8_8.so libswarm.so libswarm_ph2_8.so libswarm_ph6_8.so libswarm_ph8_8.so}; do
  timeout -k 10 200 python3 -u tools/physics_probe.py 10000000 $lib > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "$lib $(tail -1 $O/tmp.log)" | tee -a $O/ab.log
done
