#!/bin/bash
# k_tick row-walk chunk A/B, sender IDs loaded with the outbox bytes (libswarm_eager.so) or after them.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4eg
rm -rf $O; mkdir -p $O
for lib in libswarm.so libswarm_eager.so libswarm.so libswarm_eager.so libswarm.so libswarm_eager.so; do
  timeout -k 10 200 python3 -u tools/protocol_probe.py --lib $lib --modes hybrid:0.125 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "$lib $(grep -h hybrid $O/tmp.log | cut -c1-60) $(tail -1 $O/tmp.log | grep -o 'counts_sums.*')" | tee -a $O/ab.log
done
