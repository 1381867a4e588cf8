#!/bin/bash
# k_tick row-walk chunk A/B, mailing chunk: 8 hearer loads in flight (libswarm.so) against 12 and 16.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4mc
rm -rf $O; mkdir -p $O
for lib in libswarm.so libswarm_mc12.so libswarm_mc16.so libswarm.so libswarm_mc12.so libswarm_mc16.so; do
  timeout -k 10 200 python3 -u tools/protocol_probe.py --lib $lib --modes hybrid:0.125 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  echo "$lib $(grep -h hybrid $O/tmp.log | cut -c1-60) $(tail -1 $O/tmp.log | grep -o 'counts_sums.*')" | tee -a $O/ab.log
done
