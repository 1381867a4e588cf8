#!/bin/bash
# Per-launch durations of the election's round kernels (rocprofv3 kernel trace), with the rounds each
# single-XCD tail launch covered (SWARM_XCD_LOG), 10M agents: tail off, then on at $MINC changes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
for xt in 0 1; do
  SWARM_XCD_TAIL=$xt SWARM_XCD_LOG=1 SWARM_XCD_MIN_CHANGES=${MINC:-2000} timeout -k 10 300 rocprofv3 --kernel-trace \
      --output-format csv -d $O/prof$xt -o run -- python3 -u tools/elect_ab.py libswarm.so 10000000 > $O/run$xt.log 2>&1
  rc=$?; echo "xcd=$xt rc=$rc"; grep "elect ms" $O/run$xt.log
  [ $rc -eq 0 ] || exit $rc
done
