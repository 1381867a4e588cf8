#!/bin/bash
# Codec encode forms on one MI355X: kernel trace + stats and the HBM counters (FETCH_SIZE, WRITE_SIZE, one
# pass each) of tools/codec_probe.py for SWARM_ENC_PASSES=1 (one pass) and 3 (tile / base / place).
# Output: gpurun_out/codec_prof_$TAG/.  Each GPU step has its own time limit; the first failure ends it.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r5}
O=gpurun_out/codec_prof_$TAG
mkdir -p $O
for p in ${PASSES:-1 3}; do
  echo "[$(date +%T)] passes=$p trace"
  SWARM_ENC_PASSES=$p timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$p -o run \
      -- python3 tools/codec_probe.py ${M:-10000000} ${WIDTH:-narrow} > $O/p${p}_trace.log 2>&1 || { tail $O/p${p}_trace.log; exit 1; }
  for ctr in FETCH_SIZE WRITE_SIZE; do
    echo "[$(date +%T)] passes=$p pmc $ctr"
    SWARM_ENC_PASSES=$p timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $O/p${p}_$ctr -o run \
        -- python3 tools/codec_probe.py ${M:-10000000} ${WIDTH:-narrow} > $O/p${p}_$ctr.log 2>&1 || { tail $O/p${p}_$ctr.log; exit 1; }
  done
done
echo "[$(date +%T)] done"
