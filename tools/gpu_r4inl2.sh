#!/bin/bash
# Inline mail: storm fraction sweep, and per-tick kernel times (rocprofv3 trace) of both forms.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4inl2
rm -rf $O; mkdir -p $O
for inl in 1 0; do
  SWARM_FSM_INLINE=$inl timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof$inl -o run \
      -- python3 tools/protocol_probe.py --modes hybrid:0.125 > $O/prof$inl.log 2>&1 || { tail $O/prof$inl.log; exit 1; }
  python3 tools/trace_protocol.py $O/prof$inl 200 ticks > $O/ticks$inl.txt; head -3 $O/ticks$inl.txt
  rm -rf $O/prof$inl
done
for rep in 1 2; do
  SWARM_FSM_INLINE=1 timeout -k 10 300 python3 -u tools/protocol_probe.py --modes hybrid:0.0625,hybrid:0.09,hybrid:0.125,hybrid:0.18 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  grep -h '"hybrid' $O/tmp.log | cut -c1-60 | sed 's/^/inline=1 /' | tee -a $O/ab.log
done
