#!/bin/bash
# ELL rows A/B by round range: rocprofv3 kernel traces of tools/elect_ab.py at 10M agents with
# SWARM_ELL=0 (CSR), 1 (ELL in every sparse round), 2 (ELL in the agent-order tail only).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4ell2
rm -rf $O; mkdir -p $O
for e in 0 1 2; do
  SWARM_ELL=$e timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/ell$e -o run \
      -- python3 tools/elect_ab.py libswarm.so 10000000 > $O/ell$e.log 2>&1 || { tail $O/ell$e.log; exit 1; }
  grep "elect ms" $O/ell$e.log
  python3 tools/trace_ranges.py $(find $O/ell$e -name "run_kernel_trace.csv" | head -1) ell$e | tee -a $O/ranges.txt
  rm -rf $O/ell$e
done
for e in 2 0 2 0 1 2 0; do
  SWARM_ELL=$e timeout -k 10 200 python3 -u tools/elect_ab.py libswarm.so 10000000 > $O/ab_tmp.log 2>&1 \
      || { cat $O/ab_tmp.log; exit 1; }
  echo "ell=$e $(tail -1 $O/ab_tmp.log)" | tee -a $O/ab.log
done
