#!/bin/bash
# HBM traffic of the election kernels: one rocprofv3 --pmc pass per counter (FETCH_SIZE needs 3
# TCC slots, WRITE_SIZE 2: they cannot share a pass), kernel trace only, no other domains.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pmc}
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/pmc_${TAG}_$ctr -o run \
      -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --roofline-rounds 5 \
      > gpurun_out/pmc_${TAG}_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc_${TAG}_FETCH_SIZE gpurun_out/pmc_${TAG}_WRITE_SIZE > gpurun_out/pmc_${TAG}.json
cat gpurun_out/pmc_${TAG}.json
