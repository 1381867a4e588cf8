#!/bin/bash
# Per-tick HBM traffic of the protocol ticks (f2): FETCH_SIZE and WRITE_SIZE passes of
# tools/protocol_pmc.py, joined per tick by tools/protocol_pmc_join.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pp}
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/ppmc_${TAG}_$ctr -o run \
      -- python3 tools/protocol_pmc.py ${TAG}_$ctr > gpurun_out/ppmc_${TAG}_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc"; tail -1 gpurun_out/ppmc_${TAG}_$ctr.log
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/protocol_pmc_join.py gpurun_out/ppmc_${TAG}_FETCH_SIZE gpurun_out/ppmc_${TAG}_WRITE_SIZE \
    gpurun_out/protocol_ticks_${TAG}_FETCH_SIZE.json > gpurun_out/ppmc_${TAG}.json
python3 -c "import json; d=json.load(open('gpurun_out/ppmc_${TAG}.json')); d.pop('per_tick'); print(json.dumps(d))"
