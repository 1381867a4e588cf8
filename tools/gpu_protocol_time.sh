#!/bin/bash
# Per-tick k_tick durations of tools/protocol_pmc.py's 200-tick scenario by tick class
# (tools/protocol_time_join.py).  Output: gpurun_out/ptime_$TAG.json.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-pt}
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ptrace_$TAG -o run \
    -- python3 tools/protocol_pmc.py ${TAG} > gpurun_out/ptrace_$TAG.log 2>&1 || { tail gpurun_out/ptrace_$TAG.log; exit 1; }
python3 tools/protocol_time_join.py gpurun_out/ptrace_$TAG gpurun_out/protocol_ticks_${TAG}.json > gpurun_out/ptime_$TAG.json
python3 -c "import json; d=json.load(open('gpurun_out/ptime_${TAG}.json')); d.pop('per_tick_us'); print(json.dumps(d))"
