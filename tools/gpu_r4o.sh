#!/bin/bash
# Storm threshold A/B at bench scale: hybrid pull fractions (tools/protocol_probe.py, 10M agents).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4o
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u tools/protocol_probe.py --modes ${MODES:-hybrid:0.125,hybrid:0.05,hybrid:0.02,hybrid:0.01,hybrid:0.005,push:0,hybrid:0.125} > $O/ab.log 2>&1
rc=$?; echo "rc=$rc"; cut -c1-150 $O/ab.log
