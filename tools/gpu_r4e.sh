#!/bin/bash
# Round 4: protocol storm-tick pull (hybrid) -- tests, then the f2 probe at 10M agents push vs hybrid.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_protocol.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/protocol_tests_r4e.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/protocol_tests_r4e.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/protocol_probe.py --agents 10000000 --ticks 200 > gpurun_out/protocol_probe_r4e.log 2>&1
rc=$?; echo "probe rc=$rc"; grep -v amdgpu.ids gpurun_out/protocol_probe_r4e.log | tail -8
exit $rc
