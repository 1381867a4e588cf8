#!/bin/bash
# Codec GPU tests and timing on the current build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4cd
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_codec.py tests/test_physics.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for i in 1 2; do timeout -k 10 200 python3 -u tools/codec_probe.py | tail -1; done
