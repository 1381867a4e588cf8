#!/bin/bash
# One-launch ticks (inline mail only): protocol + smoke-level GPU tests, tick time, bench f2 row.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4inl3
rm -rf $O; mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_protocol.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for rep in 1 2; do
  timeout -k 10 300 python3 -u tools/protocol_probe.py --modes hybrid:0.125 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  grep -h '"hybrid' $O/tmp.log | cut -c1-80 | tee -a $O/ab.log
done
