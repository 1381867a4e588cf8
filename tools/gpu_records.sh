#!/bin/bash
# Record tail on one MI355X: its GPU parity tests, then A/B timings at 1M and 10M agents.  Stops at
# the first crash-like exit (fault / abort / timeout); test failures still let the timings run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/rec_${TAG:-a}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_records.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 $O/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
SWARM_REC_DEBUG=1 timeout -k 10 300 python3 -u tools/records_ab.py 1000000 0,1,early > $O/ab_1m.json 2> $O/ab_1m.err
rc=$?; echo "ab1m rc=$rc"; tail -1 $O/ab_1m.json; tail -3 $O/ab_1m.err
[ $rc -eq 0 ] || exit $rc
SWARM_REC_DEBUG=1 timeout -k 10 300 python3 -u tools/records_ab.py 10000000 1 > $O/ab_10m.json 2> $O/ab_10m.err
rc=$?; echo "ab10m rc=$rc"; tail -1 $O/ab_10m.json; tail -3 $O/ab_10m.err
exit $rc
