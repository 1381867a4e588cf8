#!/bin/bash
# Inline mail A/B: protocol GPU tests with SWARM_FSM_INLINE=1 (k_tick mails its own senders, no
# k_mail launch) and with the default, then tick time both ways at several storm fractions.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r4inl
rm -rf $O; mkdir -p $O
SWARM_FSM_INLINE=1 timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_protocol.py > $O/tests_inline.log 2>&1
rc=$?; echo "pytest inline rc=$rc"; tail -2 $O/tests_inline.log; [ $rc -eq 0 ] || { tail -40 $O/tests_inline.log; exit $rc; }
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_protocol.py > $O/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/tests.log; [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for inl in 0 1 0 1; do
  SWARM_FSM_INLINE=$inl timeout -k 10 300 python3 -u tools/protocol_probe.py --modes hybrid:0.125,hybrid:0.25,hybrid:0.5 > $O/tmp.log 2>&1 || { cat $O/tmp.log; exit 1; }
  for m in 0.125 0.25 0.5; do
    echo "inline=$inl $(grep -h "hybrid_$m\"" $O/tmp.log | cut -c1-60) $(tail -1 $O/tmp.log | grep -o 'same_counts.*')" | tee -a $O/ab.log
  done
done
