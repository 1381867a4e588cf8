set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/pipe_probe.py 100000 1000000 10000000 > gpurun_out/pipe_probe_a.log 2>&1
rc=$?; echo "probe rc=$rc"; cat gpurun_out/pipe_probe_a.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_pipe.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pipe_tests_a.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pipe_tests_a.log
exit $rc
