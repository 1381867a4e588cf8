#!/bin/bash
# Round-end evidence on one MI355X: GPU tests, smoke, bench, rocprofv3 kernel stats and PMC
# HBM-traffic passes of the same bench command.  Everything lands in gpurun_out/round_$TAG/;
# copy what is to be judged into profiles/<round>/.  Each GPU step has its own time limit and
# the script stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r1}
O=gpurun_out/round_$TAG
mkdir -p $O
step() { echo "[$(date +%T)] $*"; }
step tests
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
step smoke
timeout -k 10 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail $O/smoke.log; exit 1; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  step pmc $ctr
  timeout -s KILL 300 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_$ctr -o run \
      -- python3 bench.py --steps 1 --warmup 0 --cpu-baseline 0 --roofline-rounds 5 > $O/pmc_$ctr.log 2>&1 \
      || { tail $O/pmc_$ctr.log; exit 1; }
done
python3 tools/pmc_summary.py $O/pmc_FETCH_SIZE $O/pmc_WRITE_SIZE > $O/pmc_traffic.json
# the bench line's traffic figures come from profiles/LATEST: point it (in this box's copy of the
# tree) at this run's PMC summary, so bench.json cites the same run
mkdir -p profiles/$TAG && cp $O/pmc_traffic.json profiles/$TAG/ && echo $TAG > profiles/LATEST
step bench
timeout -k 10 500 python3 -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.log || { tail $O/bench.log; exit 1; }
step rocprof
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run \
    -- python3 bench.py --steps 10 --warmup 2 --cpu-baseline 0 --rows 0 > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
step done
