#!/bin/bash
# Parity tests, then a small tuning sweep of the election gather (one process per setting).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-tune}
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=30 --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" gpurun_out/gpu_tests_$TAG.log | tail -12
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
IFS=';' read -ra CFG_LIST <<< "${CFGS:-frontier;dense}"
i=0
for cfg in "${CFG_LIST[@]}"; do
  i=$((i+1))
  read -r mode envs <<< "$cfg"
  name="${TAG}_${i}_${mode}"
  env $envs timeout -k 10 300 python -u bench.py --steps 2 --elect-mode $mode --cpu-baseline 0 \
      > gpurun_out/tune_$name.json 2> gpurun_out/tune_$name.err
  rc=$?; echo "cfg [$cfg] rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/tune_$name.json'));print(' value %.3e ms/step %.1f elect %.1f alloc %.2f dom_launch_ms %.4f frac %.3f rounds %d' % (d['value'], d['ms_per_step'], d['breakdown_ms']['elect'], d['breakdown_ms']['alloc'], d['roofline']['avg_launch_ms'], d['roofline']['frac'], d['config']['rounds_exec']))"
done
if [ "${PROF:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run \
      -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline 0 > gpurun_out/prof_$TAG.log 2>&1
  rc=$?; echo "rocprof rc=$rc"
  python - <<PY
import csv
rows=list(csv.DictReader(open('gpurun_out/prof_$TAG/run_kernel_stats.csv')))
for r in rows[:12]:
    print(f"{r['Name'][:70]:70s} calls={r['Calls']:>6s} avg_us={float(r['AverageNs'])/1e3:9.2f} pct={float(r['Percentage']):6.2f}")
PY
fi
