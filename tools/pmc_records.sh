#!/bin/bash
# PMC passes over the record tail at 1M agents (tools/records_ab.py, records on): instruction mix,
# wave cycles and LDS waits of k_rec_tiles.  One rocprofv3 --pmc pass per counter group.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_rec_${TAG:-a}; mkdir -p $O
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
         "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-include-regex k_rec_tiles --output-format csv -d $O/p$i -o run \
      -- python3 tools/records_ab.py 1000000 1 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections, os
O = os.environ.get("O_DIR")
PY
for f in $O/p*/run_counter_collection.csv; do
  python3 -c "
import csv,collections,sys
t=collections.defaultdict(float); n=collections.Counter()
for r in csv.DictReader(open('$f')):
    if 'k_rec_tiles' not in r['Kernel_Name']: continue
    t[r['Counter_Name']]+=float(r['Counter_Value']); n[r['Counter_Name']]+=1
for k in sorted(t): print(k, '%.4g'%t[k], 'dispatch-rows', n[k])
"
done
