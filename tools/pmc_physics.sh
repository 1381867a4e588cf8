#!/bin/bash
# VALU / memory counters of the physics step (tools/physics_probe.py), one rocprofv3 pass each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_phys; mkdir -p $O
i=0
for P in "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU_INT32 TA_TA_BUSY_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 tools/physics_probe.py 10000000 > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
echo done
