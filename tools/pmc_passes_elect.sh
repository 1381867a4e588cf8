set -u
export TMPDIR=/tmp
O=gpurun_out/pmc2; mkdir -p $O
i=0
for P in "SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM GRBM_GUI_ACTIVE" "TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVES SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --output-format csv -d $O/p$i -o run -- python3 tools/elect_once.py > $O/p$i.log 2>&1 || { tail -5 $O/p$i.log; exit 1; }
done
echo done
