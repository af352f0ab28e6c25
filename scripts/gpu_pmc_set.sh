#!/bin/bash
# the latency / pipe-utilisation PMC set of the config-3 search, one pass per line (gpurun_out/pmcs_p<i>)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  env ${PMC_ENV} timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_(pipe|band)" --output-format csv -d $OUT/pmcs_p$i -o pmc -- python3 $R/scripts/ablate.py ${CFG:-c3} > $OUT/pmcs_p$i.log 2>&1 || exit $?
done <<'CTRS'
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT
TD_TD_BUSY_sum TD_TC_STALL_sum
TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum
SQ_WAVES SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
CTRS
echo pmc set done
