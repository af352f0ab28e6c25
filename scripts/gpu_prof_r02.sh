#!/bin/bash
# Round-2 evidence: rocprofv3 kernel trace + stats of the bench command itself,
# then PMC passes (one counter group per run) over a short search loop.
# Outputs under gpurun_out/r02prof/.  Each step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${PROF_NAME:-r02prof}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/bench.json 2> $OUT/bench.err || { echo trace failed; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_(band|flat)" --output-format csv -d $OUT/pmc_p$i -o pmc -- python3 $R/scripts/ablate.py ${CFG:-c3} > $OUT/pmc_p$i.log 2>&1 || { echo pmc pass $i failed; tail -5 $OUT/pmc_p$i.log; exit 1; }
done <<'CTRS'
TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
CTRS
echo pmc done
