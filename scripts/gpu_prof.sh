#!/bin/bash
# rocprofv3: kernel-trace stats of a short bench run, then PMC passes (one
# counter group per run, kernel-trace only alongside --pmc) on scripts/ablate.py.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps ${STEPS:-10} --warmup 3 --cpu-queries 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || exit $?
[ -n "$NO_PMC" ] && exit 0
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex score_tiles --output-format csv -d $OUT/pmc$i -o pmc -- python3 $R/scripts/ablate.py c3 > $OUT/pmc$i.log 2>&1 || exit $?
done <<'CTRS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum
TCC_EA0_RDREQ_sum
CTRS
echo prof done
