#!/bin/bash
# Dev pass: ablation sweep (VARIANTS, one process each) then PMC passes on the
# score kernels (one counter group per rocprofv3 run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
for var in ${VARIANTS:-BM25_ABLATE=0}; do
  envs=$(echo "$var" | tr ',' ' ')
  env $envs timeout -k 10 180 python scripts/ablate.py ${CFG:-c3} | sed "s/}/, \"variant\": \"$var\"}/" >> $OUT/ablate.jsonl 2>> $OUT/ablate.err || { echo "ablate $var failed"; tail $OUT/ablate.err; exit 1; }
done
cat $OUT/ablate.jsonl
[ -n "$NO_PMC" ] && exit 0
export TMPDIR=/tmp
cd /tmp
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_" --output-format csv -d $OUT/pmc$i -o pmc -- python3 $R/scripts/ablate.py ${CFG:-c3} > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail $OUT/pmc$i.log; exit 1; }
done <<CTRS
${PMC1:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS}
${PMC2:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE}
${PMC3:-FETCH_SIZE}
${PMC4:-TCC_HIT_sum TCC_MISS_sum}
CTRS
python3 $R/scripts/prof_summary.py $OUT
