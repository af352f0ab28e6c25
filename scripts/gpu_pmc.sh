#!/bin/bash
# PMC passes for the score kernels under several env variants (VARIANTS as in gpu_ablate.sh)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for var in ${VARIANTS:-BM25_TILE_SHIFT=13}; do
  tag=$(echo "$var" | tr ',=' '__')
  i=0
  while read -r ctrs; do
    [ -z "$ctrs" ] && continue
    i=$((i+1))
    env $(echo "$var" | tr ',' ' ') timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_" --output-format csv -d $OUT/pmc_$tag/p$i -o pmc -- python3 $R/scripts/ablate.py c3 > $OUT/pmc_$tag.p$i.log 2>&1 || exit $?
  done <<'CTRS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM GRBM_GUI_ACTIVE
FETCH_SIZE
TCC_HIT_sum TCC_MISS_sum
CTRS
done
echo pmc done
