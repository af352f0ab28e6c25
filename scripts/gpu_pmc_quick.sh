#!/bin/bash
# one PMC pass (CTRS) of the config-3 search per env variant (VARIANTS); csv under gpurun_out/pmcq_<variant>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
export TMPDIR=/tmp
cd /tmp
for var in ${VARIANTS:-BM25_BAND=8}; do
  tag=$(echo "$var" | tr ',=' '__')
  env $(echo "$var" | tr ',' ' ') timeout -s KILL 300 rocprofv3 --pmc ${CTRS:-TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum} --kernel-include-regex "score_pipe" --output-format csv -d $OUT/pmcq_$tag -o pmc -- python3 $R/scripts/ablate.py ${CFG:-c3} > $OUT/pmcq_$tag.log 2>&1 || exit $?
done
echo pmc done
