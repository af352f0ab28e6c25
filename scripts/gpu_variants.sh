#!/bin/bash
# dev: time variant builds (exp/libbm25mi_*.so) on the config-3 search, one
# child process per library (scripts/variant_lib_time.py); $VLIBS lists them.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 1000 python scripts/variant_lib_time.py $VLIBS | tee $R/gpurun_out/variants.jsonl
