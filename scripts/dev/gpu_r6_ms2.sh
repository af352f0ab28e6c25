#!/bin/bash
# merge_sorted window: merge tests, c3 selection counters, three W = 8 rank-3 traces.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_ms2}; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "merge or world_bounds or sharded or config4" > $OUT/pytest_sel.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_sel.log | tail -30; exit 1; }
tail -1 $OUT/pytest_sel.log
timeout -k 10 300 python -u scripts/dev/c3_stats.py > $OUT/c3_stats.txt 2>&1 || { echo stats failed; tail -5 $OUT/c3_stats.txt; exit 1; }
tail -1 $OUT/c3_stats.txt
NAME=${NAME:-r6_ms2} bash scripts/dev/gpu_r6_mstrace.sh
