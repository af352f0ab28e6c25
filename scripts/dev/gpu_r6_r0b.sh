#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_r0b}; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "world_bounds or theta_bound" > $OUT/pytest_sel.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_sel.log | tail -30; exit 1; }
tail -1 $OUT/pytest_sel.log
bash scripts/dev/gpu_r6_r0.sh
