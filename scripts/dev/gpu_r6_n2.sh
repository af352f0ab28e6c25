#!/bin/bash
# Final probe (one-collective W = 1, 2, 4, 8; two-collective W = 8; rank-3 trace)
# and an N = 2 gloo rehearsal of bench.py's multi-rank step on the one GPU.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_pf2}; mkdir -p $OUT; cd $R
NAME=${NAME:-r6_pf2} bash scripts/dev/gpu_r6_probe_final.sh || exit 1
timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 5 --warmup 2 --cpu-queries 0 --e2e-batches 0 > $OUT/bench_n2_gloo.json 2> $OUT/bench_n2_gloo.err || { echo n2 failed; tail -20 $OUT/bench_n2_gloo.err; exit 1; }
cat $OUT/bench_n2_gloo.json | cut -c1-600
