#!/bin/bash
# GPU box: -m gpu suite, short bench, option sweep on c3 (T = 8, 16).
set -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-queries 0 --e2e-batches 5 > "$out/bench.json" 2> "$out/bench.err" || exit $?
timeout -k 10 400 python -u scripts/opt_sweep.py --config c3 --terms 8,16 --sets '[{}, {"flat_bw": 4}, {"flat_bw": 2}, {"items_per_wave": 16}, {"claim_m": 8}, {"claim_ch": 2}]' > "$out/sweep.jsonl" 2> "$out/sweep.err"
