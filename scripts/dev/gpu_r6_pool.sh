#!/bin/bash
# Pooled tile bounds A/B: GPU tests, c3 bench with BM25_BOUND_POOL=1/0, W=8
# probe (one-collective) kernel trace with the pooled world bounds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_pool}; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_gpu.log | tail -30; exit 1; }
tail -1 $OUT/pytest_gpu.log
for p in 1 0 1 0; do
  BM25_BOUND_POOL=$p timeout -k 10 300 python -u bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/c3_pool$p.json 2> $OUT/c3_pool$p.err || { echo bench failed; tail -5 $OUT/c3_pool$p.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/c3_pool$p.json').read().strip().splitlines()[-1]); print('pool', $p, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['score_kernels'])"
done
export TMPDIR=/tmp
for p in 1 0; do
  ( cd /tmp; BM25_BOUND_POOL=$p PROBE_ITERS=10 PROBE_RANKS=1 PROBE_WORLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8_pool$p -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_w8_pool$p.jsonl 2> $OUT/probe_w8_pool$p.err ) || { echo probe failed; tail -5 $OUT/probe_w8_pool$p.err; exit 1; }
done
( cd /tmp; timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -o run -- python3 $R/bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/c3_rocprof.json 2> $OUT/c3_rocprof.err ) || { echo trace failed; exit 1; }
PROBE_WORLD=1 timeout -k 10 600 python -u scripts/shard_probe.py 1 8 > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err || { echo probe2 failed; tail -5 $OUT/shard_probe.err; exit 1; }
cat $OUT/shard_probe.jsonl | cut -c1-400
