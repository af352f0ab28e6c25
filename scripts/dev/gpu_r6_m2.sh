#!/bin/bash
# Merge changes: GPU tests, W = 8 probe (two passes, all ranks), rank-3 trace, c3 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_m2}; mkdir -p $OUT; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_gpu.log | tail -30; exit 1; }
tail -1 $OUT/pytest_gpu.log
PROBE_PASSES=2 PROBE_WORLD=1 timeout -k 10 900 python -u scripts/shard_probe.py 1 8 > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err || { echo probe failed; tail -5 $OUT/shard_probe.err; exit 1; }
python - <<PY
import json
for l in open("$OUT/shard_probe.jsonl"):
    d = json.loads(l); print(d["W"], [r["ms"] for r in d["per_rank"]], d["projected_ms"], d.get("speedup_vs_W1"))
PY
export TMPDIR=/tmp
( cd /tmp; PROBE_ITERS=10 PROBE_RANKS=3 PROBE_WORLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8 -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_w8_trace.jsonl 2> $OUT/probe_w8_trace.err ) || { echo trace failed; exit 1; }
timeout -k 10 300 python -u bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/c3.json 2> $OUT/c3.err || { echo bench failed; exit 1; }
python -c "import json; d=json.loads(open('$OUT/c3.json').read().strip().splitlines()[-1]); print('c3', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])"
