#!/bin/bash
# merge_sorted batched loads: its tests, the W = 1 / 8 one-collective probe
# (two passes per rank, list sizes), a W = 8 rank-0 kernel trace.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_ms}; mkdir -p $OUT; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 --timeout-method thread -k "merge_sorted or world_bounds or global_theta or merge_paths or sharded" > $OUT/pytest_sel.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_sel.log | tail -30; exit 1; }
tail -1 $OUT/pytest_sel.log
PROBE_PASSES=2 PROBE_WORLD=1 timeout -k 10 900 python -u scripts/shard_probe.py 1 8 > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err || { echo probe failed; tail -5 $OUT/shard_probe.err; exit 1; }
python - <<PY
import json
for l in open("$OUT/shard_probe.jsonl"):
    d = json.loads(l); print(d["W"], [r["ms"] for r in d["per_rank"]], d["projected_ms"], d.get("speedup_vs_W1"), d.get("list_sizes"))
PY
export TMPDIR=/tmp
( cd /tmp; PROBE_ITERS=10 PROBE_RANKS=3 PROBE_WORLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8 -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_w8_trace.jsonl 2> $OUT/probe_w8_trace.err ) || { echo trace failed; exit 1; }
