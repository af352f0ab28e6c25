#!/bin/bash
# Final round-6 probe: one-collective W = 1, 2, 4, 8 and the two-collective W = 8,
# two passes per rank; a W = 8 kernel trace of rank 3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_pf}; mkdir -p $OUT; cd $R
PROBE_PASSES=2 PROBE_WORLD=1 timeout -k 10 900 python -u scripts/shard_probe.py 1 2 4 8 > $OUT/shard_probe_world.jsonl 2> $OUT/shard_probe_world.err || { echo probe failed; tail -5 $OUT/shard_probe_world.err; exit 1; }
PROBE_PASSES=2 timeout -k 10 600 python -u scripts/shard_probe.py 8 > $OUT/shard_probe_two.jsonl 2> $OUT/shard_probe_two.err || { echo probe2 failed; tail -5 $OUT/shard_probe_two.err; exit 1; }
python - <<PY
import json
for f in ("world", "two"):
    for l in open("$OUT/shard_probe_%s.jsonl" % f):
        d = json.loads(l); print(f, d["W"], [r["ms"] for r in d["per_rank"]], d["projected_ms"], d.get("speedup_vs_W1"), d.get("list_sizes"))
PY
export TMPDIR=/tmp
( cd /tmp; PROBE_ITERS=10 PROBE_RANKS=3 PROBE_WORLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8 -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_w8_trace.jsonl 2> $OUT/probe_w8_trace.err ) || { echo trace failed; exit 1; }
