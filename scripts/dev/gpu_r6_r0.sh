#!/bin/bash
# W = 8 one-collective probe: rank 0 vs rank 3, pooled bounds on / off.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_r0}; mkdir -p $OUT; cd $R
for p in 1 0; do
  BM25_BOUND_POOL=$p PROBE_PASSES=2 PROBE_RANKS=3,0 PROBE_WORLD=1 timeout -k 10 600 python -u scripts/shard_probe.py 8 > $OUT/probe_pool$p.jsonl 2> $OUT/probe_pool$p.err || { echo probe failed; tail -5 $OUT/probe_pool$p.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/probe_pool$p.jsonl').read().strip().splitlines()[-1]); print('pool', $p, [(r['rank'], r['ms']) for r in d['per_rank']], d.get('list_sizes'))"
done
