#!/bin/bash
# W = 8 one-collective probe: REST item width (BM25_FLAT_BW) A/B, all ranks.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_bw}; mkdir -p $OUT; cd $R
for bw in ${BWS:-0 4 0 4}; do
  BM25_FLAT_BW=$bw PROBE_ITERS=20 PROBE_WORLD=1 timeout -k 10 600 python -u scripts/shard_probe.py 8 > $OUT/probe_bw$bw.jsonl 2> $OUT/probe_bw$bw.err || { echo probe failed; tail -5 $OUT/probe_bw$bw.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/probe_bw$bw.jsonl').read().strip().splitlines()[-1]); print('bw', $bw, [r['ms'] for r in d['per_rank']], d['max_rank_ms'])"
done
