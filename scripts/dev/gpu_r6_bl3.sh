#!/bin/bash
# Block-merge threshold 512: W = 8 rank-3 trace, c2 bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_bl3}; mkdir -p $OUT; cd $R
export TMPDIR=/tmp
( cd /tmp; PROBE_ITERS=10 PROBE_RANKS=3 PROBE_WORLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8 -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_w8.jsonl 2> $OUT/probe_w8.err ) || { echo trace failed; exit 1; }
timeout -k 10 300 python -u bench.py --config c2 --cpu-queries 0 --e2e-batches 0 > $OUT/c2.json 2> $OUT/c2.err || { echo c2 failed; exit 1; }
python -c "import json; d=json.loads(open('$OUT/c2.json').read().strip().splitlines()[-1]); print('c2', d['value'], d['ms_per_step'])"
