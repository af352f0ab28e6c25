#!/bin/bash
# merge_sorted duration check: the W = 8 rank-3 probe trace, three runs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_mst}; mkdir -p $OUT
export TMPDIR=/tmp
for i in 1 2 3; do
  ( cd /tmp; PROBE_ITERS=10 PROBE_RANKS=3 PROBE_WORLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8_$i -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_w8_$i.jsonl 2> $OUT/probe_w8_$i.err ) || { echo trace failed; exit 1; }
done
