#!/bin/bash
# One-wave-per-query kernels' waves per workgroup (BM25_QW variants) at W = 8:
# merge_sorted / merge_fast per-call durations, rank-3 traces, two per build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_qw}; mkdir -p $OUT
export TMPDIR=/tmp
for v in prod qw1 qw2 prod qw1 qw2; do
  lib=""; [ $v != prod ] && lib=$R/scripts/dev/libbm25mi_$v.so
  n=$(ls -d $OUT/prof_${v}_* 2>/dev/null | wc -l)
  ( cd /tmp; VLIB=$lib PROBE_ITERS=10 PROBE_RANKS=3 PROBE_WORLD=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_${v}_$n -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_${v}_$n.jsonl 2> $OUT/probe_${v}_$n.err ) || { echo trace failed; exit 1; }
done
