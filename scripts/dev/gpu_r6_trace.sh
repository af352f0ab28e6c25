#!/bin/bash
# Round-6: kernel traces of the three-stream shard probe (W = 8, rank 0), with
# the default and with more hardware queues; outputs under gpurun_out/$NAME/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r6t}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for hq in ${HQS:-4 8}; do
  GPU_MAX_HW_QUEUES=$hq PROBE_STREAMS=${PROBE_STREAMS:-3} PROBE_GRID=${PROBE_GRID:-95} PROBE_RANKS=0 PROBE_ITERS=10 \
    timeout -k 10 600 python3 $R/scripts/shard_probe.py 8 > $OUT/probe_hq$hq.jsonl 2> $OUT/probe_hq$hq.err || { echo probe hq$hq failed; tail -5 $OUT/probe_hq$hq.err; exit 1; }
  cat $OUT/probe_hq$hq.jsonl
done
GPU_MAX_HW_QUEUES=${TRACE_HQ:-8} PROBE_STREAMS=${PROBE_STREAMS:-3} PROBE_GRID=${PROBE_GRID:-95} PROBE_RANKS=0 PROBE_ITERS=10 \
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_trace.jsonl 2> $OUT/probe_trace.err || { echo trace failed; tail -5 $OUT/probe_trace.err; exit 1; }
find $OUT/trace -name "*kernel_trace.csv" | head -3
exit 0
