set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4g
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u scripts/shard_probe.py 1 8 > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err || { echo probe failed; tail -20 $OUT/shard_probe.err; exit 1; }
cat $OUT/shard_probe.jsonl
cd /tmp && export TMPDIR=/tmp
PROBE_ITERS=5 PROBE_RANKS=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/probe8_trace -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe8_under_rocprof.jsonl 2> $OUT/probe8_rocprof.err || { echo probe trace failed; tail -5 $OUT/probe8_rocprof.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o run -- python3 $R/bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/bench_under_rocprof.json 2> $OUT/bench_rocprof.err || { echo bench trace failed; tail -5 $OUT/bench_rocprof.err; exit 1; }
cat $OUT/bench_under_rocprof.json
