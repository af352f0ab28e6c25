set -o pipefail
R=$GRAFT_REPO_ROOT; OUT=$R/gpurun_out/r6_ld2; mkdir -p $OUT
export TMPDIR=/tmp; cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8 -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_w8.jsonl 2> $OUT/probe_w8.err && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -o run -- python3 $R/bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/c3.json 2> $OUT/c3.err
