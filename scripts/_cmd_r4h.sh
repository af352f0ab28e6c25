set -o pipefail
R=$GRAFT_REPO_ROOT
P=mojo-bm25_amd/bm25mi/libbm25mi.so
NAME=r4j STEPS="tests variants" VLIBS="$P" VCFGS="c3 c5" bash scripts/gpu_r4.sh || exit 1
OUT=$R/gpurun_out/r4j
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o run -- python3 $R/bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/bench_under_rocprof.json 2> $OUT/bench_rocprof.err || { echo bench trace failed; tail -5 $OUT/bench_rocprof.err; exit 1; }
python3 -c "
import csv
for r in list(csv.DictReader(open('$OUT/c3_trace/run_kernel_stats.csv')))[:10]: print('%-70s %6s %9.1f' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
"
cd $R && timeout -k 10 600 python -u scripts/shard_probe.py 1 8 > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err || { echo probe failed; tail -20 $OUT/shard_probe.err; exit 1; }
cut -c1-200 $OUT/shard_probe.jsonl; grep -o '"projected_ms.*' $OUT/shard_probe.jsonl
