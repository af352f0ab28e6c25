set -o pipefail
R=$GRAFT_REPO_ROOT
P=mojo-bm25_amd/bm25mi/libbm25mi.so
NAME=r4m STEPS="tests variants" VLIBS="$P" VCFGS="c3 c5" bash scripts/gpu_r4.sh || exit 1
OUT=$R/gpurun_out/r4m
cd $R
PROBE_RANKS=0,3,7 timeout -k 10 400 python -u scripts/shard_probe.py 1 8 > $OUT/probe.jsonl 2> $OUT/probe.err || { echo probe failed; tail -5 $OUT/probe.err; exit 1; }
grep -o '"per_rank.*' $OUT/probe.jsonl | cut -c1-400
