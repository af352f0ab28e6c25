set -o pipefail
R=$GRAFT_REPO_ROOT
P=mojo-bm25_amd/bm25mi/libbm25mi.so
NAME=r4s STEPS="tests variants" VLIBS="$P" VCFGS="c3 c5 c3:16" bash scripts/gpu_r4.sh || exit 1
OUT=$R/gpurun_out/r4s
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_large_k.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $OUT/pytest_large.log 2>&1 || { echo large failed; tail -20 $OUT/pytest_large.log; exit 1; }
tail -1 $OUT/pytest_large.log
timeout -k 10 300 python -u bench.py --k 10000 --steps 5 --warmup 2 --cpu-queries 0 --e2e-batches 0 > $OUT/bench_k10000.json 2> $OUT/bench_k10000.err || { echo k failed; tail -5 $OUT/bench_k10000.err; exit 1; }
cut -c1-200 $OUT/bench_k10000.json
