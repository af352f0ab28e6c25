set -o pipefail
OUT=gpurun_out/r5d; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_large_k.py -v -s -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_large.log 2>&1; grep -E "PASSED|FAILED|passed|failed" $OUT/pytest_large.log | tail -20
timeout -k 10 300 python -u bench.py --k 10000 --steps 5 --warmup 2 --cpu-queries 0 --e2e-batches 0 > $OUT/bench_k10000.json 2> $OUT/bench_k10000.err && tail -c 600 $OUT/bench_k10000.json
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof_k10000 -o run -- python3 bench.py --k 10000 --steps 3 --warmup 1 --cpu-queries 0 --e2e-batches 0 > $OUT/prof_k10000.log 2>&1; echo prof rc=$?
VLIB=exp/libbm25mi_trace.so timeout -k 10 300 python -u scripts/dev/rest_trace.py > $OUT/rest_trace.jsonl 2> $OUT/rest_trace.err; cat $OUT/rest_trace.jsonl
