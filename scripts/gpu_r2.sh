#!/bin/bash
# Round-2 GPU pass: full GPU tests, bench c3 (default segments), c3 with the
# sparse segment table, c5 per-rank shard. Each step has its own time limit;
# the chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
fi
timeout -k 10 600 python bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || { echo bench c3 failed; tail -20 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json
BM25_SEGMENTS=sparse timeout -k 10 600 python bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/bench_c3s.json 2> $OUT/bench_c3s.err || { echo bench c3 sparse failed; tail -20 $OUT/bench_c3s.err; exit 1; }
cat $OUT/bench_c3s.json
timeout -k 10 900 python bench.py --config c5 ${C5_ARGS} > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo bench c5 failed; tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
