#!/bin/bash
# Full GPU-box pass: parity tests, smoke, bench (N=1), rocprofv3 kernel-trace
# stats of a short bench. Each GPU step has its own time limit; the chain stops
# at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
fi
timeout -k 10 600 python bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
[ -n "$NO_PROF" ] && exit 0
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-queries 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo prof failed; tail -20 $OUT/prof_bench.err; exit 1; }
cat $OUT/prof_bench.json
python3 $R/scripts/prof_summary.py $OUT
