#!/bin/bash
# A/B pass: GPU tests on the default build, then the c3 bench with the default
# score kernel and with each alternative named in $AB (env assignments, one
# per run, e.g. AB="BM25_FLAT=0").  Each GPU step has its own time limit.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab
mkdir -p $OUT
cd $R
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python bench.py --cpu-queries 0 --e2e-batches 0 ${BENCH_ARGS} > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench failed; tail -20 $OUT/bench_default.err; exit 1; }
python -c "import json;d=json.load(open('$OUT/bench_default.json'));print('default', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
i=0
for v in $AB; do
  i=$((i+1))
  env $v timeout -k 10 300 python bench.py --cpu-queries 0 --e2e-batches 0 ${BENCH_ARGS} > $OUT/bench_ab$i.json 2> $OUT/bench_ab$i.err || { echo bench $v failed; tail -20 $OUT/bench_ab$i.err; exit 1; }
  python -c "import json;d=json.load(open('$OUT/bench_ab$i.json'));print('$v', d['value'], d['roofline']['kernel_ms'], d['roofline']['frac'])"
done
