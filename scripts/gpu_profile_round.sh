#!/bin/bash
# Round evidence on the GPU box: parity tests, bench (N=1), rocprofv3 kernel
# trace + stats of a short bench, and PMC passes (one counter group per run,
# no tracing domains beside --pmc) on the score kernels for roofline.traffic.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
if [ -z "$NO_TESTS" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
fi
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --steps 10 --warmup 3 --cpu-queries 0 > $OUT/prof_bench.json 2> $OUT/prof_bench.err || { echo prof failed; tail -20 $OUT/prof_bench.err; exit 1; }
i=0
for ctrs in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_" --output-format csv -d $OUT/pmc$i -o pmc -- python3 $R/scripts/ablate.py c3 > $OUT/pmc$i.log 2>&1 || { echo "pmc $ctrs failed"; tail -5 $OUT/pmc$i.log; exit 1; }
done
python3 $R/scripts/prof_summary.py $OUT > $OUT/summary.txt
cat $OUT/summary.txt
