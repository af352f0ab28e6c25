#!/bin/bash
# One GPU-box pass: parity tests, smoke, short bench. Each GPU step has its own
# time limit and the chain stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
STEPS=${STEPS:-10}
timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 600 python bench.py --steps $STEPS --warmup 3 ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?
echo "gpu_check rc=$rc"
exit $rc
