#!/bin/bash
# dev loop on the GPU box: (optional) GPU parity tests, then the ablation
# sweep over VARIANTS (scripts/gpu_ablate.sh); stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
if [ -z "$NO_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
fi
[ -n "$VARIANTS" ] && bash scripts/gpu_ablate.sh
exit 0
