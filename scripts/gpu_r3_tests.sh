#!/bin/bash
# GPU box: the -m gpu suite, then a short bench run (no CPU leg).
# usage: scripts/gpu_r3_tests.sh <out-subdir> [pytest -k expr]
set -o pipefail
out=gpurun_out/$1
mkdir -p "$out"
(cat /sys/fs/cgroup/cpu.max; nproc; python -c "import os; print(len(os.sched_getaffinity(0)), os.cpu_count())") > "$out/cpu.txt" 2>&1
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -s --timeout 600 --timeout-method thread "${K[@]}" > "$out/pytest.log" 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --cpu-queries 0 --e2e-batches 5 > "$out/bench.json" 2> "$out/bench.err"
