set -o pipefail
mkdir -p gpurun_out/r4e
timeout -k 10 120 python -u scripts/dev/debug_zero_fill4.py > gpurun_out/r4e/dbg4.log 2>&1; echo rc=$?
cut -c1-300 gpurun_out/r4e/dbg4.log
