set -o pipefail
NAME=r4o STEPS="lines" bash scripts/gpu_r4.sh
