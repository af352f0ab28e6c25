set -o pipefail
P=mojo-bm25_amd/bm25mi/libbm25mi.so
NAME=r4f STEPS="tests variants" VLIBS="$P $P:BM25_THETA_BOUND=0" VCFGS="c3 c5 c3:16" bash scripts/gpu_r4.sh
