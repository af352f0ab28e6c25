set -o pipefail
mkdir -p gpurun_out/r4d
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_k.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "not config3 and not config5 and not config4" > gpurun_out/r4d/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/r4d/pytest.log; exit 1; }
tail -2 gpurun_out/r4d/pytest.log
P=mojo-bm25_amd/bm25mi/libbm25mi.so
NAME=r4d STEPS="variants" VLIBS="$P $P:BM25_THETA_BOUND=0 $P:BM25_THETA_BOUND=0,BM25_TILE_BOUND=0" VCFGS="c3 c5 c3:16" bash scripts/gpu_r4.sh
