set -o pipefail
mkdir -p gpurun_out/r4b
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_large_k.py -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "not config3 and not config5 and not config4" > gpurun_out/r4b/pytest.log 2>&1 || { echo pytest failed; tail -30 gpurun_out/r4b/pytest.log; exit 1; }
tail -2 gpurun_out/r4b/pytest.log
P=mojo-bm25_amd/bm25mi/libbm25mi.so
NAME=r4b STEPS=variants VLIBS="exp/libbm25mi_r3.so $P exp/libbm25mi_h_w5fr8.so exp/libbm25mi_h_t12.so exp/libbm25mi_t12.so $P:BM25_FLAT_BW=4 $P:BM25_FLAT_BW=2" VCFGS="c3 c3:16" bash scripts/gpu_r4.sh
