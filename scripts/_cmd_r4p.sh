set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r4q
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "config3 or config4 or variants or theta_bound or merge_paths or widths or golden or rare" > $OUT/pytest.log 2>&1 || { echo pytest failed; tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 400 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so exp/libbm25mi_nosf.so > $OUT/var_c3.jsonl 2> $OUT/var_c3.err || { echo var failed; tail -5 $OUT/var_c3.err; exit 1; }
cut -c1-150 $OUT/var_c3.jsonl
PROBE_RANKS=0 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_sf.jsonl 2> $OUT/probe_sf.err || { echo probe failed; tail -5 $OUT/probe_sf.err; exit 1; }
VLIB=exp/libbm25mi_nosf.so PROBE_RANKS=0 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_nosf.jsonl 2> $OUT/probe_nosf.err || { echo probe failed; tail -5 $OUT/probe_nosf.err; exit 1; }
grep -o '"per_rank.*"max_rank_ms": [0-9.]*' $OUT/probe_sf.jsonl $OUT/probe_nosf.jsonl
