#!/bin/bash
# round-5 dev GPU call: tests, large-k emission timing, heavy-first order.
# A step that times out, aborts or faults (rc >= 124) ends the call.
OUT=gpurun_out/r5e; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; chk pytest; tail -3 $OUT/pytest_gpu.log
VK=10000 timeout -k 10 400 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so exp/libbm25mi_emit1.so exp/libbm25mi_emit2.so > $OUT/k10000_variants.jsonl 2>&1; chk var; cat $OUT/k10000_variants.jsonl
timeout -k 10 300 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so mojo-bm25_amd/bm25mi/libbm25mi.so:BM25_HEAVY_FIRST=1 > $OUT/c3_heavy.jsonl 2>&1; chk heavy; cat $OUT/c3_heavy.jsonl
PROBE_ITERS=20 timeout -k 10 400 python -u scripts/shard_probe.py 1 8 > $OUT/probe_base.jsonl 2> $OUT/probe_base.err; chk probe; cat $OUT/probe_base.jsonl
BM25_HEAVY_FIRST=1 PROBE_ITERS=20 timeout -k 10 400 python -u scripts/shard_probe.py 1 8 > $OUT/probe_heavy.jsonl 2> $OUT/probe_heavy.err; chk probe_heavy; cat $OUT/probe_heavy.jsonl
