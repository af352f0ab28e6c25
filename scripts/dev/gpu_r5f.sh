#!/bin/bash
# round-5 dev GPU call: large-k slots + LDS row sort
OUT=gpurun_out/r5f; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_large_k.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_large.log 2>&1; chk pytest_large; tail -3 $OUT/pytest_large.log
grep -q failed $OUT/pytest_large.log && exit 1
VK=10000 timeout -k 10 300 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so > $OUT/k10000.jsonl 2>&1; chk var; cat $OUT/k10000.jsonl


