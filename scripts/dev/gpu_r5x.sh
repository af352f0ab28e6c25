#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5x; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_large_k.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_large.log 2>&1; chk pytest; tail -2 $OUT/pytest_large.log
grep -q failed $OUT/pytest_large.log && exit 1
VK=10000 timeout -k 10 300 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so > $OUT/k10000.jsonl 2>&1; chk var; cat $OUT/k10000.jsonl
timeout -k 10 300 python -u bench.py --k 10000 --steps 5 --warmup 2 --cpu-queries 0 --e2e-batches 0 > $OUT/bench_k10000.json 2> $OUT/bench_k10000.err; chk bench
python -c "import json;d=json.loads(open('$OUT/bench_k10000.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])"
