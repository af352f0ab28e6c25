#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5u; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
for j in 0 1 2 3 0 2; do
  BM25_TAIL_JIT=$j PROBE_ITERS=30 PROBE_RANKS=0,1 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_$j.jsonl 2> $OUT/probe_$j.err; chk $j
  python -c "import json;d=json.loads(open('$OUT/probe_$j.jsonl').read().splitlines()[-1]);print('jit $j',d['per_rank'])"
done
P=mojo-bm25_amd/bm25mi/libbm25mi.so
timeout -k 10 300 python -u scripts/variant_lib_time.py $P $P:BM25_TAIL_JIT=1 $P:BM25_TAIL_JIT=2 $P:BM25_TAIL_JIT=3 > $OUT/c3.jsonl 2>&1; chk var; cat $OUT/c3.jsonl
