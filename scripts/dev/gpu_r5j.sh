#!/bin/bash
# round-5 dev GPU call: tail split (pieces for the last items of each XCD range)
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5j; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_parity.log 2>&1; chk pytest; tail -3 $OUT/pytest_parity.log
grep -q failed $OUT/pytest_parity.log && exit 1
P=mojo-bm25_amd/bm25mi/libbm25mi.so
timeout -k 10 500 python -u scripts/variant_lib_time.py $P:BM25_TAIL_ITEMS=0 $P $P:BM25_TAIL_ITEMS=1 $P:BM25_TAIL_ITEMS=4 $P:BM25_TAIL_BW=2 $P:BM25_TAIL_ITEMS=4,BM25_TAIL_BW=2 $P:BM25_TAIL_ITEMS=0 $P > $OUT/tail_c3.jsonl 2>&1; chk var; cat $OUT/tail_c3.jsonl
for cfg in "0 1" "2 1" "4 2" "4 1"; do
  set -- $cfg
  BM25_TAIL_ITEMS=$1 BM25_TAIL_BW=$2 PROBE_ITERS=20 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_t$1_b$2.jsonl 2> $OUT/probe_t$1_b$2.err; chk probe_$1_$2
  python -c "import json;d=json.loads(open('$OUT/probe_t$1_b$2.jsonl').read().splitlines()[-1]);print('tail',$1,$2,d['max_rank_ms'],d['projected_ms'])"
done
