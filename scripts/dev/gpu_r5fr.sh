#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5fr; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
P=mojo-bm25_amd/bm25mi/libbm25mi.so
timeout -k 10 500 python -u scripts/variant_lib_time.py $P exp/libbm25mi_fr12.so $P:VTERMS=16 exp/libbm25mi_fr12.so:VTERMS=16 $P:VCFG=c5 exp/libbm25mi_fr12.so:VCFG=c5 $P exp/libbm25mi_fr12.so > $OUT/fr.jsonl 2>&1; chk var; cut -c1-140 $OUT/fr.jsonl
for v in base fr12 base fr12; do
  if [ $v = base ]; then unset VLIB; else export VLIB=$R/exp/libbm25mi_$v.so; fi
  PROBE_ITERS=30 PROBE_RANKS=0,1 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_$v.jsonl 2> $OUT/probe_$v.err; chk $v
  python -c "import json;d=json.loads(open('$OUT/probe_$v.jsonl').read().splitlines()[-1]);print('$v',d['per_rank'])"
done
