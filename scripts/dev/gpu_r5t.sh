#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5t; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_gpu_parity.py tests/test_gpu_large_k.py -x -q --timeout 120 --timeout-method thread  > $OUT/pytest.log 2>&1; chk pytest; tail -2 $OUT/pytest.log
grep -q failed $OUT/pytest.log && exit 1
for v in base msel base msel; do
  if [ $v = base ]; then unset VLIB; else export VLIB=$R/exp/libbm25mi_$v.so; fi
  PROBE_ITERS=30 PROBE_RANKS=0,1 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_$v.jsonl 2> $OUT/probe_$v.err; chk $v
  python -c "import json;d=json.loads(open('$OUT/probe_$v.jsonl').read().splitlines()[-1]);print('$v',d['per_rank'])"
done
P=mojo-bm25_amd/bm25mi/libbm25mi.so
timeout -k 10 300 python -u scripts/variant_lib_time.py $P exp/libbm25mi_msel.so $P:VCFG=c5 exp/libbm25mi_msel.so:VCFG=c5 > $OUT/c3.jsonl 2>&1; chk var; cat $OUT/c3.jsonl
