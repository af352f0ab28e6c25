#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5n; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
for v in base nonpost; do
  if [ $v = base ]; then unset VLIB; else export VLIB=$R/exp/libbm25mi_$v.so; fi
  PROBE_ITERS=30 PROBE_RANKS=0,1 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_$v.jsonl 2> $OUT/probe_$v.err; chk $v
  python -c "import json;d=json.loads(open('$OUT/probe_$v.jsonl').read().splitlines()[-1]);print('$v',d['per_rank'])"
done
unset VLIB
PROBE_ITERS=30 PROBE_RANKS=0,1 timeout -k 10 300 python -u exp/r4/scripts/shard_probe.py 8 > $OUT/probe_r4.jsonl 2> $OUT/probe_r4.err; chk r4
python -c "import json;d=json.loads(open('$OUT/probe_r4.jsonl').read().splitlines()[-1]);print('r4',d['per_rank'])"
timeout -k 10 300 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so mojo-bm25_amd/bm25mi/libbm25mi.so:VTERMS=16 > $OUT/c3.jsonl 2>&1; chk var; cat $OUT/c3.jsonl
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest_parity.log 2>&1; chk pytest; tail -2 $OUT/pytest_parity.log
