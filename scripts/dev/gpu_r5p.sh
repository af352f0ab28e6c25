#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5p; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
for v in base nonpost base nonpost; do
  if [ $v = base ]; then unset VLIB; else export VLIB=$R/exp/libbm25mi_$v.so; fi
  PROBE_ITERS=30 PROBE_RANKS=0,1 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_$v.jsonl 2> $OUT/probe_$v.err; chk $v
  python -c "import json;d=json.loads(open('$OUT/probe_$v.jsonl').read().splitlines()[-1]);print('$v',d['per_rank'])"
done
