#!/bin/bash
# bisect the W=8 REST regression: round-4 probe over intermediate builds
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5o; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
for v in r4 c_7b8712e c_565c80d c_825e76e r4; do
  PROBE_ITERS=30 PROBE_RANKS=0,1 timeout -k 10 300 python -u exp/$v/scripts/shard_probe.py 8 > $OUT/probe_$v.jsonl 2> $OUT/probe_$v.err; chk $v
  python -c "import json;d=json.loads(open('$OUT/probe_$v.jsonl').read().splitlines()[-1]);print('$v',d['per_rank'])"
done
