#!/bin/bash
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5r; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; chk pytest; tail -2 $OUT/pytest_gpu.log
grep -q failed $OUT/pytest_gpu.log && exit 1
timeout -k 10 600 python -u bench.py --cpu-queries 0 > $OUT/bench.json 2> $OUT/bench.err; chk bench; cat $OUT/bench.json
PROBE_ITERS=20 PROBE_HYBRID=1 timeout -k 10 600 python -u scripts/shard_probe.py 1 8 > $OUT/probe.jsonl 2> $OUT/probe.err; chk probe
python - <<'PY'
import json
for l in open('gpurun_out/r5r/probe.jsonl'):
    d=json.loads(l); print(d['W'], d['shards'], d['replicas'], d['max_rank_ms'], d['projected_ms'], d.get('speedup_vs_W1'))
PY
