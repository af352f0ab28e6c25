#!/bin/bash
# round-5 dev GPU call: kernel stats of the W=8 rank, round-4 build vs current
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5m; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
export TMPDIR=/tmp
cd /tmp
PROBE_ITERS=50 PROBE_RANKS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r4 -o run -- python3 $R/exp/r4/scripts/shard_probe.py 8 > $OUT/probe_r4.jsonl 2> $OUT/probe_r4.err; chk r4
PROBE_ITERS=50 PROBE_RANKS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_r5 -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_r5.jsonl 2> $OUT/probe_r5.err; chk r5
