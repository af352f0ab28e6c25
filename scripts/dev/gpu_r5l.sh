#!/bin/bash
# round-5 dev GPU call: W=8 regression hunt — the round-4 build and its probe
# (exp/r4) next to the current build, same box
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5l; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
PROBE_ITERS=20 timeout -k 10 300 python -u exp/r4/scripts/shard_probe.py 8 > $OUT/probe_r4.jsonl 2> $OUT/probe_r4.err; chk r4
cut -c1-400 $OUT/probe_r4.jsonl
PROBE_ITERS=20 timeout -k 10 300 python -u scripts/shard_probe.py 8 > $OUT/probe_r5.jsonl 2> $OUT/probe_r5.err; chk r5
cut -c1-400 $OUT/probe_r5.jsonl
