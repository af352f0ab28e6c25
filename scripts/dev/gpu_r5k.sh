#!/bin/bash
# round-5 dev GPU call: W=8 rank kernel breakdown, k=10000 after the pack change
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5k; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
VK=10000 timeout -k 10 300 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so > $OUT/k10000.jsonl 2>&1; chk var; cat $OUT/k10000.jsonl
export TMPDIR=/tmp
cd /tmp
PROBE_ITERS=10 PROBE_RANKS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_w8 -o run -- python3 $R/scripts/shard_probe.py 8 > $OUT/probe_w8.jsonl 2> $OUT/probe_w8.err; chk prof_w8
cat $OUT/probe_w8.jsonl | cut -c1-300
