#!/bin/bash
# round-5 dev GPU call: L2-miss traffic of the base and clamped-row builds
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5g; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
VK=10000 timeout -k 10 300 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so > $OUT/k10000.jsonl 2>&1; chk var; cat $OUT/k10000.jsonl
timeout -k 10 300 python -u scripts/variant_lib_time.py mojo-bm25_amd/bm25mi/libbm25mi.so exp/libbm25mi_clamp.so mojo-bm25_amd/bm25mi/libbm25mi.so:VTERMS=16 exp/libbm25mi_clamp.so:VTERMS=16 > $OUT/clamp_time.jsonl 2>&1; chk var2; cat $OUT/clamp_time.jsonl
export TMPDIR=/tmp
cd /tmp
for lib in base clamp; do
  if [ $lib = base ]; then export VLIB=$R/mojo-bm25_amd/bm25mi/libbm25mi.so; else export VLIB=$R/exp/libbm25mi_clamp.so; fi
  for t in 8 16; do
    timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "score_flat|bound_keys" --output-format csv -d $OUT/pmc_${lib}_t$t -o pmc -- python3 $R/scripts/pmc_workload.py --config c3 --terms $t > $OUT/pmc_${lib}_t$t.log 2>&1; chk pmc_${lib}_$t
  done
done
