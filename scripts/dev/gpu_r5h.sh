#!/bin/bash
# round-5 dev GPU call: structured clamped row loads (CLAMP=2 default) vs 0 / 1
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r5h; mkdir -p $OUT
chk() { rc=$?; echo "$1 rc=$rc"; [ $rc -ge 124 ] && exit $rc; return 0; }
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; chk pytest; tail -3 $OUT/pytest_gpu.log
grep -q failed $OUT/pytest_gpu.log && exit 1
P=mojo-bm25_amd/bm25mi/libbm25mi.so
timeout -k 10 500 python -u scripts/variant_lib_time.py $P exp/libbm25mi_clamp0.so exp/libbm25mi_clamp1.so $P:VTERMS=16 exp/libbm25mi_clamp0.so:VTERMS=16 $P:VCFG=c5 exp/libbm25mi_clamp0.so:VCFG=c5 > $OUT/clamp_time.jsonl 2>&1; chk var; cat $OUT/clamp_time.jsonl
export TMPDIR=/tmp
cd /tmp
for t in 8 16; do
  timeout -s KILL 200 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "score_flat|bound_keys" --output-format csv -d $OUT/pmc_t$t -o pmc -- python3 $R/scripts/pmc_workload.py --config c3 --terms $t > $OUT/pmc_t$t.log 2>&1; chk pmc_$t
done
