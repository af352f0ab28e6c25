#!/bin/bash
# Round-6 GPU steps (outputs under gpurun_out/$NAME/); each GPU step has its
# own time limit and the chain stops at the first failure.
#   STEPS=tests   pytest -m gpu + smoke
#   STEPS=lines   bench lines: c3 (CPU legs), c2 (CPU legs), replica proxy
#                 (rank 0 of 8), c3 at k=10000 (large-k path), c3 at 16
#                 terms, c5 (one rank's shard)
#   STEPS=prof    rocprofv3 kernel traces (c3, k=10000) and PMC traffic passes
#   STEPS=probe   scripts/shard_probe.py (W = PROBE_WS)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=${NAME:-r6}
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd $R
for step in ${STEPS:-tests lines}; do
  case $step in
  tests)
    timeout -k 10 900 python -u -m pytest tests -m gpu ${PYTEST_X--x} -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|passed|failed" $OUT/pytest_gpu.log | tail -30; [ -n "$PYTEST_CONTINUE" ] || exit 1; }
    tail -1 $OUT/pytest_gpu.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
    ;;
  btrace)  # kernel trace + stats of one bench command: BARGS="--config c2 ..."
    ( export TMPDIR=/tmp; cd /tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/btrace -o run -- python3 $R/bench.py $BARGS --cpu-queries 0 --e2e-batches 0 > $OUT/btrace.json 2> $OUT/btrace.err ) || { echo btrace failed; tail -5 $OUT/btrace.err; exit 1; }
    ;;
  sel)  # selected GPU tests: TESTS="path::name ..."
    timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/pytest_sel.log 2>&1 || { echo "pytest sel failed"; grep -E "FAILED|Error|passed|failed" $OUT/pytest_sel.log | tail -30; exit 1; }
    tail -1 $OUT/pytest_sel.log
    ;;
  c3)  # the headline line only
    timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
    cat $OUT/bench.json
    ;;
  k10000)  # the large-k side line
    timeout -k 10 300 python -u bench.py --k 10000 --steps 5 --warmup 2 --cpu-queries 0 --e2e-batches 0 > $OUT/bench_k10000.json 2> $OUT/bench_k10000.err || { echo bench k10000 failed; tail -20 $OUT/bench_k10000.err; exit 1; }
    cat $OUT/bench_k10000.json
    ;;
  side)  # the threshold side lines: uniform weights (default options, and theta_bound 0), lucene-scored
    timeout -k 10 400 python -u bench.py --config c3u --cpu-queries 0 --e2e-batches 0 > $OUT/bench_c3u.json 2> $OUT/bench_c3u.err || { echo bench c3u failed; tail -20 $OUT/bench_c3u.err; exit 1; }
    cat $OUT/bench_c3u.json
    BM25_THETA_BOUND=0 timeout -k 10 400 python -u bench.py --config c3u --cpu-queries 0 --e2e-batches 0 > $OUT/bench_c3u_tb0.json 2> $OUT/bench_c3u_tb0.err || { echo bench c3u tb0 failed; tail -20 $OUT/bench_c3u_tb0.err; exit 1; }
    cat $OUT/bench_c3u_tb0.json
    timeout -k 10 500 python -u bench.py --config c3l --cpu-queries 0 --e2e-batches 0 > $OUT/bench_c3l.json 2> $OUT/bench_c3l.err || { echo bench c3l failed; tail -20 $OUT/bench_c3l.err; exit 1; }
    cat $OUT/bench_c3l.json
    ;;
  lines)
    timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
    cat $OUT/bench.json
    timeout -k 10 300 python -u bench.py --config c2 > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo bench c2 failed; tail -20 $OUT/bench_c2.err; exit 1; }
    timeout -k 10 300 python -u bench.py --replica-of 8 --cpu-queries 0 > $OUT/bench_replica8.json 2> $OUT/bench_replica8.err || { echo bench replica failed; tail -20 $OUT/bench_replica8.err; exit 1; }
    timeout -k 10 300 python -u bench.py --k 10000 --steps 5 --warmup 2 --cpu-queries 0 --e2e-batches 0 > $OUT/bench_k10000.json 2> $OUT/bench_k10000.err || { echo bench k10000 failed; tail -20 $OUT/bench_k10000.err; exit 1; }
    timeout -k 10 300 python -u bench.py --terms 16 --cpu-queries 0 > $OUT/bench_t16.json 2> $OUT/bench_t16.err || { echo bench t16 failed; tail -20 $OUT/bench_t16.err; exit 1; }
    timeout -k 10 600 python -u bench.py --config c5 --cpu-queries 0 --e2e-batches 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo bench c5 failed; tail -20 $OUT/bench_c5.err; exit 1; }
    ;;
  variants)  # VLIBS: variant libraries timed against the product (scripts/variant_lib_time.py)
    for cfg in ${VCFGS:-c3}; do
      VCFG=${cfg%%:*} VTERMS=$([ "${cfg#*:}" != "$cfg" ] && echo ${cfg#*:}) timeout -k 10 900 python -u scripts/variant_lib_time.py $VLIBS > $OUT/variants_${cfg/:/_t}.jsonl 2> $OUT/variants_${cfg/:/_t}.err || { echo variants failed; tail -20 $OUT/variants_${cfg/:/_t}.err; exit 1; }
      cat $OUT/variants_${cfg/:/_t}.jsonl
    done
    ;;
  prof)  # rocprofv3 kernel trace + stats of the c3 and k=10000 bench commands; PMC
         # passes (one counter group per run) of the score kernels: c3, 16 terms, c5 shard
    ( export TMPDIR=/tmp; cd /tmp
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -o run -- python3 $R/bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/bench_c3_rocprof.json 2> $OUT/bench_c3_rocprof.err || { echo trace c3 failed; exit 1; }
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_k10000 -o run -- python3 $R/bench.py --k 10000 --steps 5 --warmup 2 --cpu-queries 0 --e2e-batches 0 > $OUT/bench_k10000_rocprof.json 2> $OUT/bench_k10000_rocprof.err || { echo trace k10000 failed; exit 1; }
      while read -r tag args ctrs; do
        [ -z "$ctrs" ] && continue
        timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_flat|bound_keys" --output-format csv -d $OUT/pmc_${tag}_${ctrs%% *} -o pmc -- python3 $R/scripts/pmc_workload.py ${args//,/ } > $OUT/pmc_${tag}_${ctrs%% *}.log 2>&1 || { echo pmc $tag failed; exit 1; }
      done <<'CTRS'
c3 --config,c3 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum
c3 --config,c3 WRITE_SIZE
c3 --config,c3 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
c3 --config,c3 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
t16 --config,c3,--terms,16 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum
t16 --config,c3,--terms,16 WRITE_SIZE
c5 --config,c5 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum
c5 --config,c5 WRITE_SIZE
CTRS
    ) || exit 1
    echo prof done
    ;;
  probe)  # per-rank config-3 shard work with real sample keys + modelled collectives
    timeout -k 10 900 python -u scripts/shard_probe.py ${PROBE_WS:-1 2 4 8} > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err || { echo probe failed; tail -20 $OUT/shard_probe.err; exit 1; }
    cat $OUT/shard_probe.jsonl
    ;;
  esac
done
exit 0
