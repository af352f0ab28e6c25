#!/bin/bash
# Round evidence on one GPU box (outputs under gpurun_out/$NAME/); each GPU
# step has its own time limit and the chain stops at the first failure.
#   PART=tests : pytest -m gpu, smoke, bench lines (c3 with the CPU legs,
#                c3 at 16 terms per query, c5 one rank's shard)
#   PART=prof  : rocprofv3 kernel trace + stats of the c3 bench command, PMC
#                passes (one counter group per run) of the score kernels on
#                c3, c3 at 16 terms and the c5 rank shard, the shard probe
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=${NAME:-evidence}
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd $R
if [ "${PART:-tests}" = tests ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s -p no:cacheprovider --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
  timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
  timeout -k 10 300 python -u bench.py --terms 16 --cpu-queries 0 > $OUT/bench_t16.json 2> $OUT/bench_t16.err || { echo bench t16 failed; tail -20 $OUT/bench_t16.err; exit 1; }
  timeout -k 10 600 python -u bench.py --config c5 --cpu-queries 0 --e2e-batches 5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo bench c5 failed; tail -20 $OUT/bench_c5.err; exit 1; }
  exit 0
fi
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/bench_under_rocprof.json 2> $OUT/bench_rocprof.err || { echo trace failed; tail -5 $OUT/bench_rocprof.err; exit 1; }
i=0
while read -r tag args ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_flat|bound_keys" --output-format csv -d $OUT/pmc_${tag}_p$i -o pmc -- python3 $R/scripts/pmc_workload.py ${args//,/ } > $OUT/pmc_${tag}_p$i.log 2>&1 || { echo pmc pass $i failed; tail -5 $OUT/pmc_${tag}_p$i.log; exit 1; }
done <<'CTRS'
c3 --config,c3 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum
c3 --config,c3 WRITE_SIZE
c3 --config,c3 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
c3 --config,c3 SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
t16 --config,c3,--terms,16 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum
t16 --config,c3,--terms,16 WRITE_SIZE
t16 --config,c3,--terms,16 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT
c5 --config,c5 TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum TCC_HIT_sum TCC_MISS_sum
c5 --config,c5 WRITE_SIZE
c5 --config,c5 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT
CTRS
echo pmc done
cd $R
timeout -k 10 600 python scripts/shard_probe.py > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err || { echo shard probe failed; tail -5 $OUT/shard_probe.err; exit 1; }
cat $OUT/shard_probe.jsonl
