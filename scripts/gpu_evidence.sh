#!/bin/bash
# Round evidence on one GPU box: GPU tests, smoke, the default bench line,
# rocprofv3 kernel trace + stats of the bench command, PMC passes (one
# counter group per run) of the score kernels, and the per-rank shard probe.
# Outputs under gpurun_out/$NAME/.  Each GPU step has its own time limit; the
# chain stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
NAME=${NAME:-evidence}
OUT=$R/gpurun_out/$NAME
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo smoke failed; tail -20 $OUT/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/bench_under_rocprof.json 2> $OUT/bench_rocprof.err || { echo trace failed; tail -5 $OUT/bench_rocprof.err; exit 1; }
i=0
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "score_(band|flat)" --output-format csv -d $OUT/pmc_p$i -o pmc -- python3 $R/scripts/ablate.py c3 > $OUT/pmc_p$i.log 2>&1 || { echo pmc pass $i failed; tail -5 $OUT/pmc_p$i.log; exit 1; }
done <<'CTRS'
TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE
CTRS
echo pmc done
cd $R
timeout -k 10 600 python scripts/shard_probe.py > $OUT/shard_probe.jsonl 2> $OUT/shard_probe.err || { echo shard probe failed; tail -5 $OUT/shard_probe.err; exit 1; }
cat $OUT/shard_probe.jsonl
