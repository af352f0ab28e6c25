#!/bin/bash
# Round-6: PMC of the per-batch latency-bound kernels (theta, bound keys,
# merges) in the W = 8 shard probe, rank 0, serial protocol; plus a kernel
# trace of the same run.  Outputs under gpurun_out/$NAME/.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${NAME:-r6p}
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
export PROBE_RANKS=0 PROBE_ITERS=10
RX="merge_sorted|merge_fast|theta_wave|bound_keys|merge_tail|score_flat_kernel<11, 0"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/scripts/shard_probe.py ${PROBE_W:-8} > $OUT/probe_trace.jsonl 2> $OUT/probe_trace.err || { echo trace failed; tail -5 $OUT/probe_trace.err; exit 1; }
i=0
[ -n "$SKIP_PMC" ] && { echo done; exit 0; }
while read -r ctrs; do
  [ -z "$ctrs" ] && continue
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $ctrs --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc$i -o pmc -- python3 $R/scripts/shard_probe.py ${PROBE_W:-8} > $OUT/pmc$i.log 2>&1 || { echo pmc $i failed; tail -5 $OUT/pmc$i.log; exit 1; }
done <<'CTRS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SMEM GRBM_GUI_ACTIVE
CTRS
echo done
exit 0
