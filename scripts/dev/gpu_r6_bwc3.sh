#!/bin/bash
# c3 REST item width A/B (BM25_FLAT_BW 0 = auto (8), 4), bench lines without CPU legs.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; OUT=$R/gpurun_out/${NAME:-r6_bwc3}; mkdir -p $OUT; cd $R
for bw in 0 4 0 4; do
  BM25_FLAT_BW=$bw timeout -k 10 300 python -u bench.py --cpu-queries 0 --e2e-batches 0 > $OUT/c3_bw$bw.json 2> $OUT/c3_bw$bw.err || { echo bench failed; tail -5 $OUT/c3_bw$bw.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/c3_bw$bw.json').read().strip().splitlines()[-1]); print('bw', $bw, d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['config']['tiles_per_item'])"
done
