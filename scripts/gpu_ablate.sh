#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for rb in ${RBS:-8}; do
for sh in ${SHIFTS:-14}; do
for m in ${MODES:-0 1 2 3 7 15}; do
  BM25_RB=$rb BM25_TILE_SHIFT=$sh BM25_ABLATE=$m timeout -k 10 180 python scripts/ablate.py ${CFG:-c3} | sed "s/}/, \"rb\": $rb}/" >> gpurun_out/ablate.jsonl 2>> gpurun_out/ablate.err || exit $?
done; done; done
echo ablate done
