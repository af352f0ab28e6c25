#!/bin/bash
# sweep: VARIANTS is a list of "ENV=VAL,ENV2=VAL2" settings; each runs scripts/ablate.py
set -o pipefail
mkdir -p gpurun_out
for var in ${VARIANTS:-BM25_TILE_SHIFT=13}; do
  envs=$(echo "$var" | tr ',' ' ')
  echo "== $var" >> gpurun_out/ablate.err
  env $envs timeout -k 10 180 python scripts/ablate.py ${CFG:-c3} 2>> gpurun_out/ablate.err | sed "s|}|, \"variant\": \"$var\"}|" >> gpurun_out/ablate.jsonl || exit $?
done
echo ablate done
