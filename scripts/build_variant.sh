#!/bin/bash
# Dev tool: build a variant of libbm25mi.so with compile-time knobs into
# exp/libbm25mi_<name>.so (kernels recompiled with the -D flags, the C-ABI and
# build objects reused from the product build), for scripts/variant_lib_time.py.
#   scripts/build_variant.sh NAME -DBM25_X=1 ...
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
OBJ=$R/mojo-bm25_amd/bm25mi/_obj
OUTD=${OUTD:-$R/exp}
mkdir -p $OUTD
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -Wno-unused-value \
  "$@" -c -o $OUTD/k_$NAME.o $R/mojo-bm25_amd/csrc/bm25mi_kernels.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $OUTD/libbm25mi_$NAME.so \
  $OUTD/k_$NAME.o $OBJ/bm25mi_large.o $OBJ/bm25mi_build.o $OBJ/bm25mi_sort.o $OBJ/bm25mi_dense.o $OBJ/bm25mi_capi.o
rm -f $OUTD/k_$NAME.o
echo $OUTD/libbm25mi_$NAME.so
