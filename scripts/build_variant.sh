#!/bin/bash
# dev: build a variant of libbm25mi.so with extra compile flags into exp/
#   scripts/build_variant.sh NAME -DBM25_KJ2=3 ...   ->  exp/libbm25mi_NAME.so
# (load it with BM25MI_LIB=exp/libbm25mi_NAME.so)
set -e
cd "$(dirname "$0")/.."
name=$1; shift
mkdir -p exp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wno-unused-result -Wno-unused-value "$@" \
  -o exp/libbm25mi_$name.so mojo-bm25_amd/csrc/bm25mi_kernels.hip mojo-bm25_amd/csrc/bm25mi_build.hip mojo-bm25_amd/csrc/bm25mi_capi.cpp
echo exp/libbm25mi_$name.so
