// bm25mi_dense.hip — float64 scoring and ranking of bm25.BM25 (the dense
// model's API, bm25.py:124-178) on the device, from the float64 values of its
// BM25 matrix (bm25_build_scores method 1 writes them; bm25_index_set_values_f64
// keeps them beside the index).
//
//   get_scores  np.sum(bm25_matrix[:, ids], axis=1) (bm25.py:143): numpy
//               walks the gathered [N, T] block column by column, so every
//               document's float64 sum is 0 + v(t0) + v(t1) + ... in query order
//               (a document without the term adds 0.0).  A one-document corpus
//               is the exception: the reduction then runs over one contiguous
//               row, numpy's pairwise sum (8 partial sums per block of <= 128,
//               halves above) — reproduced as such.
//   get_top_n   np.argsort(scores)[::-1][:n] (bm25.py:172-176): the n best by
//               (score desc, doc asc) — a stable radix sort of the sortable
//               float64 bits, descending (bm25mi_sort.hip); the reference's
//               order among equal scores is numpy-implementation-defined.
#include "bm25mi_internal.h"

#include <algorithm>

namespace bm25mi {

namespace {

// One wave per tile: an f64 LDS accumulator of the tile's documents, the
// query's terms added in order (a term's postings hold distinct documents; a
// wave's LDS accesses execute in program order, so each document's adds are
// in query order), then stored.
template <int S>
__global__ __launch_bounds__(64) void dense64_kernel(
    const int64_t* __restrict__ indptr, const uint32_t* __restrict__ rel,
    const int64_t* __restrict__ tl_ptr, const uint16_t* __restrict__ tl_tile,
    const uint32_t* __restrict__ tl_start, int32_t sparse, const uint16_t* __restrict__ ldoc,
    const double* __restrict__ val64, int64_t V, int64_t ntiles, int64_t n_docs,
    const int32_t* __restrict__ query, int32_t T, double* __restrict__ out) {
  constexpr int D = 1 << S;
  __shared__ double acc[D];
  const int64_t tile = blockIdx.x;
  const uint32_t lane = threadIdx.x;
  for (int j = (int)lane; j < D; j += 64) acc[j] = 0.0;
  for (int32_t i = 0; i < T; ++i) {
    const int32_t t = query[i];
    if (t < 0 || t >= V) continue;
    uint32_t r0, r1;
    if (!sparse) {
      r0 = rel[t * (ntiles + 1) + tile];
      r1 = rel[t * (ntiles + 1) + tile + 1];
    } else {  // binary search of the term's non-empty tiles
      const int64_t b = tl_ptr[t], e = tl_ptr[t + 1];
      int64_t lo = b, hi = e;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)tl_tile[mid] < tile) lo = mid + 1;
        else hi = mid;
      }
      const uint32_t df = (uint32_t)(indptr[t + 1] - indptr[t]);
      r0 = r1 = lo < e ? tl_start[lo] : df;
      if (lo < e && (int64_t)tl_tile[lo] == tile) r1 = lo + 1 < e ? tl_start[lo + 1] : df;
    }
    const int64_t p0 = indptr[t];
    for (uint32_t p = r0 + lane; p < r1; p += 64u) {
      const uint32_t slot = (uint32_t)ldoc[p0 + p] >> 2;
      acc[slot] += val64[p0 + p];
    }
  }
  const int64_t base = tile << S;
  for (int j = (int)lane; j < D; j += 64)
    if (base + j < n_docs) out[base + j] = acc[j];
}

// numpy's pairwise sum of v(0 .. n) (npy pairwise_sum: blocks of <= 128 with
// 8 partial sums, halves above, the cut on a multiple of 8), iteratively with
// an explicit stack; v(i) = the i-th query term's value for document 0.
template <class F>
__device__ double pairwise(F v, int64_t n0) {
  struct Fr { int64_t s, n; int st; double left; };
  Fr stk[40];
  int sp = 0;
  stk[0] = Fr{0, n0, 0, 0.0};
  double ret = 0.0;
  for (;;) {
    Fr& f = stk[sp];
    if (f.n <= 128 || f.st == 0) {
      if (f.n < 8) {
        double r = 0.0;
        for (int64_t i = 0; i < f.n; ++i) r += v(f.s + i);
        ret = r;
      } else if (f.n <= 128) {
        double r[8];
        for (int j = 0; j < 8; ++j) r[j] = v(f.s + j);
        int64_t i = 8;
        for (; i < f.n - (f.n % 8); i += 8)
          for (int j = 0; j < 8; ++j) r[j] += v(f.s + i + j);
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < f.n; ++i) res += v(f.s + i);
        ret = res;
      } else {  // descend into the left half
        int64_t n2 = f.n / 2;
        n2 -= n2 % 8;
        f.st = 1;
        stk[++sp] = Fr{f.s, n2, 0, 0.0};
        continue;
      }
    } else if (f.st == 1) {  // left done: descend into the right half
      int64_t n2 = f.n / 2;
      n2 -= n2 % 8;
      f.left = ret;
      f.st = 2;
      stk[++sp] = Fr{f.s + n2, f.n - n2, 0, 0.0};
      continue;
    } else {  // both halves done
      ret = f.left + ret;
    }
    if (sp == 0) return ret;
    --sp;
  }
}

__global__ __launch_bounds__(64) void dense64_one_doc_kernel(
    const int64_t* __restrict__ indptr, const double* __restrict__ val64, int64_t V,
    const int32_t* __restrict__ query, int32_t T, double* __restrict__ out) {
  if (threadIdx.x != 0) return;
  // only the query's valid ids are gathered (bm25.py:140); a column's single
  // posting, if any, is document 0's
  int32_t n = 0;
  for (int32_t i = 0; i < T; ++i) n += (query[i] >= 0 && query[i] < V) ? 1 : 0;
  auto v = [&](int64_t j) -> double {
    int32_t c = -1;
    for (int32_t i = 0; i < T; ++i) {
      if (query[i] >= 0 && query[i] < V && ++c == j) {
        const int32_t t = query[i];
        return indptr[t + 1] > indptr[t] ? val64[indptr[t]] : 0.0;
      }
    }
    return 0.0;
  };
  out[0] = 0.0 + pairwise(v, n);  // (the reduction starts from add's identity)
}

// Sortable float64 bits (larger key = larger score) and the document.
__global__ __launch_bounds__(256) void f64_keys_kernel(const double* __restrict__ s, int64_t n,
                                                       uint64_t* __restrict__ keys,
                                                       uint32_t* __restrict__ docs) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    uint64_t u;
    const double x = s[i];
    __builtin_memcpy(&u, &x, 8);
    keys[i] = (u >> 63) ? ~u : (u | (1ull << 63));
    docs[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(256) void f64_take_kernel(const uint32_t* __restrict__ docs,
                                                       const double* __restrict__ s, int64_t n,
                                                       int32_t* __restrict__ out_docs,
                                                       double* __restrict__ out_scores) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint32_t d = docs[i];
    out_docs[i] = (int32_t)d;
    out_scores[i] = s[d];
  }
}

inline unsigned grid_of(int64_t n) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

}  // namespace

hipError_t launch_dense_f64(const DevIndex& ix, const double* val64, const int32_t* d_query,
                            int64_t T, double* d_out, hipStream_t st) {
  if (ix.n_docs == 0) return hipSuccess;
  if (ix.tile_shift != kDefaultTileShift) return hipErrorInvalidValue;
  if (ix.n_docs == 1) {
    hipLaunchKernelGGL(dense64_one_doc_kernel, dim3(1), dim3(64), 0, st, ix.indptr, val64,
                       ix.n_terms, d_query, (int32_t)T, d_out);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dense64_kernel<kDefaultTileShift>, dim3((unsigned)ix.ntiles), dim3(64), 0, st,
                     ix.indptr, ix.rel, ix.tl_ptr, ix.tl_tile, ix.tl_start, ix.sparse ? 1 : 0,
                     ix.ldoc, val64, ix.n_terms, ix.ntiles, ix.n_docs, d_query, (int32_t)T, d_out);
  return hipGetLastError();
}

size_t topn_f64_scratch_bytes(int64_t n_docs) {
  return (size_t)n_docs * (2 * sizeof(uint64_t) + 2 * sizeof(uint32_t)) +
         radix_sort_scratch_bytes(n_docs) + 64;
}

hipError_t launch_topn_f64(const double* d_scores, int64_t n_docs, int64_t n, void* scratch,
                           int32_t* d_docs, double* d_out_scores, hipStream_t st) {
  if (n_docs == 0 || n == 0) return hipSuccess;
  uint64_t* keys = (uint64_t*)scratch;
  uint64_t* keys_alt = keys + n_docs;
  uint32_t* docs = (uint32_t*)(keys_alt + n_docs);
  uint32_t* docs_alt = docs + n_docs;
  void* rs = (void*)(((uintptr_t)(docs_alt + n_docs) + 15) & ~(uintptr_t)15);
  hipLaunchKernelGGL(f64_keys_kernel, dim3(grid_of(n_docs)), dim3(256), 0, st, d_scores, n_docs,
                     keys, docs);
  bool alt = false;
  // stable: equal scores keep the documents' ascending order
  const hipError_t e =
      radix_sort_pairs(keys, docs, keys_alt, docs_alt, n_docs, 0, 64, true, 0, rs, &alt, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(f64_take_kernel, dim3(grid_of(n)), dim3(256), 0, st, alt ? docs_alt : docs,
                     d_scores, n, d_docs, d_out_scores);
  return hipGetLastError();
}

}  // namespace bm25mi
