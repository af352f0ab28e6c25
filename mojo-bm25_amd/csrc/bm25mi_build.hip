// bm25mi_build.hip — GPU index build: (doc, term, tf) triples + document
// lengths -> the CSC score matrix the search path reads (SURVEY.md §8(f)
// row 2: the step upstream of the path).
//
//   1. validate + pack keys  term << 32 | doc           (one thread per triple)
//   2. radix sort of the keys with the triple ordinal as payload
//      (bm25mi_sort.hip): term-major, doc-ascending = canonical CSC order
//   3. document frequencies (atomic count per term) + duplicate detection
//   4. idf per term, unless the caller passes it
//   5. per-posting score, written as CSC indices/data (+ optional f64 data)
//   6. indptr = exclusive scan of the document frequencies
//
// Two scoring rules, each with the operation order (and precision) of the
// code it stands in for, so that the values are bit-identical:
//   kLucene — bm25s 0.2.12 (the writer of the on-disk index the reference
//     loads, params.index.json "method": "lucene"; bm25s itself is not in the
//     reference): per document norm = k1 * ((1 - b) + b * dl / avgdl) in f64,
//     cast to f32; score = f32(tf / (tf + norm)) * idf, f32; idf =
//     f32(ln(1 + (N - df + 0.5) / (df + 0.5))).  Pinned by the 20 values of
//     animal_index_bm25/data.csc.index.npy (tests/golden/animal.npz).
//   kBm25Py — bm25.py:108-121 with NumPy 2 promotion: f32(b * dl) / avgdl in
//     f64, lnf = k1 * ((1 - b) + that), den = tf + lnf (f64), num =
//     f32(tf * (k1 + 1)), score = num / den * idf (f64; idf f32 as
//     bm25.py:119) — the float64 bm25_matrix entry; data = its f32 cast.
// No FMA contraction anywhere in the formulas (#pragma clang fp contract(off)).
#include "bm25mi_internal.h"

#include <algorithm>

namespace bm25mi {

namespace {

__global__ __launch_bounds__(256) void pack_keys_kernel(const int32_t* __restrict__ docs,
                                                        const int32_t* __restrict__ terms,
                                                        const float* __restrict__ tfs, int64_t n,
                                                        int64_t n_docs, int64_t n_terms,
                                                        uint64_t* __restrict__ keys,
                                                        uint32_t* __restrict__ ord,
                                                        int32_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = docs[i], t = terms[i];
    const float tf = tfs[i];
    if (d < 0 || d >= n_docs || t < 0 || t >= n_terms) atomicOr(err, 1);
    if (!(tf > 0.f) || !(tf < INFINITY)) atomicOr(err, 2);
    keys[i] = ((uint64_t)(uint32_t)t << 32) | (uint32_t)d;
    ord[i] = (uint32_t)i;
  }
}

__global__ __launch_bounds__(256) void count_terms_kernel(const uint64_t* __restrict__ keys,
                                                          int64_t n, int64_t n_terms,
                                                          unsigned long long* __restrict__ df,
                                                          int32_t* __restrict__ err) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    if (i > 0 && keys[i - 1] == k) atomicOr(err, 4);  // one triple per (doc, term)
    const uint32_t t = (uint32_t)(k >> 32);
    if (t < (uint64_t)n_terms) atomicAdd(df + t, 1ull);
  }
}

// idf = ln(1 + (N - df + 0.5) / (df + 0.5))  (bm25s "lucene" idf, and
// bm25.py:100 math.log((N - df + 0.5) / (df + 0.5) + 1) — the same value)
__global__ __launch_bounds__(256) void idf_kernel(const unsigned long long* __restrict__ df,
                                                  int64_t n_terms, int64_t n_docs,
                                                  float* __restrict__ idf) {
#pragma clang fp contract(off)
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_terms;
       t += (int64_t)gridDim.x * blockDim.x) {
    const double f = (double)df[t];
    const double num = (double)n_docs - f + 0.5, den = f + 0.5;
    idf[t] = (num > 0.0 && den > 0.0) ? (float)log(num / den + 1.0) : 0.f;
  }
}

template <int METHOD>
__global__ __launch_bounds__(256) void score_postings_kernel(
    const uint64_t* __restrict__ keys, const uint32_t* __restrict__ ord,
    const float* __restrict__ tfs, const int32_t* __restrict__ doc_len,
    const float* __restrict__ idf, int64_t n, int64_t n_docs, int64_t n_terms, double avgdl,
    double k1, double b, int32_t* __restrict__ out_indices, float* __restrict__ out_data,
    double* __restrict__ out_data64) {
#pragma clang fp contract(off)
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t k = keys[i];
    const int32_t doc = (int32_t)(uint32_t)k;
    const uint32_t term = (uint32_t)(k >> 32);
    const float tf = tfs[ord[i]];
    const bool ok = doc >= 0 && (int64_t)doc < n_docs && (int64_t)term < n_terms;  // (checked
    const float w = ok ? idf[term] : 0.f;                                        // by the host)
    const int32_t dl = ok ? doc_len[doc] : 0;
    float v32;
    double v64;
    if (METHOD == kLucene) {
      const double norm = avgdl == 0.0 ? k1 * (1.0 - b) : k1 * ((1.0 - b) + b * (double)dl / avgdl);
      const float r = tf / (tf + (float)norm);
      v32 = r * w;
      v64 = (double)v32;
    } else {
      double lnf;
      if (avgdl == 0.0) {
        lnf = k1 * (1.0 - b);
      } else {
        const float bd = (float)b * (float)dl;  // f32 array * python float
        lnf = k1 * ((1.0 - b) + (double)bd / avgdl);
      }
      const double den = (double)tf + lnf;
      const float num = tf * (float)(k1 + 1.0);
      v64 = ((double)num / den) * (double)w;
      v32 = (float)v64;
    }
    out_indices[i] = doc;
    out_data[i] = v32;
    if (out_data64) out_data64[i] = v64;
  }
}

int grid_for(int64_t n) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 256 * 64));
}

}  // namespace

hipError_t build_scores(int64_t n_docs, int64_t n_terms, int64_t n, const int32_t* d_docs,
                        const int32_t* d_terms, const float* d_tfs, const int32_t* d_doc_len,
                        double avgdl, double k1, double b, int method, const float* d_idf_in,
                        int64_t* d_indptr, int32_t* d_indices, float* d_data, double* d_data64,
                        int32_t* d_err, hipStream_t st) {
  hipError_t e = hipSuccess;
  uint64_t *keys = nullptr, *keys2 = nullptr;
  uint32_t *ord = nullptr, *ord2 = nullptr;
  unsigned long long* df = nullptr;
  float* idf = nullptr;
  void* tmp = nullptr;
  size_t tmp_bytes = 0, b1 = 0, b2 = 0;
  int end_bit = 32;
  while (end_bit < 64 && (n_terms >> (end_bit - 32)) > 0) ++end_bit;
  auto done = [&](hipError_t r) {
    hipStreamSynchronize(st);
    hipFree(keys);
    hipFree(keys2);
    hipFree(ord);
    hipFree(ord2);
    hipFree(df);
    hipFree(idf);
    hipFree(tmp);
    return r;
  };
#define BTRY(x)                             \
  do {                                      \
    e = (x);                                \
    if (e != hipSuccess) return done(e);    \
  } while (0)
  const size_t m = (size_t)std::max<int64_t>(n, 1);
  BTRY(hipMalloc(&df, sizeof(unsigned long long) * (n_terms + 1)));
  BTRY(hipMemsetAsync(df, 0, sizeof(unsigned long long) * (n_terms + 1), st));
  if (n > 0) {
    BTRY(hipMalloc(&keys, sizeof(uint64_t) * m));
    BTRY(hipMalloc(&keys2, sizeof(uint64_t) * m));
    BTRY(hipMalloc(&ord, sizeof(uint32_t) * m));
    BTRY(hipMalloc(&ord2, sizeof(uint32_t) * m));
    hipLaunchKernelGGL(pack_keys_kernel, dim3(grid_for(n)), dim3(256), 0, st, d_docs, d_terms,
                       d_tfs, n, n_docs, n_terms, keys, ord, d_err);
    BTRY(hipGetLastError());
    // ids out of range stop the build here: the scoring pass indexes doc_len
    // and idf with them (the caller reports d_err as EINVAL)
    int32_t herr = 0;
    BTRY(hipMemcpyAsync(&herr, d_err, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    BTRY(hipStreamSynchronize(st));
    if (herr & 1) return done(hipSuccess);
    b1 = radix_sort_scratch_bytes(n);
    b2 = exclusive_scan_scratch_bytes(n_terms + 1);
    tmp_bytes = std::max(b1, b2);
    BTRY(hipMalloc(&tmp, std::max<size_t>(tmp_bytes, 16)));
    bool alt = false;
    BTRY(radix_sort_pairs(keys, ord, keys2, ord2, n, 0, end_bit, false, 0, tmp, &alt, st));
    const uint64_t* sk = alt ? keys2 : keys;
    const uint32_t* so = alt ? ord2 : ord;
    hipLaunchKernelGGL(count_terms_kernel, dim3(grid_for(n)), dim3(256), 0, st, sk, n, n_terms,
                       df, d_err);
    BTRY(hipGetLastError());
    const float* w = d_idf_in;
    if (!w) {
      BTRY(hipMalloc(&idf, sizeof(float) * std::max<int64_t>(n_terms, 1)));
      hipLaunchKernelGGL(idf_kernel, dim3(grid_for(n_terms)), dim3(256), 0, st, df, n_terms,
                         n_docs, idf);
      BTRY(hipGetLastError());
      w = idf;
    }
    if (method == kLucene)
      hipLaunchKernelGGL(score_postings_kernel<kLucene>, dim3(grid_for(n)), dim3(256), 0, st, sk,
                         so, d_tfs, d_doc_len, w, n, n_docs, n_terms, avgdl, k1, b, d_indices, d_data,
                         d_data64);
    else
      hipLaunchKernelGGL(score_postings_kernel<kBm25Py>, dim3(grid_for(n)), dim3(256), 0, st, sk,
                         so, d_tfs, d_doc_len, w, n, n_docs, n_terms, avgdl, k1, b, d_indices, d_data,
                         d_data64);
    BTRY(hipGetLastError());
    BTRY(exclusive_scan_u64(df, d_indptr, n_terms + 1, tmp, st));
  } else {
    BTRY(hipMemsetAsync(d_indptr, 0, sizeof(int64_t) * (n_terms + 1), st));
  }
#undef BTRY
  return done(hipGetLastError());
}

}  // namespace bm25mi
