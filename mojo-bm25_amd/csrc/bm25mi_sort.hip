// bm25mi_sort.hip — hand-written device sort and scan for gfx950, in place
// of hipCUB's DeviceRadixSort / DeviceSegmentedRadixSort / DeviceScan:
//   * the index build's (term, doc) key sort and its indptr scan
//     (bm25mi_build.hip; bm25s's CSC order, bm25_test.py:19-38),
//   * the large-k path's row sorts (bm25mi_large.hip; the argsort of the k
//     survivors, bm25_native.py:209-212),
//   * bm25.BM25's float64 ranking (bm25mi_dense.hip; bm25.py:172-178).
//
// Radix sort: least-significant digit first, 8 bits per pass, stable, over
// (u64 key, u32 value) pairs.  A pass is three launches:
//   rs_hist_kernel     per tile of 4096 pairs, a 256-bin LDS histogram of the
//                      pass's digit (a wave's pairs that share a digit add once)
//                      -> hist[digit][tile]
//   rs_scan_kernel     one workgroup per digit: exclusive scan of its row over
//                      the tiles, and the digit's total
//   rs_scatter_kernel  per tile, in input order: each pair's rank among the
//                      tile's pairs of its digit (wave match by 8 ballots +
//                      the earlier waves' counts in LDS), written at
//                      base[digit] + hist[digit][tile] + rank
// The digit comes from the key (complemented for a descending sort) or from
// the value: sorting by key bits and then by value bits (the row of a
// segmented sort) leaves every row contiguous and ordered inside — the
// segmented sort of the large-k path in one sequence of passes.
#include "bm25mi_internal.h"

#include <algorithm>

namespace bm25mi {

namespace {

constexpr int kRsT = 256;             // threads per workgroup (4 waves)
constexpr int kRsR = 16;              // rounds per tile
constexpr int64_t kRsTile = kRsT * kRsR;  // pairs per tile

struct RsPass {
  int shift;      // digit = (source >> shift) & mask
  uint32_t mask;
  int from_val;   // 1: the value's bits, 0: the key's
  int desc;       // key digits of ~key (descending keys)
};

__device__ __forceinline__ uint32_t rs_digit(uint64_t k, uint32_t v, const RsPass& p) {
  if (p.from_val) return (v >> p.shift) & p.mask;
  const uint64_t kk = p.desc ? ~k : k;
  return (uint32_t)(kk >> p.shift) & p.mask;
}

__device__ __forceinline__ uint32_t rs_lane() { return threadIdx.x & 63u; }

// Lanes of the wave (among `valid` ones) whose digit equals this lane's.
__device__ __forceinline__ uint64_t rs_match(uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t bb = __ballot(((d >> b) & 1u) != 0u);
    m &= ((d >> b) & 1u) ? bb : ~bb;
  }
  return m;
}

__device__ __forceinline__ uint32_t rs_below(uint64_t m) {  // set bits of m below this lane
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__global__ __launch_bounds__(kRsT) void rs_hist_kernel(const uint64_t* __restrict__ keys,
                                                       const uint32_t* __restrict__ vals,
                                                       int64_t n, RsPass p, int64_t nb,
                                                       uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0u;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kRsTile;
  for (int r = 0; r < kRsR; ++r) {
    const int64_t i = base + (int64_t)r * kRsT + threadIdx.x;
    const bool valid = i < n;
    const uint32_t d = valid ? rs_digit(keys[i], p.from_val ? vals[i] : 0u, p) : 0u;
    const uint64_t m = rs_match(d, valid);
    if (valid && rs_below(m) == 0u) atomicAdd(&h[d], (uint32_t)__popcll(m));
  }
  __syncthreads();
  hist[(int64_t)threadIdx.x * nb + blockIdx.x] = h[threadIdx.x];
}

// Exclusive scan of 256 values held one per thread (block of kRsT threads).
__device__ __forceinline__ uint32_t rs_block_excl(uint32_t x, uint32_t* wsum, uint32_t* total) {
  const uint32_t lane = rs_lane(), w = threadIdx.x >> 6;
  uint32_t incl = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
    if ((int)lane >= o) incl += y;
  }
  if (lane == 63u) wsum[w] = incl;
  __syncthreads();
  uint32_t pre = 0u;
  for (uint32_t j = 0; j < w; ++j) pre += wsum[j];
  if (total) *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return pre + incl - x;
}

__global__ __launch_bounds__(kRsT) void rs_scan_kernel(uint32_t* __restrict__ hist, int64_t nb,
                                                       uint32_t* __restrict__ totals) {
  __shared__ uint32_t wsum[4];
  uint32_t* row = hist + (int64_t)blockIdx.x * nb;
  uint32_t carry = 0u;
  for (int64_t c = 0; c < nb; c += kRsT) {
    const int64_t i = c + threadIdx.x;
    const uint32_t x = i < nb ? row[i] : 0u;
    uint32_t tot = 0u;
    const uint32_t ex = rs_block_excl(x, wsum, &tot);
    if (i < nb) row[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) totals[blockIdx.x] = carry;
}

__global__ __launch_bounds__(kRsT) void rs_scatter_kernel(
    const uint64_t* __restrict__ keys, const uint32_t* __restrict__ vals,
    uint64_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out, int64_t n, RsPass p,
    int64_t nb, const uint32_t* __restrict__ hist, const uint32_t* __restrict__ totals) {
  __shared__ uint32_t off[256];
  __shared__ uint32_t wc[4][256];
  __shared__ uint32_t wsum[4];
  const uint32_t t = threadIdx.x, w = t >> 6;
  {
    const uint32_t base = rs_block_excl(totals[t], wsum, nullptr);
    off[t] = base + hist[(int64_t)t * nb + blockIdx.x];
    wc[0][t] = wc[1][t] = wc[2][t] = wc[3][t] = 0u;
  }
  __syncthreads();
  const int64_t b0 = (int64_t)blockIdx.x * kRsTile;
  for (int r = 0; r < kRsR; ++r) {
    const int64_t i = b0 + (int64_t)r * kRsT + t;
    const bool valid = i < n;
    const uint64_t k = valid ? keys[i] : 0ull;
    const uint32_t v = (valid && vals) ? vals[i] : 0u;
    const uint32_t d = valid ? rs_digit(k, v, p) : 0u;
    const uint64_t m = rs_match(d, valid);
    const uint32_t rank = rs_below(m);
    if (valid && rank == 0u) wc[w][d] = (uint32_t)__popcll(m);
    __syncthreads();
    if (valid) {
      uint32_t dst = off[d] + rank;
      for (uint32_t j = 0; j < w; ++j) dst += wc[j][d];
      keys_out[dst] = k;
      if (vals_out) vals_out[dst] = v;
    }
    __syncthreads();
    off[t] += wc[0][t] + wc[1][t] + wc[2][t] + wc[3][t];
    wc[0][t] = wc[1][t] = wc[2][t] = wc[3][t] = 0u;
    __syncthreads();
  }
}

// vals[i] = i / n (the row of pair i in rows of n pairs).
__global__ __launch_bounds__(256) void rs_rows_kernel(uint32_t* __restrict__ vals, int64_t total,
                                                      int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * 256)
    vals[i] = (uint32_t)(i / n);
}

// --- exclusive scan of u64 counts (index build indptr) ---------------------
constexpr int kScanChunk = 1024;  // elements per workgroup (256 x 4)

__device__ __forceinline__ unsigned long long scan_wave_incl(unsigned long long x) {
  const uint32_t lane = rs_lane();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long y = __shfl_up(x, o, 64);
    if ((int)lane >= o) x += y;
  }
  return x;
}

// Exclusive scan of the 1024 values of this workgroup's chunk (4 per thread,
// consecutive): returns each thread's 4 exclusive prefixes; *total = the sum.
__device__ void scan_chunk(const unsigned long long (&x)[4], unsigned long long (&ex)[4],
                           unsigned long long* wsum, unsigned long long* total) {
  const uint32_t lane = rs_lane(), w = threadIdx.x >> 6;
  const unsigned long long s = x[0] + x[1] + x[2] + x[3];
  const unsigned long long incl = scan_wave_incl(s);
  if (lane == 63u) wsum[w] = incl;
  __syncthreads();
  unsigned long long pre = 0ull;
  for (uint32_t j = 0; j < w; ++j) pre += wsum[j];
  *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  unsigned long long run = pre + incl - s;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    ex[j] = run;
    run += x[j];
  }
}

__global__ __launch_bounds__(256) void scan_sums_kernel(const unsigned long long* __restrict__ in,
                                                        int64_t n,
                                                        unsigned long long* __restrict__ bsum) {
  __shared__ unsigned long long wsum[4];
  const int64_t c = (int64_t)blockIdx.x * kScanChunk + 4 * threadIdx.x;
  unsigned long long x[4], ex[4], tot;
#pragma unroll
  for (int j = 0; j < 4; ++j) x[j] = c + j < n ? in[c + j] : 0ull;
  scan_chunk(x, ex, wsum, &tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void scan_bsum_kernel(unsigned long long* __restrict__ bsum,
                                                        int64_t nb) {
  __shared__ unsigned long long wsum[4];
  unsigned long long carry = 0ull;
  for (int64_t c = 0; c < nb; c += kScanChunk) {
    const int64_t e = c + 4 * threadIdx.x;
    unsigned long long x[4], ex[4], tot;
#pragma unroll
    for (int j = 0; j < 4; ++j) x[j] = e + j < nb ? bsum[e + j] : 0ull;
    scan_chunk(x, ex, wsum, &tot);
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (e + j < nb) bsum[e + j] = carry + ex[j];
    carry += tot;
  }
}

__global__ __launch_bounds__(256) void scan_out_kernel(const unsigned long long* __restrict__ in,
                                                       int64_t n,
                                                       const unsigned long long* __restrict__ bsum,
                                                       int64_t* __restrict__ out) {
  __shared__ unsigned long long wsum[4];
  const int64_t c = (int64_t)blockIdx.x * kScanChunk + 4 * threadIdx.x;
  unsigned long long x[4], ex[4], tot;
#pragma unroll
  for (int j = 0; j < 4; ++j) x[j] = c + j < n ? in[c + j] : 0ull;
  scan_chunk(x, ex, wsum, &tot);
  const unsigned long long b = bsum[blockIdx.x];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (c + j < n) out[c + j] = (int64_t)(b + ex[j]);
}

inline int64_t rs_tiles(int64_t n) { return (n + kRsTile - 1) / kRsTile; }

}  // namespace

size_t radix_sort_scratch_bytes(int64_t n) {
  return sizeof(uint32_t) * (size_t)(256 * std::max<int64_t>(rs_tiles(n), 1) + 256);
}

hipError_t radix_sort_pairs(uint64_t* keys, uint32_t* vals, uint64_t* keys_alt, uint32_t* vals_alt,
                            int64_t n, int key_bits_lo, int key_bits_hi, bool descending,
                            int val_bits_hi, void* scratch, bool* result_in_alt,
                            hipStream_t st) {
  *result_in_alt = false;
  if (n <= 1) return hipSuccess;
  if (n > (int64_t)UINT32_MAX || (val_bits_hi > 0 && (!vals || !vals_alt)))
    return hipErrorInvalidValue;
  const int64_t nb = rs_tiles(n);
  uint32_t* hist = (uint32_t*)scratch;
  uint32_t* totals = hist + 256 * nb;
  uint64_t *ki = keys, *ko = keys_alt;
  uint32_t *vi = vals, *vo = vals_alt;
  auto pass = [&](const RsPass& p) -> hipError_t {
    hipLaunchKernelGGL(rs_hist_kernel, dim3((unsigned)nb), dim3(kRsT), 0, st, ki, vi, n, p, nb,
                       hist);
    hipLaunchKernelGGL(rs_scan_kernel, dim3(256), dim3(kRsT), 0, st, hist, nb, totals);
    hipLaunchKernelGGL(rs_scatter_kernel, dim3((unsigned)nb), dim3(kRsT), 0, st, ki, vi, ko, vo,
                       n, p, nb, hist, totals);
    std::swap(ki, ko);
    std::swap(vi, vo);
    *result_in_alt = !*result_in_alt;
    return hipGetLastError();
  };
  for (int s = key_bits_lo; s < key_bits_hi; s += 8) {
    const int w = std::min(8, key_bits_hi - s);
    const hipError_t e = pass(RsPass{s, (1u << w) - 1u, 0, descending ? 1 : 0});
    if (e != hipSuccess) return e;
  }
  for (int s = 0; s < val_bits_hi; s += 8) {
    const int w = std::min(8, val_bits_hi - s);
    const hipError_t e = pass(RsPass{s, (1u << w) - 1u, 1, 0});
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t radix_sort_rows_desc(uint64_t* keys, uint64_t* keys_alt, uint32_t* rows,
                                uint32_t* rows_alt, int64_t G, int64_t n, void* scratch,
                                bool* result_in_alt, hipStream_t st) {
  const int64_t total = G * n;
  *result_in_alt = false;
  if (total <= 1) return hipSuccess;
  int row_bits = 0;
  while (row_bits < 32 && (G - 1) >> row_bits) ++row_bits;
  if (G > 1) {
    hipLaunchKernelGGL(rs_rows_kernel, dim3((unsigned)std::min<int64_t>((total + 255) / 256, 8192)),
                       dim3(256), 0, st, rows, total, n);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return radix_sort_pairs(keys, G > 1 ? rows : nullptr, keys_alt, G > 1 ? rows_alt : nullptr,
                          total, 0, 64, true, G > 1 ? row_bits : 0, scratch, result_in_alt, st);
}

size_t exclusive_scan_scratch_bytes(int64_t n) {
  return sizeof(unsigned long long) * (size_t)std::max<int64_t>((n + kScanChunk - 1) / kScanChunk, 1);
}

hipError_t exclusive_scan_u64(const unsigned long long* in, int64_t* out, int64_t n, void* scratch,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t nb = (n + kScanChunk - 1) / kScanChunk;
  unsigned long long* bsum = (unsigned long long*)scratch;
  hipLaunchKernelGGL(scan_sums_kernel, dim3((unsigned)nb), dim3(256), 0, st, in, n, bsum);
  hipLaunchKernelGGL(scan_bsum_kernel, dim3(1), dim3(256), 0, st, bsum, nb);
  hipLaunchKernelGGL(scan_out_kernel, dim3((unsigned)nb), dim3(256), 0, st, in, n, bsum, out);
  return hipGetLastError();
}

}  // namespace bm25mi
