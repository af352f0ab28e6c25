// bm25mi_large.hip — exact top-k for any k <= n_docs: the path of k > kMaxK.
//
// Replaces bm25_native._topk for large k (bm25_native.py:204-214:
// argpartition(doc_scores, -k) then argsort of the k survivors, any k <= N;
// output rows sized [Q, k] at :147-148).  The sampled-threshold pipeline of
// bm25mi_kernels.hip keeps ~P k keys per query in LDS-sized lists, which is
// what limits it to k <= kMaxK; above that the selection works on the whole
// dense score vector, one chunk of G queries at a time:
//
//   1. scores_batch_kernel      the chunk's dense fp32 sums [G][Np] (the same
//                               adds in query-term order as the main path)
//   2. radix selection          the k-th largest key (score desc, doc asc) of
//                               every query, 8 bits per pass from the top:
//                               lk_hist_kernel (LDS histogram of the keys that
//                               share the prefix decided so far) +
//                               lk_pick_kernel (the digit holding the k-th key);
//                               a query is decided as soon as every key with
//                               its prefix is needed (usually 4-5 passes)
//   3. lk_compact_kernel        the k keys >= the k-th key (unordered)
//   4. row sort                 descending, every row of the chunk in one
//                               sequence of radix passes (bm25mi_sort.hip)
//   5. lk_write_kernel          keys -> doc ids (+ doc_offset) and scores;
//                               rows of a shard with fewer than k docs are
//                               padded with doc -1 / score bits ~0
//
// Keys: (sortable score bits) << 32 | (0xFFFFFFFF - doc), as everywhere in
// the engine (bm25mi_internal.h), so equal scores order by doc ascending and
// zero-score (untouched) documents fill a row the same way.
#include "bm25mi_internal.h"

#include <cfloat>

#include <algorithm>
#include <vector>

namespace bm25mi {

namespace {

struct SelState {
  uint64_t prefix;  // key bits decided so far (the bits below the pass's digit are 0)
  uint32_t need;    // rank of the k-th key among the keys that share the prefix
  uint32_t done;    // 1: every key with the prefix is in the top-k; kth = prefix
};

__device__ __forceinline__ uint64_t doc_key(float s, uint32_t d) {
  return ((uint64_t)score_key(s) << 32) | (uint64_t)(0xFFFFFFFFu - d);
}

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o, 64);
  return v;
}

// Inclusive prefix sum over the 64 lanes.
__device__ __forceinline__ uint32_t wave_scan(uint32_t x) {
  const int lane = (int)(threadIdx.x & 63);
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

__global__ __launch_bounds__(64) void lk_init_kernel(SelState* __restrict__ st, int64_t G,
                                                     uint32_t k, int32_t* __restrict__ cnt) {
  for (int64_t g = threadIdx.x; g < G; g += 64) {
    st[g] = SelState{0ull, k, 0u};
    cnt[g] = 0;
  }
}

// One digit pass: hist[g][digit] += the keys of query g whose bits above
// (shift + 8) equal its prefix.  Exact zero sums (untouched documents, most
// of a row) share one digit while shift >= 32 (their doc bits lie below it):
// they are counted in a register, not with same-address LDS atomics.
__global__ __launch_bounds__(256) void lk_hist_kernel(const float* __restrict__ scores,
                                                      int64_t stride, int64_t n_docs, int shift,
                                                      const SelState* __restrict__ st,
                                                      uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[256];
  const int64_t g = blockIdx.y;
  const SelState s = st[g];
  if (s.done) return;  // block-uniform; before the only barriers
  h[threadIdx.x] = 0u;
  __syncthreads();
  const int hs = shift + 8;
  const uint64_t pre = s.prefix;
  auto match = [&](uint64_t key) { return hs >= 64 || ((key ^ pre) >> hs) == 0ull; };
  const bool zfast = shift >= 32;
  const uint64_t zkey = (uint64_t)score_key(0.f) << 32;
  const bool zmatch = match(zkey);
  const uint32_t zdig = (uint32_t)(zkey >> shift) & 255u;
  const float4* row = reinterpret_cast<const float4*>(scores + g * stride);
  const int64_t n4 = (n_docs + 3) >> 2;
  uint32_t zeros = 0;
  const uint32_t lane = threadIdx.x & 63u;
  // every lane of a wave runs the same rounds (the ballots below)
  const int64_t step = (int64_t)gridDim.x * 256;
  const int64_t rounds = (n4 + step - 1) / step;
  for (int64_t r = 0; r < rounds; ++r) {
    const int64_t i = r * step + (int64_t)blockIdx.x * 256 + threadIdx.x;
    float fe[4] = {0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
      const float4 f = row[i];
      fe[0] = f.x;
      fe[1] = f.y;
      fe[2] = f.z;
      fe[3] = f.w;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t d = 4 * i + c;
      bool pend = d < n_docs;
      if (pend && zfast && __float_as_uint(fe[c]) == 0u) {
        zeros += zmatch ? 1u : 0u;
        pend = false;
      }
      const uint64_t key = doc_key(fe[c], (uint32_t)d);
      pend = pend && match(key);
      const uint32_t dig = (uint32_t)(key >> shift) & 255u;
      // the high digits of a row's scores are few (one exponent range): the
      // lanes that share the first pending lane's digit add once, twice over,
      // and the rest (distinct digits, no same-address serialisation) add
      // one by one
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        const uint64_t m = __ballot(pend);
        if (m == 0ull) break;  // wave-uniform
        const int leader = __builtin_ctzll(m);
        const uint32_t dl = (uint32_t)__shfl((int)dig, leader, 64);
        const bool same = pend && dig == dl;
        const uint64_t sm = __ballot(same);
        if ((int)lane == leader) atomicAdd(&h[dl], (uint32_t)__popcll(sm));
        pend = pend && !same;
      }
      if (pend) atomicAdd(&h[dig], 1u);
    }
  }
  zeros = wave_sum(zeros);
  if ((threadIdx.x & 63) == 0 && zeros) atomicAdd(&h[zdig], zeros);
  __syncthreads();
  if (h[threadIdx.x]) atomicAdd(&hist[g * 256 + threadIdx.x], h[threadIdx.x]);
}

// The digit of the pass that holds each query's k-th key (one wave per
// query): bins scanned from the top; the histogram row is cleared for the
// next pass.
__global__ __launch_bounds__(64) void lk_pick_kernel(SelState* __restrict__ st,
                                                     uint32_t* __restrict__ hist, int shift) {
  const int64_t g = blockIdx.x;
  const SelState s = st[g];
  if (s.done) return;  // wave-uniform; no barriers
  const uint32_t lane = threadIdx.x & 63;
  uint32_t* h = hist + g * 256;
  uint32_t c[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = h[4 * lane + j];
    h[4 * lane + j] = 0u;
  }
  const uint32_t t = c[0] + c[1] + c[2] + c[3];
  const uint32_t incl = wave_scan(t);
  const uint32_t tot = __shfl((int)incl, 63, 64);
  uint32_t above = tot - incl;  // keys in the bins of the higher lanes
#pragma unroll
  for (int j = 3; j >= 0; --j) {
    if (above < s.need && s.need <= above + c[j]) {  // exactly one (lane, bin)
      const uint32_t need = s.need - above;
      SelState n;
      n.prefix = s.prefix | ((uint64_t)(4 * lane + j) << shift);
      n.need = need;
      n.done = (c[j] == need || shift == 0) ? 1u : 0u;
      st[g] = n;
    }
    above += c[j];
  }
}

// The keys >= the k-th key of each query (exactly k: keys are unique),
// appended in any order.  A workgroup stages its keys in LDS (an LDS atomic
// per wave and round) and claims its range of the row with ONE global atomic
// at the end: the keys are sparse (k of ~N per row, ~k / gridDim.x per
// workgroup), and a global atomic per wave-round on the row's one counter
// serialised the pass (8.6 ms per 100-query chunk at k = 10 000).  Keys past
// the stage's capacity (a zero-fill row's keys crowd into its first docs) take
// the global atomic directly.
constexpr int kCompactStage = 2048;
__global__ __launch_bounds__(256) void lk_compact_kernel(const float* __restrict__ scores,
                                                         int64_t stride, int64_t n_docs,
                                                         const SelState* __restrict__ st,
                                                         int32_t* __restrict__ cnt,
                                                         uint64_t* __restrict__ keys, int64_t kk) {
  __shared__ uint64_t stage[kCompactStage];
  __shared__ int32_t n_stage, base;
  const int64_t g = blockIdx.y;
  const uint64_t kth = st[g].prefix;
  const uint32_t lane = threadIdx.x & 63;
  if (threadIdx.x == 0) n_stage = 0;
  __syncthreads();
  const float4* row = reinterpret_cast<const float4*>(scores + g * stride);
  const int64_t n4 = (n_docs + 3) >> 2;
  // every lane of a wave runs the same rounds (ballots below)
  const int64_t step = (int64_t)gridDim.x * 256;
  const int64_t rounds = (n4 + step - 1) / step;
  for (int64_t r = 0; r < rounds; ++r) {
    const int64_t i = r * step + (int64_t)blockIdx.x * 256 + threadIdx.x;
    float fe[4] = {0.f, 0.f, 0.f, 0.f};
    if (i < n4) {
      const float4 f = row[i];
      fe[0] = f.x;
      fe[1] = f.y;
      fe[2] = f.z;
      fe[3] = f.w;
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int64_t d = 4 * i + c;
      const uint64_t key = d < n_docs ? doc_key(fe[c], (uint32_t)d) : 0ull;
      const bool keep = key != 0ull && key >= kth;
      const uint64_t m = __ballot(keep);
      if (m == 0ull) continue;
      int p0 = 0;
      if (lane == 0) p0 = atomicAdd(&n_stage, (int)__popcll(m));
      p0 = __shfl(p0, 0, 64);
      const int pos = p0 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      if (keep) {
        if (pos < kCompactStage) {
          stage[pos] = key;
        } else {  // stage full: straight to the row
          const int gp = atomicAdd(cnt + g, 1);
          if (gp < kk) keys[g * kk + gp] = key;
        }
      }
    }
  }
  __syncthreads();
  const int ns = min(n_stage, kCompactStage);
  if (threadIdx.x == 0) base = ns > 0 ? atomicAdd(cnt + g, ns) : 0;
  __syncthreads();
  for (int j = threadIdx.x; j < ns; j += 256)
    if (base + j < kk) keys[g * kk + base + j] = stage[j];
}

// Keys of W best-first lists -> keys[q][w * k + j] (padding maps to key 0).
__global__ __launch_bounds__(256) void lk_list_keys_kernel(const int32_t* __restrict__ docs,
                                                           const float* __restrict__ scores,
                                                           int64_t W, int64_t q0, int64_t G, int k,
                                                           int64_t rstride,
                                                           uint64_t* __restrict__ keys) {
  const int64_t n = W * k;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < G * n;
       e += (int64_t)gridDim.x * 256) {
    const int64_t g = e / n, i = e - g * n;
    const int64_t w = i / k, j = i - w * k;
    const int64_t o = w * rstride + (q0 + g) * k + j;
    keys[e] = make_key(scores[o], (uint32_t)docs[o]);
  }
}

// Sorted rows [G][n] -> the first k of each: docs (+ doc_offset) and scores
// of rows q0 .. q0 + G; positions >= k_valid, and key 0, are padding.
__global__ __launch_bounds__(256) void lk_write_kernel(const uint64_t* __restrict__ keys,
                                                       int64_t n, int64_t G, int k, int k_valid,
                                                       int64_t doc_offset,
                                                       int32_t* __restrict__ docs,
                                                       float* __restrict__ scores) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < G * k;
       e += (int64_t)gridDim.x * 256) {
    const int64_t g = e / k, i = e - g * k;
    const uint64_t key = i < k_valid ? keys[g * n + i] : 0ull;
    if (key == 0ull) {
      docs[e] = -1;
      scores[e] = __uint_as_float(0xFFFFFFFFu);
    } else {
      docs[e] = (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)key) + doc_offset);
      scores[e] = key_score((uint32_t)(key >> 32));
    }
  }
}

// Rows of n <= kLdsSortMax keys sorted descending in one workgroup's LDS and
// written out as lk_write_kernel does (docs + doc_offset and scores; columns
// n..k-1 and zero keys padded with doc -1 / score bits ~0): a bitonic network
// over the row padded with zero keys to N = 1024 E, the strides below E inside
// each thread's E consecutive keys (registers), the others across the LDS.
// One launch for the sort and the write, and every pass stays on chip: the
// device-wide radix sort of (row, key) pairs moves 10 passes of 12 B per key
// through memory.
constexpr int kLdsSortT = 1024;
constexpr int kLdsSortMax = 16384;

template <int E>
__device__ __forceinline__ void bitonic_regs(uint64_t (&r)[E], uint32_t i0, uint32_t size,
                                             uint32_t j_top) {
  // the strides j_top, j_top / 2, ..., 1 of merge size `size` (j_top < E)
#pragma unroll
  for (uint32_t j = E / 2; j >= 1; j >>= 1) {
    if (j > j_top) continue;
#pragma unroll
    for (uint32_t a = 0; a < (uint32_t)E; ++a) {
      if (a & j) continue;
      const bool asc = ((i0 + a) & size) != 0u;
      const uint64_t x = r[a], y = r[a + j];
      const bool sw = asc ? (x > y) : (x < y);
      r[a] = sw ? y : x;
      r[a + j] = sw ? x : y;
    }
  }
}

template <int E>
__global__ __launch_bounds__(kLdsSortT) void row_sort_write_kernel(
    const uint64_t* __restrict__ keys, int64_t n, int k, int64_t doc_offset,
    int32_t* __restrict__ docs, float* __restrict__ scores) {
  constexpr uint32_t N = (uint32_t)kLdsSortT * E;
  __shared__ uint64_t buf[N];
  const int64_t row = blockIdx.x;
  const uint32_t t = threadIdx.x;
  const uint32_t i0 = t * E;
  uint64_t r[E];
  const uint64_t* src = keys + row * n;
#pragma unroll
  for (int a = 0; a < E; ++a) r[a] = (int64_t)(i0 + a) < n ? src[i0 + a] : 0ull;
  for (uint32_t size = 2; size <= (uint32_t)E; size <<= 1) bitonic_regs<E>(r, i0, size, size / 2);
#pragma unroll
  for (int a = 0; a < E; ++a) buf[i0 + a] = r[a];
  __syncthreads();
  for (uint32_t size = 2 * E; size <= N; size <<= 1) {
    for (uint32_t j = size / 2; j >= (uint32_t)E; j >>= 1) {
      const uint32_t lg = (uint32_t)__builtin_ctz(j);
#pragma unroll
      for (uint32_t m = 0; m < (uint32_t)E / 2; ++m) {
        const uint32_t p = t + m * kLdsSortT;                // pair p: i has bit j clear
        const uint32_t i = ((p >> lg) << (lg + 1)) | (p & (j - 1u));
        const bool asc = (i & size) != 0u;
        const uint64_t x = buf[i], y = buf[i + j];
        if (asc ? (x > y) : (x < y)) {
          buf[i] = y;
          buf[i + j] = x;
        }
      }
      __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < E; ++a) r[a] = buf[i0 + a];
    bitonic_regs<E>(r, i0, size, E / 2);
#pragma unroll
    for (int a = 0; a < E; ++a) buf[i0 + a] = r[a];
    __syncthreads();
  }
  for (int64_t i = t; i < k; i += kLdsSortT) {
    const uint64_t key = i < n ? buf[i] : 0ull;
    const int64_t e = row * k + i;
    if (key == 0ull) {
      docs[e] = -1;
      scores[e] = __uint_as_float(0xFFFFFFFFu);
    } else {
      docs[e] = (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)key) + doc_offset);
      scores[e] = key_score((uint32_t)(key >> 32));
    }
  }
}

// Sorts and writes rows [G][n] (n <= kLdsSortMax) into [G][k] results; false
// when the rows are too long for the LDS sort.
bool lds_sort_write(const uint64_t* keys, int64_t G, int64_t n, int k, int64_t doc_offset,
                    int32_t* docs, float* scores, hipStream_t st) {
  if (n > kLdsSortMax || G <= 0) return false;
  if (n <= kLdsSortT * 8)
    hipLaunchKernelGGL(row_sort_write_kernel<8>, dim3((unsigned)G), dim3(kLdsSortT), 0, st, keys, n,
                       k, doc_offset, docs, scores);
  else
    hipLaunchKernelGGL(row_sort_write_kernel<16>, dim3((unsigned)G), dim3(kLdsSortT), 0, st, keys,
                       n, k, doc_offset, docs, scores);
  return true;
}

// Scratch bytes of sorting G rows of n keys (descending): the radix passes'
// histograms + the row numbers (two buffers).
int64_t sort_bytes(int64_t G, int64_t n) {
  return (int64_t)radix_sort_scratch_bytes(G * n) + 8 * G * n;
}

// Sorts rows [G][n] of `in` descending; *out = the buffer that holds them
// (in or alt).
hipError_t sort_rows(uint64_t* in, uint64_t* alt, int64_t G, int64_t n, char* tmp,
                     const uint64_t** out, hipStream_t st) {
  uint32_t* rows = (uint32_t*)tmp;
  uint32_t* rows_alt = rows + G * n;
  bool in_alt = false;
  const hipError_t e =
      radix_sort_rows_desc(in, alt, rows, rows_alt, G, n, rows_alt + G * n, &in_alt, st);
  *out = in_alt ? alt : in;
  return e;
}

// Device memory this path may take per launch sequence.
int64_t large_budget() {
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 1ull << 30;
  return std::max<int64_t>(64ll << 20, std::min<int64_t>((int64_t)free_b / 4, 4ll << 30));
}

// Scratch of one launch sequence.  With a handle's arena (LargeArena) the
// buffers come from it; what does not fit is allocated stream-ordered,
// released on `st` after everything enqueued so far, and counted, so the host
// grows the arena before the handle's next search: a large-k search then
// allocates nothing (each stream-ordered allocation and free cost the host
// ~0.1 ms: ~2 ms per search at c3, k = 10 000, before its first kernel).  The
// device's default pool keeps its default release threshold (the process's
// other users of the pool are not affected); what a handle retains is its
// arena, at most its budget (large_budget at first use), plus what the first
// search allocated stream-ordered until the pool trims it at a
// synchronisation.  At most budget bytes at a time: a nested launch sequence
// (the list path's dense rows) gets what its caller's scratch leaves.
struct Scratch {
  hipStream_t st;
  std::vector<void*> ptrs;
  LargeArena* ar;
  size_t start, total = 0;
  explicit Scratch(hipStream_t s, LargeArena* a = nullptr)
      : st(s), ar(a), start(a ? a->used : 0) {}
  template <class T>
  hipError_t get(T** p, int64_t n) {
    *p = nullptr;
    const size_t size = (sizeof(T) * (size_t)std::max<int64_t>(n, 1) + 255) & ~(size_t)255;
    total += size;
    if (ar && ar->base && ar->used + size <= ar->bytes) {
      *p = reinterpret_cast<T*>(ar->base + ar->used);
      ar->used += size;
      return hipSuccess;
    }
    const hipError_t e = hipMallocAsync((void**)p, size, st);
    if (e == hipSuccess) ptrs.push_back((void*)*p);
    return e;
  }
  ~Scratch() {
    if (ar) {
      ar->need = std::max(ar->need, start + total);
      ar->used = start;
    }
    for (void* p : ptrs) hipFreeAsync(p, st);
  }
};

// The byte budget of one large-k launch sequence: the arena's, fixed at its
// first use (hipMemGetInfo costs the host too), else the device's free memory.
int64_t budget_of(LargeArena* ar) {
  if (!ar) return large_budget();
  if (ar->budget == 0) ar->budget = large_budget();
  return ar->budget;
}

#define LK_TRY(expr)                    \
  do {                                  \
    const hipError_t e_ = (expr);       \
    if (e_ != hipSuccess) return e_;    \
  } while (0)

inline unsigned grid_for(int64_t work, int64_t per_block, int64_t cap) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(cap, (work + per_block - 1) / per_block));
}

}  // namespace

hipError_t launch_search_large(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                               int k, int32_t* d_docs, float* d_scores, hipStream_t st,
                               LargeArena* arena, int64_t budget) {
  if (Q == 0 || k == 0) return hipSuccess;
  ix.disp.kernels |= kKLarge;
  const int kv = (int)std::min<int64_t>(k, ix.n_docs);  // a doc shard may hold fewer than k
  if (kv == 0) {  // an empty shard: all padding
    LK_TRY(hipMemsetAsync(d_docs, 0xFF, sizeof(int32_t) * Q * k, st));
    return hipMemsetAsync(d_scores, 0xFF, sizeof(float) * Q * k, st);
  }
  const int64_t Np = ix.ntiles << ix.tile_shift;  // row stride: whole tiles
  const int64_t per_q = Np * 4 + (int64_t)kv * 16 + 256 * 4 + 64 + sort_bytes(1, kv);
  if (budget <= 0) budget = budget_of(arena);
  int64_t G = std::max<int64_t>(1, std::min<int64_t>(Q, budget / per_q));
  G = std::min<int64_t>(G, 65535);
  G = std::min<int64_t>(G, std::max<int64_t>(1, (int64_t)INT32_MAX / kv - 1));
  const int64_t sb = sort_bytes(G, kv);
  Scratch sc(st, arena);
  float* scores = nullptr;
  uint32_t* hist = nullptr;
  SelState* state = nullptr;
  int32_t* cnt = nullptr;
  uint64_t *keys = nullptr, *alt = nullptr;
  char* tmp = nullptr;
  LK_TRY(sc.get(&scores, G * Np));
  LK_TRY(sc.get(&hist, G * 256));
  LK_TRY(sc.get(&state, G));
  LK_TRY(sc.get(&cnt, G));
  LK_TRY(sc.get(&keys, G * kv));
  LK_TRY(sc.get(&alt, G * kv));
  LK_TRY(sc.get(&tmp, sb));
  LK_TRY(hipMemsetAsync(hist, 0, sizeof(uint32_t) * G * 256, st));
  const int64_t n4 = (ix.n_docs + 3) >> 2;
  for (int64_t q0 = 0; q0 < Q; q0 += G) {
    const int64_t g = std::min<int64_t>(G, Q - q0);
    LK_TRY(launch_scores_batch(ix, d_queries + q0 * T, g, T, Np, scores, st));
    hipLaunchKernelGGL(lk_init_kernel, dim3(1), dim3(64), 0, st, state, g, (uint32_t)kv, cnt);
    const dim3 grid(grid_for(n4, 256 * 8, 1024), (unsigned)g);
    for (int shift = 56; shift >= 0; shift -= 8) {
      hipLaunchKernelGGL(lk_hist_kernel, grid, dim3(256), 0, st, scores, Np, ix.n_docs, shift,
                         state, hist);
      hipLaunchKernelGGL(lk_pick_kernel, dim3((unsigned)g), dim3(64), 0, st, state, hist, shift);
    }
    hipLaunchKernelGGL(lk_compact_kernel, grid, dim3(256), 0, st, scores, Np, ix.n_docs, state, cnt,
                       keys, (int64_t)kv);
    if (!lds_sort_write(keys, g, kv, k, ix.doc_offset, d_docs + q0 * k, d_scores + q0 * k, st)) {
      const uint64_t* sorted = nullptr;
      LK_TRY(sort_rows(keys, alt, g, kv, tmp, &sorted, st));
      hipLaunchKernelGGL(lk_write_kernel, dim3(grid_for(g * k, 256, 4096)), dim3(256), 0, st,
                         sorted, (int64_t)kv, g, k, kv, ix.doc_offset, d_docs + q0 * k,
                         d_scores + q0 * k);
    }
    LK_TRY(hipGetLastError());
  }
  return hipSuccess;
}

namespace {

// ---------------------------------------------------------------------------
// The list path (k in (kMaxK, kLargeListMaxK]): no dense score rows.  A
// SAMPLE pass keeps the best key of each 256-doc slice of every P-th tile
// group (launch_sample_large); theta = the k-th best of those keys — k real
// documents score at least theta, so it is a lower bound of the k-th key;
// the REST pass appends every key >= theta to the query's list
// (launch_rest_lists); the k-th key of the list by radix selection, the k
// keys >= it compacted, the rows sorted (bm25mi_sort.hip) and written.  A
// query whose list overflowed, or whose sample or list holds fewer than k
// keys (zero-fill), is answered by the dense path above, on its own.
// ---------------------------------------------------------------------------
constexpr int kSelT = 256;

// Wave-aggregated LDS histogram add (a wave's keys that share a digit add once).
__device__ __forceinline__ void hist_add(uint32_t* h, uint32_t d, bool valid) {
  uint64_t m = __ballot(valid);
#pragma unroll
  for (int b = 0; b < 8; ++b) {
    const uint64_t bb = __ballot(((d >> b) & 1u) != 0u);
    m &= ((d >> b) & 1u) ? bb : ~bb;
  }
  const uint32_t below =
      __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (valid && below == 0u) atomicAdd(&h[d], (uint32_t)__popcll(m));
}

// Exclusive scan of one value per thread of a 256-thread workgroup.
__device__ __forceinline__ uint32_t block_excl256(uint32_t x, uint32_t* wsum) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint32_t incl = wave_scan(x);
  if (lane == 63u) wsum[w] = incl;
  __syncthreads();
  uint32_t pre = 0u;
  for (uint32_t j = 0; j < w; ++j) pre += wsum[j];
  __syncthreads();
  return pre + incl - x;
}

// The k-th largest non-zero key of each row (one workgroup per row), 8 bits
// per pass from the top; a row decided early (every key of its prefix is
// needed) ends with the prefix (lower bits 0), which selects the same keys.
//   MODE 0 (threshold from the sample keys, rows of `stride` keys): out =
//     theta moved into the index's doc frame (sample keys carry global ids),
//     or, with fewer than k keys, the zero-fill threshold (every positive
//     document is listed); lens[row] = 0 (the list count the REST pass
//     appends to); fb[row] = 0.
//   MODE 1 (list select, rows of lens[row] <= cap keys): out = the k-th key,
//     or 0 when the list holds fewer than k keys (all of them, then the
//     smallest zero-score documents: list_compact_kernel); fb = 1 when the
//     list overflowed.
template <int MODE>
__global__ __launch_bounds__(kSelT) void row_kth_kernel(const uint64_t* __restrict__ keys,
                                                        int64_t stride, int32_t* __restrict__ lens,
                                                        int32_t cap, uint32_t k, int64_t doc_offset,
                                                        uint64_t* __restrict__ out,
                                                        int32_t* __restrict__ fb) {
  __shared__ uint32_t h[256];
  __shared__ uint32_t wsum[4];
  __shared__ uint64_t s_prefix;
  __shared__ uint32_t s_need, s_state;  // s_state: 0 continue, 1 decided, 2 too few keys
  const int64_t row = blockIdx.x;
  const uint32_t t = threadIdx.x;
  int64_t n = stride;
  bool over = false;
  if (MODE == 1) {
    const int32_t c = lens[row];
    over = c > cap;
    n = over ? 0 : c;
  }
  const uint64_t* r = keys + row * stride;
  uint64_t prefix = 0ull;
  uint32_t need = k;
  bool found = !over;
  for (int shift = 56; found && shift >= 0; shift -= 8) {
    h[t] = 0u;
    if (t == 0) s_state = 2u;
    __syncthreads();
    const int hs = shift + 8;
    const int64_t rounds = (n + kSelT - 1) / kSelT;  // every lane runs every round (ballots)
    for (int64_t i0 = 0; i0 < rounds; ++i0) {
      const int64_t i = i0 * kSelT + t;
      const uint64_t key = i < n ? r[i] : 0ull;
      const bool in = key != 0ull && (hs >= 64 || ((key ^ prefix) >> hs) == 0ull);
      hist_add(h, (uint32_t)(key >> shift) & 255u, in);
    }
    __syncthreads();
    const uint32_t x = h[255 - t];  // thread t: digit 255 - t (from the top)
    const uint32_t above = block_excl256(x, wsum);
    if (above < need && need <= above + x) {
      s_prefix = prefix | ((uint64_t)(255 - t) << shift);
      s_need = need - above;
      s_state = (x == need - above || shift == 0) ? 1u : 0u;
    }
    __syncthreads();
    const uint32_t st = s_state;
    if (st == 2u) {
      found = false;
      break;
    }
    prefix = s_prefix;
    need = s_need;
    __syncthreads();
    if (st == 1u) break;
  }
  if (t != 0) return;
  if (MODE == 0) {
    lens[row] = 0;
    if (found) {  // into the index's frame: tie doc global -> local (a key of this shard)
      const uint64_t lo = (prefix & 0xFFFFFFFFull) + (uint64_t)doc_offset;
      out[row] = lo <= 0xFFFFFFFFull ? (prefix & ~0xFFFFFFFFull) | lo
                                     : ((prefix >> 32) + 1ull) << 32;
    } else {
      out[row] = (uint64_t)score_key(FLT_MIN) << 32;  // every positive doc (zero fill)
    }
    fb[row] = 0;
  } else {
    out[row] = found ? prefix : 0ull;
    if (over) fb[row] = 1;
  }
}

// The k keys >= kth[row] of each list row (exactly k: keys are unique),
// appended in any order to out[row][0..k); fallback rows are skipped.  A
// row of fewer than k keys (kth = 0: its query has fewer than k positive
// documents) takes all of them and then the smallest document ids it does
// not hold, at score 0 (the reference's argpartition fills its top-k with
// zero-score documents; the (score desc, doc asc) order takes the smallest):
// an LDS bitmap of the held ids below k, scanned in order.
constexpr int kZeroFillWords = (int)(kLargeListMaxK / 32);
__global__ __launch_bounds__(kSelT) void list_compact_kernel(const uint64_t* __restrict__ list,
                                                             int64_t C,
                                                             const int32_t* __restrict__ lens,
                                                             const uint64_t* __restrict__ kth,
                                                             const int32_t* __restrict__ fb,
                                                             int64_t k, uint64_t* __restrict__ out) {
  __shared__ int32_t s_pos;
  __shared__ uint32_t bm[kZeroFillWords];
  __shared__ uint32_t wsum[4];
  const int64_t row = blockIdx.x;
  if (fb[row]) return;  // block-uniform; before the barriers
  const uint64_t th = kth[row];
  const int64_t n = lens[row];
  if (th == 0ull) {  // zero fill: all n < k keys, then the first k - n ids not held
    const uint64_t* r = list + row * C;
    const int64_t words = (k + 31) >> 5;
    for (int64_t w = threadIdx.x; w < words; w += kSelT) bm[w] = 0u;
    __syncthreads();
    for (int64_t i = threadIdx.x; i < n; i += kSelT) {
      const uint64_t key = r[i];
      out[row * k + i] = key;
      const uint32_t d = 0xFFFFFFFFu - (uint32_t)key;
      if ((int64_t)d < k) atomicOr(&bm[d >> 5], 1u << (d & 31u));
    }
    __syncthreads();
    const uint64_t zkey = (uint64_t)score_key(0.f) << 32;
    uint32_t carry = 0u;
    for (int64_t w0 = 0; w0 < words; w0 += kSelT) {
      const int64_t w = w0 + threadIdx.x;
      uint32_t free_bits = 0u;
      if (w < words) {
        free_bits = ~bm[w];
        const int64_t hi = k - 32 * w;  // ids past k - 1 are not candidates
        if (hi < 32) free_bits &= (1u << hi) - 1u;
      }
      const uint32_t c = (uint32_t)__popc(free_bits);
      const uint32_t ex = block_excl256(c, wsum);
      uint32_t pos = carry + ex;
      while (free_bits != 0u && (int64_t)(n + pos) < k) {
        const uint32_t b = (uint32_t)__builtin_ctz(free_bits);
        free_bits &= free_bits - 1u;
        const uint32_t d = (uint32_t)(32 * w) + b;
        out[row * k + n + pos] = zkey | (uint64_t)(0xFFFFFFFFu - d);
        ++pos;
      }
      // every thread needs the round's total: the last thread's ex + c
      __shared__ uint32_t s_tot;
      if (threadIdx.x == kSelT - 1) s_tot = ex + c;
      __syncthreads();
      carry += s_tot;
      __syncthreads();
    }
    return;
  }
  if (threadIdx.x == 0) s_pos = 0;
  __syncthreads();
  const uint64_t* r = list + row * C;
  const uint32_t lane = threadIdx.x & 63u;
  const int64_t rounds = (n + kSelT - 1) / kSelT;
  for (int64_t i0 = 0; i0 < rounds; ++i0) {
    const int64_t i = i0 * kSelT + threadIdx.x;
    const uint64_t key = i < n ? r[i] : 0ull;
    const bool keep = key != 0ull && key >= th;
    const uint64_t m = __ballot(keep);
    if (m == 0ull) continue;
    int p0 = 0;
    if (lane == 0) p0 = atomicAdd(&s_pos, (int)__popcll(m));
    p0 = __shfl(p0, 0, 64);
    const int pos = p0 + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (keep && pos < k) out[row * k + pos] = key;
  }
}

// The REST pass's per-tile slots (emit_rest_slot, bm25mi_kernels.hip) of each
// query gathered into its list: the slots' keys in tile order, then the
// overflow keys; lens[row] = their number, or cap + 1 when they do not fit
// (row_kth_kernel<1> then sends the query to the dense path).  One workgroup
// per query.
__global__ __launch_bounds__(kSelT) void slot_pack_kernel(const uint64_t* __restrict__ slots,
                                                          const int32_t* __restrict__ slot_cnt,
                                                          int64_t ntiles, int32_t Cb,
                                                          const uint64_t* __restrict__ ovf,
                                                          int32_t Co, int32_t* __restrict__ lens,
                                                          uint64_t* __restrict__ list, int64_t C) {
  __shared__ uint32_t wsum[4];
  __shared__ uint32_t s_tot;
  __shared__ uint32_t offs[kSelT];
  const int64_t row = blockIdx.x;
  const int32_t* cn = slot_cnt + row * ntiles;
  const uint64_t* sl = slots + row * ntiles * Cb;
  const int32_t no = lens[row];  // overflow keys (the REST pass's list count)
  uint64_t* out = list + row * C;
  if (no > Co) {  // block-uniform, before the barriers
    if (threadIdx.x == 0) lens[row] = (int32_t)(C + 1);
    return;
  }
  uint32_t carry = 0u;
  for (int64_t t0 = 0; t0 < ntiles; t0 += kSelT) {
    const int64_t t = t0 + threadIdx.x;
    const uint32_t n = t < ntiles ? (uint32_t)min(cn[t], Cb) : 0u;
    const uint32_t ex = block_excl256(n, wsum);
    offs[threadIdx.x] = ex;
    if (threadIdx.x == kSelT - 1) s_tot = ex + n;
    __syncthreads();
    // the round's keys copied by all threads at once (independent loads): key
    // e is in the last slot whose offset is <= e
    const uint32_t tot = s_tot;
    for (uint32_t e = threadIdx.x; e < tot; e += kSelT) {
      uint32_t lo = 0u, hi = kSelT - 1u;
      while (lo < hi) {
        const uint32_t mid = (lo + hi + 1u) >> 1;
        if (offs[mid] <= e) lo = mid;
        else hi = mid - 1u;
      }
      if ((int64_t)(carry + e) < C) out[carry + e] = sl[(t0 + lo) * Cb + (e - offs[lo])];
    }
    carry += tot;
    __syncthreads();
  }
  for (int32_t i = threadIdx.x; i < no; i += kSelT)
    if ((int64_t)carry + i < C) out[carry + i] = ovf[row * Co + i];
  if (threadIdx.x == 0) {
    const int64_t total = (int64_t)carry + no;
    lens[row] = total > C ? (int32_t)(C + 1) : (int32_t)total;
  }
}

// Rows of the fallback queries: ids[j] = the j-th row with fb set (host-built),
// queries gathered / results scattered.
__global__ __launch_bounds__(256) void gather_rows_kernel(const int32_t* __restrict__ src,
                                                          const int32_t* __restrict__ ids,
                                                          int64_t n, int64_t width,
                                                          int32_t* __restrict__ dst) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n * width;
       e += (int64_t)gridDim.x * 256) {
    const int64_t j = e / width, c = e - j * width;
    dst[e] = src[(int64_t)ids[j] * width + c];
  }
}

__global__ __launch_bounds__(256) void scatter_rows_kernel(const int32_t* __restrict__ sd,
                                                           const float* __restrict__ ss,
                                                           const int32_t* __restrict__ ids,
                                                           int64_t n, int64_t width,
                                                           int32_t* __restrict__ dd,
                                                           float* __restrict__ ds) {
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n * width;
       e += (int64_t)gridDim.x * 256) {
    const int64_t j = e / width, c = e - j * width;
    dd[(int64_t)ids[j] * width + c] = sd[e];
    ds[(int64_t)ids[j] * width + c] = ss[e];
  }
}

}  // namespace

// Geometry of the list path: sampling stride P (the largest of 8, 4, 2 whose
// sample holds >= 2k keys, else 2 when it holds >= k), kLargeM keys per
// sample tile; P = 0: the list path does not apply.
SampleGeom large_geom(const DevIndex& ix, int64_t k) {
  for (int need = 2; need >= 1; --need)
    for (int P = 8; P >= 2; P >>= 1) {
      if (ix.ntiles < 2 * P) continue;
      const int G = ix.ntiles >= 4 * kSampleGroup * P ? kSampleGroup : 1;
      // sample_count (bm25mi_kernels.hip): groups of G tiles every G * P
      const int64_t r = ix.ntiles % (G * P);
      const int64_t nS = (ix.ntiles / (G * P)) * G + (r < G ? r : G);
      if (nS * kLargeM >= need * k && (need == 2 || P == 2)) return SampleGeom{P, kLargeM, nS * kLargeM, G};
    }
  return SampleGeom{0, 0, 0, 1};
}

hipError_t launch_search_large_lists(const DevIndex& ix, const int32_t* d_queries, int64_t Q,
                                     int64_t T, int k, const Workspace& ws, int32_t* d_docs,
                                     float* d_scores, int64_t* n_fallback, hipStream_t st) {
  *n_fallback = 0;
  if (Q == 0 || k == 0) return hipSuccess;
  const SampleGeom g = large_geom(ix, k);
  if (g.P == 0 || k > ix.n_docs || !large_list_supported(ix, T, Q)) return hipErrorInvalidValue;
  ix.disp.kernels |= kKLarge | kKFlatSample | kKFlatRest;
  ix.disp.sample_p = g.P;
  // list capacity: the list_cap option, else 4 P k (the k-th sample key of a
  // 1-in-P sample sits near the (P k)-th key; 4x headroom for slice effects)
  const int64_t C = ix.opt.list_cap > 0 ? (int64_t)ix.opt.list_cap
                                        : std::min<int64_t>(1 << 20, 4 * (int64_t)g.P * k);
  // REST's per-tile slots: Cb keys each, ~4x the mean a tile lists when the
  // list reaches its capacity C; keys past a slot go to an overflow list of C / 2
  const int32_t Cb = (int32_t)std::min<int64_t>(
      512, std::max<int64_t>(8, ((C + ix.ntiles - 1) / ix.ntiles + 7) / 8 * 8));
  const int64_t Co = std::max<int64_t>(1, C / 2);
  const int64_t per_q = (g.S + C + 2 * (int64_t)k + ix.ntiles * Cb + Co) * 8 + ix.ntiles * 4 +
                        64 + 8 * (int64_t)k + (int64_t)radix_sort_scratch_bytes(k) + 64;
  int64_t G = std::max<int64_t>(1, std::min<int64_t>(Q, budget_of(ws.arena) / per_q));
  G = std::min<int64_t>(G, std::max<int64_t>(1, (int64_t)INT32_MAX / C - 1));
  Scratch sc(st, ws.arena);
  uint64_t *skeys = nullptr, *theta = nullptr, *list = nullptr, *kth = nullptr, *keys = nullptr,
           *alt = nullptr, *slots = nullptr, *ovf = nullptr;
  int32_t *cnt = nullptr, *fb = nullptr, *slot_cnt = nullptr;
  char* tmp = nullptr;
  LK_TRY(sc.get(&slots, G * ix.ntiles * Cb));
  LK_TRY(sc.get(&slot_cnt, G * ix.ntiles));
  LK_TRY(sc.get(&ovf, G * Co));
  LK_TRY(sc.get(&skeys, G * g.S));
  LK_TRY(sc.get(&theta, G));
  LK_TRY(sc.get(&list, G * C));
  LK_TRY(sc.get(&kth, G));
  LK_TRY(sc.get(&keys, G * k));
  LK_TRY(sc.get(&alt, G * k));
  LK_TRY(sc.get(&cnt, G));
  LK_TRY(sc.get(&fb, Q));
  LK_TRY(sc.get(&tmp, sort_bytes(G, k)));
  Workspace w = ws;  // the handle's claim counters, counters and segment table
  w.theta = theta;
  w.list = ovf;  // REST: the slots' overflow
  w.list_cnt = cnt;
  w.list_cap = (int32_t)Co;
  w.slots = slots;
  w.slot_cnt = slot_cnt;
  w.slot_cap = Cb;
  for (int64_t q0 = 0; q0 < Q; q0 += G) {
    const int64_t gq = std::min<int64_t>(G, Q - q0);
    const int32_t* q = d_queries + q0 * T;
    LK_TRY(launch_sample_large(ix, q, gq, T, g, skeys, w, st));
    hipLaunchKernelGGL(row_kth_kernel<0>, dim3((unsigned)gq), dim3(kSelT), 0, st, skeys, g.S, cnt,
                       0, (uint32_t)k, ix.doc_offset, theta, fb + q0);
    LK_TRY(hipMemsetAsync(ws.counters, 0, sizeof(int32_t) * kCounters, st));
    LK_TRY(hipMemsetAsync(slot_cnt, 0, sizeof(int32_t) * gq * ix.ntiles, st));
    LK_TRY(launch_rest_lists(ix, q, gq, T, g, w, st));
    hipLaunchKernelGGL(slot_pack_kernel, dim3((unsigned)gq), dim3(kSelT), 0, st, slots, slot_cnt,
                       ix.ntiles, Cb, ovf, (int32_t)Co, cnt, list, C);
    hipLaunchKernelGGL(row_kth_kernel<1>, dim3((unsigned)gq), dim3(kSelT), 0, st, list, C, cnt,
                       (int32_t)C, (uint32_t)k, 0ll, kth, fb + q0);
    hipLaunchKernelGGL(list_compact_kernel, dim3((unsigned)gq), dim3(kSelT), 0, st, list, C, cnt,
                       kth, fb + q0, (int64_t)k, keys);
    if (!lds_sort_write(keys, gq, k, k, ix.doc_offset, d_docs + q0 * k, d_scores + q0 * k, st)) {
      const uint64_t* sorted = nullptr;
      LK_TRY(sort_rows(keys, alt, gq, k, tmp, &sorted, st));
      hipLaunchKernelGGL(lk_write_kernel, dim3(grid_for(gq * k, 256, 4096)), dim3(256), 0, st,
                         sorted, (int64_t)k, gq, k, k, ix.doc_offset, d_docs + q0 * k,
                         d_scores + q0 * k);
    }
    LK_TRY(hipGetLastError());
  }
  // the queries the lists could not serve: the dense path, on their own (the
  // one host synchronisation of this path: their number sizes that pass)
  std::vector<int32_t> hfb((size_t)Q);
  LK_TRY(hipMemcpyAsync(hfb.data(), fb, sizeof(int32_t) * Q, hipMemcpyDeviceToHost, st));
  LK_TRY(hipStreamSynchronize(st));
  std::vector<int32_t> ids;
  for (int64_t i = 0; i < Q; ++i)
    if (hfb[(size_t)i]) ids.push_back((int32_t)i);
  *n_fallback = (int64_t)ids.size();
  if (ids.empty()) return hipSuccess;
  const int64_t nf = (int64_t)ids.size();
  int32_t *d_ids = nullptr, *fq = nullptr, *fd = nullptr;
  float* fs = nullptr;
  LK_TRY(sc.get(&d_ids, nf));
  LK_TRY(sc.get(&fq, nf * std::max<int64_t>(T, 1)));
  LK_TRY(sc.get(&fd, nf * k));
  LK_TRY(sc.get(&fs, nf * k));
  LK_TRY(hipMemcpyAsync(d_ids, ids.data(), sizeof(int32_t) * nf, hipMemcpyHostToDevice, st));
  if (T > 0)
    hipLaunchKernelGGL(gather_rows_kernel, dim3(grid_for(nf * T, 256, 4096)), dim3(256), 0, st,
                       d_queries, d_ids, nf, T, fq);
  // the dense rows get what this sequence's scratch leaves of the budget
  const int64_t left = budget_of(ws.arena) - (int64_t)sc.total;
  LK_TRY(launch_search_large(ix, fq, nf, T, k, fd, fs, st, ws.arena,
                             std::max<int64_t>(left, 64ll << 20)));
  hipLaunchKernelGGL(scatter_rows_kernel, dim3(grid_for(nf * k, 256, 4096)), dim3(256), 0, st, fd,
                     fs, d_ids, nf, (int64_t)k, d_docs, d_scores);
  // (ids lives on the host until the copy above has run)
  LK_TRY(hipStreamSynchronize(st));
  return hipGetLastError();
}

hipError_t launch_merge_large(const int32_t* d_docs, const float* d_scores, int64_t W, int64_t Q,
                              int k, int64_t rank_stride, int32_t* d_out_docs,
                              float* d_out_scores, hipStream_t st) {
  if (Q == 0 || k == 0) return hipSuccess;
  const int64_t n = W * (int64_t)k;
  if (n > INT32_MAX / 2) return hipErrorInvalidValue;
  const int64_t per_q = n * 16 + 64 + sort_bytes(1, n);
  int64_t G = std::max<int64_t>(1, std::min<int64_t>(Q, large_budget() / per_q));
  G = std::min<int64_t>(G, std::max<int64_t>(1, (int64_t)INT32_MAX / n - 1));
  const int64_t sb = sort_bytes(G, n);
  Scratch sc(st);
  uint64_t *keys = nullptr, *alt = nullptr;
  char* tmp = nullptr;
  LK_TRY(sc.get(&keys, G * n));
  LK_TRY(sc.get(&alt, G * n));
  LK_TRY(sc.get(&tmp, sb));
  for (int64_t q0 = 0; q0 < Q; q0 += G) {
    const int64_t g = std::min<int64_t>(G, Q - q0);
    hipLaunchKernelGGL(lk_list_keys_kernel, dim3(grid_for(g * n, 256, 8192)), dim3(256), 0, st,
                       d_docs, d_scores, W, q0, g, k, rank_stride, keys);
    const uint64_t* sorted = nullptr;
    LK_TRY(sort_rows(keys, alt, g, n, tmp, &sorted, st));
    hipLaunchKernelGGL(lk_write_kernel, dim3(grid_for(g * k, 256, 4096)), dim3(256), 0, st, sorted,
                       n, g, k, k, 0ll, d_out_docs + q0 * k, d_out_scores + q0 * k);
    LK_TRY(hipGetLastError());
  }
  return hipSuccess;
}

}  // namespace bm25mi
