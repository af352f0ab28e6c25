// bm25mi_kernels.hip — gfx950 kernels of the BM25 CSC query path.
//
// Replaces the reference's GPU path (MAX graph ops.gather -> ops.sum ->
// ops.top_k, gpu_bm25/common.py:64-80, vendored as
// operations/gather_scatter.mojo:683-763 and operations/topk.mojo:576-963)
// and its CPU scorer (bm25_native.py:149-158, 204-214) with a doc-tiled
// sparse design:
//
//   score_tiles   one workgroup per (doc tile, query): gathers the query's
//                 posting segments inside the tile (coalesced reads of the
//                 CSC `data` + u16 local doc ids), scatter-adds them into an
//                 fp32 LDS accumulator term by term in query order (the exact
//                 fp32 arithmetic of scipy csc_matvec, bm25_native.py:152),
//                 then extracts the tile's top-kTileM keys with wave64
//                 shuffle/ballot argmax rounds.
//   merge         one workgroup per query: bitonic-sorts the per-tile
//                 candidates in LDS, picks the top-k and flags the (rare)
//                 tiles whose kTileM-th candidate beats the k-th key.
//   rescore       persistent: exact top-k of each flagged tile.
//   merge(final)  merges the exact lists of flagged tiles.
// The result is exactly the top-k under (score desc, doc asc) of the dense
// score vector, with untouched documents scoring 0.
#include "bm25mi_internal.h"

namespace bm25mi {

constexpr int kTG = 16;  // query terms staged in LDS per group
constexpr int kR = 8;    // postings held in registers per thread per chunk
constexpr int kE = 32;   // accumulator entries owned by a thread in selection

struct IndexArgs {
  const int64_t* indptr;
  const uint32_t* rel;
  const uint16_t* ldoc;
  const float* val;
  int64_t V, ntiles, n_docs;
};

static IndexArgs args_of(const DevIndex& ix) {
  return IndexArgs{ix.indptr, ix.rel, ix.ldoc, ix.val, ix.n_terms, ix.ntiles, ix.n_docs};
}

struct TileShared {
  int64_t base[kTG];        // global posting index = base[s] + concat position
  uint32_t start[kTG + 1];  // prefix of segment lengths
  uint32_t red[2][16];      // per-wave argmax values, double-buffered
  int32_t item;
};

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint32_t w = (uint32_t)__shfl_xor((int)v, o, 64);
    v = v > w ? v : w;
  }
  return v;
}

// ---------------------------------------------------------------------------
// Scatter phase: acc[d] = sum over query terms (in order) of the term's score
// for doc d of this tile.  Replaces doc_toks[:, query].sum(axis=1)
// (bm25_native.py:152 -> scipy csc_matvec): same fp32 adds, same order per doc.
// ---------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void accumulate_tile(const IndexArgs& a, int64_t tile,
                                                const int32_t* __restrict__ qterms,
                                                int T, float* acc, TileShared& sm) {
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  const int tid = threadIdx.x;

  float4* acc4 = reinterpret_cast<float4*>(acc);
#pragma unroll
  for (int j = 0; j < kE / 4; ++j) acc4[j * NT + tid] = make_float4(0.f, 0.f, 0.f, 0.f);

  for (int g0 = 0; g0 < T; g0 += kTG) {
    const int ng = min(kTG, T - g0);
    __syncthreads();  // zeroing / previous group's reads of sm are done
    if (tid < ng) {
      const int32_t term = qterms[g0 + tid];
      int64_t lo = 0;
      uint32_t len = 0;
      if (term >= 0 && term < a.V) {  // negative ids are padding (bm25_native.py:151)
        const uint32_t* r = a.rel + (int64_t)term * (a.ntiles + 1) + tile;
        const uint32_t r0 = r[0], r1 = r[1];
        lo = a.indptr[term] + r0;
        len = r1 - r0;
      }
      sm.base[tid] = lo;
      sm.start[tid + 1] = len;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t s = 0;
      sm.start[0] = 0;
      for (int i = 0; i < ng; ++i) {
        const uint32_t len = sm.start[i + 1];
        sm.base[i] -= (int64_t)s;
        s += len;
        sm.start[i + 1] = s;
      }
    }
    __syncthreads();
    const uint32_t total = sm.start[ng];
    for (uint32_t cb = 0; cb < total; cb += NT * kR) {
      // 1) positions -> global posting indices (no memory traffic)
      int64_t gidx[kR];
      int sg[kR];
      int s = 0;
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        uint32_t P = cb + r * NT + tid;
        sg[r] = P < total ? 0 : -1;
        P = P < total ? P : total - 1;
        while (s + 1 < ng && P >= sm.start[s + 1]) ++s;
        sg[r] = sg[r] < 0 ? -1 : s;
        gidx[r] = sm.base[s] + (int64_t)P;
      }
      // 2) issue every load of the chunk before the first use
      uint32_t ld[kR];
      float v[kR];
#pragma unroll
      for (int r = 0; r < kR; ++r) {
        ld[r] = a.ldoc[gidx[r]];
        v[r] = a.val[gidx[r]];
      }
      // 3) LDS adds, one term after the other (a doc occurs once per term, so
      //    within a term the adds commute; across terms the barrier keeps
      //    query order, bm25_native.py:152 / csc_matvec)
      const uint32_t ce = cb + NT * kR;
      for (int s2 = 0; s2 < ng; ++s2) {
        if (sm.start[s2 + 1] <= cb || sm.start[s2] >= ce) continue;  // block-uniform
#pragma unroll
        for (int r = 0; r < kR; ++r)
          if (sg[r] == s2) atomicAdd(&acc[ld[r]], v[r]);
        __syncthreads();
      }
    }
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------
// Selection phase: the m best keys of the tile, best first, written to out[].
// Thread t owns docs [t*kE, t*kE + kE) of the tile, so "first wave, first
// lane, first entry" among equal scores is the smallest doc id.
// ---------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void select_tile(const float* acc, int64_t tile, int64_t n_docs,
                                            int m, uint64_t* __restrict__ out,
                                            TileShared& sm) {
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  constexpr int NW = NT / 64;
  constexpr int C4 = kE / 4;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float4* acc4 = reinterpret_cast<const float4*>(acc);
  const int swz = tid & 7;  // rotate chunk order across lanes: spreads LDS banks
  const int64_t doc0 = tile * D + (int64_t)tid * kE;

  uint32_t key[kE];
#pragma unroll
  for (int j = 0; j < C4; ++j) {
    const float4 f = acc4[tid * C4 + (j ^ swz)];
    key[j * 4 + 0] = score_key(f.x);
    key[j * 4 + 1] = score_key(f.y);
    key[j * 4 + 2] = score_key(f.z);
    key[j * 4 + 3] = score_key(f.w);
  }
  if (doc0 + kE > n_docs) {
#pragma unroll
    for (int j = 0; j < C4; ++j)
#pragma unroll
      for (int c = 0; c < 4; ++c)
        if (doc0 + ((j ^ swz) * 4 + c) >= n_docs) key[j * 4 + c] = 0;
  }
  uint32_t lmax = 0;
#pragma unroll
  for (int i = 0; i < kE; ++i) lmax = lmax > key[i] ? lmax : key[i];

  for (int r = 0; r < m; ++r) {
    const uint32_t wm = wave_max_u32(lmax);
    const unsigned long long bal = __ballot(lmax == wm);
    const int wl = __ffsll(bal) - 1;
    if (lane == 0) sm.red[r & 1][wave] = wm;
    __syncthreads();
    uint32_t bm = 0;
    int ws = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint32_t x = sm.red[r & 1][w];
      if (x > bm) { bm = x; ws = w; }
    }
    if (bm == 0) {  // no valid entry left (tile smaller than m)
      if (tid == 0) out[r] = 0;
      continue;
    }
    if (wave == ws && lane == wl) {
      int eb = kE;
#pragma unroll
      for (int j = 0; j < C4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int e = (j ^ swz) * 4 + c;
          if (key[j * 4 + c] == bm && e < eb) eb = e;
        }
      out[r] = ((uint64_t)bm << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(doc0 + eb));
      lmax = 0;
#pragma unroll
      for (int j = 0; j < C4; ++j)
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          if ((j ^ swz) * 4 + c == eb) key[j * 4 + c] = 0;
          lmax = lmax > key[j * 4 + c] ? lmax : key[j * 4 + c];
        }
    }
  }
}

// One workgroup per (tile, query); blocks are dealt round-robin over the 8
// XCDs (b % 8), so block b maps to item (b % 8) * per + b / 8: each XCD walks
// its own contiguous run of tiles, all queries of a tile back to back, and the
// tile's hot posting segments stay in that XCD's L2.
template <int S>
__global__ __launch_bounds__((1 << S) / kE) void score_tiles_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t Q, int32_t T,
    uint64_t* __restrict__ cand) {
  __shared__ __attribute__((aligned(16))) float acc[1 << S];
  __shared__ TileShared sm;
  const int64_t nitems = a.ntiles * (int64_t)Q;
  const int64_t per = (nitems + 7) >> 3;
  const int64_t b = blockIdx.x;
  const int64_t item = (b & 7) * per + (b >> 3);
  if (item >= nitems) return;
  const int64_t tile = item / Q;
  const int64_t q = item - tile * Q;
  accumulate_tile<S>(a, tile, queries + q * T, T, acc, sm);
  select_tile<S>(acc, tile, a.n_docs, kTileM, cand + (q * a.ntiles + tile) * kTileM, sm);
}

// Exact top-k of each flagged tile; persistent, pulls items from the queue
// the merge kernel filled (every wave reaches the exit test each iteration).
template <int S>
__global__ __launch_bounds__((1 << S) / kE) void rescore_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, int32_t k,
    int64_t maxflag, Workspace ws) {
  __shared__ __attribute__((aligned(16))) float acc[1 << S];
  __shared__ TileShared sm;
  const int32_t n_items = ws.counters[0];
  for (;;) {
    __syncthreads();
    if (threadIdx.x == 0) sm.item = atomicAdd(&ws.counters[1], 1);
    __syncthreads();
    const int32_t it = sm.item;
    if (it >= n_items) break;
    const int32_t code = ws.queue[it];
    const int64_t q = code / maxflag;
    const int64_t tile = ws.flag_tiles[code];
    accumulate_tile<S>(a, tile, queries + q * T, T, acc, sm);
    select_tile<S>(acc, tile, a.n_docs, k, ws.cand2 + (int64_t)code * k, sm);
  }
}

template <int S>
__global__ __launch_bounds__((1 << S) / kE) void scores_dense_kernel(
    IndexArgs a, const int32_t* __restrict__ query, int32_t T, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float acc[1 << S];
  __shared__ TileShared sm;
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  const int64_t tile = blockIdx.x;
  accumulate_tile<S>(a, tile, query, T, acc, sm);
  const int64_t d0 = tile * D;
  if (d0 + D <= a.n_docs) {
    float4* o4 = reinterpret_cast<float4*>(out + d0);
    const float4* acc4 = reinterpret_cast<const float4*>(acc);
#pragma unroll
    for (int j = 0; j < kE / 4; ++j) o4[j * NT + threadIdx.x] = acc4[j * NT + threadIdx.x];
  } else {
    for (int64_t e = threadIdx.x; d0 + e < a.n_docs; e += NT) out[d0 + e] = acc[e];
  }
}

// ---------------------------------------------------------------------------
// Index build: u16 local doc ids + per-(term, tile) segment table, one wave
// per term.  Flags non-canonical input (unsorted / duplicate / out-of-range
// doc ids inside a column) in *err.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void build_tables_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, int64_t V,
    int64_t n_docs, int S, int64_t ntiles, uint32_t* __restrict__ rel,
    uint16_t* __restrict__ ldoc, int32_t* __restrict__ err) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const uint32_t mask = (1u << S) - 1u;
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < V;
       t += waves) {
    const int64_t a0 = indptr[t], a1 = indptr[t + 1];
    uint32_t* row = rel + t * (ntiles + 1);
    for (int64_t p = a0 + lane; p < a1; p += 64) {
      const int32_t d = indices[p];
      const int32_t dp = p > a0 ? indices[p - 1] : -1;
      const bool ok = d >= 0 && (int64_t)d < n_docs && d > dp;
      if (!ok) atomicOr(err, 1);
      ldoc[p] = (uint16_t)((uint32_t)d & mask);
      if (ok) {
        const int64_t tp = dp >= 0 ? ((int64_t)dp >> S) : -1;
        const int64_t tc = (int64_t)d >> S;
        for (int64_t j = tp + 1; j <= tc; ++j) row[j] = (uint32_t)(p - a0);
      }
    }
    int64_t last = -1;
    if (a1 > a0) {
      const int32_t dl = indices[a1 - 1];
      last = (dl >= 0 && (int64_t)dl < n_docs) ? ((int64_t)dl >> S) : ntiles - 1;
    }
    for (int64_t j = last + 1 + lane; j <= ntiles; j += 64) row[j] = (uint32_t)(a1 - a0);
  }
}

// ---------------------------------------------------------------------------
// Merge: one workgroup per query, bitonic sort of u64 keys in LDS.
// ---------------------------------------------------------------------------
constexpr int kMergeNT = 1024;
constexpr int kMaxFlagBits = 65536;  // tiles per query addressable by the flag bitmap

__device__ __forceinline__ void bitonic_sort_desc(uint64_t* keys, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = threadIdx.x; i < (n >> 1); i += blockDim.x) {
        const int lo = 2 * stride * (i / stride) + (i % stride);
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const uint64_t x = keys[lo], y = keys[hi];
        if ((x < y) == desc) { keys[lo] = y; keys[hi] = x; }
      }
      __syncthreads();
    }
  }
}

__device__ __forceinline__ int next_pow2(int64_t x) {
  int n = 1;
  while (n < x) n <<= 1;
  return n;
}

// keys[0..k) <- the k largest candidates of src (src(i), i < n_total), sorted.
template <class Src>
__device__ void topk_of(const Src& src, int64_t n_total, int k, uint64_t* keys) {
  const int B = next_pow2(k);
  int64_t done = n_total < kMergeP ? n_total : kMergeP;
  int n = next_pow2(done > B ? done : B);
  for (int i = threadIdx.x; i < n; i += blockDim.x) keys[i] = i < done ? src(i) : 0ull;
  __syncthreads();
  bitonic_sort_desc(keys, n);
  while (done < n_total) {
    const int64_t rem = n_total - done;
    const int chunk = (int)(rem < kMergeP - B ? rem : kMergeP - B);
    const int n2 = next_pow2(B + chunk);
    for (int i = threadIdx.x; i < n2 - B; i += blockDim.x)
      keys[B + i] = i < chunk ? src(done + i) : 0ull;
    __syncthreads();
    bitonic_sort_desc(keys, n2);
    done += chunk;
  }
}

__device__ __forceinline__ void write_result(const uint64_t* keys, int k, int64_t row,
                                             int64_t doc_offset, int32_t* __restrict__ docs,
                                             float* __restrict__ scores) {
  for (int i = threadIdx.x; i < k; i += blockDim.x) {
    const uint64_t key = keys[i];
    docs[row * k + i] = (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)key) + doc_offset);
    scores[row * k + i] = key_score((uint32_t)(key >> 32));
  }
}

struct SrcFirst {
  const uint64_t* c;
  __device__ uint64_t operator()(int64_t i) const { return c[i]; }
};

struct SrcFinal {
  const uint64_t* c;      // this query's [ntiles][M] candidates
  const uint64_t* c2;     // this query's flagged tiles' exact lists, contiguous
  const uint32_t* bits;   // LDS bitmap of flagged tiles
  int64_t n1;
  __device__ uint64_t operator()(int64_t i) const {
    if (i < n1) {
      const int64_t j = i / kTileM;
      return ((bits[j >> 5] >> (j & 31)) & 1u) ? 0ull : c[i];
    }
    return c2[i - n1];
  }
};

struct SrcLists {
  const int32_t* docs;
  const float* scores;
  int64_t Q, q;
  int k;
  __device__ uint64_t operator()(int64_t i) const {
    const int64_t w = i / k, j = i - w * k;
    const int64_t o = (w * Q + q) * k + j;
    return make_key(scores[o], (uint32_t)docs[o]);
  }
};

__global__ __launch_bounds__(kMergeNT) void merge_first_kernel(
    const uint64_t* __restrict__ cand, int64_t ntiles, int32_t k, int64_t maxflag,
    int64_t doc_offset, Workspace ws, int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  __shared__ int32_t s_nflag;
  const int64_t q = blockIdx.x;
  const uint64_t* c = cand + q * ntiles * kTileM;
  if (threadIdx.x == 0) s_nflag = 0;
  topk_of(SrcFirst{c}, ntiles * kTileM, k, keys);
  const uint64_t theta = keys[k - 1];
  if (k > kTileM) {
    // A tile whose kTileM-th candidate beats theta may hold unreported docs
    // of the top-k: schedule it for an exact rescore (at most (k-1)/kTileM).
    for (int64_t j = threadIdx.x; j < ntiles; j += blockDim.x) {
      if (c[j * kTileM + kTileM - 1] > theta) {
        const int i = atomicAdd(&s_nflag, 1);
        if (i < maxflag) ws.flag_tiles[q * maxflag + i] = (int32_t)j;
      }
    }
  }
  __syncthreads();
  const int nf = s_nflag < maxflag ? s_nflag : (int)maxflag;
  if (threadIdx.x == 0) {
    ws.nflag[q] = nf;
    if (nf > 0) {
      const int base = atomicAdd(&ws.counters[0], nf);
      for (int i = 0; i < nf; ++i) ws.queue[base + i] = (int32_t)(q * maxflag + i);
    }
  }
  if (nf == 0) write_result(keys, k, q, doc_offset, docs, scores);
}

__global__ __launch_bounds__(kMergeNT) void merge_final_kernel(
    const uint64_t* __restrict__ cand, int64_t ntiles, int32_t k, int64_t maxflag,
    int64_t doc_offset, Workspace ws, int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  __shared__ uint32_t bits[kMaxFlagBits / 32];
  const int64_t q = blockIdx.x;
  const int nf = ws.nflag[q];
  if (nf == 0) return;
  const int64_t nwords = (ntiles + 31) >> 5;
  for (int64_t i = threadIdx.x; i < nwords; i += blockDim.x) bits[i] = 0;
  __syncthreads();
  if ((int)threadIdx.x < nf) {
    const int32_t j = ws.flag_tiles[q * maxflag + threadIdx.x];
    atomicOr(&bits[j >> 5], 1u << (j & 31));
  }
  __syncthreads();
  SrcFinal src{cand + q * ntiles * kTileM, ws.cand2 + q * maxflag * (int64_t)k, bits,
               ntiles * kTileM};
  topk_of(src, ntiles * kTileM + (int64_t)nf * k, k, keys);
  write_result(keys, k, q, doc_offset, docs, scores);
}

__global__ __launch_bounds__(kMergeNT) void merge_lists_kernel(
    const int32_t* __restrict__ in_docs, const float* __restrict__ in_scores, int64_t W,
    int64_t Q, int32_t k, int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  const int64_t q = blockIdx.x;
  topk_of(SrcLists{in_docs, in_scores, Q, q, k}, W * k, k, keys);
  write_result(keys, k, q, 0, docs, scores);
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
bool tile_shift_supported(int s) { return s == 13 || s == 14 || s == 15; }

hipError_t launch_build_tables(const DevIndex& ix, const int32_t* d_indices, int32_t* d_err,
                               hipStream_t stream) {
  if (ix.n_terms == 0) return hipSuccess;
  int64_t blocks = (ix.n_terms + 3) / 4;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(build_tables_kernel, dim3((unsigned)blocks), dim3(256), 0, stream,
                     ix.indptr, d_indices, ix.n_terms, ix.n_docs, ix.tile_shift, ix.ntiles,
                     ix.rel, ix.ldoc, d_err);
  return hipGetLastError();
}

template <int S>
static void launch_score_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T,
                           const Workspace& ws, hipStream_t st) {
  const int64_t nitems = ix.ntiles * Q;
  const int64_t grid = ((nitems + 7) >> 3) << 3;
  hipLaunchKernelGGL(score_tiles_kernel<S>, dim3((unsigned)grid), dim3((1 << S) / kE), 0, st,
                     args_of(ix), q, (int32_t)Q, (int32_t)T, ws.cand);
}

hipError_t launch_score_tiles(const DevIndex& ix, const int32_t* d_queries, int64_t Q,
                              int64_t T, const Workspace& ws, hipStream_t stream) {
  if (Q == 0 || ix.ntiles == 0) return hipSuccess;
  switch (ix.tile_shift) {
    case 13: launch_score_s<13>(ix, d_queries, Q, T, ws, stream); break;
    case 14: launch_score_s<14>(ix, d_queries, Q, T, ws, stream); break;
    case 15: launch_score_s<15>(ix, d_queries, Q, T, ws, stream); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

template <int S>
static void launch_rescore_s(const DevIndex& ix, const int32_t* q, int64_t T, int k,
                             int64_t maxflag, const Workspace& ws, hipStream_t st) {
  hipLaunchKernelGGL(rescore_kernel<S>, dim3(512), dim3((1 << S) / kE), 0, st, args_of(ix), q,
                     (int32_t)T, (int32_t)k, maxflag, ws);
}

hipError_t launch_select(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                         int k, const Workspace& ws, int32_t* d_docs, float* d_scores,
                         hipStream_t stream) {
  if (Q == 0 || k == 0) return hipSuccess;
  const int64_t maxflag = maxflag_for(k, ix.ntiles);
  hipError_t e = hipMemsetAsync(ws.counters, 0, 4 * sizeof(int32_t), stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(merge_first_kernel, dim3((unsigned)Q), dim3(kMergeNT), 0, stream, ws.cand,
                     ix.ntiles, (int32_t)k, maxflag, ix.doc_offset, ws, d_docs, d_scores);
  if (k > kTileM) {
    switch (ix.tile_shift) {
      case 13: launch_rescore_s<13>(ix, d_queries, T, k, maxflag, ws, stream); break;
      case 14: launch_rescore_s<14>(ix, d_queries, T, k, maxflag, ws, stream); break;
      case 15: launch_rescore_s<15>(ix, d_queries, T, k, maxflag, ws, stream); break;
      default: return hipErrorInvalidValue;
    }
    hipLaunchKernelGGL(merge_final_kernel, dim3((unsigned)Q), dim3(kMergeNT), 0, stream,
                       ws.cand, ix.ntiles, (int32_t)k, maxflag, ix.doc_offset, ws, d_docs,
                       d_scores);
  }
  return hipGetLastError();
}

hipError_t launch_scores_dense(const DevIndex& ix, const int32_t* d_query, int64_t T,
                               float* d_out, hipStream_t stream) {
  if (ix.ntiles == 0) return hipSuccess;
  const dim3 grid((unsigned)ix.ntiles);
  switch (ix.tile_shift) {
    case 13: hipLaunchKernelGGL(scores_dense_kernel<13>, grid, dim3((1 << 13) / kE), 0, stream, args_of(ix), d_query, (int32_t)T, d_out); break;
    case 14: hipLaunchKernelGGL(scores_dense_kernel<14>, grid, dim3((1 << 14) / kE), 0, stream, args_of(ix), d_query, (int32_t)T, d_out); break;
    case 15: hipLaunchKernelGGL(scores_dense_kernel<15>, grid, dim3((1 << 15) / kE), 0, stream, args_of(ix), d_query, (int32_t)T, d_out); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_merge_lists(const int32_t* d_docs, const float* d_scores, int64_t W,
                              int64_t Q, int k, int32_t* d_out_docs, float* d_out_scores,
                              hipStream_t stream) {
  if (Q == 0 || k == 0) return hipSuccess;
  hipLaunchKernelGGL(merge_lists_kernel, dim3((unsigned)Q), dim3(kMergeNT), 0, stream, d_docs,
                     d_scores, W, Q, (int32_t)k, d_out_docs, d_out_scores);
  return hipGetLastError();
}

}  // namespace bm25mi
