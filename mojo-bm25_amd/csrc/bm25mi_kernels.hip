// bm25mi_kernels.hip — gfx950 kernels of the BM25 CSC query path.
//
// Replaces the reference's GPU path (MAX graph ops.gather -> ops.sum ->
// ops.top_k, gpu_bm25/common.py:64-80, vendored as
// operations/gather_scatter.mojo:683-763 and operations/topk.mojo:576-963)
// and its CPU scorer (bm25_native.py:149-158, 204-214) with a doc-tiled
// sparse design:
//
//   score_tiles<SAMPLE>  one workgroup per (sample doc tile, query): gathers
//                 the query's posting segments inside the tile (row-uniform,
//                 4 postings per lane: u16x4 doc ids + f32x4 scores), adds them
//                 into an fp32 LDS accumulator term by term in query order
//                 (the exact fp32 arithmetic of scipy csc_matvec,
//                 bm25_native.py:152), then extracts the tile's exact top-4
//                 keys with wave64 DPP argmax rounds.
//   theta         per query, the k-th best sample candidate: a lower bound of
//                 the final k-th key.
//   score_tiles<REST>    every other tile: same accumulation, then a compare
//                 against theta; the (typically 0-2) keys above it are
//                 emitted, and only a tile with more than 4 runs the argmax.
//   merge         one workgroup per query: bitonic-sorts the per-tile
//                 candidates in LDS, picks the top-k and flags the (rare)
//                 tiles whose 4th candidate beats the k-th key.
//   rescore       persistent: exact top-k of each flagged tile.
//   merge(final)  merges the exact lists of flagged tiles.
// The result is exactly the top-k under (score desc, doc asc) of the dense
// score vector, with untouched documents scoring 0.
#include "bm25mi_internal.h"

#include <cstdlib>

namespace bm25mi {

constexpr int kTG = 16;  // query terms staged in LDS per group
constexpr int kE = 32;   // accumulator entries owned by a thread in selection

enum Phase { kAll = 0, kSample = 1, kRest = 2 };

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
  int64_t abeg[kTG];          // a term's first posting in the tile, aligned down to 4
  uint32_t off[kTG];          // first posting - abeg (0..3)
  uint32_t len[kTG];          // postings of the term in the tile
  uint32_t rstart[kTG + 1];   // prefix of row counts
  uint32_t red[2][16];        // per-wave argmax values, double-buffered
  int32_t nsel;               // keys emitted by the threshold pass
  int32_t item;
};

__device__ __forceinline__ uint32_t sgpr(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ int64_t sgpr64(int64_t v) {
  const uint32_t lo = sgpr((uint32_t)v), hi = sgpr((uint32_t)((uint64_t)v >> 32));
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// Max over the 64 lanes of a wave: DPP inside each 16-lane row, then the four
// row results through SGPRs.
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false));   // quad [1,0,3,2]
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false));   // quad [2,3,0,1]
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false));  // row_half_mirror
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false));  // row_mirror
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return max(max(a, b), max(c, d));
}

// ---------------------------------------------------------------------------
// Scatter phase: acc[d] = sum over query terms (in order) of the term's score
// for doc d of this tile.  Replaces doc_toks[:, query].sum(axis=1)
// (bm25_native.py:152 -> scipy csc_matvec): same fp32 adds, same order per doc.
//
// Each term's segment is cut into rows of 4*NT postings aligned down to a
// multiple of 4; lane t of a row loads postings [4t, 4t+4) of it as one u16x4
// (accumulator slots, acc_slot() applied at build time) and one f32x4 from a
// block-uniform base (SGPR base + lane offset).  A row belongs to one term, so
// a barrier between rows of different terms keeps the per-document add order;
// inside a term every doc occurs once, so plain LDS read-add-writes never
// race.  Lanes outside the segment are redirected to a private dummy slot
// (acc[D + lane]) instead of branching around their LDS accesses.
// ---------------------------------------------------------------------------
template <int S, int kRB = 4>
__device__ __forceinline__ void accumulate_tile(const IndexArgs& a, int64_t tile,
                                                const int32_t* __restrict__ qterms,
                                                int T, float* acc, TileShared& sm,
                                                int mode = 0) {
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  constexpr uint32_t RW = 4 * NT;  // postings per row
  const int tid = threadIdx.x;
  const uint32_t dummy = D + (tid & 63);

  float4* acc4 = reinterpret_cast<float4*>(acc);
  if (!(mode & 8)) {
#pragma unroll
    for (int j = 0; j < kE / 4; ++j) acc4[j * NT + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (tid == 0) sm.nsel = 0;

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
      sm.abeg[tid] = lo & ~3ll;
      sm.off[tid] = (uint32_t)(lo & 3);
      sm.len[tid] = len;
      sm.rstart[tid + 1] = len ? (uint32_t)(((lo & 3) + len + RW - 1) / RW) : 0u;
    }
    __syncthreads();
    if (tid == 0) {
      uint32_t s = 0;
      sm.rstart[0] = 0;
      for (int i = 0; i < ng; ++i) {
        s += sm.rstart[i + 1];
        sm.rstart[i + 1] = s;
      }
    }
    __syncthreads();
    const uint32_t R = (mode & 4) ? 0u : sgpr(sm.rstart[ng]);
    int s = 0;          // term of the current row (block-uniform)
    int last_s = -1;    // term of the last added row
    for (uint32_t rb = 0; rb < R; rb += kRB) {
      ushort4 ld[kRB];
      float4 v[kRB];
      int32_t i0[kRB];
      int rs[kRB];
#pragma unroll
      for (int b = 0; b < kRB; ++b) {
        const uint32_t row = rb + b;
        rs[b] = -1;
        if (row < R) {
          while (row >= sgpr(sm.rstart[s + 1])) ++s;
          const uint32_t rr = row - sgpr(sm.rstart[s]);
          const int64_t A0 = sgpr64(sm.abeg[s]) + (int64_t)rr * RW;
          // last 4-aligned group of the segment, relative to this row: lanes
          // past it re-read that group (one cache line for all of them)
          // instead of fetching postings of other terms
          const uint32_t off = sgpr(sm.off[s]);
          const uint32_t lastg = ((off + sgpr(sm.len[s]) - 1) & ~3u) - rr * RW;
          const uint32_t g = min(4u * tid, lastg) >> 2;
          ld[b] = reinterpret_cast<const ushort4*>(a.ldoc + A0)[g];
          v[b] = reinterpret_cast<const float4*>(a.val + A0)[g];
          i0[b] = (int32_t)(rr * RW) + 4 * tid - (int32_t)off;
          rs[b] = s;
        }
      }
      if (mode & 2) {
#pragma unroll
        for (int b = 0; b < kRB; ++b)
          asm volatile("" ::"v"(ld[b].x), "v"(ld[b].w), "v"(v[b].x), "v"(v[b].w));
        continue;
      }
#pragma unroll
      for (int b = 0; b < kRB; ++b) {
        if (rs[b] < 0) break;
        if (rs[b] != last_s) {
          if (last_s >= 0) __syncthreads();  // previous term's adds complete
          last_s = rs[b];
        }
        const uint32_t len = sgpr(sm.len[rs[b]]);
        const uint32_t d0 = (uint32_t)(i0[b] + 0) < len ? (uint32_t)ld[b].x : dummy;
        const uint32_t d1 = (uint32_t)(i0[b] + 1) < len ? (uint32_t)ld[b].y : dummy;
        const uint32_t d2 = (uint32_t)(i0[b] + 2) < len ? (uint32_t)ld[b].z : dummy;
        const uint32_t d3 = (uint32_t)(i0[b] + 3) < len ? (uint32_t)ld[b].w : dummy;
        // four distinct docs of one term (or the dummy slot): read all, write all
        const float x0 = acc[d0], x1 = acc[d1], x2 = acc[d2], x3 = acc[d3];
        acc[d0] = x0 + v[b].x;
        acc[d1] = x1 + v[b].y;
        acc[d2] = x2 + v[b].z;
        acc[d3] = x3 + v[b].w;
      }
    }
  }
  __syncthreads();
}

// Load this thread's 32 accumulator entries (entry e = tile-local doc
// tid*32 + e), conflict-free float4 reads.
template <int S>
__device__ __forceinline__ void load_entries(const float* acc, float (&fv)[kE]) {
  constexpr int NT = (1 << S) / kE;
  const float4* acc4 = reinterpret_cast<const float4*>(acc);
#pragma unroll
  for (int j = 0; j < kE / 4; ++j) {
    const float4 f = acc4[j * NT + threadIdx.x];
    fv[j * 4 + 0] = f.x;
    fv[j * 4 + 1] = f.y;
    fv[j * 4 + 2] = f.z;
    fv[j * 4 + 3] = f.w;
  }
}

// Order-preserving u32 keys of the entries (0 = past n_docs).
template <int S>
__device__ __forceinline__ void make_keys(const float (&fv)[kE], int64_t tile, int64_t n_docs,
                                          uint32_t (&key)[kE]) {
  constexpr int D = 1 << S;
  const int64_t doc0 = tile * D + (int64_t)threadIdx.x * kE;
#pragma unroll
  for (int e = 0; e < kE; ++e) key[e] = score_key(fv[e]);
  if (doc0 + kE > n_docs) {
#pragma unroll
    for (int e = 0; e < kE; ++e)
      if (doc0 + e >= n_docs) key[e] = 0;
  }
}

// ---------------------------------------------------------------------------
// Exact selection: the m best keys of the tile, best first, into out[0..m).
// Thread t owns docs [t*32, t*32+32), so "first wave, first lane, first entry"
// among equal scores is the smallest doc id.
// ---------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void select_tile(uint32_t (&key)[kE], int64_t tile, int m,
                                            uint64_t* __restrict__ out, TileShared& sm) {
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  constexpr int NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t doc0 = tile * D + (int64_t)tid * kE;
  uint32_t lmax = 0;
#pragma unroll
  for (int i = 0; i < kE; ++i) lmax = max(lmax, key[i]);

  for (int r = 0; r < m; ++r) {
    const uint32_t wm = wave_max_u32(lmax);
    const unsigned long long bal = __ballot(lmax == wm);
    const int wl = (int)__builtin_ctzll(bal);
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
      int eb = 0;
#pragma unroll
      for (int e = kE - 1; e >= 0; --e)
        if (key[e] == bm) eb = e;
      out[r] = ((uint64_t)bm << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(doc0 + eb));
      lmax = 0;
#pragma unroll
      for (int e = 0; e < kE; ++e) {
        key[e] = e == eb ? 0u : key[e];
        lmax = max(lmax, key[e]);
      }
    }
  }
}

// Threshold emission (REST tiles): write the keys > theta (at most kTileM;
// slots past the count are zeroed) and return the block-wide count; above
// kTileM the caller runs the exact selection instead.  The test runs on the
// fp32 sums directly (one compare per entry); only a lane holding theta's
// exact score compares doc ids.  Accumulators are never -0.0 (a sum that
// starts at +0.0 cannot produce it) and docs past n_docs hold 0.0, which can
// only pass when theta's score is negative — those are masked explicitly.
template <int S>
__device__ __forceinline__ int emit_above(const float (&fv)[kE], int64_t tile, int64_t n_docs,
                                          uint64_t theta, uint64_t* __restrict__ out,
                                          TileShared& sm) {
  constexpr int D = 1 << S;
  const int tid = threadIdx.x;
  const float th = key_score((uint32_t)(theta >> 32));
  const uint32_t th_doc = 0xFFFFFFFFu - (uint32_t)theta;
  const int64_t doc0 = tile * D + (int64_t)tid * kE;
  const int64_t lim_hi = n_docs - doc0;  // entries e >= lim_hi are past n_docs
  int c = 0;
  bool tie = false;
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    c += fv[e] > th;
    tie |= fv[e] == th;
  }
  if (tie || lim_hi < kE) {  // rare: exact per-entry rule
    const int64_t lim_tie = (int64_t)th_doc - doc0;  // ties pass for e < lim_tie
    c = 0;
#pragma unroll
    for (int e = 0; e < kE; ++e)
      c += (e < lim_hi) & ((fv[e] > th) | ((fv[e] == th) & (e < lim_tie)));
  }
  if (c > 0) {
    const int64_t lim_tie = (int64_t)th_doc - doc0;
    int pos = atomicAdd(&sm.nsel, c);
#pragma unroll
    for (int e = 0; e < kE; ++e) {
      const bool pass = (e < lim_hi) & ((fv[e] > th) | ((fv[e] == th) & (e < lim_tie)));
      if (pass) {
        if (pos < kTileM)
          out[pos] = ((uint64_t)score_key(fv[e]) << 32) |
                     (uint64_t)(0xFFFFFFFFu - (uint32_t)(doc0 + e));
        ++pos;
      }
    }
  }
  __syncthreads();
  const int n = sm.nsel;
  if (n < kTileM && tid < kTileM - n) out[n + tid] = 0;
  return n;
}

// Work item -> (tile, query).  Blocks are dealt round-robin over the 8 XCDs
// (b % 8), so block b runs item (b % 8) * per + b / 8: each XCD walks its own
// contiguous run of tiles, all queries of a tile back to back, and the tile's
// hot posting segments stay in that XCD's L2.
template <int PH>
__device__ __forceinline__ bool item_of(int64_t ntiles, int64_t Q, int P, int64_t& tile,
                                        int64_t& q) {
  const int64_t nS = (ntiles + P - 1) / P;
  const int64_t nt = PH == kAll ? ntiles : (PH == kSample ? nS : ntiles - nS);
  const int64_t nitems = nt * Q;
  const int64_t per = (nitems + 7) >> 3;
  const int64_t b = blockIdx.x;
  const int64_t item = (b & 7) * per + (b >> 3);
  if (item >= nitems) return false;
  const int64_t ti = item / Q;
  q = item - ti * Q;
  if (PH == kAll) tile = ti;
  else if (PH == kSample) tile = ti * P;
  else tile = (ti / (P - 1)) * P + (ti % (P - 1)) + 1;
  return true;
}

template <int S, int PH, int RB>
__global__ __launch_bounds__((1 << S) / kE) void score_tiles_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t Q, int32_t T, int32_t P,
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand, int mode) {
  __shared__ __attribute__((aligned(16))) float acc[(1 << S) + 64];
  __shared__ TileShared sm;
  int64_t tile, q;
  if (!item_of<PH>(a.ntiles, Q, P, tile, q)) return;
  accumulate_tile<S, RB>(a, tile, queries + q * T, T, acc, sm, mode);
  uint64_t* out = cand + (q * a.ntiles + tile) * kTileM;
  if (mode & 1) {  // ablation: no selection
    if (threadIdx.x == 0) out[0] = __float_as_uint(acc[0]);
    return;
  }
  float fv[kE];
  load_entries<S>(acc, fv);
  if (PH == kRest) {
    if (emit_above<S>(fv, tile, a.n_docs, theta[q], out, sm) <= kTileM) return;
  }
  uint32_t key[kE];
  make_keys<S>(fv, tile, a.n_docs, key);
  select_tile<S>(key, tile, kTileM, out, sm);
}

// ---------------------------------------------------------------------------
// Streaming (persistent) score kernel: the same per-item work as
// score_tiles_kernel, software-pipelined across items so that memory latency
// overlaps compute.  While item n is accumulated and selected, the first
// posting rows of item n+1 are in flight (registers) and the segment
// metadata of item n+2 (rel/indptr) is in flight; the query terms of item n+3
// are loaded one iteration ahead of that.  Items are handed out in chunks
// from one counter per XCD group (blockIdx % 8), in tile-major order, so the
// workgroups of an XCD work on the same tile together (L2 reuse of the hot
// posting segments across queries).  Requires T <= kTG.
// ---------------------------------------------------------------------------
struct ItemMeta {
  int64_t abeg[kTG];
  uint32_t off[kTG];
  uint32_t len[kTG];
  uint32_t rstart[kTG + 1];
};

constexpr int kFifo = 16;
struct StreamShared {
  ItemMeta meta[3];
  int64_t fifo[kFifo];  // upcoming items of this workgroup
  int32_t fhead, fcount, exhausted;
  uint32_t red[2][16];
  int32_t nsel[2];
};

template <int PH>
__device__ __forceinline__ void item_tile(int64_t item, int64_t Q, int P, int64_t& tile,
                                          int64_t& q) {
  const int64_t ti = item / Q;
  q = item - ti * Q;
  if (PH == kAll) tile = ti;
  else if (PH == kSample) tile = ti * P;
  else tile = (ti / (P - 1)) * P + (ti % (P - 1)) + 1;
}

// Issue the segment-metadata loads of one query term (thread < T).
struct MetaRegs {
  uint32_t r0, r1;
  int64_t ip;
  bool ok;
};
__device__ __forceinline__ MetaRegs meta_issue(const IndexArgs& a, int32_t term, int64_t tile) {
  MetaRegs m;
  m.ok = term >= 0 && term < a.V;  // negative ids are padding (bm25_native.py:151)
  const int64_t t = m.ok ? term : 0;
  const uint32_t* r = a.rel + t * (a.ntiles + 1) + tile;
  m.r0 = r[0];
  m.r1 = r[1];
  m.ip = a.indptr[t];
  return m;
}

// Threads 0..T-1 (wave 0) publish their term's segment into `mt`: row counts
// and their prefix via a wave scan (no block barrier needed inside).
template <int S>
__device__ __forceinline__ void meta_store(const MetaRegs& m, int T, ItemMeta& mt) {
  constexpr uint32_t RW = 4 * ((1 << S) / kE);
  const int tid = threadIdx.x;
  uint32_t rows = 0;
  if (tid < T) {
    const int64_t lo = m.ip + m.r0;
    const uint32_t len = m.ok ? m.r1 - m.r0 : 0u;
    mt.abeg[tid] = lo & ~3ll;
    mt.off[tid] = (uint32_t)(lo & 3);
    mt.len[tid] = len;
    rows = len ? (uint32_t)(((lo & 3) + len + RW - 1) / RW) : 0u;
  }
  if (tid < 64) {
    uint32_t x = rows;
#pragma unroll
    for (int o = 1; o < kTG; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
      if ((tid & 63) >= o) x += y;
    }
    if (tid < T) mt.rstart[tid + 1] = x;
    if (tid == 0) mt.rstart[0] = 0;
  }
}

// Issue the loads of rows [row0, row0 + RB) of an item (block-uniform).
// Every call issues exactly 2*RB loads, none under a branch (rows past the
// item read a fixed in-bounds address and are marked rs = -1): the compiler's
// vmcnt bookkeeping then stays exact across the software pipeline.
template <int S, int RB>
__device__ __forceinline__ void rows_issue(const IndexArgs& a, const ItemMeta& mt, int T,
                                           uint32_t row0, ushort4 (&ld)[RB], float4 (&v)[RB],
                                           int32_t (&i0)[RB], int (&rs)[RB]) {
  constexpr uint32_t RW = 4 * ((1 << S) / kE);
  const int tid = threadIdx.x;
  const uint32_t R = sgpr(mt.rstart[T]);
  int s = 0;
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    const uint32_t row = row0 + b;
    int64_t A0 = 0;
    uint32_t lastg = 0, rr = 0, off = 0;
    rs[b] = -1;
    if (row < R) {
      while (row >= sgpr(mt.rstart[s + 1])) ++s;
      rr = row - sgpr(mt.rstart[s]);
      A0 = sgpr64(mt.abeg[s]) + (int64_t)rr * RW;
      off = sgpr(mt.off[s]);
      lastg = ((off + sgpr(mt.len[s]) - 1) & ~3u) - rr * RW;
      rs[b] = s;
    }
    const uint32_t g = min(4u * tid, lastg) >> 2;
    ld[b] = reinterpret_cast<const ushort4*>(a.ldoc + A0)[g];
    v[b] = reinterpret_cast<const float4*>(a.val + A0)[g];
    i0[b] = (int32_t)(rr * RW) + 4 * tid - (int32_t)off;
  }
}

// Add a batch of rows (barrier between rows of different terms).
template <int S, int RB>
__device__ __forceinline__ void rows_add(const ItemMeta& mt, float* acc, const ushort4 (&ld)[RB],
                                         const float4 (&v)[RB], const int32_t (&i0)[RB],
                                         const int (&rs)[RB], int& last_s) {
  constexpr int D = 1 << S;
  const uint32_t dummy = D + (threadIdx.x & 63);
#pragma unroll
  for (int b = 0; b < RB; ++b) {
    if (rs[b] < 0) break;
    if (rs[b] != last_s) {
      if (last_s >= 0) __syncthreads();  // previous term's adds complete
      last_s = rs[b];
    }
    const uint32_t len = sgpr(mt.len[rs[b]]);
    const uint32_t d0 = (uint32_t)(i0[b] + 0) < len ? (uint32_t)ld[b].x : dummy;
    const uint32_t d1 = (uint32_t)(i0[b] + 1) < len ? (uint32_t)ld[b].y : dummy;
    const uint32_t d2 = (uint32_t)(i0[b] + 2) < len ? (uint32_t)ld[b].z : dummy;
    const uint32_t d3 = (uint32_t)(i0[b] + 3) < len ? (uint32_t)ld[b].w : dummy;
    const float x0 = acc[d0], x1 = acc[d1], x2 = acc[d2], x3 = acc[d3];
    acc[d0] = x0 + v[b].x;
    acc[d1] = x1 + v[b].y;
    acc[d2] = x2 + v[b].z;
    acc[d3] = x3 + v[b].w;
  }
}

__device__ __forceinline__ void fifo_refill(StreamShared& ss, int32_t* ctr, int64_t g_lo,
                                            int64_t g_hi, int chunk) {
  while (!ss.exhausted && ss.fcount + chunk <= kFifo) {
    const int64_t c = g_lo + atomicAdd(ctr, chunk);
    for (int i = 0; i < chunk; ++i) {
      if (c + i >= g_hi) { ss.exhausted = 1; break; }
      ss.fifo[(ss.fhead + ss.fcount) % kFifo] = c + i;
      ++ss.fcount;
    }
  }
}

__device__ __forceinline__ int64_t fifo_peek(const StreamShared& ss, int j) {
  return j < ss.fcount ? ss.fifo[(ss.fhead + j) % kFifo] : -1;
}

template <int S, int PH, int RB>
__global__ __launch_bounds__((1 << S) / kE) void score_stream_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t Q, int32_t T, int32_t P,
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand, int32_t* __restrict__ wctr,
    int32_t chunk) {
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  __shared__ __attribute__((aligned(16))) float acc[D + 64];
  __shared__ StreamShared ss;
  __shared__ TileShared sm;  // red / nsel of the selection helpers
  const int tid = threadIdx.x;
  const bool refiller = tid == NT - 64;  // lane 0 of the last wave grabs chunks
  const int64_t nS = (a.ntiles + P - 1) / P;
  const int64_t nt = PH == kAll ? a.ntiles : (PH == kSample ? nS : a.ntiles - nS);
  const int64_t nitems = nt * Q;
  const int64_t per = (nitems + 7) >> 3;
  const int g = blockIdx.x & 7;
  const int64_t g_lo = g * per, g_hi = min(nitems, g_lo + per);
  int32_t* ctr = wctr + g;
  const int tq = min(tid, T - 1);  // every thread loads a valid query slot

  // ---- prologue: item list, zeroed accumulator, metadata of items 0 and 1
  if (refiller) {
    ss.fhead = 0;
    ss.fcount = 0;
    ss.exhausted = 0;
    fifo_refill(ss, ctr, g_lo, g_hi, chunk);
  }
  float4* acc4 = reinterpret_cast<float4*>(acc);
#pragma unroll
  for (int j = 0; j < kE / 4; ++j) acc4[j * NT + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const int64_t it0 = sgpr64(fifo_peek(ss, 0));
  if (it0 < 0) return;  // block-uniform
  int32_t qn;           // query term (thread tq) of the item two ahead
  {
    int64_t tile, q;
    item_tile<PH>(it0, Q, P, tile, q);
    const MetaRegs m0 = meta_issue(a, tid < T ? queries[q * T + tq] : -1, tile);
    const int64_t it1 = sgpr64(fifo_peek(ss, 1));
    item_tile<PH>(it1 >= 0 ? it1 : it0, Q, P, tile, q);
    const MetaRegs m1 = meta_issue(a, tid < T ? queries[q * T + tq] : -1, tile);
    const int64_t it2 = sgpr64(fifo_peek(ss, 2));
    item_tile<PH>(it2 >= 0 ? it2 : it0, Q, P, tile, q);
    qn = queries[q * T + tq];
    meta_store<S>(m0, T, ss.meta[0]);
    if (it1 >= 0) meta_store<S>(m1, T, ss.meta[1]);
    if (tid == 0) sm.nsel = 0;
  }
  __syncthreads();
  ushort4 ldA[RB], ldB[RB];
  float4 vA[RB], vB[RB];
  int32_t iA[RB], iB[RB];
  int rsA[RB], rsB[RB];
  rows_issue<S, RB>(a, ss.meta[0], T, 0, ldA, vA, iA, rsA);

  // One pipeline step: item n's first rows are in (ld, v, i, rs); item n+1's
  // first rows are issued into (ldN, ...).  Returns false after the last item.
  auto step = [&](int n, ushort4 (&ld)[RB], float4 (&v)[RB], int32_t (&i0)[RB], int (&rs)[RB],
                  ushort4 (&ldN)[RB], float4 (&vN)[RB], int32_t (&iN)[RB],
                  int (&rsN)[RB]) -> bool {
    const int64_t it = sgpr64(fifo_peek(ss, 0));
    const int64_t nx = sgpr64(fifo_peek(ss, 1));
    const int64_t n2 = sgpr64(fifo_peek(ss, 2));
    const int64_t n3 = sgpr64(fifo_peek(ss, 3));
    const ItemMeta& mc = ss.meta[n % 3];
    int64_t tile, q;
    item_tile<PH>(it, Q, P, tile, q);
    // (a) metadata of item n+2, query terms of item n+3 (fixed load count)
    int64_t t2, q2;
    item_tile<PH>(n2 >= 0 ? n2 : it, Q, P, t2, q2);
    const MetaRegs m2 = meta_issue(a, tid < T ? qn : -1, t2);
    item_tile<PH>(n3 >= 0 ? n3 : it, Q, P, t2, q2);
    qn = queries[q2 * T + tq];
    // (b) first rows of item n+1 (without a next item the loads still go out,
    //     from the current item's valid segments, and are never used)
    rows_issue<S, RB>(a, nx >= 0 ? ss.meta[(n + 1) % 3] : mc, T, 0, ldN, vN, iN, rsN);
    // (c) accumulate item n: prefetched rows, then any further rows
    int last_s = -1;
    rows_add<S, RB>(mc, acc, ld, v, i0, rs, last_s);
    const uint32_t R = sgpr(mc.rstart[T]);
    for (uint32_t rb = RB; rb < R; rb += RB) {
      ushort4 ldX[RB];
      float4 vX[RB];
      int32_t iX[RB];
      int rsX[RB];
      rows_issue<S, RB>(a, mc, T, rb, ldX, vX, iX, rsX);
      rows_add<S, RB>(mc, acc, ldX, vX, iX, rsX, last_s);
    }
    __syncthreads();
    // (d) selection of item n; the entries are zeroed for item n+1 as read
    {
      float fv[kE];
      load_entries<S>(acc, fv);
#pragma unroll
      for (int j = 0; j < kE / 4; ++j) acc4[j * NT + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
      uint64_t* out = cand + (q * a.ntiles + tile) * kTileM;
      bool exact = true;
      if (PH == kRest) exact = emit_above<S>(fv, tile, a.n_docs, theta[q], out, sm) > kTileM;
      if (exact) {
        uint32_t key[kE];
        make_keys<S>(fv, tile, a.n_docs, key);
        select_tile<S>(key, tile, kTileM, out, sm);
      }
    }
    __syncthreads();  // every read of sm.nsel / red and of meta[n % 3] is done
    // (e) publish item n+2's metadata, advance the item list
    if (n2 >= 0) meta_store<S>(m2, T, ss.meta[(n + 2) % 3]);
    if (tid == 0) sm.nsel = 0;
    if (refiller) {
      ss.fhead = (ss.fhead + 1) % kFifo;
      --ss.fcount;
      fifo_refill(ss, ctr, g_lo, g_hi, chunk);
    }
    __syncthreads();
    return nx >= 0;
  };

  for (int n = 0;; n += 2) {
    if (!step(n, ldA, vA, iA, rsA, ldB, vB, iB, rsB)) break;
    if (!step(n + 1, ldB, vB, iB, rsB, ldA, vA, iA, rsA)) break;
  }
}

// Exact top-k of each flagged tile; persistent, pulls items from the queue
// the merge kernel filled (every wave reaches the exit test each iteration).
template <int S>
__global__ __launch_bounds__((1 << S) / kE) void rescore_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, int32_t k,
    int64_t maxflag, Workspace ws) {
  __shared__ __attribute__((aligned(16))) float acc[(1 << S) + 64];
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
    float fv[kE];
    load_entries<S>(acc, fv);
    uint32_t key[kE];
    make_keys<S>(fv, tile, a.n_docs, key);
    select_tile<S>(key, tile, k, ws.cand2 + (int64_t)code * k, sm);
  }
}

template <int S>
__global__ __launch_bounds__((1 << S) / kE) void scores_dense_kernel(
    IndexArgs a, const int32_t* __restrict__ query, int32_t T, float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float acc[(1 << S) + 64];
  __shared__ TileShared sm;
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  const int64_t tile = blockIdx.x;
  accumulate_tile<S>(a, tile, query, T, acc, sm);
  const float4* acc4 = reinterpret_cast<const float4*>(acc);
  const int64_t d0 = tile * D + (int64_t)threadIdx.x * kE;  // this thread's 32 docs
  if (d0 + kE <= a.n_docs) {
    float4* o4 = reinterpret_cast<float4*>(out + d0);
#pragma unroll
    for (int j = 0; j < kE / 4; ++j) o4[j] = acc4[j * NT + threadIdx.x];
  } else {
    for (int e = 0; e < kE && d0 + e < a.n_docs; ++e) {
      const float4 f = acc4[(e >> 2) * NT + threadIdx.x];
      out[d0 + e] = (e & 3) == 0 ? f.x : (e & 3) == 1 ? f.y : (e & 3) == 2 ? f.z : f.w;
    }
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
      ldoc[p] = (uint16_t)acc_slot((uint32_t)d & mask, S);
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

struct SrcSample {  // the kTileM slots of every P-th tile
  const uint64_t* c;
  int P;
  __device__ uint64_t operator()(int64_t i) const {
    return c[(i / kTileM) * P * kTileM + (i % kTileM)];
  }
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

// theta[q] = k-th best key among the sample tiles' candidates (0 when there
// are fewer than k): k real documents score at least this, so it is a lower
// bound of the final k-th key.
__global__ __launch_bounds__(kMergeNT) void theta_kernel(const uint64_t* __restrict__ cand,
                                                         int64_t ntiles, int32_t P, int32_t k,
                                                         uint64_t* __restrict__ theta) {
  __shared__ uint64_t keys[kMergeP];
  const int64_t q = blockIdx.x;
  const int64_t nS = (ntiles + P - 1) / P;
  topk_of(SrcSample{cand + q * ntiles * kTileM, P}, nS * kTileM, k, keys);
  if (threadIdx.x == 0) theta[q] = keys[k - 1];
}

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

static int env_mode() {
  static const int mode = getenv("BM25_ABLATE") ? atoi(getenv("BM25_ABLATE")) : 0;
  return mode;
}

// Sampling stride: every P-th tile is a sample tile; P is the largest of
// {8, 4, 2} whose sample still yields >= 2k candidates (else one exact pass).
static int sample_stride(int64_t ntiles, int k) {
  static const bool off = getenv("BM25_NO_SAMPLE") != nullptr;
  if (off) return 1;
  for (int P = 8; P >= 2; P >>= 1) {
    const int64_t nS = (ntiles + P - 1) / P;
    if (ntiles >= 2 * P && nS * kTileM >= 2 * (int64_t)k) return P;
  }
  return 1;
}

template <int S, int PH, int RB>
static void launch_stream(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int P,
                          const Workspace& ws, int32_t* wctr, hipStream_t st) {
  static int grid = 0;
  if (grid == 0) {
    int dev = 0, cus = 0, occ = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, score_stream_kernel<S, PH, RB>,
                                                 (1 << S) / kE, 0);
    const char* e = getenv("BM25_STREAM_WG_PER_CU");
    if (e) occ = atoi(e);
    grid = ((cus * (occ > 0 ? occ : 1) + 7) / 8) * 8;
    if (grid < 8) grid = 8;
  }
  hipLaunchKernelGGL((score_stream_kernel<S, PH, RB>), dim3((unsigned)grid), dim3((1 << S) / kE),
                     0, st, args_of(ix), q, (int32_t)Q, (int32_t)T, (int32_t)P, ws.theta, ws.cand,
                     wctr, (int32_t)8);
}

static bool use_stream(int64_t T) {
  static const bool off = getenv("BM25_NO_STREAM") != nullptr;
  return !off && T >= 1 && T <= kTG;
}

template <int S, int PH>
static void launch_phase(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int P,
                         const Workspace& ws, hipStream_t st) {
  const int64_t nS = (ix.ntiles + P - 1) / P;
  const int64_t nt = PH == kAll ? ix.ntiles : (PH == kSample ? nS : ix.ntiles - nS);
  const int64_t grid = ((nt * Q + 7) >> 3) << 3;
  if (grid == 0) return;
  if (use_stream(T)) {
    launch_stream<S, PH, 4>(ix, q, Q, T, P, ws, ws.wctr + (PH == kRest ? 8 : 0), st);
    return;
  }
  static const int rb = getenv("BM25_RB") ? atoi(getenv("BM25_RB")) : 8;
  if (rb == 4)
    hipLaunchKernelGGL((score_tiles_kernel<S, PH, 4>), dim3((unsigned)grid), dim3((1 << S) / kE),
                       0, st, args_of(ix), q, (int32_t)Q, (int32_t)T, (int32_t)P, ws.theta,
                       ws.cand, env_mode());
  else
    hipLaunchKernelGGL((score_tiles_kernel<S, PH, 8>), dim3((unsigned)grid), dim3((1 << S) / kE),
                       0, st, args_of(ix), q, (int32_t)Q, (int32_t)T, (int32_t)P, ws.theta,
                       ws.cand, env_mode());
}

template <int S>
static void launch_score_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int k,
                           const Workspace& ws, hipStream_t st) {
  const int P = sample_stride(ix.ntiles, k);
  if (P == 1) {
    launch_phase<S, kAll>(ix, q, Q, T, 1, ws, st);
    return;
  }
  launch_phase<S, kSample>(ix, q, Q, T, P, ws, st);
  hipLaunchKernelGGL(theta_kernel, dim3((unsigned)Q), dim3(kMergeNT), 0, st, ws.cand, ix.ntiles,
                     (int32_t)P, (int32_t)k, ws.theta);
  launch_phase<S, kRest>(ix, q, Q, T, P, ws, st);
}

hipError_t launch_score_tiles(const DevIndex& ix, const int32_t* d_queries, int64_t Q,
                              int64_t T, int k, const Workspace& ws, hipStream_t stream) {
  if (Q == 0 || ix.ntiles == 0) return hipSuccess;
  if (use_stream(T)) {
    const hipError_t e = hipMemsetAsync(ws.wctr, 0, 16 * sizeof(int32_t), stream);
    if (e != hipSuccess) return e;
  }
  switch (ix.tile_shift) {
    case 13: launch_score_s<13>(ix, d_queries, Q, T, k, ws, stream); break;
    case 14: launch_score_s<14>(ix, d_queries, Q, T, k, ws, stream); break;
    case 15: launch_score_s<15>(ix, d_queries, Q, T, k, ws, stream); break;
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
