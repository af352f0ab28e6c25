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

// Candidate-slot marker of a REST tile with >= kTileM keys above theta (never
// a real key: that would be a NaN score at doc 0).
constexpr uint64_t kOverflowKey = ~0ull;

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

// Value of lane `l` (block-uniform l) of a VGPR, as a scalar.
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ int64_t lane_i64(int64_t v, int l) {
  const uint32_t lo = lane_u32((uint32_t)v, l), hi = lane_u32((uint32_t)((uint64_t)v >> 32), l);
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
                                                int mode = 0,
                                                const SegDesc* __restrict__ dsc = nullptr) {
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
    if (dsc) {  // segments precomputed for the batch (desc_kernel): one load level
      if (tid < 64) {
        uint32_t rows = 0;
        if (tid < ng) {
          const SegDesc d = dsc[tid];
          sm.abeg[tid] = d.beg & ~3ll;
          sm.off[tid] = (uint32_t)(d.beg & 3);
          sm.len[tid] = d.len;
          rows = d.len ? (uint32_t)(((d.beg & 3) + d.len + RW - 1) / RW) : 0u;
        }
        uint32_t x = rows;  // inclusive scan of row counts over the wave
#pragma unroll
        for (int o = 1; o < kTG; o <<= 1) {
          const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
          if (tid >= o) x += y;
        }
        if (tid < ng) sm.rstart[tid + 1] = x;
        if (tid == 0) sm.rstart[0] = 0;
      }
      __syncthreads();
    } else {
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
    }
    // Per-term metadata into VGPR lanes (lane s holds term s): uniform values
    // are then v_readlane'd, with no LDS round trip on the address path.
    const int li = min(tid & 63, kTG - 1);
    const int64_t m_abeg = sm.abeg[li];
    const uint32_t m_off = sm.off[li], m_len = sm.len[li];
    const uint32_t m_rs0 = sm.rstart[li], m_rs1 = sm.rstart[li + 1];
    const uint32_t R = (mode & 4) ? 0u : lane_u32(m_rs1, ng - 1);
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
          while (row >= lane_u32(m_rs1, s)) ++s;
          const uint32_t rr = row - lane_u32(m_rs0, s);
          const int64_t A0 = lane_i64(m_abeg, s) + (int64_t)rr * RW;
          // last 4-aligned group of the segment, relative to this row: lanes
          // past it re-read that group (one cache line for all of them)
          // instead of fetching postings of other terms
          const uint32_t off = lane_u32(m_off, s);
          const uint32_t lastg = ((off + lane_u32(m_len, s) - 1) & ~3u) - rr * RW;
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
        const uint32_t len = lane_u32(m_len, rs[b]);
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

// Threshold emission (REST tiles), barrier-free: the keys > theta go to the
// tile's candidate slots (pre-zeroed for the search) through an LDS slot
// counter.  With at most kTileM - 1 keys above theta the tile is complete
// (its last slot stays empty, so the merge never flags it).  With more, the
// lane that holds the kTileM-th key appends the tile to the overflow queue,
// and fixup_kernel rewrites its slots with the tile's exact top-kTileM.  The
// test runs on the fp32 sums (one compare per entry, after a max early-out);
// only a lane holding theta's exact score compares doc ids.  Accumulators are
// never -0.0 (a sum that starts at +0.0 cannot produce it) and docs past
// n_docs hold 0.0, which can only pass when theta's score is negative: those
// are masked explicitly.
template <int S>
__device__ __forceinline__ void emit_above(const float (&fv)[kE], int64_t tile, int64_t n_docs,
                                           uint64_t theta, uint64_t* __restrict__ out,
                                           TileShared& sm, int32_t* ovq, int32_t* ovn,
                                           int32_t code) {
  constexpr int D = 1 << S;
  const int tid = threadIdx.x;
  const float th = key_score((uint32_t)(theta >> 32));
  const uint32_t th_doc = 0xFFFFFFFFu - (uint32_t)theta;
  const int64_t doc0 = tile * D + (int64_t)tid * kE;
  const int64_t lim_hi = n_docs - doc0;  // entries e >= lim_hi are past n_docs
  float mx = fv[0];
#pragma unroll
  for (int e = 1; e < kE; ++e) mx = fmaxf(mx, fv[e]);
  if (mx < th && lim_hi >= kE) return;  // common: nothing of this lane passes
  const int64_t lim_tie = (int64_t)th_doc - doc0;  // ties pass for e < lim_tie
  int c = 0;
#pragma unroll
  for (int e = 0; e < kE; ++e)
    c += (e < lim_hi) & ((fv[e] > th) | ((fv[e] == th) & (e < lim_tie)));
  if (c == 0) return;
  int pos = atomicAdd(&sm.nsel, c);
  const int first = pos;
#pragma unroll
  for (int e = 0; e < kE; ++e) {
    const bool pass = (e < lim_hi) & ((fv[e] > th) | ((fv[e] == th) & (e < lim_tie)));
    if (pass) {
      if (pos < kTileM - 1)
        out[pos] = ((uint64_t)score_key(fv[e]) << 32) |
                   (uint64_t)(0xFFFFFFFFu - (uint32_t)(doc0 + e));
      ++pos;
    }
  }
  if (first <= kTileM - 1 && pos > kTileM - 1) ovq[atomicAdd(ovn, 1)] = code;  // one lane
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
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand,
    const SegDesc* __restrict__ desc, int32_t* __restrict__ ovq, int32_t* __restrict__ ovn,
    int mode) {
  __shared__ __attribute__((aligned(16))) float acc[(1 << S) + 64];
  __shared__ TileShared sm;
  int64_t tile, q;
  if (!item_of<PH>(a.ntiles, Q, P, tile, q)) return;
  accumulate_tile<S, RB>(a, tile, queries + q * T, T, acc, sm, mode,
                         desc ? desc + (tile * Q + q) * T : nullptr);
  uint64_t* out = cand + (q * a.ntiles + tile) * kTileM;
  if (mode & 1) {  // ablation: no selection
    if (threadIdx.x == 0) out[0] = __float_as_uint(acc[0]);
    return;
  }
  float fv[kE];
  load_entries<S>(acc, fv);
  if (PH == kRest) {
    emit_above<S>(fv, tile, a.n_docs, theta[q], out, sm, ovq, ovn,
                  (int32_t)(q * a.ntiles + tile));
    return;
  }
  uint32_t key[kE];
  make_keys<S>(fv, tile, a.n_docs, key);
  select_tile<S>(key, tile, kTileM, out, sm);
}

// ---------------------------------------------------------------------------
// Pipelined score kernel (persistent).  An item's postings are read as one
// concatenated stream (term after term, positions 0..total); thread t holds
// positions t + NT*j, j < J ("slots", 2 VGPRs each: LDS slot | term << 16,
// and the score).  While item n is accumulated and selected, the slots of
// item n+1 are in flight and the segment descriptors of item n+2 (from
// desc_kernel) are in flight, so an item's memory latency overlaps the
// previous item's compute.  Items come in chunks from one counter per XCD
// group (blockIdx % 8) in tile-major order: the workgroups of an XCD share a
// tile (L2 reuse of its hot posting segments across queries).  Every
// pipeline step issues a fixed number of global loads, none under a branch,
// and the two slot register sets alternate by unrolling (no copies), so the
// compiler's vmcnt waits stay counted instead of draining the pipeline.
// Requires 1 <= T <= kTG.
// ---------------------------------------------------------------------------
constexpr int kFifo = 16;
constexpr uint32_t kNoTerm = 31u;

struct PipeMeta {
  int64_t delta[kTG];       // global posting index - stream position, per term
  uint32_t start[kTG + 1];  // stream position of each term's first posting; [T] = total
};

struct PipeShared {
  PipeMeta meta[3];
  int64_t fifo[kFifo];  // upcoming items of this workgroup
  int32_t fhead, fcount, exhausted;
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

__device__ __forceinline__ void fifo_refill(PipeShared& ps, int32_t* ctr, int64_t g_lo,
                                            int64_t g_hi, int chunk) {
  while (!ps.exhausted && ps.fcount + chunk <= kFifo) {
    const int64_t c = g_lo + atomicAdd(ctr, chunk);
    for (int i = 0; i < chunk; ++i) {
      if (c + i >= g_hi) { ps.exhausted = 1; break; }
      ps.fifo[(ps.fhead + ps.fcount) % kFifo] = c + i;
      ++ps.fcount;
    }
  }
}

__device__ __forceinline__ int64_t fifo_peek(const PipeShared& ps, int j) {
  return j < ps.fcount ? ps.fifo[(ps.fhead + j) % kFifo] : -1;
}

// Descriptor registers of one term (thread < T) -> the stage's PipeMeta.
__device__ __forceinline__ void meta_put(const SegDesc& d, int T, PipeMeta& m) {
  const int tid = threadIdx.x;
  if (tid < T) {
    m.delta[tid] = d.beg - (int64_t)d.pre;
    m.start[tid] = d.pre;
    if (tid == T - 1) m.start[T] = d.pre + d.len;
  }
}

// The stage's per-term metadata in VGPR lanes (lane s = term s): uniform
// values are v_readlane'd on the address path instead of read from LDS.
struct MetaLanes {
  int64_t delta;
  uint32_t start, start1;  // start[s], start[s + 1]
  uint32_t total;
};
__device__ __forceinline__ MetaLanes meta_lanes(const PipeMeta& m, int T) {
  const int li = min((int)(threadIdx.x & 63), kTG - 1);
  MetaLanes r;
  r.delta = m.delta[li];
  r.start = m.start[li];
  r.start1 = m.start[li + 1];
  r.total = sgpr(m.start[T]);
  return r;
}

// Issue the J slot loads of stream positions [p0 + NT*j + t].  Exactly 2*J
// loads per call, unconditionally (positions past the stream re-read the
// row's first posting and are tagged kNoTerm).
template <int S, int J>
__device__ __forceinline__ void slots_issue(const IndexArgs& a, const MetaLanes& ml, int T,
                                            uint32_t p0, uint32_t (&lt)[J], float (&v)[J]) {
  constexpr uint32_t NT = (1u << S) / kE;
  const uint32_t tid = threadIdx.x;
  int s = 0;  // term of the current slot-row's first position (block-uniform)
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t r0 = p0 + NT * j;
    uint32_t P = r0 + tid;
    uint32_t st = kNoTerm;
    int64_t delta = 0;
    if (r0 < ml.total) {
      while (s + 1 < T && lane_u32(ml.start1, s) <= r0) ++s;
      st = s;
      delta = lane_i64(ml.delta, s);
      const uint32_t rend = min(r0 + NT, ml.total);
      for (int sl = s + 1; sl < T && lane_u32(ml.start, sl) < rend; ++sl) {
        if (P >= lane_u32(ml.start, sl)) {
          st = sl;
          delta = lane_i64(ml.delta, sl);
        }
      }
      if (P >= ml.total) {  // past the stream: reload row position r0 (term s)
        P = r0;
        st = kNoTerm;
        delta = lane_i64(ml.delta, s);
      }
    } else {
      P = 0;
    }
    const int64_t g = (int64_t)P + delta;
    lt[j] = (uint32_t)a.ldoc[g] | (st << 16);
    v[j] = a.val[g];
  }
}

// Add the slots of stream positions [p0, p0 + NT*J) in term order.
template <int S, int J>
__device__ __forceinline__ void slots_add(const MetaLanes& ml, int T, uint32_t p0, float* acc,
                                          const uint32_t (&lt)[J], const float (&v)[J],
                                          int& last_s) {
  constexpr uint32_t NT = (1u << S) / kE;
  const uint32_t dummy = (1u << S) + (threadIdx.x & 63);
  int s = 0;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const uint32_t r0 = p0 + NT * j;
    if (r0 >= ml.total) break;
    while (s + 1 < T && lane_u32(ml.start1, s) <= r0) ++s;
    const uint32_t rend = min(r0 + NT, ml.total);
    for (int sc = s; sc < T && lane_u32(ml.start, sc) < rend; ++sc) {
      if (lane_u32(ml.start1, sc) == lane_u32(ml.start, sc)) continue;  // empty term
      if (sc != last_s) {
        if (last_s >= 0) __syncthreads();  // previous term's adds complete
        last_s = sc;
      }
      const uint32_t d = (lt[j] >> 16) == (uint32_t)sc ? (lt[j] & 0xFFFFu) : dummy;
      const float x = acc[d];
      acc[d] = x + v[j];
    }
  }
}

template <int S, int PH, int J>
__global__ __launch_bounds__((1 << S) / kE, 4) void score_pipe_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t Q, int32_t T, int32_t P,
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand,
    const SegDesc* __restrict__ desc, int32_t* __restrict__ wctr, int32_t chunk,
    int32_t* __restrict__ ovq, int32_t* __restrict__ ovn) {
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  __shared__ __attribute__((aligned(16))) float acc[D + 64];
  __shared__ PipeShared ps;
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
  const int td = min(tid, T - 1);  // every thread loads a valid descriptor slot

  if (refiller) {
    ps.fhead = 0;
    ps.fcount = 0;
    ps.exhausted = 0;
    fifo_refill(ps, ctr, g_lo, g_hi, chunk);
  }
  if (tid == 0) sm.nsel = 0;
  float4* acc4 = reinterpret_cast<float4*>(acc);
#pragma unroll
  for (int j = 0; j < kE / 4; ++j) acc4[j * NT + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
  __syncthreads();
  const int64_t it0 = sgpr64(fifo_peek(ps, 0));
  if (it0 < 0) return;  // block-uniform
  {
    int64_t tile, q;
    item_tile<PH>(it0, Q, P, tile, q);
    const SegDesc d0 = desc[(tile * Q + q) * T + td];
    const int64_t it1 = sgpr64(fifo_peek(ps, 1));
    item_tile<PH>(it1 >= 0 ? it1 : it0, Q, P, tile, q);
    const SegDesc d1 = desc[(tile * Q + q) * T + td];
    meta_put(d0, T, ps.meta[0]);
    meta_put(d1, T, ps.meta[1]);
  }
  __syncthreads();
  uint32_t ltA[J], ltB[J];
  float vA[J], vB[J];
  slots_issue<S, J>(a, meta_lanes(ps.meta[0], T), T, 0, ltA, vA);

  auto step = [&](int n, uint32_t (&lt)[J], float (&v)[J], uint32_t (&ltN)[J],
                  float (&vN)[J]) -> bool {
    const int64_t it = sgpr64(fifo_peek(ps, 0));
    const int64_t nx = sgpr64(fifo_peek(ps, 1));
    const int64_t n2 = sgpr64(fifo_peek(ps, 2));
    const PipeMeta& mc = ps.meta[n % 3];
    int64_t tile, q, t2, q2;
    item_tile<PH>(it, Q, P, tile, q);
    // (a) descriptors of item n+2
    item_tile<PH>(n2 >= 0 ? n2 : it, Q, P, t2, q2);
    const SegDesc d2 = desc[(t2 * Q + q2) * T + td];
    const MetaLanes mlc = meta_lanes(mc, T);
    // (b) slots of item n+1 (without a next item: harmless reloads of item n)
    slots_issue<S, J>(a, nx >= 0 ? meta_lanes(ps.meta[(n + 1) % 3], T) : mlc, T, 0, ltN, vN);
    // (c) accumulate item n: prefetched slots, then the rest of its stream
    int last_s = -1;
    slots_add<S, J>(mlc, T, 0, acc, lt, v, last_s);
    for (uint32_t p0 = NT * J; p0 < mlc.total; p0 += NT * J) {
      uint32_t ltX[J];
      float vX[J];
      slots_issue<S, J>(a, mlc, T, p0, ltX, vX);
      slots_add<S, J>(mlc, T, p0, acc, ltX, vX, last_s);
    }
    __syncthreads();
    // (d) selection of item n; entries are zeroed for item n+1 as they are read
    {
      float fv[kE];
      load_entries<S>(acc, fv);
#pragma unroll
      for (int j = 0; j < kE / 4; ++j) acc4[j * NT + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
      uint64_t* out = cand + (q * a.ntiles + tile) * kTileM;
      if (PH == kRest) {
        emit_above<S>(fv, tile, a.n_docs, theta[q], out, sm, ovq, ovn,
                      (int32_t)(q * a.ntiles + tile));
      } else {
        uint32_t key[kE];
        make_keys<S>(fv, tile, a.n_docs, key);
        select_tile<S>(key, tile, kTileM, out, sm);
      }
    }
    __syncthreads();  // reads of sm.nsel / red and of meta[n % 3] are done
    // (e) publish item n+2's descriptors, advance the item list
    if (n2 >= 0) meta_put(d2, T, ps.meta[(n + 2) % 3]);
    if (tid == 0) sm.nsel = 0;
    if (refiller) {
      ps.fhead = (ps.fhead + 1) % kFifo;
      --ps.fcount;
      fifo_refill(ps, ctr, g_lo, g_hi, chunk);
    }
    __syncthreads();
    return nx >= 0;
  };

  for (int n = 0;; n += 2) {
    if (!step(n, ltA, vA, ltB, vB)) break;
    if (!step(n + 1, ltB, vB, ltA, vA)) break;
  }
}

// ---------------------------------------------------------------------------
// Slot score kernel: one workgroup per (tile, query) like score_tiles_kernel,
// but the item's postings are read as one dense concatenated stream (thread t
// takes positions t + NT*j): every lane of a load carries a posting, each
// load is 2 + 4 bytes per lane, and the RMW touches one posting per lane per
// slot-row, instead of 4-wide rows of which ~3/4 of the lanes idle on short
// segments.  Needs the batch's segment descriptors (1 <= T <= kTG).
// ---------------------------------------------------------------------------
template <int S, int PH, int J>
__global__ __launch_bounds__((1 << S) / kE) void score_slots_kernel(
    IndexArgs a, int32_t Q, int32_t T, int32_t P, const uint64_t* __restrict__ theta,
    uint64_t* __restrict__ cand, const SegDesc* __restrict__ desc, int32_t* __restrict__ ovq,
    int32_t* __restrict__ ovn) {
  constexpr int D = 1 << S;
  constexpr int NT = D / kE;
  __shared__ __attribute__((aligned(16))) float acc[D + 64];
  __shared__ PipeMeta pm;
  __shared__ TileShared sm;
  const int tid = threadIdx.x;
  int64_t tile, q;
  if (!item_of<PH>(a.ntiles, Q, P, tile, q)) return;
  float4* acc4 = reinterpret_cast<float4*>(acc);
#pragma unroll
  for (int j = 0; j < kE / 4; ++j) acc4[j * NT + tid] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (tid == 0) sm.nsel = 0;
  if (tid < T) meta_put(desc[(tile * Q + q) * T + tid], T, pm);
  __syncthreads();
  const MetaLanes ml = meta_lanes(pm, T);
  int last_s = -1;
  for (uint32_t p0 = 0; p0 < ml.total; p0 += NT * J) {
    uint32_t lt[J];
    float v[J];
    slots_issue<S, J>(a, ml, T, p0, lt, v);
    slots_add<S, J>(ml, T, p0, acc, lt, v, last_s);
  }
  __syncthreads();
  float fv[kE];
  load_entries<S>(acc, fv);
  uint64_t* out = cand + (q * a.ntiles + tile) * kTileM;
  if (PH == kRest) {
    emit_above<S>(fv, tile, a.n_docs, theta[q], out, sm, ovq, ovn,
                  (int32_t)(q * a.ntiles + tile));
    return;
  }
  uint32_t key[kE];
  make_keys<S>(fv, tile, a.n_docs, key);
  select_tile<S>(key, tile, kTileM, out, sm);
}

// Segment descriptors of every (tile, query, term) of the batch, tile-major
// like the score kernels' items: one thread per (tile, query).
template <int S>
__global__ __launch_bounds__(256) void desc_kernel(IndexArgs a, const int32_t* __restrict__ queries,
                                                   int32_t Q, int32_t T,
                                                   SegDesc* __restrict__ desc) {
  constexpr uint32_t RW = 4 * ((1 << S) / kE);
  const int64_t item = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= a.ntiles * Q) return;
  const int64_t tile = item / Q, q = item - tile * Q;
  uint32_t pre = 0;
  (void)RW;
  for (int s = 0; s < T; ++s) {
    const int32_t term = queries[q * T + s];
    int64_t beg = 0;
    uint32_t len = 0;
    if (term >= 0 && term < a.V) {  // negative ids are padding (bm25_native.py:151)
      const uint32_t* r = a.rel + (int64_t)term * (a.ntiles + 1) + tile;
      const uint32_t r0 = r[0], r1 = r[1];
      beg = a.indptr[term] + r0;
      len = r1 - r0;
    }
    desc[item * T + s] = SegDesc{beg, len, pre};
    pre += len;
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

// Exact top-kTileM of the REST tiles that overflowed the threshold pass;
// persistent, queue-driven like rescore_kernel.
template <int S>
__global__ __launch_bounds__((1 << S) / kE) void fixup_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, uint64_t* __restrict__ cand,
    const int32_t* __restrict__ ovq, int32_t* __restrict__ counters) {
  __shared__ __attribute__((aligned(16))) float acc[(1 << S) + 64];
  __shared__ TileShared sm;
  const int32_t n_items = counters[2];
  for (;;) {
    __syncthreads();
    if (threadIdx.x == 0) sm.item = atomicAdd(&counters[3], 1);
    __syncthreads();
    const int32_t it = sm.item;
    if (it >= n_items) break;
    const int32_t code = ovq[it];
    const int64_t q = code / a.ntiles, tile = code - q * a.ntiles;
    accumulate_tile<S>(a, tile, queries + q * T, T, acc, sm);
    float fv[kE];
    load_entries<S>(acc, fv);
    uint32_t key[kE];
    make_keys<S>(fv, tile, a.n_docs, key);
    select_tile<S>(key, tile, kTileM, cand + (int64_t)code * kTileM, sm);
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

// Same result as topk_of when at least k candidates are >= lo: candidates
// below lo (or empty) are dropped while compacting into LDS (wave ballots, one
// LDS atomic per wave), so only the survivors are sorted.
template <class Src>
__device__ void topk_compact(const Src& src, int64_t n_total, int k, uint64_t lo, uint64_t* keys,
                             int* cnt) {
  const int B = next_pow2(k);
  if (threadIdx.x == 0) *cnt = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t rounds = (n_total + blockDim.x - 1) / blockDim.x;
  for (int64_t r = 0; r < rounds; ++r) {
    const int64_t i = r * blockDim.x + threadIdx.x;
    const uint64_t key = i < n_total ? src(i) : 0ull;
    const bool keep = key != 0ull && key != kOverflowKey && key >= lo;
    const unsigned long long m = __ballot(keep);
    int base = 0;
    if (lane == 0 && m) base = atomicAdd(cnt, (int)__popcll(m));
    base = __shfl(base, 0, 64);
    const int pos = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                          __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (keep && pos < kMergeP) keys[pos] = key;
  }
  __syncthreads();
  const int c = *cnt;
  if (c > kMergeP) {  // too many survivors: full chunked sort
    __syncthreads();
    topk_of(src, n_total, k, keys);
    return;
  }
  const int n = next_pow2(c > B ? c : B);
  for (int i = c + threadIdx.x; i < n; i += blockDim.x) keys[i] = 0ull;
  __syncthreads();
  bitonic_sort_desc(keys, n);
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
    int64_t doc_offset, Workspace ws, const uint64_t* __restrict__ theta_s,
    int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  __shared__ int32_t s_nflag, s_cnt;
  const int64_t q = blockIdx.x;
  const uint64_t* c = cand + q * ntiles * kTileM;
  if (threadIdx.x == 0) s_nflag = 0;
  // theta_s (sampling pass): k sample candidates are >= it, so nothing below
  // it can reach the top-k
  topk_compact(SrcFirst{c}, ntiles * kTileM, k, theta_s ? theta_s[q] : 0ull, keys, &s_cnt);
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
bool tile_shift_supported(int s) { return s >= 12 && s <= 15; }

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
  if (getenv("BM25_NO_SAMPLE")) return 1;
  for (int P = 8; P >= 2; P >>= 1) {
    const int64_t nS = (ntiles + P - 1) / P;
    if (ntiles >= 2 * P && nS * kTileM >= 2 * (int64_t)k) return P;
  }
  return 1;
}

static bool use_desc(int64_t T) {
  return !getenv("BM25_NO_DESC") && T >= 1 && T <= kDescMaxT;
}

// The pipelined kernel is opt-in (BM25_PIPE=1): on config 3 it is still
// slower than the per-item kernel (measurements).
static bool use_pipe(int64_t T) {
  return getenv("BM25_PIPE") && use_desc(T) && T <= kTG;
}

template <int S, int PH>
static void launch_pipe(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int P,
                        const Workspace& ws, hipStream_t st) {
  constexpr int J = 8;
  static int grid = 0;
  if (grid == 0) {
    int dev = 0, cus = 0, occ = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, score_pipe_kernel<S, PH, J>,
                                                 (1 << S) / kE, 0);
    const char* e = getenv("BM25_PIPE_WG_PER_CU");
    if (e) occ = atoi(e);
    grid = ((cus * (occ > 0 ? occ : 1) + 7) / 8) * 8;
  }
  hipLaunchKernelGGL((score_pipe_kernel<S, PH, J>), dim3((unsigned)grid), dim3((1 << S) / kE), 0,
                     st, args_of(ix), q, (int32_t)Q, (int32_t)T, (int32_t)P, ws.theta, ws.cand,
                     ws.desc, ws.wctr + (PH == kRest ? 8 : 0), (int32_t)8, ws.ovq,
                     ws.counters + 2);
}

static bool use_slots(int64_t T) {
  return getenv("BM25_SLOTS") && use_desc(T) && T <= kTG;
}

template <int S, int PH>
static void launch_phase(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int P,
                         const Workspace& ws, hipStream_t st) {
  const int64_t nS = (ix.ntiles + P - 1) / P;
  const int64_t nt = PH == kAll ? ix.ntiles : (PH == kSample ? nS : ix.ntiles - nS);
  const int64_t grid = ((nt * Q + 7) >> 3) << 3;
  if (grid == 0) return;
  if (use_pipe(T)) {
    launch_pipe<S, PH>(ix, q, Q, T, P, ws, st);
    return;
  }
  if (use_slots(T)) {
    const int J = getenv("BM25_J") ? atoi(getenv("BM25_J")) : 8;
    if (J == 16)
      hipLaunchKernelGGL((score_slots_kernel<S, PH, 16>), dim3((unsigned)grid),
                         dim3((1 << S) / kE), 0, st, args_of(ix), (int32_t)Q, (int32_t)T,
                         (int32_t)P, ws.theta, ws.cand, ws.desc, ws.ovq, ws.counters + 2);
    else
      hipLaunchKernelGGL((score_slots_kernel<S, PH, 8>), dim3((unsigned)grid),
                         dim3((1 << S) / kE), 0, st, args_of(ix), (int32_t)Q, (int32_t)T,
                         (int32_t)P, ws.theta, ws.cand, ws.desc, ws.ovq, ws.counters + 2);
    return;
  }
  const int rb = getenv("BM25_RB") ? atoi(getenv("BM25_RB")) : 8;
  if (rb == 4)
    hipLaunchKernelGGL((score_tiles_kernel<S, PH, 4>), dim3((unsigned)grid), dim3((1 << S) / kE),
                       0, st, args_of(ix), q, (int32_t)Q, (int32_t)T, (int32_t)P, ws.theta,
                       ws.cand, use_desc(T) ? ws.desc : nullptr, ws.ovq, ws.counters + 2,
                       env_mode());
  else
    hipLaunchKernelGGL((score_tiles_kernel<S, PH, 8>), dim3((unsigned)grid), dim3((1 << S) / kE),
                       0, st, args_of(ix), q, (int32_t)Q, (int32_t)T, (int32_t)P, ws.theta,
                       ws.cand, use_desc(T) ? ws.desc : nullptr, ws.ovq, ws.counters + 2,
                       env_mode());
}

template <int S>
static void launch_score_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int k,
                           const Workspace& ws, hipStream_t st) {
  if (use_pipe(T)) hipMemsetAsync(ws.wctr, 0, 16 * sizeof(int32_t), st);
  hipMemsetAsync(ws.counters, 0, 4 * sizeof(int32_t), st);
  hipMemsetAsync(ws.cand, 0, sizeof(uint64_t) * Q * ix.ntiles * kTileM, st);
  if (use_desc(T)) {
    const int64_t n = ix.ntiles * Q;
    hipLaunchKernelGGL(desc_kernel<S>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st,
                       args_of(ix), q, (int32_t)Q, (int32_t)T, ws.desc);
  }
  const int P = sample_stride(ix.ntiles, k);
  if (P == 1) {
    launch_phase<S, kAll>(ix, q, Q, T, 1, ws, st);
    return;
  }
  launch_phase<S, kSample>(ix, q, Q, T, P, ws, st);
  hipLaunchKernelGGL(theta_kernel, dim3((unsigned)Q), dim3(kMergeNT), 0, st, ws.cand, ix.ntiles,
                     (int32_t)P, (int32_t)k, ws.theta);
  launch_phase<S, kRest>(ix, q, Q, T, P, ws, st);
  hipLaunchKernelGGL(fixup_kernel<S>, dim3(256), dim3((1 << S) / kE), 0, st, args_of(ix), q,
                     (int32_t)T, ws.cand, ws.ovq, ws.counters);
}

hipError_t launch_score_tiles(const DevIndex& ix, const int32_t* d_queries, int64_t Q,
                              int64_t T, int k, const Workspace& ws, hipStream_t stream) {
  if (Q == 0 || ix.ntiles == 0) return hipSuccess;

  switch (ix.tile_shift) {
    case 12: launch_score_s<12>(ix, d_queries, Q, T, k, ws, stream); break;
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
  hipError_t e = hipMemsetAsync(ws.counters, 0, 2 * sizeof(int32_t), stream);
  if (e != hipSuccess) return e;
  const bool sampled = sample_stride(ix.ntiles, k) > 1;
  hipLaunchKernelGGL(merge_first_kernel, dim3((unsigned)Q), dim3(kMergeNT), 0, stream, ws.cand,
                     ix.ntiles, (int32_t)k, maxflag, ix.doc_offset, ws,
                     sampled ? ws.theta : nullptr, d_docs, d_scores);
  if (k > kTileM) {
    switch (ix.tile_shift) {
      case 12: launch_rescore_s<12>(ix, d_queries, T, k, maxflag, ws, stream); break;
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
    case 12: hipLaunchKernelGGL(scores_dense_kernel<12>, grid, dim3((1 << 12) / kE), 0, stream, args_of(ix), d_query, (int32_t)T, d_out); break;
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
