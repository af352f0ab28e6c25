// bm25mi_kernels.hip — gfx950 kernels of the BM25 CSC query path.
//
// Replaces the reference's GPU path (MAX graph ops.gather -> ops.sum ->
// ops.top_k, gpu_bm25/common.py:64-80, vendored as
// operations/gather_scatter.mojo:683-763 and operations/topk.mojo:576-963)
// and its CPU scorer (bm25_native.py:149-158, 204-214).  DESIGN.md §4.
//
// Unit of work: an ITEM = (tile, query), a tile being 2^S consecutive docs
// (S = 11: 2048 docs).  One wavefront owns one item at a time and keeps the
// tile's fp32 accumulators in its own LDS slice, so the query-term order of
// each document's adds (the exact fp32 arithmetic of scipy csc_matvec,
// bm25_native.py:152) is simply the wave's program order: no barriers.
//
//   score_wave<SAMPLE>  every P-th tile: the tile's exact top-4 keys
//   theta               per query: the k-th best sample key, a lower bound of
//                       the final k-th key
//   score_wave<REST>    every other tile: appends the keys above theta to the
//                       query's candidate list
//   merge_first         per query: top-k of the sample keys + list; flags the
//                       (rare) sample tiles whose 4th key beats the k-th key;
//                       a query whose list overflowed goes to the fallback
//   rescore             exact top-k of every flagged tile
//   merge_final         merges those exact lists in
//   fallback stage      the overflowed queries through the same pipeline with
//                       every tile a sample tile (exact top-4 everywhere)
// The result is exactly the top-k under (score desc, doc asc) of the dense
// score vector, with untouched documents scoring 0.
#include "bm25mi_internal.h"

#include <map>
#include <mutex>
#include <cstdio>
#include <cstdlib>
#include <vector>

namespace bm25mi {

enum Phase { kAll = 0, kSample = 1, kRest = 2 };

#ifndef BM25_KJ
#define BM25_KJ 8
#endif
constexpr int kJ = BM25_KJ;  // posting rows (64 postings each) in flight per wave
constexpr int kWaves = 4;   // independent waves per score workgroup
constexpr int kGroup = 64;  // query terms per descriptor group (one per lane)

struct IndexArgs {
  const int64_t* indptr;
  const uint32_t* rel;
  const uint16_t* ldoc;
  const float* val;
  int64_t V, ntiles, n_docs, nnz;
  int64_t doc_offset;  // global id of the index's first doc (sample keys are global)
  int32_t nonneg;
  int32_t sparse;           // segment table form (DevIndex)
  const int64_t* tl_ptr;    // sparse: tile lists
  const uint16_t* tl_tile;
  const uint32_t* tl_start;
  const uint64_t* seg;      // sparse + band kernel: this search's per-item segments
};

static IndexArgs args_of(const DevIndex& ix) {
  return IndexArgs{ix.indptr, ix.rel, ix.ldoc, ix.val, ix.n_terms, ix.ntiles, ix.n_docs,
                   ix.nnz, ix.doc_offset, ix.nonneg ? 1 : 0, ix.sparse ? 1 : 0, ix.tl_ptr,
                   ix.tl_tile, ix.tl_start, nullptr};
}

// Segment bounds [r0, r1) (relative to indptr[term]) of a valid term in a
// tile.  Sparse: a binary search of the term's tile list (the cold paths; the
// band kernel reads a per-search table instead, seg_table_kernel).
__device__ __forceinline__ void segment(const IndexArgs& a, int64_t term, int64_t tile,
                                        uint32_t& r0, uint32_t& r1) {
  if (!a.sparse) {
    const uint32_t* r = a.rel + term * (a.ntiles + 1) + tile;
    r0 = r[0];
    r1 = r[1];
    return;
  }
  const int64_t b = a.tl_ptr[term], e = a.tl_ptr[term + 1];
  int64_t lo = b, hi = e;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)a.tl_tile[mid] < tile) lo = mid + 1;
    else hi = mid;
  }
  const uint32_t df = (uint32_t)(a.indptr[term + 1] - a.indptr[term]);
  const uint32_t at = lo < e ? a.tl_start[lo] : df;
  r0 = r1 = at;
  if (lo < e && (int64_t)a.tl_tile[lo] == tile) r1 = lo + 1 < e ? a.tl_start[lo + 1] : df;
}

// Sample tiles: groups of G consecutive tiles, one group in every G*P tiles
// (tile of sample index si, and the number of sample tiles of an index).
// Consecutive sample tiles of a query then share the boundary cache lines of
// its terms' posting segments, as the REST tiles do.
__host__ __device__ inline int64_t sample_tile(int64_t si, int64_t P, int64_t G) {
  return (si / G) * G * P + si % G;
}
__host__ __device__ inline int64_t sample_count(int64_t ntiles, int64_t P, int64_t G) {
  const int64_t r = ntiles % (G * P);
  return (ntiles / (G * P)) * G + (r < G ? r : G);
}

// One search stage of candidate selection (see the merge kernels).
struct Stage {
  const uint64_t* cand;      // [nq][nt][kTileM] exact top-kTileM keys of the stage's tiles
  uint64_t* cand_out;        // where the score pass writes its keys (SAMPLE / ALL)
  int64_t cstride;           // keys per query row of cand_out
  int64_t nt;                // candidate tiles per query
  int32_t P;                 // SAMPLE: sampling stride (sample_tile)
  int32_t G;                 // SAMPLE: sample tiles per group (sample_tile)
  int32_t M;                 // SAMPLE: keys per sample tile
  const uint64_t* theta;     // [nq] lower bound of the k-th key (null: none)
  const uint64_t* list;      // [nq][C] keys of the other tiles above theta (null: none)
  const int32_t* list_cnt;   // [nq]
  int32_t C;
  const uint64_t* sample_keys;  // REST: this shard's sample keys [nq][sample_stride] (null: none)
  int64_t sample_stride;
  const int32_t* qmap;       // stage query -> batch row (null: identity)
  const int32_t* nq_dev;     // stage queries, on the device (null: nq_host)
  int32_t nq_host;           // stage queries (host bound)
  int32_t* fb;               // overflowed queries are appended here
  int32_t* fb_cnt;
  int32_t ctr_region;        // claim counters of the launch: ws.wctr + region * kWctrInts
  bool ctr_zeroed;           // ... already zeroed by the search's zero_search_kernel
};

__device__ __forceinline__ int lane_id() { return (int)(threadIdx.x & 63); }

// Value of lane `l` (wave-uniform l) of a VGPR, as a scalar.
__device__ __forceinline__ uint32_t lane_u32(uint32_t v, int l) {
  return (uint32_t)__builtin_amdgcn_readlane((int)v, l);
}
__device__ __forceinline__ int64_t lane_i64(int64_t v, int l) {
  const uint32_t lo = lane_u32((uint32_t)v, l), hi = lane_u32((uint32_t)((uint64_t)v >> 32), l);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

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

// Sum over the 64 lanes of a wave (DPP inside 16-lane rows, then SGPRs).
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) + (uint32_t)__builtin_amdgcn_readlane((int)v, 16) +
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) + (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
}

// Inclusive prefix sum over the wave.
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  const int lane = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= o) x += y;
  }
  return x;
}

// LDS fp32 add without return (ds_add_f32): IEEE round-to-nearest-even, the
// same rounding as scipy's `y[i] += data[p]`.
__device__ __forceinline__ void lds_add(float* p, float v) {
  __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// ---------------------------------------------------------------------------
// Scatter phase of one item: acc[slot(d)] += the query terms' scores of doc d,
// term by term in query order.  Replaces doc_toks[:, query].sum(axis=1)
// (bm25_native.py:152 -> scipy csc_matvec): same fp32 adds, same order per doc.
//
// Lane s of the wave holds the segment of query term s inside the tile
// ([beg, beg + len) of the CSC arrays, from indptr + the rel table).  The
// segments are read as one concatenated stream, 64 positions per row (lane l
// of row r reads position 64r + l), so every lane of a load carries a
// posting: a u16 LDS slot and an f32 score.  kJ rows are loaded before the
// first add.  The adds are LDS float atomics issued row by row in stream
// order; the LDS executes one wave's instructions in order, so each doc's adds
// happen in term order.  Inside a row, two lanes of one term never share a doc
// (a CSC column holds a doc once); a row that spans a term boundary is issued
// once per term under an exec mask.
// ---------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void add_group(const IndexArgs& a, int64_t beg, uint32_t len, int ng,
                                          float* acc) {
  const int lane = lane_id();
  const uint32_t incl = wave_incl_scan(len);
  const uint32_t start = incl - len;                // lane s: stream position of term s
  const int64_t delta = beg - (int64_t)start;       // posting index - stream position
  const uint32_t total = lane_u32(incl, ng - 1);
  int s_cur = 0;  // term of the current row's first position (wave-uniform)
  for (uint32_t r0 = 0; r0 < total; r0 += 64u * kJ) {
    uint32_t dl[kJ];
    float v[kJ];
    int ts[kJ], sf[kJ], sl[kJ];
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      const uint32_t rs = r0 + 64u * j;
      sf[j] = -1;
      sl[j] = -1;
      ts[j] = 0;
      dl[j] = 0;
      v[j] = 0.f;
      if (rs < total) {
        while (s_cur + 1 < ng && lane_u32(start, s_cur + 1) <= rs) ++s_cur;
        const uint32_t p = rs + lane;
        const uint32_t re = min(rs + 64u, total);
        int s = s_cur, last = s_cur;
        int64_t d = lane_i64(delta, s_cur);
        for (int sc = s_cur + 1; sc < ng && lane_u32(start, sc) < re; ++sc) {
          if (p >= lane_u32(start, sc)) {
            s = sc;
            d = lane_i64(delta, sc);
          }
          last = sc;
        }
        sf[j] = s_cur;
        sl[j] = last;
        ts[j] = s;
        if (p < total) {
          const int64_t g = (int64_t)p + d;
          dl[j] = a.ldoc[g];
          v[j] = a.val[g];
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      if (sf[j] < 0) break;
      const bool live = r0 + 64u * j + lane < total;
      if (sf[j] == sl[j]) {
        if (live) lds_add(acc + dl[j], v[j]);
      } else {
        for (int sc = sf[j]; sc <= sl[j]; ++sc)
          if (live && ts[j] == sc) lds_add(acc + dl[j], v[j]);
      }
    }
  }
}

// All query terms of one item, in groups of 64 (one term per lane).
template <int S>
__device__ __forceinline__ void add_item(const IndexArgs& a, int64_t tile,
                                         const int32_t* __restrict__ qterms, int T, float* acc) {
  const int lane = lane_id();
  for (int g0 = 0; g0 < T; g0 += kGroup) {
    const int ng = min(kGroup, T - g0);
    int64_t beg = 0;
    uint32_t len = 0;
    if (lane < ng) {
      const int32_t term = qterms[g0 + lane];
      if (term >= 0 && term < a.V) {  // negative ids are padding (bm25_native.py:151)
        uint32_t r0, r1;
        segment(a, term, tile, r0, r1);
        beg = a.indptr[term] + r0;
        len = r1 - r0;
      }
    }
    add_group<S>(a, beg, len, ng, acc);
  }
}

template <int S>
__device__ __forceinline__ void zero_acc(float* acc) {
  float4* a4 = reinterpret_cast<float4*>(acc);
#pragma unroll
  for (int j = 0; j < (1 << S) / 256; ++j) a4[j * 64 + lane_id()] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// Accumulator layout: tile-local doc d lives at LDS float d (identity), so
// the sorted doc ids of a posting row fall on consecutive banks.  A lane reads
// float4 j*64 + lane: its entry e is tile-local doc entry_doc(e, lane) =
// 256*(e/4) + 4*lane + e%4 (conflict-free ds_read_b128), cleared for the next
// item as it is read.
__device__ __forceinline__ uint32_t entry_doc(int e, uint32_t lane) {
  return ((uint32_t)(e >> 2) << 8) | (lane << 2) | (uint32_t)(e & 3);
}

template <int S>
__device__ __forceinline__ void take_entries(float* acc, float (&fv)[(1 << S) / 64]) {
  float4* a4 = reinterpret_cast<float4*>(acc);
  const int lane = lane_id();
#pragma unroll
  for (int j = 0; j < (1 << S) / 256; ++j) {
    const float4 f = a4[j * 64 + lane];
    a4[j * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    fv[j * 4 + 0] = f.x;
    fv[j * 4 + 1] = f.y;
    fv[j * 4 + 2] = f.z;
    fv[j * 4 + 3] = f.w;
  }
}

// ---------------------------------------------------------------------------
// Exact selection: the m best keys of the tile, best first, into out[0..m).
// Each lane keeps its best entry (the first of equal keys: its entries are in
// doc order); a round takes the wave's best key, then the smallest doc among
// the lanes holding it, whose lane and entry follow from the doc id.  Docs
// past n_docs never qualify.
// ---------------------------------------------------------------------------
template <int S>
__device__ __forceinline__ void select_top(const float (&fv)[(1 << S) / 64], int64_t tile,
                                           int64_t n_docs, int m, uint32_t idoff,
                                           uint64_t* __restrict__ out) {
  constexpr int E = (1 << S) / 64;
  const uint32_t lane = lane_id();
  const int64_t base = tile << S;
  const int lim = (int)min<int64_t>(1 << S, n_docs - base);  // docs >= lim: past n_docs
  uint32_t key[E];
#pragma unroll
  for (int e = 0; e < E; ++e) key[e] = (int)entry_doc(e, lane) < lim ? score_key(fv[e]) : 0u;
  uint32_t lmax = 0, ldoc = 0;
#pragma unroll
  for (int e = 0; e < E; ++e)
    if (key[e] > lmax) {
      lmax = key[e];
      ldoc = entry_doc(e, lane);
    }
  for (int r = 0; r < m; ++r) {
    const uint32_t wm = wave_max_u32(lmax);
    if (wm == 0) {  // no valid entry left (tile smaller than m)
      if (lane == 0) out[r] = 0;
      continue;
    }
    const uint32_t doc = 0xFFFFFFFFu - wave_max_u32(lmax == wm ? 0xFFFFFFFFu - ldoc : 0u);
    if (lane == ((doc >> 2) & 63u)) {
      out[r] = ((uint64_t)wm << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + doc) - idoff);
      const int eb = (int)(((doc >> 8) << 2) | (doc & 3u));
      lmax = 0;
#pragma unroll
      for (int e = 0; e < E; ++e) {
        key[e] = e == eb ? 0u : key[e];
        if (key[e] > lmax) {
          lmax = key[e];
          ldoc = entry_doc(e, lane);
        }
      }
    }
  }
}

// Threshold emission (REST tiles): every key > theta is appended to the
// query's list (one atomic per wave).  A list that overflows its capacity C
// only counts: the merge sends that query to the exact fallback stage.  The
// test runs on the fp32 sums (one compare per entry, after a max early-out);
// only an entry equal to theta's score compares doc ids.  Accumulators are
// never -0.0 (a sum that starts at +0.0 cannot produce it); docs past n_docs
// are masked.
template <int S>
__device__ __forceinline__ void emit_above(const float (&fv)[(1 << S) / 64], int64_t tile,
                                           int64_t n_docs, uint64_t theta,
                                           uint64_t* __restrict__ list, int32_t* __restrict__ cnt,
                                           int32_t C) {
  constexpr int E = (1 << S) / 64;
  const uint32_t lane = lane_id();
  const float th = key_score((uint32_t)(theta >> 32));
  const int64_t base = tile << S;
  constexpr int64_t D = 1 << S;
  // tile-local bounds, clamped to [-1, D]: docs >= lim are past n_docs, ties
  // pass for docs < tie
  const int lim = (int)max<int64_t>(-1, min<int64_t>(D, n_docs - base));
  const int tie = (int)max<int64_t>(
      -1, min<int64_t>(D, (int64_t)(0xFFFFFFFFu - (uint32_t)theta) - base + 1));
  float mx = fv[0];
#pragma unroll
  for (int e = 1; e < E; ++e) mx = fmaxf(mx, fv[e]);
  int c = 0;
  if (!(mx < th && lim == D)) {
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const int d = (int)entry_doc(e, lane);
      c += (d < lim) & ((fv[e] > th) | ((fv[e] == th) & (d < tie)));
    }
  }
  if (__ballot(c > 0) == 0) return;  // common: nothing of this tile passes
  const uint32_t incl = wave_incl_scan((uint32_t)c);
  int pos = 0;
  if (lane == 63) pos = atomicAdd(cnt, (int)incl);
  pos = __shfl(pos, 63, 64) + (int)incl - c;
  if (c == 0) return;
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const int d = (int)entry_doc(e, lane);
    const bool pass = (d < lim) & ((fv[e] > th) | ((fv[e] == th) & (d < tie)));
    if (pass) {
      if (pos < C)
        list[pos] = ((uint64_t)score_key(fv[e]) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + d));
      ++pos;
    }
  }
}

// ---------------------------------------------------------------------------
// Selection straight from the LDS accumulators, 8 entries (2 float4) per lane
// at a time, so no item keeps all 2^S/64 entries in registers.
// ---------------------------------------------------------------------------
// Key of entry e of this lane (0 past n_docs); `lim` = n_docs - tile base.
__device__ __forceinline__ uint32_t entry_key(float f, int e, uint32_t lane, int lim) {
  return (int)entry_doc(e, lane) < lim ? score_key(f) : 0u;
}

// This lane's best key over its entries (first of equal keys = smallest doc).
template <int S>
__device__ __forceinline__ void lane_best(const float* acc, int lim, uint32_t& bk, uint32_t& bd) {
  const float4* a4 = reinterpret_cast<const float4*>(acc);
  const uint32_t lane = lane_id();
  bk = 0;
  bd = 0;
#pragma unroll 2
  for (int j = 0; j < (1 << S) / 256; ++j) {
    const float4 f = a4[j * 64 + lane];
    const float fe[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint32_t k = entry_key(fe[c], 4 * j + c, lane, lim);
      if (k > bk) {
        bk = k;
        bd = entry_doc(4 * j + c, lane);
      }
    }
  }
}

// SAMPLE / ALL tiles: the m best keys of the tile, best first, into out[0..m),
// then the accumulators are cleared.  A round takes the wave's best key, then
// the smallest doc among the lanes holding it; the winner marks that entry
// taken (score bits 0xFFFFFFFF: key 0) and rescans its entries.
template <int S>
__device__ __forceinline__ void select_top_lds(float* acc, int64_t tile, int64_t n_docs, int m,
                                               uint64_t* __restrict__ out) {
  const uint32_t lane = lane_id();
  const int64_t base = tile << S;
  const int lim = (int)min<int64_t>(1 << S, n_docs - base);
  uint32_t bk, bd;
  lane_best<S>(acc, lim, bk, bd);
  for (int r = 0; r < m; ++r) {
    const uint32_t wm = wave_max_u32(bk);
    if (wm == 0) {  // no valid entry left (tile smaller than m)
      if (lane == 0) out[r] = 0;
      continue;
    }
    const uint32_t doc = 0xFFFFFFFFu - wave_max_u32(bk == wm ? 0xFFFFFFFFu - bd : 0u);
    if (lane == ((doc >> 2) & 63u)) {
      out[r] = ((uint64_t)wm << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + doc));
      acc[doc] = __uint_as_float(0xFFFFFFFFu);
      lane_best<S>(acc, lim, bk, bd);
    }
  }
  zero_acc<S>(acc);
}

// REST tiles: every key > theta is appended to the query's list (one atomic
// per wave and chunk that has any), and the accumulators are cleared.  A list
// that overflows its capacity C only counts: the merge sends that query to the
// exact fallback stage.  The test runs on the fp32 sums (one compare per
// entry, after a max early-out); only an entry equal to theta's score compares
// doc ids.  Accumulators are never -0.0 (a sum that starts at +0.0 cannot
// produce it); docs past n_docs are masked.
template <int S>
__device__ __forceinline__ void emit_rest(float* acc, int64_t tile, int64_t n_docs, uint64_t theta,
                                          uint64_t* __restrict__ list, int32_t* __restrict__ cnt,
                                          int32_t C) {
  constexpr int D = 1 << S;
  float4* a4 = reinterpret_cast<float4*>(acc);
  const uint32_t lane = lane_id();
  const float th = key_score((uint32_t)(theta >> 32));
  const int64_t base = tile << S;
  // tile-local bounds, clamped to [-1, D]: docs >= lim are past n_docs, ties
  // pass for docs < tie
  const int lim = (int)max<int64_t>(-1, min<int64_t>(D, n_docs - base));
  const int tie = (int)max<int64_t>(
      -1, min<int64_t>(D, (int64_t)(0xFFFFFFFFu - (uint32_t)theta) - base + 1));
#pragma unroll 1
  for (int j0 = 0; j0 < D / 256; j0 += 2) {  // not unrolled: 8 entries live at a time
    const float4 f0 = a4[j0 * 64 + lane], f1 = a4[(j0 + 1) * 64 + lane];
    a4[j0 * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    a4[(j0 + 1) * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
    const float fe[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
    const float mx = fmaxf(fmaxf(fmaxf(fe[0], fe[1]), fmaxf(fe[2], fe[3])),
                           fmaxf(fmaxf(fe[4], fe[5]), fmaxf(fe[6], fe[7])));
    int c = 0;
    if (!(mx < th && lim == D)) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int d = (int)entry_doc(4 * j0 + e, lane);
        c += (d < lim) & ((fe[e] > th) | ((fe[e] == th) & (d < tie)));
      }
    }
    if (__ballot(c > 0) == 0) continue;  // common: nothing of this chunk passes
    const uint32_t incl = wave_incl_scan((uint32_t)c);
    int pos = 0;
    if (lane == 63) pos = atomicAdd(cnt, (int)incl);
    pos = __shfl(pos, 63, 64) + (int)incl - c;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int d = (int)entry_doc(4 * j0 + e, lane);
      const bool pass = (d < lim) & ((fe[e] > th) | ((fe[e] == th) & (d < tie)));
      if (pass) {
        if (pos < C)
          list[pos] = ((uint64_t)score_key(fe[e]) << 32) |
                      (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + d));
        ++pos;
      }
    }
  }
}

// Tiles of a phase: SAMPLE visits the sample tiles (sample_tile), ALL and
// REST every tile.
template <int PH>
__device__ __forceinline__ int64_t tile_of(int64_t ti, int P, int G) {
  return PH == kSample ? sample_tile(ti, P, G) : ti;
}
template <int PH>
__device__ __forceinline__ int32_t tile_of32(uint32_t ti, uint32_t P, uint32_t G) {
  // G (1 or kSampleGroup) is a power of two: no integer division
  return (int32_t)(PH == kSample ? ((ti & ~(G - 1u)) * P) | (ti & (G - 1u)) : ti);
}


// ---------------------------------------------------------------------------
// Software-pipelined pieces of the scatter phase (score_pipe_kernel).  An
// item's dependent loads — query terms -> (indptr, rel) -> postings — are
// issued three, two and one items ahead of its adds, so the latency of each
// level hides behind the work of the items in between.  Every stage issues a
// fixed number of loads, none under a branch (lanes with nothing to load read
// a valid dummy address), so the compiler's vmcnt waits stay counted instead
// of draining the queue.
// ---------------------------------------------------------------------------
struct Desc {  // lane s < T: raw segment bounds of query term s
  int64_t ip;
  uint32_t r0, r1;
  bool ok;
};

__device__ __forceinline__ Desc load_desc(const IndexArgs& a, int32_t term, int64_t tile) {
  Desc d;
  d.ok = term >= 0 && term < a.V;  // negative ids are padding (bm25_native.py:151)
  const int64_t t = d.ok ? term : 0;
  d.ip = a.indptr[t];
  segment(a, t, tile, d.r0, d.r1);
  return d;
}

// Inclusive prefix sum inside 16-lane rows (DPP row_shr; enough for T <= 16
// because lanes >= T hold 0).
__device__ __forceinline__ uint32_t scan16(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
  return x;
}

// An item's posting rows: each query term's segment is cut into rows of 64
// postings (one per lane), so a row belongs to one term and needs no term
// mask.  Lane j of the table describes row j0 + j of the item.
// (Rows aligned to 64-posting boundaries touch 3 cache lines instead of ~5 —
// 271 M vs 307 M L1->L2 requests per config-3 REST pass — but add ~8 % rows
// and more items past kJ rows: 5.64 vs 4.91 ms.)
struct Rows {
  int64_t base;    // posting index of the row's first posting (0 past the end)
  uint32_t cnt;    // postings in the row (0: past the item's rows)
  uint32_t term;   // the row's query term (T past the end)
  uint32_t nrows;  // rows of the item (uniform)
};

__device__ __forceinline__ Rows make_rows(const Desc& d, int T, uint32_t j0) {
  const uint32_t lane = lane_id();
  const uint32_t len = ((int)lane < T && d.ok) ? d.r1 - d.r0 : 0u;
  const int64_t beg = d.ip + (int64_t)d.r0;
  const uint32_t nr = (len + 63u) >> 6;
  const uint32_t rincl = T <= 16 ? scan16(nr) : wave_incl_scan(nr);
  Rows r;
  r.nrows = lane_u32(rincl, T - 1);
  const uint32_t j = j0 + lane;  // the row this lane describes
  // its term s = #{s < T : rincl[s] <= j}, by binary lifting over ds_bpermute
  int pos = 0;
#pragma unroll
  for (int step = 64; step >= 1; step >>= 1) {
    if (step > T) continue;  // uniform
    const int c = pos + step;
    const uint32_t x = (uint32_t)__shfl((int)rincl, min(c, T) - 1, 64);
    if (c <= T && x <= j) pos = c;
  }
  const uint32_t st = (uint32_t)__shfl((int)(rincl - nr), pos, 64);
  const uint32_t l = (uint32_t)__shfl((int)len, pos, 64);
  const uint32_t blo = (uint32_t)__shfl((int)(uint32_t)beg, pos, 64);
  const uint32_t bhi = (uint32_t)__shfl((int)(uint32_t)((uint64_t)beg >> 32), pos, 64);
  const uint32_t k = j - st;  // row index inside its term
  const bool in = j < r.nrows;
  r.base = in ? (int64_t)(((uint64_t)bhi << 32) | blo) + 64 * (int64_t)k : 0;
  r.cnt = in ? min(64u, l - 64u * k) : 0u;
  r.term = in ? (uint32_t)pos : (uint32_t)T;
  return r;
}

// Buffer descriptors over the whole posting arrays (built once per kernel
// from kernel arguments): a row's loads are then one scalar offset (its base)
// plus the constant lane offset, with no per-lane address arithmetic.  Needs
// (nnz + pad) * 4 < 2^32 bytes (use_pipe checks it; larger indices take the
// plain kernel).
struct PostingRsrc {
  __amdgpu_buffer_rsrc_t ldoc, val;
};

__device__ __forceinline__ PostingRsrc posting_rsrc(const IndexArgs& a) {
  PostingRsrc r;
  // num_records = the arrays' exact byte sizes
  const int np = (int)(a.nnz + kPostingPad);
  r.ldoc = __builtin_amdgcn_make_buffer_rsrc((void*)a.ldoc, 0, (int)((uint32_t)np * 2u), 0x00020000);
  r.val = __builtin_amdgcn_make_buffer_rsrc((void*)a.val, 0, (int)((uint32_t)np * 4u), 0x00020000);
  return r;
}

// Loads of table rows [j0, j0 + kJ): slot + score per lane.  Lanes past a
// row's postings read the next postings (or the zeroed pad after the last
// one) and are masked by add_rows.  Every load is issued, so
// the vmcnt waits stay counted.
// (Giving the masked lanes an out-of-range buffer offset instead — no fetch —
// made the config-3 score pass slower, 5.05 vs 4.77 ms, round 1.)
template <int DIAG>
__device__ __forceinline__ void issue_rows(const PostingRsrc& pr, const Rows& R, int j0,
                                           uint32_t (&ld)[kJ], float (&v)[kJ]) {
  const uint32_t lane = lane_id();
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    const uint32_t base = lane_u32((uint32_t)R.base, j0 + j);
    ld[j] = __builtin_amdgcn_raw_buffer_load_b16(pr.ldoc, (int)(lane * 2u), (int)(base * 2u), 0);
    v[j] = __uint_as_float(
        __builtin_amdgcn_raw_buffer_load_b32(pr.val, (int)(lane * 4u), (int)(base * 4u), 0));
  }
}

// Rows of a block processed: the first 4 or all kJ (a uniform choice from the
// block's row count n); rows past n in the processed range are all-trash.
__device__ __forceinline__ int rows_done(uint32_t n) { return n == 0 ? 0 : (n <= kJ / 2 ? kJ / 2 : kJ); }

// Read-add-write of NR loaded rows, in order.  Lanes past a row's postings
// are redirected to the lane's own trash slot (acc[2^S + lane], always 0) with
// a zero score, so every LDS access runs unmasked (no exec-mask branches; the
// compiler keeps its lgkmcnt waits counted); the redirected slots are written
// back into ld for the sparse emission.  Each row is read, added and written
// back before the next row of ANOTHER term is read — the LDS executes a
// wave's instructions in order, so each doc's adds stay in query-term order
// (scipy csc_matvec's sequence) — while the next row of the SAME term (distinct
// docs) is read one row ahead.  (An LDS float atomic per row, ds_add_f32, ran
// the config-3 score pass 4.7x slower: 24.8 vs 5.3 ms.)
template <int S, int NR>
__device__ __forceinline__ void rmw_rows(float* acc, const Rows& R, int j0, uint32_t (&ld)[kJ],
                                         float (&v)[kJ], float th, uint64_t& hit) {
  const uint32_t lane = lane_id();
  const uint32_t trash = (1u << S) + lane;
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const bool m = lane < lane_u32(R.cnt, j0 + j);
    ld[j] = m ? ld[j] : trash;
    v[j] = m ? v[j] : 0.f;
  }
  // bit j of bm: row j0 + j starts a new term
  const uint32_t tprev = (uint32_t)__shfl_up((int)R.term, 1, 64);
  const uint32_t bm = (uint32_t)(__ballot(R.term != tprev) >> j0);
  float x[NR];
  x[0] = acc[ld[0]];
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const bool same = j + 1 < NR && !((bm >> (j + 1)) & 1u);
    if (same) x[j + 1] = acc[ld[j + 1]];
    const float y = x[j] + v[j];
    acc[ld[j]] = y;
    hit |= __ballot(y >= th);  // th = NaN: never
    if (j + 1 < NR && !same) x[j + 1] = acc[ld[j + 1]];
  }
}

//
// hit collects the lanes whose new running sum reached th (the REST threshold
// score, NaN otherwise): with non-negative values a doc's running sums only
// grow, so an item whose hit stays 0 holds no doc with a final sum >= th.
template <int S, int DIAG>
__device__ __forceinline__ void add_rows(float* acc, const Rows& R, int j0, uint32_t (&ld)[kJ],
                                         float (&v)[kJ], uint32_t n, float th, uint64_t& hit) {
  if (DIAG & 1) {  // ablation: consume the loads, no adds
#pragma unroll
    for (int j = 0; j < kJ; ++j) asm volatile("" ::"v"(ld[j]), "v"(v[j]));
    return;
  }
  const int nr = rows_done(n);
  if (nr == kJ)
    rmw_rows<S, kJ>(acc, R, j0, ld, v, th, hit);
  else if (nr > 0)
    rmw_rows<S, kJ / 2>(acc, R, j0, ld, v, th, hit);
}

// The final sums of an item's processed rows (add_rows' ranges of the D and
// X blocks, nr rows in all), each read once and cleared; x = 0 elsewhere.
__device__ __forceinline__ void read_clear(float* acc, const uint32_t (&l0)[kJ],
                                           const uint32_t (&l1)[kJ], uint32_t nr,
                                           float (&x)[2 * kJ]) {
  const uint32_t n0 = min(nr, (uint32_t)kJ), n1 = nr > (uint32_t)kJ ? nr - kJ : 0u;
  const int r0 = rows_done(n0), r1 = rows_done(n1);
#pragma unroll
  for (int j = 0; j < 2 * kJ; ++j) x[j] = 0.f;
#pragma unroll
  for (int j = 0; j < kJ; ++j) {
    if (r0 > 0 && (j < kJ / 2 || r0 == kJ)) {
      x[j] = acc[l0[j]];
      acc[l0[j]] = 0.f;
    }
  }
  if (r1 > 0) {
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      if (j < kJ / 2 || r1 == kJ) {
        x[kJ + j] = acc[l1[j]];
        acc[l1[j]] = 0.f;
      }
    }
  }
}

// Clears the processed rows' slots (read_clear without the reads).
__device__ __forceinline__ void clear_rows(float* acc, const uint32_t (&l0)[kJ],
                                           const uint32_t (&l1)[kJ], uint32_t nr) {
  const uint32_t n0 = min(nr, (uint32_t)kJ), n1 = nr > (uint32_t)kJ ? nr - kJ : 0u;
  const int r0 = rows_done(n0), r1 = rows_done(n1);
#pragma unroll
  for (int j = 0; j < kJ; ++j)
    if (r0 > 0 && (j < kJ / 2 || r0 == kJ)) acc[l0[j]] = 0.f;
  if (r1 > 0) {
#pragma unroll
    for (int j = 0; j < kJ; ++j)
      if (j < kJ / 2 || r1 == kJ) acc[l1[j]] = 0.f;
  }
}

// REST emission from the item's own postings (items of at most 2 kJ rows,
// whose slots are still in registers): each touched doc's final sum is read
// once — the first read of a doc clears it, so a doc seen again under a later
// term reads 0 — and passes iff its key beats theta.  Exact when theta's
// score is > 0: untouched docs (sum 0) and cleared re-reads can never pass,
// and every touched doc is read after its last add.  The same reads return
// the accumulator to all zeros for the next item.  Slots are add_rows'
// (masked lanes hold their trash slot, which reads 0).
__device__ __forceinline__ void emit_sparse(float* acc, const uint32_t (&l0)[kJ],
                                            const uint32_t (&l1)[kJ], uint32_t nr, int64_t tile,
                                            int S, uint64_t theta, uint64_t* __restrict__ list,
                                            int32_t* __restrict__ cnt, int32_t C) {
  const uint32_t lane = lane_id();
  float x[2 * kJ];
  read_clear(acc, l0, l1, nr, x);
  const float th = key_score((uint32_t)(theta >> 32));
  const int64_t base = tile << S;
  // ties pass for tile-local docs < tie (clamped to [-1, 2^S])
  const int tie = (int)max<int64_t>(
      -1, min<int64_t>(1 << S, (int64_t)(0xFFFFFFFFu - (uint32_t)theta) - base + 1));
  uint32_t pm = 0;
#pragma unroll
  for (int j = 0; j < 2 * kJ; ++j) {
    const int l = (int)(j < kJ ? l0[j] : l1[j - kJ]);
    pm |= (uint32_t)((x[j] > th) | ((x[j] == th) & (l < tie))) << j;
  }
  if (__ballot(pm != 0) == 0) return;  // common: nothing of this item passes
  const int c = __popc(pm);
  const uint32_t incl = wave_incl_scan((uint32_t)c);
  int pos = 0;
  if (lane == 63) pos = atomicAdd(cnt, (int)incl);
  pos = __shfl(pos, 63, 64) + (int)incl - c;
#pragma unroll
  for (int j = 0; j < 2 * kJ; ++j) {
    if ((pm >> j) & 1u) {
      const uint32_t l = j < kJ ? l0[j] : l1[j - kJ];
      if (pos < C)
        list[pos] = ((uint64_t)score_key(x[j]) << 32) |
                    (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + l));
      ++pos;
    }
  }
}

// Item distribution of the pipelined kernel.  An XCD's items (one contiguous
// range of the tile-major item order per XCD) are handed out kClaimCH at a
// time by kClaimM counters per XCD (counter c serves chunks c, c + kClaimM,
// ...; each on a 256-B line of its own), so at any moment the XCD's waves work
// on a window of about (waves x kClaimCH) consecutive items: a few tiles, whose
// posting segments stay in the XCD's L2 across the queries.  A static stride
// lets waves drift apart (items differ in cost) until the window spans far more
// tiles than L2 holds.
// (kClaimCH, kClaimM, kCtrStride: bm25mi_internal.h)

// SAMPLE keys of an item: the best key of each of M equal doc slices of the
// tile (M distinct real documents; key 0 for a slice without one).  Any M
// distinct real documents' keys serve theta (a lower bound of the k-th key),
// and slice maxima cost one pass instead of M extraction rounds.
//
// Sparse form (items of at most 2 kJ rows): the touched docs with a positive
// sum, read and cleared as in emit_sparse.
template <int M>
__device__ __forceinline__ void best_sparse(float* acc, const uint32_t (&l0)[kJ],
                                            const uint32_t (&l1)[kJ], uint32_t nr, int64_t tile,
                                            int S, uint32_t idoff, uint64_t* __restrict__ out) {
  float x[2 * kJ];
  read_clear(acc, l0, l1, nr, x);
  const int sh = S - (M == 1 ? 0 : (M == 2 ? 1 : 2));  // slice of tile-local doc l: l >> sh
  uint32_t bk[M], bd[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    bk[i] = 0;
    bd[i] = 0xFFFFFFFFu;
  }
#pragma unroll
  for (int j = 0; j < 2 * kJ; ++j) {
    const uint32_t l = j < kJ ? l0[j] : l1[j - kJ];
    const uint32_t key = x[j] > 0.f ? score_key(x[j]) : 0u;
    const uint32_t sl = M == 1 ? 0u : (l >> sh);
#pragma unroll
    for (int i = 0; i < M; ++i) {
      const bool better = sl == (uint32_t)i && (key > bk[i] || (key == bk[i] && key != 0u && l < bd[i]));
      bd[i] = better ? l : bd[i];
      bk[i] = better ? key : bk[i];
    }
  }
  const uint32_t base = (uint32_t)(tile << S) + idoff;  // global doc ids (theta_wave_kernel)
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const uint32_t wm = wave_max_u32(bk[i]);
    uint64_t key = 0ull;
    if (wm != 0) {
      const uint32_t doc = 0xFFFFFFFFu - wave_max_u32(bk[i] == wm ? 0xFFFFFFFFu - bd[i] : 0u);
      key = ((uint64_t)wm << 32) | (uint64_t)(0xFFFFFFFFu - (base + doc));
    }
    if (lane_id() == 0) out[i] = key;
  }
}

// Dense form (heavier items): every accumulator of the tile (docs past n_docs
// excluded), then the accumulators are cleared.  Lane entries are in doc
// order inside each lane (entry_doc), so a slice is a contiguous run of them.
// POS: only positive sums are keyed (a tile without one reports key 0), as the
// touched-slot form.
template <int S, int M, bool POS = false>
__device__ __forceinline__ void best_dense(float* acc, int64_t tile, int64_t n_docs,
                                           uint32_t idoff, uint64_t* __restrict__ out) {
  constexpr int E = (1 << S) / 64;  // entries per lane
  const float4* a4 = reinterpret_cast<const float4*>(acc);
  const uint32_t lane = lane_id();
  const int64_t base = tile << S;
  const int lim = (int)min<int64_t>(1 << S, n_docs - base);
  uint32_t bk[M], bd[M];
#pragma unroll
  for (int i = 0; i < M; ++i) {
    bk[i] = 0;
    bd[i] = 0;
  }
  constexpr int per = E / 4 / M;  // float4 groups per slice
#pragma unroll
  for (int i = 0; i < M; ++i) {
#pragma unroll 2
    for (int jj = 0; jj < per; ++jj) {  // not unrolled: few accumulators live at a time
      const int j = i * per + jj;
      const float4 f = a4[j * 64 + lane];
      const float fe[4] = {f.x, f.y, f.z, f.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const uint32_t key =
            (POS && !(fe[c] > 0.f)) ? 0u : entry_key(fe[c], 4 * j + c, lane, lim);
        if (key > bk[i]) {
          bk[i] = key;
          bd[i] = entry_doc(4 * j + c, lane);
        }
      }
    }
  }
  zero_acc<S>(acc);
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const uint32_t wm = wave_max_u32(bk[i]);
    uint64_t key = 0ull;
    if (wm != 0) {
      const uint32_t doc = 0xFFFFFFFFu - wave_max_u32(bk[i] == wm ? 0xFFFFFFFFu - bd[i] : 0u);
      key = ((uint64_t)wm << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + doc) - idoff);
    }
    if (lane_id() == 0) out[i] = key;
  }
}

// One key per tile, positive sums only (the flat kernel's SAMPLE epilogue):
// the tile's best score by a float max over each lane's entries (sums >= 0
// compare as their bit patterns), then the smallest doc holding it from a
// second read; the accumulators are cleared.  Same key as best_dense<S, 1,
// true>, about half its VALU work.
template <int S>
__device__ __forceinline__ void best1_pos(float* acc, int64_t tile, uint32_t idoff,
                                          uint64_t* __restrict__ out) {
  constexpr int E4 = (1 << S) / 256;  // float4 groups per lane
  float4* a4 = reinterpret_cast<float4*>(acc);
  const uint32_t lane = lane_id();
  float m = 0.f;
#pragma unroll
  for (int j = 0; j < E4; ++j) {
    const float4 f = a4[j * 64 + lane];
    m = fmaxf(m, fmaxf(fmaxf(f.x, f.y), fmaxf(f.z, f.w)));
  }
  const uint32_t wm = wave_max_u32(__float_as_uint(m));
  uint64_t key = 0ull;
  if (wm != 0u) {
    const float fm = __uint_as_float(wm);
    uint32_t bd = 0xFFFFFFFFu;
#pragma unroll
    for (int j = E4 - 1; j >= 0; --j) {  // last match written = smallest doc
      const float4 f = a4[j * 64 + lane];
      bd = f.w == fm ? entry_doc(4 * j + 3, lane) : bd;
      bd = f.z == fm ? entry_doc(4 * j + 2, lane) : bd;
      bd = f.y == fm ? entry_doc(4 * j + 1, lane) : bd;
      bd = f.x == fm ? entry_doc(4 * j + 0, lane) : bd;
    }
    const uint32_t doc = 0xFFFFFFFFu - wave_max_u32(0xFFFFFFFFu - bd);
    key = ((uint64_t)score_key(fm) << 32) |
          (uint64_t)(0xFFFFFFFFu - (uint32_t)((tile << S) + doc) - idoff);
  }
  zero_acc<S>(acc);
  if (lane == 0) *out = key;
}

// Item of the pipelined kernel: XCD-relative ordinal rit (end = its chunk's
// end), phase tile ti = the tib-th tile of a band of bw tiles, query qi, and
// the tile it scores.
struct Cursor {
  int32_t rit, end, ti, qi, tile, tib, bw;
};

// ---------------------------------------------------------------------------
// Persistent score kernel: kWaves independent waves per workgroup, each with a
// private 2^S-float LDS accumulator.  The phase's items are tile-major
// (item = ti * nq + qi) and split into 8 contiguous ranges, one per XCD
// (workgroups are dealt round-robin over the XCDs, blockIdx % 8): an XCD's
// waves walk their range together, all queries of a tile back to back, so
// the tile's posting segments stay in that XCD's L2.
// ---------------------------------------------------------------------------
template <int S, int PH>
__global__ __launch_bounds__(64 * kWaves) void score_wave_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, Stage sg,
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand, uint64_t* __restrict__ list,
    int32_t* __restrict__ list_cnt, int32_t C) {
  constexpr int D = 1 << S;
  __shared__ __attribute__((aligned(16))) float acc_all[kWaves * D];
  const int wave = uniform((int)(threadIdx.x >> 6));
  float* acc = acc_all + wave * D;
  const int64_t nq = sg.nq_dev ? (int64_t)*sg.nq_dev : (int64_t)sg.nq_host;
  const int P = sg.P;
  const int64_t nt = PH == kSample ? sample_count(a.ntiles, P, sg.G) : a.ntiles;
  const int64_t nitems = nt * nq;
  const int64_t per = (nitems + 7) >> 3;
  const int64_t grp = blockIdx.x & 7;
  const int64_t lo = grp * per;
  const int64_t hi = min(nitems, lo + per);
  const int64_t stride = (int64_t)(gridDim.x >> 3) * kWaves;
  int64_t it = lo + (int64_t)(blockIdx.x >> 3) * kWaves + wave;
  if (it >= hi) return;  // wave-uniform; no barriers in this kernel
  zero_acc<S>(acc);
  for (; it < hi; it += stride) {
    const int64_t ti = it / nq;
    const int64_t qi = it - ti * nq;
    const int64_t q = sg.qmap ? (int64_t)sg.qmap[qi] : qi;
    const int64_t tile = tile_of<PH>(ti, P, sg.G);
    add_item<S>(a, tile, queries + q * T, T, acc);
    float fv[D / 64];
    take_entries<S>(acc, fv);
    if (PH == kRest)
      emit_above<S>(fv, tile, a.n_docs, theta[qi], list + qi * C, list_cnt + qi, C);
    else
      select_top<S>(fv, tile, a.n_docs, PH == kSample ? sg.M : kTileM,
                    PH == kSample ? (uint32_t)a.doc_offset : 0u,
                    sg.cand_out + qi * sg.cstride + ti * (PH == kSample ? sg.M : kTileM));
  }
}

// ---------------------------------------------------------------------------
// Pipelined persistent score kernel (1 <= T <= 64): same items and the same
// per-document add order as score_wave_kernel.  Item order: band-major — the
// phase's tiles are cut into bands of `band` consecutive tiles, and inside a
// band the items run query by query, each query over the band's tiles — so a
// claimed chunk is one query over consecutive tiles: its terms' segments of
// neighbouring tiles share cache lines (a light term has a few postings per
// tile), and the XCD's waves read the same band of every popular term.
// (Tile-major order, all queries of a tile back to back, re-fetched each
// light term's lines from beyond L2 for every tile: 17 GB per config-3 REST
// launch against 1.9 GB of batch-distinct postings.)  Iteration n issues
//   (1) the query terms of item n+3,
//   (2) the (indptr, rel) segment bounds of item n+2,
//   (3) item n's second block of kJ posting rows and item n+1's first block,
// and then (4) adding item n's rows (a heavy item's further rows are loaded in
// place) and selecting / emitting its candidates.
// ---------------------------------------------------------------------------
template <int S, int PH, bool QMAP, int DIAG, int SM>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(4, 4))) void score_pipe_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, int32_t P, int32_t nq_host,
    const int32_t* __restrict__ nq_dev, const int32_t* __restrict__ qmap,
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand, uint64_t* __restrict__ list,
    int32_t* __restrict__ list_cnt, int32_t C, int32_t* __restrict__ wctr, int32_t claim_ch,
    int32_t claim_m, int64_t cstride, int32_t G, int32_t band, uint64_t* __restrict__ stamps) {
  constexpr int D = 1 << S;
  constexpr int DP = D + 64;  // accumulators + one trash slot per lane (add_rows)
  __shared__ __attribute__((aligned(16))) float acc_all[kWaves * DP];
  const int wave = uniform((int)(threadIdx.x >> 6));
  float* acc = acc_all + wave * DP;
  // diagnostic build only (DIAG & 32): cycles per loop segment
  uint64_t seg[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t_last = 0;
#define BM25_STAMP(k)                                                           \
  if (DIAG & 32) {                                                              \
    __builtin_amdgcn_sched_barrier(0);                                          \
    uint64_t t_;                                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                          \
    seg[k] += t_ - t_last;                                                      \
    t_last = t_;                                                                \
  }
  BM25_STAMP(7);
  const int32_t nq = QMAP ? *nq_dev : nq_host;
  const int32_t nt = PH == kSample ? (int32_t)sample_count(a.ntiles, P, G) : (int32_t)a.ntiles;
  const int64_t nitems = (int64_t)nt * nq;
  const int64_t per = (nitems + 7) >> 3;
  const int grp = (int)(blockIdx.x & 7);
  const uint32_t lo = (uint32_t)(grp * per);
  const int32_t ngi = (int32_t)max<int64_t>(0, min<int64_t>(nitems, lo + per) - lo);
  if (ngi == 0) return;  // wave-uniform; no barriers in this kernel
  const int32_t cm = (int32_t)((blockIdx.x >> 3) * kWaves + wave) % claim_m;
  int32_t* ctr = wctr + (grp * kClaimM + cm) * kCtrStride;
  const int tl = min(lane_id(), T - 1);
  const PostingRsrc pr = posting_rsrc(a);

  // Claims: lane 0 holds the ordinal of the wave's next chunk on its counter,
  // claimed one chunk ahead of use.
  auto claim = [&]() -> int32_t {
    int32_t v = 0;
    if (lane_id() == 0) v = atomicAdd(ctr, 1);
    return v;
  };
  int32_t pending = claim();
  // cursor of the next item after c: the next one of c's chunk, else the
  // first of the pending chunk; past the end it stays on c's item with
  // rit = ngi, so every stage keeps loading valid addresses
  const int32_t nfb = nt / band;  // full bands
  const uint32_t full_items = (uint32_t)nfb * (uint32_t)band * (uint32_t)nq;
  auto next = [&](Cursor c) -> Cursor {
    if (c.rit >= ngi) return c;
    if (c.rit + 1 < c.end) {
      ++c.rit;
      if (++c.tib == c.bw) {  // the query's last tile of the band
        c.tib = 0;
        c.ti -= c.bw - 1;
        if (++c.qi == nq) {  // next band
          c.qi = 0;
          c.ti += c.bw;
          c.bw = min(band, nt - c.ti);
        }
      } else {
        ++c.ti;
      }
      c.tile = tile_of32<PH>((uint32_t)c.ti, (uint32_t)P, (uint32_t)G);
      return c;
    }
    const int64_t b = ((int64_t)uniform(pending) * claim_m + cm) * claim_ch;
    if (b >= ngi) {
      c.rit = c.end = ngi;
      return c;
    }
    pending = claim();
    Cursor n;
    n.rit = (int32_t)b;
    n.end = (int32_t)min<int64_t>(ngi, b + claim_ch);
    const uint32_t it = lo + (uint32_t)b;
    uint32_t bb, r, bw;
    if (it < full_items) {
      bb = it / ((uint32_t)band * (uint32_t)nq);
      r = it - bb * (uint32_t)band * (uint32_t)nq;
      bw = (uint32_t)band;
    } else {  // the last, partial band
      bb = (uint32_t)nfb;
      r = it - full_items;
      bw = (uint32_t)(nt - nfb * band);
    }
    n.qi = (int32_t)(r / bw);
    n.tib = (int32_t)(r - (uint32_t)n.qi * bw);
    n.bw = (int32_t)bw;
    n.ti = (int32_t)(bb * (uint32_t)band) + n.tib;
    n.tile = tile_of32<PH>((uint32_t)n.ti, (uint32_t)P, (uint32_t)G);
    return n;
  };
  auto terms_of = [&](const Cursor& c) -> int32_t {
    const int32_t q = QMAP ? qmap[c.qi] : c.qi;
    return queries[(int64_t)q * T + tl];
  };

  Cursor c0;  // a chunk "before" the first one: next() takes the pending claim
  c0.rit = -1;
  c0.end = 0;
  c0.ti = c0.qi = c0.tile = c0.tib = 0;
  c0.bw = 1;
  Cursor cD = next(c0);
  if (cD.rit >= ngi) return;
  zero_acc<S>(acc);
  acc[D + lane_id()] = 0.f;
  Cursor cC = next(cD), cB = next(cC), cA = next(cB);
  // prologue: item 0's first rows, item 1's bounds, item 2's terms
  int32_t tmD = terms_of(cD), tmC = terms_of(cC), tmB = terms_of(cB);
  Desc dC = load_desc(a, tmC, cC.tile);
  Rows rD = make_rows(load_desc(a, tmD, cD.tile), T, 0);
  uint32_t ltD[kJ];
  float vD[kJ];
  issue_rows<DIAG>(pr, rD, 0, ltD, vD);
  uint64_t thD = PH == kRest ? theta[cD.qi] : 0ull;
  int32_t nitem = 0;
  BM25_STAMP(7);

  while (cD.rit < ngi) {
    ++nitem;
    // (1) item n's second row block, (2) terms of item n+3, (3) bounds of
    // item n+2, (4) item n+1's first rows: all issued before item n's adds
    const uint32_t nrD = rD.nrows;
    uint32_t ltX[kJ];
    float vX[kJ];
    if (nrD > kJ) issue_rows<DIAG>(pr, rD, kJ, ltX, vX);  // (unconditional: 4.98 vs 4.77 ms)
    const int32_t tmA = terms_of(cA);
    const Desc dB = load_desc(a, tmB, cB.tile);
    BM25_STAMP(0);
    const Rows rC = make_rows(dC, T, 0);
    uint32_t ltC[kJ];
    float vC[kJ];
    issue_rows<DIAG>(pr, rC, 0, ltC, vC);
    const uint64_t thC = PH == kRest ? theta[cC.qi] : 0ull;
    BM25_STAMP(1);
    // (5) item n: adds in row order, then selection
    const int64_t tile = cD.tile;
    // REST over a non-negative index: candidates are flagged while adding
    const bool flagged = PH == kRest && a.nonneg && (uint32_t)(thD >> 32) > score_key(0.f);
    const float thf = flagged ? key_score((uint32_t)(thD >> 32)) : __builtin_nanf("");
    uint64_t hit = 0;
    add_rows<S, DIAG>(acc, rD, 0, ltD, vD, min(nrD, (uint32_t)kJ), thf, hit);
    if (nrD > kJ) add_rows<S, DIAG>(acc, rD, kJ, ltX, vX, min(nrD - kJ, (uint32_t)kJ), thf, hit);
    if (nrD > 2 * kJ) {  // heavy item: the remaining rows, block j + kJ issued before block j's adds
      const Desc dD = load_desc(a, tmD, tile);
      Rows t = rD;
      if ((2 * kJ & 63) == 0) t = make_rows(dD, T, 2 * kJ);
      uint32_t ltY[kJ];
      float vY[kJ];
      issue_rows<DIAG>(pr, t, (2 * kJ) & 63, ltY, vY);
      for (uint32_t j = 2 * kJ; j < nrD; j += kJ) {
        const uint32_t jn = j + kJ;
        Rows tn = t;
        uint32_t ltZ[kJ];
        float vZ[kJ];
        if (jn < nrD) {
          if ((jn & 63) == 0) tn = make_rows(dD, T, jn);
          issue_rows<DIAG>(pr, tn, (int)(jn & 63), ltZ, vZ);
        }
        add_rows<S, DIAG>(acc, t, (int)(j & 63), ltY, vY, min(nrD - j, (uint32_t)kJ), thf, hit);
        t = tn;
#pragma unroll
        for (int i = 0; i < kJ; ++i) {
          ltY[i] = ltZ[i];
          vY[i] = vZ[i];
        }
      }
    }
    BM25_STAMP(2);
    BM25_STAMP(3);
    if (DIAG & 4) {  // ablation: no selection
      zero_acc<S>(acc);
    } else if (flagged && hit == 0) {  // no doc of this item reaches theta
      if (nrD <= 2 * kJ)
        clear_rows(acc, ltD, ltX, nrD);
      else
        zero_acc<S>(acc);
    } else if (PH == kRest && nrD <= 2 * kJ && (uint32_t)(thD >> 32) > score_key(0.f)) {
      emit_sparse(acc, ltD, ltX, nrD, tile, S, thD, list + (int64_t)cD.qi * C,
                  list_cnt + cD.qi, C);
    } else if (PH == kRest) {
      emit_rest<S>(acc, tile, a.n_docs, thD, list + (int64_t)cD.qi * C, list_cnt + cD.qi, C);
    } else if (PH == kSample) {
      uint64_t* out = cand + (int64_t)cD.qi * cstride + (int64_t)cD.ti * SM;
      if (nrD <= 2 * kJ)
        best_sparse<SM>(acc, ltD, ltX, nrD, tile, S, (uint32_t)a.doc_offset, out);
      else
        best_dense<S, SM>(acc, tile, a.n_docs, (uint32_t)a.doc_offset, out);
    } else {
      select_top_lds<S>(acc, tile, a.n_docs, kTileM,
                        cand + (int64_t)cD.qi * cstride + (int64_t)cD.ti * kTileM);
    }
    BM25_STAMP(4);
    // rotate the pipeline
    cD = cC;
    cC = cB;
    cB = cA;
    cA = next(cA);
    tmD = tmC;
    tmC = tmB;
    tmB = tmA;
    dC = dB;
    rD = rC;
    thD = thC;
#pragma unroll
    for (int j = 0; j < kJ; ++j) {
      ltD[j] = ltC[j];
      vD[j] = vC[j];
    }
    BM25_STAMP(5);
  }
  if ((DIAG & 32) && lane_id() == 0) {
    uint64_t* o = stamps + ((int64_t)blockIdx.x * kWaves + wave) * 8;
    seg[6] = (uint64_t)nitem;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = seg[k];
  }
#undef BM25_STAMP
}

// ===========================================================================
// Band score kernel (queries of 1..8 terms; SAMPLE and REST phases).
//
// An ITEM is (query, band of up to 8 consecutive phase tiles); a wave scores
// the band's tiles one after another in its private LDS accumulator.
//   * The segment table (indptr + rel of every (tile, term)) is loaded once
//     per item, one item ahead: lane i * 8 + t holds term t's segment in
//     tile i.  (Per-tile items load terms, indptr and a rel pair per tile.)
//   * Postings move in DOUBLE ROWS: lane l holds postings base + 2l and
//     base + 2l + 1 (base even) — one b32 load of two u16 slots and one
//     8-byte load of two f32 scores per 128 postings, half the load
//     instructions of 64-posting rows.
//   * Every tile iteration issues the SAME loads: the next tile's first two
//     blocks of kJ2 double rows (rows past its end read posting 0), so the
//     compiler's vmcnt waits are exact counts; a load issued under a branch
//     and still in flight makes every later wait drain it (LLVM merges the
//     paths pessimistically), which is what exposed the per-tile kernel's
//     second row block.  The next item's first tile is issued during the
//     current item's last tile.
// Per tile the adds follow the query-term order exactly, so every document's
// fp32 sum has the reference's rounding sequence (bm25_native.py:152, scipy
// csc_matvec).
// ===========================================================================
constexpr int kBandT = 8;    // terms served (T <= kBandT)
constexpr int kBandW = BM25_BANDW;  // tiles per band item
#ifndef BM25_BAND_ABL  // dev ablations of the band kernel (timing only, wrong results)
#define BM25_BAND_ABL 0
#endif
#ifndef BM25_HL  // row blocks in flight ahead of the adds in a heavy tile (1 or 2)
#define BM25_HL 1
#endif
#ifndef BM25_KJ2
#define BM25_KJ2 2
#endif
constexpr int kJ2 = BM25_KJ2;  // double rows per streamed block
#ifndef BM25_NB
#define BM25_NB 2
#endif
constexpr int kNB = BM25_NB;   // blocks of the next tile issued one tile ahead

struct BandDesc {  // lane i * 8 + t: term t's segment bounds in tile i (raw)
  uint32_t ip, r0, r1;  // indptr[term] (nnz < 2^30 on this path), rel pair
  uint32_t ok;          // segment present (t < T, i < bw, valid term)
  uint64_t skey;        // REST: best sample key of tile i, ~0: no skip information
};

struct BandCur {  // XCD-relative item ordinal, its chunk end, band, query, band width
  int32_t rit, end, b, q, bw;
};

struct BandTab {  // an item's segment table (lane i * 8 + t) and its threshold
  uint32_t sb, sl;  // segment [sb, sb + sl) of the posting arrays (sl = 0: none)
  uint64_t th;      // REST: theta of the item's query
};

// Row base of the rows past a table's end (issue_rows2).
constexpr uint32_t kNoRow = 0u;

// A tile's double rows: lane j of the table describes row j0 + j.
struct Rows2 {
  uint32_t base;    // even posting index of the row's first posting pair
  uint32_t lo, hi;  // the row's term segment [lo, hi): its valid postings
  uint32_t term;    // query term (T past the end)
  uint32_t nrows;   // rows of the tile (uniform)
};

// Segment of term s (lane s < T): [beg, beg + len), cut into double rows from
// beg & ~1.
__device__ __forceinline__ Rows2 make_rows2(uint32_t beg, uint32_t len, int T, uint32_t j0) {
  const uint32_t lane = lane_id();
  len = (int)lane < T ? len : 0u;
  const uint32_t nr = len == 0 ? 0u : ((beg & 1u) + len + 127u) >> 7;
  const uint32_t rincl = scan16(nr);  // T <= 8: lanes >= T hold 0
  Rows2 r;
  r.nrows = lane_u32(rincl, T - 1);
  const uint32_t j = j0 + lane;
  int pos = 0;
#pragma unroll
  for (int step = 8; step >= 1; step >>= 1) {
    if (step > T) continue;  // uniform
    const int c = pos + step;
    const uint32_t x = (uint32_t)__shfl((int)rincl, min(c, T) - 1, 64);
    if (c <= T && x <= j) pos = c;
  }
  const uint32_t st = (uint32_t)__shfl((int)(rincl - nr), pos, 64);
  const uint32_t b = (uint32_t)__shfl((int)beg, pos, 64);
  const uint32_t l = (uint32_t)__shfl((int)len, pos, 64);
  const bool in = j < r.nrows;
  r.base = in ? (b & ~1u) + 128u * (j - st) : kNoRow;
  r.lo = in ? b : 1u;
  r.hi = in ? b + l : 0u;
  r.term = in ? (uint32_t)pos : (uint32_t)T;
  return r;
}

// Loads of double rows [j0, j0 + kJ2) of a table: slot pair + score pair per
// lane.  Every load is issued (static counts); rows past the table read
// posting 0 (an L1 hit) and are masked later.  (Loading them through a
// descriptor of zero records instead — range-checked, no memory access — ran
// the config-3 score pass slower: 5.12 vs 4.75 ms.)
__device__ __forceinline__ void issue_rows2(const PostingRsrc& pr, const Rows2& R, int j0,
                                            uint32_t (&ld)[kJ2], float (&v0)[kJ2],
                                            float (&v1)[kJ2], bool abl = false) {
  const uint32_t lane = lane_id();
#if BM25_BAND_ABL & 1  // dev ablation: no posting loads (slots = the lane's own pair)
  if (abl) {
#pragma unroll
    for (int j = 0; j < kJ2; ++j) {
      ld[j] = (2u * lane + (uint32_t)j * 128u) | ((2u * lane + 1u + (uint32_t)j * 128u) << 16);
      v0[j] = 1.f;
      v1[j] = 1.f;
    }
    return;
  }
#endif
#pragma unroll
  for (int j = 0; j < kJ2; ++j) {
    const uint32_t base = lane_u32(R.base, j0 + j);
    ld[j] = __builtin_amdgcn_raw_buffer_load_b32(pr.ldoc, (int)(lane * 4u), (int)(base * 2u), 0);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(pr.val, (int)(lane * 8u), (int)(base * 4u), 0);
    v0[j] = __uint_as_float((uint32_t)v[0]);
    v1[j] = __uint_as_float((uint32_t)v[1]);
  }
}

#ifndef BM25_BAND_WAVES
#define BM25_BAND_WAVES 1
#endif
#ifndef BM25_BAND_WPE
#define BM25_BAND_WPE 5
#endif
constexpr int kBandWaves = BM25_BAND_WAVES;  // independent waves per band workgroup

template <int S, int PH, int SM, bool SP>
__global__ __launch_bounds__(64 * kBandWaves) __attribute__((amdgpu_waves_per_eu(BM25_BAND_WPE, BM25_BAND_WPE))) void score_band_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, int32_t P, int32_t G, int32_t nq,
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand, int64_t cstride,
    uint64_t* __restrict__ list, int32_t* __restrict__ list_cnt, int32_t C,
    int32_t* __restrict__ wctr, int32_t claim_ch, int32_t claim_m,
    const uint64_t* __restrict__ skeys, int64_t sstride) {
  constexpr int D = 1 << S;
  constexpr int DP = D + 64;
  __shared__ __attribute__((aligned(16))) float acc_all[kBandWaves * DP];
  const int wave = uniform((int)(threadIdx.x >> 6));
  float* acc = acc_all + wave * DP;
  const uint32_t lane = lane_id();
  const uint32_t trash = (uint32_t)D + lane;  // this lane's always-zero slot
  const int32_t nt = PH == kSample ? (int32_t)sample_count(a.ntiles, P, G) : (int32_t)a.ntiles;
  const int32_t nb = (nt + kBandW - 1) / kBandW;
  const int64_t nitems = (int64_t)nb * nq;
  const int64_t per = (nitems + 7) >> 3;
  const int grp = (int)(blockIdx.x & 7);
  const uint32_t lo = (uint32_t)(grp * per);
  const int32_t ngi = (int32_t)max<int64_t>(0, min<int64_t>(nitems, lo + per) - lo);
  if (ngi == 0) return;  // wave-uniform; no barriers in this kernel
  const int32_t cm = (int32_t)((blockIdx.x >> 3) * kBandWaves + wave) % claim_m;
  int32_t* ctr = wctr + (grp * kClaimM + cm) * kCtrStride;
  const PostingRsrc pr = posting_rsrc(a);
  const uint32_t lt = lane & 7u, li = lane >> 3;  // segment lane: tile li, term lt
  const int64_t nbp = (a.ntiles + 7) >> 3;          // physical bands (sparse seg rows)

  auto claim = [&]() -> int32_t {
    int32_t v = 0;
    if (lane == 0) v = atomicAdd(ctr, 1);
    return v;
  };
  int32_t pending = claim();
  auto next = [&](BandCur c) -> BandCur {  // as score_pipe_kernel's next(), items = bands
    if (c.rit >= ngi) return c;
    if (c.rit + 1 < c.end) {
      ++c.rit;
      if (++c.q == nq) {
        c.q = 0;
        ++c.b;
        c.bw = min(kBandW, nt - c.b * kBandW);
      }
      return c;
    }
    const int64_t bb = ((int64_t)uniform(pending) * claim_m + cm) * claim_ch;
    if (bb >= ngi) {
      c.rit = c.end = ngi;
      return c;
    }
    pending = claim();
    BandCur n;
    n.rit = (int32_t)bb;
    n.end = (int32_t)min<int64_t>(ngi, bb + claim_ch);
    const uint32_t it = lo + (uint32_t)bb;
    n.b = (int32_t)(it / (uint32_t)nq);
    n.q = (int32_t)(it - (uint32_t)n.b * (uint32_t)nq);
    n.bw = min(kBandW, nt - n.b * kBandW);
    return n;
  };
  auto terms_of = [&](const BandCur& c) -> int32_t {
    return queries[(int64_t)c.q * T + (int)min(lt, (uint32_t)(T - 1))];
  };
  // REST: tile li of band b is a sample tile (sample groups of 8 tiles =
  // bands) iff b % P == 0; its best sample key is skeys[q][(b / P) * 8 + li]
  const bool skipping = PH == kRest && skeys != nullptr && G == kBandW;
  auto load_bdesc = [&](const BandCur& c, int32_t tm) -> BandDesc {
    BandDesc d;
    const int32_t term = __shfl(tm, (int)lt, 64);
    const bool ok = (int)lt < T && (int)li < c.bw && term >= 0 && term < a.V;
    const int64_t tt = ok ? term : 0;
    const int64_t tile = ok ? (int64_t)tile_of32<PH>((uint32_t)(c.b * kBandW + li), (uint32_t)P,
                                                      (uint32_t)G)
                            : 0;
    if constexpr (SP) {  // this search's segment table (seg_table_kernel)
      const uint64_t e =
          ok ? a.seg[((int64_t)c.q * nbp + (tile >> 3)) * 64 + lt * 8 + (tile & 7)] : 0ull;
      d.ip = 0u;
      d.r0 = (uint32_t)e;
      d.r1 = (uint32_t)e + (uint32_t)(e >> 32);
    } else {
      const uint32_t* r = a.rel + tt * (a.ntiles + 1) + tile;
      d.ip = (uint32_t)a.indptr[tt];
      d.r0 = r[0];
      d.r1 = r[1];
    }
    d.ok = ok ? 1u : 0u;
    const int64_t si = (int64_t)(c.b / P) * kBandW + min(li, (uint32_t)(c.bw - 1));
    d.skey = skipping ? skeys[(int64_t)c.q * sstride + min<int64_t>(si, sstride - 1)] : ~0ull;
    if (!(skipping && (c.b % P) == 0)) d.skey = ~0ull;
    return d;
  };
  // the item's table; REST: a sample tile whose best key scores below theta
  // holds no key of the list, so its segments are dropped (exact for m = 1
  // samples; only when theta is a positive score — no threshold and the
  // zero-fill case must still see every doc)
  auto make_tab = [&](const BandDesc& d, uint64_t th) -> BandTab {
    BandTab tb;
    const bool th_pos = PH == kRest && (uint32_t)(th >> 32) > score_key(0.f);
    const bool skip = skipping && th_pos && (uint32_t)(d.skey >> 32) < (uint32_t)(th >> 32);
    tb.sb = d.ip + d.r0;
    tb.sl = (d.ok && !skip) ? d.r1 - d.r0 : 0u;
    tb.th = th;
    return tb;
  };
  auto tile_rows = [&](const BandTab& tb, int i, uint32_t j0) -> Rows2 {
    const int src = i * 8 + (int)lt;
    return make_rows2((uint32_t)__shfl((int)tb.sb, src, 64), (uint32_t)__shfl((int)tb.sl, src, 64),
                      T, j0);
  };

  BandCur c0;
  c0.rit = -1;
  c0.end = 0;
  c0.b = c0.q = 0;
  c0.bw = 1;
  BandCur cur = next(c0);
  if (cur.rit >= ngi) return;
  zero_acc<S>(acc);
  acc[D + lane] = 0.f;
  // prologue: the first item's table (one exposed load chain), the next
  // item's descriptors in flight
  BandTab tab = make_tab(load_bdesc(cur, terms_of(cur)), PH == kRest ? theta[cur.q] : 0ull);
  BandCur nx = next(cur);
  BandDesc dN = load_bdesc(nx, terms_of(nx));
  uint64_t thN = PH == kRest ? theta[nx.q] : 0ull;
  BandCur nx2 = next(nx);
  int32_t tmN2 = terms_of(nx2);
  Rows2 rD = tile_rows(tab, 0, 0);
  uint32_t ltD[kNB][kJ2];
  float vD0[kNB][kJ2], vD1[kNB][kJ2];
#pragma unroll
  for (int k = 0; k < kNB; ++k) issue_rows2(pr, rD, k * kJ2, ltD[k], vD0[k], vD1[k], PH == kRest);
  BandCur nx3 = nx2;
  int32_t tmN3 = tmN2;

  while (cur.rit < ngi) {
    BandTab ntab = tab;
    for (int i = 0; i < cur.bw; ++i) {
      const bool last = i + 1 == cur.bw;
      const int64_t ti = (int64_t)cur.b * kBandW + i;  // phase tile (SAMPLE: sample index)
      const int64_t tile = tile_of32<PH>((uint32_t)ti, (uint32_t)P, (uint32_t)G);
      const uint32_t nrD = rD.nrows;
      // ---- on the item's last tile: the next item's table (descriptors
      // loaded one item ago), the descriptors of the one after it and the
      // terms of the one after that (claims are consumed here, where only
      // this tile's old row blocks are in flight)
      if (last) {
        nx3 = next(nx2);
        tmN3 = terms_of(nx3);
        ntab = make_tab(dN, thN);
        dN = load_bdesc(nx2, tmN2);
        thN = PH == kRest ? theta[nx2.q] : 0ull;
      }
      // ---- the next tile's first kNB blocks (of this item or the next)
      Rows2 rC = last ? tile_rows(ntab, 0, 0) : tile_rows(tab, i + 1, 0);
      if (last && nx.rit >= ngi) rC.nrows = 0;
      uint32_t ltC[kNB][kJ2];
      float vC0[kNB][kJ2], vC1[kNB][kJ2];
#pragma unroll
      for (int k = 0; k < kNB; ++k) issue_rows2(pr, rC, k * kJ2, ltC[k], vC0[k], vC1[k], PH == kRest);

      const uint64_t th = tab.th;
      const float thf_raw = key_score((uint32_t)(th >> 32));
      const bool th_pos = PH == kRest && (uint32_t)(th >> 32) > score_key(0.f);
      // REST over a non-negative index: candidates are flagged while adding
      const bool flagged = PH == kRest && a.nonneg && th_pos;
      const float thf = flagged ? thf_raw : __builtin_nanf("");
      uint64_t hit = 0;
      // ---- adds in row order (= query-term order: a term's rows are
      // consecutive); the next row's reads go before this row's writes when
      // both rows are of one term (distinct docs), after them otherwise
      auto block = [&](const Rows2& R, int j0, uint32_t (&ld)[kJ2], float (&v0)[kJ2],
                       float (&v1)[kJ2], uint32_t n) {
        int tm[kJ2];
#pragma unroll
        for (int j = 0; j < kJ2; ++j) {
          tm[j] = (uint32_t)j < n ? (int)lane_u32(R.term, j0 + j) : -1 - j;
          const uint32_t p = lane_u32(R.base, j0 + j) + 2u * lane;
          const uint32_t l0 = lane_u32(R.lo, j0 + j), l1 = lane_u32(R.hi, j0 + j);
          const bool m0 = p >= l0 && p < l1, m1 = p + 1u >= l0 && p + 1u < l1;
          ld[j] = (m0 ? (ld[j] & 0xFFFFu) : trash) | ((m1 ? (ld[j] >> 16) : trash) << 16);
          v0[j] = m0 ? v0[j] : 0.f;
          v1[j] = m1 ? v1[j] : 0.f;
        }
        if (n == 0) return;
#if BM25_BAND_ABL & 2  // dev ablation: no LDS adds (loads consumed by the hit flags)
        if (PH == kRest) {
#pragma unroll
        for (int j = 0; j < kJ2; ++j)
          if ((uint32_t)j < n)
            hit |= __ballot(v0[j] + v1[j] + (float)ld[j] >= 1e30f);
        return;
        }
#endif
        float x0 = acc[ld[0] & 0xFFFFu], x1 = acc[ld[0] >> 16];
#pragma unroll
        for (int j = 0; j < kJ2; ++j) {
          if ((uint32_t)j < n) {
            const bool same = j + 1 < kJ2 && tm[j + 1] == tm[j];
            float n0 = 0.f, n1 = 0.f;
            if (same) {
              n0 = acc[ld[j + 1] & 0xFFFFu];
              n1 = acc[ld[j + 1] >> 16];
            }
            const float y0 = x0 + v0[j], y1 = x1 + v1[j];
            acc[ld[j] & 0xFFFFu] = y0;
            acc[ld[j] >> 16] = y1;
            hit |= __ballot(y0 >= thf) | __ballot(y1 >= thf);
            if (j + 1 < kJ2 && (uint32_t)(j + 1) < n && !same) {
              n0 = acc[ld[j + 1] & 0xFFFFu];
              n1 = acc[ld[j + 1] >> 16];
            }
            x0 = n0;
            x1 = n1;
          }
        }
      };
#pragma unroll
      for (int k = 0; k < kNB; ++k)
        block(rD, k * kJ2, ltD[k], vD0[k], vD1[k],
              nrD > (uint32_t)(k * kJ2) ? min(nrD - k * kJ2, (uint32_t)kJ2) : 0u);

#if BM25_BAND_ABL & 4  // dev ablation: REST emits nothing
      if (PH == kRest) hit = 0;
#endif
      if (nrD > kNB * kJ2) {
        // ---- a heavy tile: the remaining rows, block j + kJ2 always issued
        // before block j's adds (past the end: posting 0); dense selection
        Rows2 t = rD;
        if (((kNB * kJ2) & 63) == 0) t = tile_rows(tab, i, kNB * kJ2);
        uint32_t ltY[kJ2];
        float vY0[kJ2], vY1[kJ2];
        issue_rows2(pr, t, (kNB * kJ2) & 63, ltY, vY0, vY1, PH == kRest);
#if BM25_HL == 2
        // a second block in flight: rows kNB * kJ2 + kJ2 .. (dead past the end)
        Rows2 tw = t;
        {
          const uint32_t jw = kNB * kJ2 + kJ2;
          if (jw < nrD && (jw & 63) == 0) tw = tile_rows(tab, i, jw);
          if (jw >= nrD) {
            tw.base = kNoRow;
            tw.hi = 0u;
          }
        }
        uint32_t ltW[kJ2];
        float vW0[kJ2], vW1[kJ2];
        issue_rows2(pr, tw, (int)((kNB * kJ2 + kJ2) & 63), ltW, vW0, vW1, PH == kRest);
#endif
        for (uint32_t j = kNB * kJ2; j < nrD; j += kJ2) {
          const uint32_t jn = j + BM25_HL * kJ2;
#if BM25_HL == 2
          Rows2 tn = tw;
#else
          Rows2 tn = t;
#endif
          if (jn < nrD && (jn & 63) == 0) tn = tile_rows(tab, i, jn);
          if (jn >= nrD) {  // nothing left: a dead block keeps the load count static
            tn.base = kNoRow;
            tn.hi = 0u;
          }
          uint32_t ltZ[kJ2];
          float vZ0[kJ2], vZ1[kJ2];
          issue_rows2(pr, tn, (int)(jn & 63), ltZ, vZ0, vZ1, PH == kRest);
          block(t, (int)(j & 63), ltY, vY0, vY1, min(nrD - j, (uint32_t)kJ2));
#if BM25_HL == 2
          t = tw;
          tw = tn;
#pragma unroll
          for (int u = 0; u < kJ2; ++u) {
            ltY[u] = ltW[u];
            vY0[u] = vW0[u];
            vY1[u] = vW1[u];
            ltW[u] = ltZ[u];
            vW0[u] = vZ0[u];
            vW1[u] = vZ1[u];
          }
#else
          t = tn;
#pragma unroll
          for (int u = 0; u < kJ2; ++u) {
            ltY[u] = ltZ[u];
            vY0[u] = vZ0[u];
            vY1[u] = vZ1[u];
          }
#endif
        }
        if (flagged && hit == 0)
          zero_acc<S>(acc);
        else if (PH == kRest)
          emit_rest<S>(acc, tile, a.n_docs, th, list + (int64_t)cur.q * C, list_cnt + cur.q, C);
        else
          best_dense<S, SM>(acc, tile, a.n_docs, (uint32_t)a.doc_offset,
                            cand + (int64_t)cur.q * cstride + ti * SM);
      } else {
        // ---- selection / emission from the touched slots (the D blocks'
        // masked slot pairs); the accumulator is left zeroed
        auto for_ops = [&](auto&& f) {
#pragma unroll
          for (int k = 0; k < kNB; ++k)
#pragma unroll
            for (int j = 0; j < kJ2; ++j)
              if ((uint32_t)(k * kJ2 + j) < nrD) {
                f(ltD[k][j] & 0xFFFFu);
                f(ltD[k][j] >> 16);
              }
        };
        auto clear_ops = [&]() { for_ops([&](uint32_t s) { acc[s] = 0.f; }); };
        if (flagged && hit == 0) {  // no doc of this tile reaches theta
          clear_ops();
        } else if (PH == kRest && th_pos && a.nonneg) {
          // two passes: count (a passing sum is marked by negating it — sums
          // are >= 0 here — so a doc reached twice counts once), then write
          // the marked ones in the same order
          const int64_t base = tile << S;
          const int tie = (int)max<int64_t>(
              -1, min<int64_t>(D, (int64_t)(0xFFFFFFFFu - (uint32_t)th) - base + 1));
          int cnt = 0;
          for_ops([&](uint32_t s) {
            const float x = acc[s];
            const bool pass = (x > thf_raw) | ((x == thf_raw) & ((int)s < tie));
            if (pass) acc[s] = -x;
            cnt += pass;
          });
          if (__ballot(cnt > 0) != 0) {
            const uint32_t incl = wave_incl_scan((uint32_t)cnt);
            int pos = 0;
            if (lane == 63) pos = atomicAdd(list_cnt + cur.q, (int)incl);
            pos = __shfl(pos, 63, 64) + (int)incl - cnt;
            uint64_t* lq = list + (int64_t)cur.q * C;
            for_ops([&](uint32_t s) {
              const float x = acc[s];
              if (x < 0.f) {
                if (pos < C) lq[pos] = ((uint64_t)score_key(-x) << 32) |
                                       (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + s));
                ++pos;
                acc[s] = 0.f;
              }
            });
          }
          clear_ops();
        } else if (PH == kRest) {
          emit_rest<S>(acc, tile, a.n_docs, th, list + (int64_t)cur.q * C, list_cnt + cur.q, C);
        } else {  // SAMPLE: the best key of each of SM doc slices of the tile
          const int sh = S - (SM == 1 ? 0 : (SM == 2 ? 1 : 2));
          uint32_t bk[SM], bd[SM];
#pragma unroll
          for (int u = 0; u < SM; ++u) {
            bk[u] = 0;
            bd[u] = 0xFFFFFFFFu;
          }
          for_ops([&](uint32_t s) {
            const float x = acc[s];
            const uint32_t key = (x > 0.f && s < (uint32_t)D) ? score_key(x) : 0u;
            const uint32_t sli = SM == 1 ? 0u : (s >> sh);
#pragma unroll
            for (int u = 0; u < SM; ++u) {
              const bool better =
                  sli == (uint32_t)u && (key > bk[u] || (key == bk[u] && key != 0u && s < bd[u]));
              bd[u] = better ? s : bd[u];
              bk[u] = better ? key : bk[u];
            }
          });
          clear_ops();
          const uint32_t base = (uint32_t)(tile << S) + (uint32_t)a.doc_offset;
          uint64_t* out = cand + (int64_t)cur.q * cstride + ti * SM;
#pragma unroll
          for (int u = 0; u < SM; ++u) {
            const uint32_t wm = wave_max_u32(bk[u]);
            uint64_t key = 0ull;
            if (wm != 0) {
              const uint32_t doc =
                  0xFFFFFFFFu - wave_max_u32(bk[u] == wm ? 0xFFFFFFFFu - bd[u] : 0u);
              key = ((uint64_t)wm << 32) | (uint64_t)(0xFFFFFFFFu - (base + doc));
            }
            if (lane == 0) out[u] = key;
          }
        }
      }
      // ---- rotate
      rD = rC;
#pragma unroll
      for (int k = 0; k < kNB; ++k)
#pragma unroll
        for (int j = 0; j < kJ2; ++j) {
          ltD[k][j] = ltC[k][j];
          vD0[k][j] = vC0[k][j];
          vD1[k][j] = vC1[k][j];
        }
    }
    // ---- next item (its first tile is in flight)
    tab = ntab;
    cur = nx;
    nx = nx2;
    nx2 = nx3;
    tmN2 = tmN3;
  }
}

// ===========================================================================
// Flat score kernel (queries of 1..8 terms; SAMPLE and REST).  DESIGN.md §4.
//
// The band kernel's items — (query, band of up to 8 phase tiles), claimed per
// XCD — but the wave streams the posting rows of all its items as ONE
// sequence that ignores tile and item boundaries:
//   * an item's rows (double rows, each inside one (tile, term) segment;
//     tile-major, query-term order inside a tile) are numbered once per item
//     by a scan over its 64 (tile, term) segments; a CHUNK of up to 64 rows is
//     one table, lane r = row r (flat_chunk: a binary search of the scan);
//   * a ring of kFR rows is in flight: the step that adds row r issues row
//     r + kFR into the registers row r freed, so loads never pause at a tile
//     or item edge and every step issues the same loads (static vmcnt);
//   * a row of another tile than the accumulator's first runs that tile's
//     epilogue (REST: the keys >= theta, or a plain clear when no add reached
//     theta; SAMPLE: the tile's best key per slice).
// Per tile there is no row-table work, no refill of the pipeline and no
// per-tile branch structure: the per-item fixed cost of the band kernel
// (ablation: 2.49 of its 4.35 ms with no loads, adds or emission) is what
// this removes.  Each doc's adds stay in query-term order (bm25_native.py:152).
// ===========================================================================
#ifndef BM25_FR    // rows in flight (ring slots): REST, SAMPLE
#define BM25_FR 10
#endif
#ifndef BM25_FR_S
#define BM25_FR_S 8
#endif
constexpr uint32_t kDeadSid = 0xFFFFFFFFu;   // padding row: no adds, no tile
constexpr uint32_t kNoTag = 0xFFFFFFFFu;     // accumulator holds no tile

#ifndef BM25_FLAT_WPE
#define BM25_FLAT_WPE 5
#endif

// Inclusive prefix sum over the wave (DPP: rows of 16, then the row carries).
__device__ __forceinline__ uint32_t scan64(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false); // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false); // row_bcast:31
  return x;
}

struct FlatDesc {   // lane i * 8 + t: term t's segment in tile i (raw; r1 == r0: none)
  uint32_t ip, r0, r1;
  uint32_t sk;      // REST: score-key half of the tile's best sample key (sample tiles)
};

struct FlatTab {    // one chunk of an item's rows: lane r = row j0 + r
  uint32_t base;    // even posting index of the row's first pair (0: dead row)
  uint32_t pk;      // valid postings [lo, hi) of the row's 128 (lo = pk & 1, hi = pk >> 1)
  uint32_t sid;     // (item serial << 6) | tile * 8 + term; kDeadSid: padding
};

struct FlatCtx {    // the item a chunk (or the accumulator's tile) belongs to
  int32_t q, b;
  uint64_t th;
};

// Rows [j0, j0 + 64) of an item whose (tile, term) lane s holds segment
// [sb, sb + sl), rows [excl, incl) of the item.
__device__ __forceinline__ FlatTab flat_chunk(uint32_t sb, uint32_t sl, uint32_t incl,
                                              uint32_t excl, uint32_t total, uint32_t j0,
                                              uint32_t ser) {
  const uint32_t lane = lane_id();
  const uint32_t j = j0 + lane;
  int pos = 0;  // segments ending at or before row j (binary lifting)
#pragma unroll
  for (int step = 32; step >= 1; step >>= 1) {
    const uint32_t x = (uint32_t)__shfl((int)incl, pos + step - 1, 64);
    if (x <= j) pos += step;
  }
  const uint32_t e = (uint32_t)__shfl((int)excl, pos, 64);
  const uint32_t b = (uint32_t)__shfl((int)sb, pos, 64);
  const uint32_t l = (uint32_t)__shfl((int)sl, pos, 64);
  const bool in = j < total;
  FlatTab t;
  const uint32_t k = j - e;  // row of its segment
  t.base = (in && l != 0u) ? (b & ~1u) + 128u * k : 0u;
  // row positions p of the segment: p + base in [b, b + l)
  const uint32_t rlo = k == 0u ? (b & 1u) : 0u;
  const uint32_t rhi = min(128u, (b & 1u) + l - 128u * k);
  t.pk = (in && l != 0u) ? (rlo | (rhi << 1)) : 1u;
  t.sid = in ? (ser << 6) | (uint32_t)pos : kDeadSid;
  return t;
}

template <int S, int PH, int SM, bool SP>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BM25_FLAT_WPE, BM25_FLAT_WPE))) void score_flat_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, int32_t P, int32_t G, int32_t nq,
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand, int64_t cstride,
    uint64_t* __restrict__ list, int32_t* __restrict__ list_cnt, int32_t C,
    int32_t* __restrict__ wctr, int32_t claim_ch, int32_t claim_m,
    const uint64_t* __restrict__ skeys, int64_t sstride, int32_t BW) {
  constexpr int D = 1 << S;
  constexpr int kFR = PH == kSample ? BM25_FR_S : BM25_FR;  // ring slots (>= 2)
  __shared__ __attribute__((aligned(16))) float acc[D + 64];
  const uint32_t lane = lane_id();
  const uint32_t trash = (uint32_t)D + lane;  // this lane's always-zero slot
  const int32_t nt = PH == kSample ? (int32_t)sample_count(a.ntiles, P, G) : (int32_t)a.ntiles;
  const int32_t nb = (nt + BW - 1) / BW;  // items: (query, BW <= 8 consecutive phase tiles)
  const int64_t nitems = (int64_t)nb * nq;
  const int64_t per = (nitems + 7) >> 3;
  const int grp = (int)(blockIdx.x & 7);
  const uint32_t lo = (uint32_t)(grp * per);
  const int32_t ngi = (int32_t)max<int64_t>(0, min<int64_t>(nitems, lo + per) - lo);
  if (ngi == 0) return;  // wave-uniform; no barriers in this kernel
  const int32_t cm = (int32_t)(blockIdx.x >> 3) % claim_m;
  int32_t* ctr = wctr + (grp * kClaimM + cm) * kCtrStride;
  const PostingRsrc pr = posting_rsrc(a);
  const uint32_t lt = lane & 7u, li = lane >> 3;  // segment lane: tile li, term lt
  const int64_t nbp = (a.ntiles + 7) >> 3;          // physical bands (sparse seg rows)

  // ---- items: claims, terms -> segment descriptors (as score_band_kernel)
  auto claim = [&]() -> int32_t {
    int32_t v = 0;
    if (lane == 0) v = atomicAdd(ctr, 1);
    return v;
  };
  int32_t pending = claim();
  auto next = [&](BandCur c) -> BandCur {
    if (c.rit >= ngi) return c;
    if (c.rit + 1 < c.end) {
      ++c.rit;
      if (++c.q == nq) {
        c.q = 0;
        ++c.b;
        c.bw = min(BW, nt - c.b * BW);
      }
      return c;
    }
    const int64_t bb = ((int64_t)uniform(pending) * claim_m + cm) * claim_ch;
    if (bb >= ngi) {
      c.rit = c.end = ngi;
      return c;
    }
    pending = claim();
    BandCur n;
    n.rit = (int32_t)bb;
    n.end = (int32_t)min<int64_t>(ngi, bb + claim_ch);
    const uint32_t it = lo + (uint32_t)bb;
    n.b = (int32_t)(it / (uint32_t)nq);
    n.q = (int32_t)(it - (uint32_t)n.b * (uint32_t)nq);
    n.bw = min(BW, nt - n.b * BW);
    return n;
  };
  auto terms_of = [&](const BandCur& c) -> int32_t {
    return queries[(int64_t)c.q * T + (int)min(lt, (uint32_t)(T - 1))];
  };
  // REST: sample tiles (groups of G = kSampleGroup tiles, one group per G * P)
  // whose best sample key is below theta are skipped
  const bool skipping = PH == kRest && skeys != nullptr && G == kSampleGroup;
  const uint32_t lgG = (uint32_t)__builtin_ctz((unsigned)G), lgP = (uint32_t)__builtin_ctz((unsigned)P);
  // an item's segment descriptors (4 VGPRs: a lane outside the item reads its
  // r1 from r0's address, so r1 - r0 = 0 needs no flag; the sample-tile test
  // is redone from the item cursor at enter_item)
  auto load_bdesc = [&](const BandCur& c, int32_t tm) -> FlatDesc {
    FlatDesc d;
    const int32_t term = __shfl(tm, (int)lt, 64);
    const bool ok = (int)lt < T && (int)li < c.bw && term >= 0 && term < a.V;
    const int64_t tt = ok ? term : 0;
    const int64_t tile = ok ? (int64_t)tile_of32<PH>((uint32_t)(c.b * BW + li), (uint32_t)P,
                                                      (uint32_t)G)
                            : 0;
    if constexpr (SP) {  // outside the item: the zero entry past the table
      const uint64_t e = a.seg[ok ? ((int64_t)c.q * nbp + (tile >> 3)) * 64 + lt * 8 + (tile & 7)
                                  : (int64_t)nq * nbp * 64];
      d.ip = 0u;
      d.r0 = (uint32_t)e;
      d.r1 = (uint32_t)e + (uint32_t)(e >> 32);
    } else {
      const uint32_t* r = a.rel + tt * (a.ntiles + 1) + tile;
      d.ip = (uint32_t)a.indptr[tt];
      d.r0 = r[0];
      d.r1 = *(ok ? r + 1 : r);
    }
    if (skipping) {  // the score-key half of this tile's best sample key
      // G and P are powers of two (sample_geom): shifts, no integer division
      const uint32_t t32 = (uint32_t)tile;
      const int64_t si = (int64_t)(((t32 >> (lgG + lgP)) << lgG) | (t32 & (uint32_t)(G - 1)));
      d.sk = reinterpret_cast<const uint32_t*>(skeys)[2 * ((int64_t)c.q * sstride +
                                                             min<int64_t>(si, sstride - 1)) + 1];
    } else {
      d.sk = 0u;
    }
    return d;
  };
  auto th_positive = [&](uint64_t th) -> bool {
    return (uint32_t)(th >> 32) > score_key(0.f);
  };

  // ---- the issue side's item: its segments (lane s = tile * 8 + term) and
  // row numbering; the item prefetch pipeline one and two items ahead
  uint32_t iSb = 0, iSl = 0, iIncl = 0, iExcl = 0;
  uint32_t iTotal = 0, iR = 0, iJ0 = 0, iSer = 0;
  FlatCtx ctxI{0, 0, 0ull};
  BandCur nx, nx2;
  FlatDesc dN;
  uint64_t thN = 0ull;
  int32_t tmN2 = 0;
  // enter item nx (descriptors dN) on the issue side; advance the prefetch
  auto enter_item = [&]() {
    const bool th_pos = PH == kRest && th_positive(thN);
    const uint32_t t32 = (uint32_t)(nx.b * BW) + li;  // REST: phase tile = tile
    const bool smp = skipping && ((t32 >> lgG) & (uint32_t)(P - 1)) == 0u;
    const bool skip = smp && th_pos && dN.sk < (uint32_t)(thN >> 32);
    iSb = dN.ip + dN.r0;
    iSl = skip ? 0u : dN.r1 - dN.r0;
    uint32_t nr = iSl == 0u ? 0u : ((iSb & 1u) + iSl + 127u) >> 7;
    // no positive threshold: every tile of the band runs its epilogue (one
    // row, possibly empty, in each tile)
    if (PH == kRest && !th_pos && lt == 0u && (int)li < nx.bw) nr = max(nr, 1u);
    iIncl = scan64(nr);
    iExcl = iIncl - nr;
    iTotal = lane_u32(iIncl, 63);
    uint32_t R = max(iTotal, (uint32_t)kFR);
    if ((R & 63u) != 0u && (R & 63u) < (uint32_t)kFR) R += (uint32_t)kFR - (R & 63u);
    iR = R;
    iJ0 = 0;
    iSer = (iSer + 1u) & 0x3FFFFFFu;  // tags of consecutive items differ
    ctxI.q = nx.q;
    ctxI.b = nx.b;
    ctxI.th = thN;
    // prefetch: descriptors of the item after, terms of the one after that
    BandCur nx3 = next(nx2);
    dN = load_bdesc(nx2, tmN2);
    thN = PH == kRest ? theta[nx2.q] : 0ull;
    tmN2 = terms_of(nx3);
    nx = nx2;
    nx2 = nx3;
  };

  BandCur c0;
  c0.rit = -1;
  c0.end = 0;
  c0.b = c0.q = 0;
  c0.bw = 1;
  nx = next(c0);
  if (nx.rit >= ngi) return;
  dN = load_bdesc(nx, terms_of(nx));
  thN = PH == kRest ? theta[nx.q] : 0ull;
  nx2 = next(nx);
  tmN2 = terms_of(nx2);
  for (int j = 0; j < D / 256; ++j)
    reinterpret_cast<float4*>(acc)[j * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  acc[D + lane] = 0.f;

  // issue table: the chunk the next issued row comes from
  bool items_left = true, iDead = false;
  FlatTab tI;
  uint32_t nI = 0, il = 0;
  auto next_chunk = [&]() {  // tI <- the chunk after it (or the dead tail)
    if (iJ0 + 64u < iR) {
      iJ0 += 64u;
    } else if (items_left && nx.rit < ngi) {
      enter_item();
    } else {
      items_left = false;
      iDead = true;
      tI.base = 0u;
      tI.pk = 1u;
      tI.sid = kDeadSid;
      nI = 0x7FFFFFFFu;
      il = 0;
      return;
    }
    tI = flat_chunk(iSb, iSl, iIncl, iExcl, iTotal, iJ0, iSer);
    nI = min(64u, iR - iJ0);
    il = 0;
  };
  enter_item();
  tI = flat_chunk(iSb, iSl, iIncl, iExcl, iTotal, 0u, iSer);
  nI = min(64u, iR);
  il = 0;

  // ring: slot s holds the raw loads of rows r == s (mod kFR)
  uint32_t ldR[kFR];
  float v0R[kFR], v1R[kFR];
  auto issue = [&](int s) {
    if (il == nI) next_chunk();
    const uint32_t base = lane_u32(tI.base, (int)il);
    ldR[s] = __builtin_amdgcn_raw_buffer_load_b32(pr.ldoc, (int)(lane * 4u), (int)(base * 2u), 0);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(pr.val, (int)(lane * 8u), (int)(base * 4u), 0);
    v0R[s] = __uint_as_float((uint32_t)v[0]);
    v1R[s] = __uint_as_float((uint32_t)v[1]);
    ++il;
  };
#pragma unroll
  for (int s = 0; s < kFR; ++s) issue(s);  // the first chunk holds >= kFR rows

  // process side
  uint32_t tPpk = tI.pk, tPsid = tI.sid;  // the process side's chunk (no bases)
  uint32_t nP = nI, pl = 0;
  FlatCtx ctxP = ctxI, ctxE = ctxI;
  auto thf_of = [&](uint64_t th) -> float {
    return (PH == kRest && a.nonneg && th_positive(th)) ? key_score((uint32_t)(th >> 32))
                                                         : __builtin_nanf("");
  };
  float thfP = thf_of(ctxP.th);
  uint32_t curTag = kNoTag;
  uint64_t hit = 0;
  bool done = false;

  auto epilogue = [&]() {
    const int32_t ti = ctxE.b * BW + (int32_t)(curTag & 7u);
    const int64_t tile = tile_of32<PH>((uint32_t)ti, (uint32_t)P, (uint32_t)G);
    if constexpr (PH == kRest) {
      const bool flagged = a.nonneg && th_positive(ctxE.th);
      if (flagged && hit == 0)
        zero_acc<S>(acc);
      else
        emit_rest<S>(acc, tile, a.n_docs, ctxE.th, list + (int64_t)ctxE.q * C,
                     list_cnt + ctxE.q, C);
    } else {
      uint64_t* out = cand + (int64_t)ctxE.q * cstride + (int64_t)ti * SM;
      if constexpr (SM == 1)
        best1_pos<S>(acc, tile, (uint32_t)a.doc_offset, out);
      else
        best_dense<S, SM, true>(acc, tile, a.n_docs, (uint32_t)a.doc_offset, out);
    }
  };

  // the current row (its slot already consumed): masked slots and scores,
  // the accumulator values read one step early, its segment id
  uint32_t sc0, sc1, sidC;
  float ac0, ac1, xc0, xc1;
  auto prepare = [&](int s) {  // row pl of the process chunk, from slot s
    sidC = lane_u32(tPsid, (int)pl);
    const uint32_t pk = lane_u32(tPpk, (int)pl);
    const uint32_t p0 = 2u * lane, rhi = pk >> 1;
    const bool m0 = p0 >= (pk & 1u) && p0 < rhi, m1 = p0 + 1u < rhi;
    sc0 = m0 ? (ldR[s] & 0xFFFFu) : trash;
    sc1 = m1 ? (ldR[s] >> 16) : trash;
    ac0 = m0 ? v0R[s] : 0.f;
    ac1 = m1 ? v1R[s] : 0.f;
    xc0 = acc[sc0];
    xc1 = acc[sc1];
  };
  prepare(0);

  // step of ring slot s: row r (prepared) is added, row r + kFR goes into slot
  // s (consumed by the previous step), row r + 1 is prepared from slot s + 1
  auto step = [&](int s) {
    issue(s);
    if (sidC != kDeadSid) {
      const uint32_t tag = sidC >> 3;
      if (tag != curTag) {
        if (curTag != kNoTag) epilogue();
        hit = 0;
        curTag = tag;
        ctxE = ctxP;
        xc0 = 0.f;  // read before the epilogue cleared the accumulator
        xc1 = 0.f;
      }
    }
    const float y0 = xc0 + ac0, y1 = xc1 + ac1;
    acc[sc0] = y0;
    acc[sc1] = y1;
    if (PH == kRest) hit |= __ballot(fmaxf(y0, y1) >= thfP);
    if (++pl == nP) {  // the process side enters the issue side's chunk
      tPpk = tI.pk;
      tPsid = tI.sid;
      nP = nI;
      pl = 0;
      ctxP = ctxI;
      thfP = thf_of(ctxP.th);
      done = iDead;
    }
    prepare((s + 1) % kFR);
  };

  while (!done) {
#pragma unroll
    for (int s = 0; s < kFR; ++s) step(s);
  }
  if (curTag != kNoTag) epilogue();
}

// ---------------------------------------------------------------------------
// Exact top-k of each flagged tile (persistent, queue-driven; every wave
// reaches the exit test each iteration).  Wave 0 accumulates the tile; the
// workgroup bitonic-sorts its 2^S keys in LDS.
// ---------------------------------------------------------------------------
constexpr int kRescoreNT = 256;

__device__ __forceinline__ void bitonic_sort_desc(uint64_t* keys, int n) {
  for (int size = 2; size <= n; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int ls = __builtin_ctz((unsigned)stride);  // stride is a power of two:
      for (int i = threadIdx.x; i < (n >> 1); i += blockDim.x) {  // no integer division
        const int lo = ((i >> ls) << (ls + 1)) + (i & (stride - 1));
        const int hi = lo + stride;
        const bool desc = (lo & size) == 0;
        const uint64_t x = keys[lo], y = keys[hi];
        if ((x < y) == desc) {
          keys[lo] = y;
          keys[hi] = x;
        }
      }
      __syncthreads();
    }
  }
}

template <int S>
__global__ __launch_bounds__(kRescoreNT) void rescore_kernel(IndexArgs a,
                                                             const int32_t* __restrict__ queries,
                                                             int32_t T, int32_t k, int64_t maxflag,
                                                             Stage sg, Workspace ws) {
  constexpr int D = 1 << S;
  __shared__ __attribute__((aligned(16))) float acc[D];
  __shared__ uint64_t keys[D];
  __shared__ int32_t s_item;
  const int32_t n_items = ws.counters[0];
  for (;;) {
    __syncthreads();
    if (threadIdx.x == 0) s_item = atomicAdd(&ws.counters[1], 1);
    __syncthreads();
    const int32_t it = s_item;
    if (it >= n_items) break;
    const int32_t code = ws.queue[it];
    const int64_t qi = code / maxflag;
    const int64_t q = sg.qmap ? (int64_t)sg.qmap[qi] : qi;
    const int64_t tile = sample_tile(ws.flag_tiles[code], sg.P, sg.G);
    if (threadIdx.x < 64) {
      zero_acc<S>(acc);
      add_item<S>(a, tile, queries + q * T, T, acc);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < D; i += blockDim.x) {
      const int64_t doc = (tile << S) + i;
      keys[i] = doc < a.n_docs ? make_key(acc[i], (uint32_t)doc) : 0ull;
    }
    __syncthreads();
    bitonic_sort_desc(keys, D);
    uint64_t* out = ws.cand2 + (int64_t)code * k;
    for (int i = threadIdx.x; i < k; i += blockDim.x) out[i] = i < D ? keys[i] : 0ull;
  }
}

// Dense per-doc scores of one query: one wave per tile, coalesced stores.
template <int S>
__global__ __launch_bounds__(64) void scores_dense_kernel(IndexArgs a,
                                                          const int32_t* __restrict__ query,
                                                          int32_t T, float* __restrict__ out) {
  constexpr int D = 1 << S, E = D / 64;
  __shared__ __attribute__((aligned(16))) float acc[D];
  const int64_t tile = blockIdx.x;
  zero_acc<S>(acc);
  add_item<S>(a, tile, query, T, acc);
  float fv[E];
  take_entries<S>(acc, fv);
  const int64_t base = tile << S;
  const uint32_t lane = lane_id();
  if (base + D <= a.n_docs) {
#pragma unroll
    for (int j = 0; j < E / 4; ++j)  // docs base + 256 j + 4 lane + (0..3)
      *reinterpret_cast<float4*>(out + base + entry_doc(4 * j, lane)) =
          make_float4(fv[4 * j], fv[4 * j + 1], fv[4 * j + 2], fv[4 * j + 3]);
  } else {
#pragma unroll
    for (int e = 0; e < E; ++e)
      if (base + entry_doc(e, lane) < a.n_docs) out[base + entry_doc(e, lane)] = fv[e];
  }
}

// ---------------------------------------------------------------------------
// Index build: u16 accumulator slots + per-(term, tile) segment table, one
// wave per term.  Terms with at least ntiles/4 postings fill their rel row
// from the tile boundaries between consecutive postings; lighter terms fill
// it entry by entry with a binary search (coalesced stores either way).
// Flags non-canonical input (unsorted / duplicate / out-of-range doc ids
// inside a column) in *err.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void build_tables_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, int64_t V,
    int64_t n_docs, int S, int64_t ntiles, uint32_t* __restrict__ rel,
    uint16_t* __restrict__ ldoc, int32_t* __restrict__ err) {
  const int lane = lane_id();
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const uint32_t mask = (1u << S) - 1u;
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < V;
       t += waves) {
    const int64_t a0 = indptr[t], a1 = indptr[t + 1];
    const int64_t df = a1 - a0;
    uint32_t* row = rel + t * (ntiles + 1);
    const bool heavy = df * 4 >= ntiles;
    for (int64_t p = a0 + lane; p < a1; p += 64) {
      const int32_t d = indices[p];
      const int32_t dp = p > a0 ? indices[p - 1] : -1;
      const bool ok = d >= 0 && (int64_t)d < n_docs && d > dp;
      if (!ok) atomicOr(err, 1);
      ldoc[p] = (uint16_t)((uint32_t)d & mask);  // tile-local doc = LDS slot
      if (heavy && ok) {
        const int64_t tp = dp >= 0 ? ((int64_t)dp >> S) : -1;
        const int64_t tc = (int64_t)d >> S;
        for (int64_t j = tp + 1; j <= tc; ++j) row[j] = (uint32_t)(p - a0);
      }
    }
    if (heavy) {
      int64_t last = -1;
      if (df > 0) {
        const int32_t dl = indices[a1 - 1];
        last = (dl >= 0 && (int64_t)dl < n_docs) ? ((int64_t)dl >> S) : ntiles - 1;
      }
      for (int64_t j = last + 1 + lane; j <= ntiles; j += 64) row[j] = (uint32_t)df;
    } else {
      for (int64_t j = lane; j <= ntiles; j += 64) {
        const int64_t target = j << S;  // first doc of tile j
        int64_t lo = 0, hi = df;
        while (lo < hi) {
          const int64_t mid = (lo + hi) >> 1;
          if ((int64_t)indices[a0 + mid] < target) lo = mid + 1;
          else hi = mid;
        }
        row[j] = (uint32_t)lo;
      }
    }
  }
}

// Sparse segment table, pass 1: ldoc + validation (as build_tables_kernel)
// and the number of non-empty tiles of every term (one wave per term).
__global__ __launch_bounds__(256) void count_tiles_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, int64_t V,
    int64_t n_docs, int S, uint16_t* __restrict__ ldoc, int64_t* __restrict__ cnt,
    int32_t* __restrict__ err) {
  const int lane = lane_id();
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  const uint32_t mask = (1u << S) - 1u;
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < V;
       t += waves) {
    const int64_t a0 = indptr[t], a1 = indptr[t + 1];
    uint32_t n = 0;
    for (int64_t p = a0 + lane; p < a1; p += 64) {
      const int32_t d = indices[p];
      const int32_t dp = p > a0 ? indices[p - 1] : -1;
      const bool ok = d >= 0 && (int64_t)d < n_docs && d > dp;
      if (!ok) atomicOr(err, 1);
      ldoc[p] = (uint16_t)((uint32_t)d & mask);
      n += (dp < 0 || (d >> S) != (dp >> S)) ? 1u : 0u;
    }
    const uint32_t tot = wave_incl_scan(n);
    if (lane == 63) cnt[t] = (int64_t)tot;
  }
}

// Pass 2: the tile lists (tl_ptr = exclusive scan of the counts).
__global__ __launch_bounds__(256) void fill_tiles_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ indices, int64_t V, int S,
    const int64_t* __restrict__ tl_ptr, uint16_t* __restrict__ tl_tile,
    uint32_t* __restrict__ tl_start) {
  const int lane = lane_id();
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x >> 6);
  for (int64_t t = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < V;
       t += waves) {
    const int64_t a0 = indptr[t], a1 = indptr[t + 1];
    int64_t o = tl_ptr[t];
    for (int64_t p0 = a0; p0 < a1; p0 += 64) {
      const int64_t p = p0 + lane;
      bool first = false;
      int32_t d = 0;
      if (p < a1) {
        d = indices[p];
        const int32_t dp = p > a0 ? indices[p - 1] : -1;
        first = dp < 0 || (d >> S) != (dp >> S);
      }
      const uint64_t m = __ballot(first);
      if (first) {
        const int64_t i = o + __popcll(m & ((1ull << lane) - 1ull));
        tl_tile[i] = (uint16_t)(d >> S);
        tl_start[i] = (uint32_t)(p - a0);
      }
      o += __popcll(m);
    }
  }
}

// ---------------------------------------------------------------------------
// Merge: one workgroup per query, bitonic sort of u64 keys in LDS.
// ---------------------------------------------------------------------------
constexpr int kMergeNT = 1024;
constexpr int kMaxFlagBits = 65536;  // tiles per query addressable by the flag bitmap

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
  const int lane = lane_id();
  const int64_t rounds = (n_total + blockDim.x - 1) / blockDim.x;
  for (int64_t r = 0; r < rounds; ++r) {
    const int64_t i = r * blockDim.x + threadIdx.x;
    const uint64_t key = i < n_total ? src(i) : 0ull;
    const bool keep = key != 0ull && key >= lo;
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
    if (key == 0ull) {  // padding (a shard's list under a global theta): maps back to key 0
      docs[row * k + i] = -1;
      scores[row * k + i] = __uint_as_float(0xFFFFFFFFu);
      continue;
    }
    docs[row * k + i] = (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)key) + doc_offset);
    scores[row * k + i] = key_score((uint32_t)(key >> 32));
  }
}

struct SrcFirst {
  const uint64_t* c;
  __device__ uint64_t operator()(int64_t i) const { return c[i]; }
};

struct SrcCat {  // the stage's tile candidates, then the query's list
  const uint64_t* c;
  const uint64_t* l;
  int64_t n1;
  __device__ uint64_t operator()(int64_t i) const { return i < n1 ? c[i] : l[i - n1]; }
};

struct SrcFinal {
  const uint64_t* c;      // this query's [nt][kTileM] candidates
  const uint64_t* l;      // this query's list
  const uint64_t* c2;     // this query's flagged tiles' exact lists, contiguous
  const uint32_t* bits;   // LDS bitmap of flagged tiles
  int64_t n1, n2;
  __device__ uint64_t operator()(int64_t i) const {
    if (i < n1) {
      const int64_t j = i / kTileM;
      return ((bits[j >> 5] >> (j & 31)) & 1u) ? 0ull : c[i];
    }
    if (i < n1 + n2) return l[i - n1];
    return c2[i - n1 - n2];
  }
};

struct SrcLists {  // list w of query q at element w * rstride + q * k
  const int32_t* docs;
  const float* scores;
  int64_t Q, q;
  int k;
  int64_t rstride;
  __device__ uint64_t operator()(int64_t i) const {
    const int64_t w = i / k, j = i - w * k;
    const int64_t o = w * rstride + q * k + j;
    return make_key(scores[o], (uint32_t)docs[o]);
  }
};

// theta of a query whose sample holds fewer than k keys, on a non-negative
// index (values 0 or normal positive, so every sum is 0 or >= FLT_MIN): every
// doc with a positive sum (key >= (FLT_MIN, any doc)) goes to the list, and
// merge_first completes the top-k with the smallest doc ids outside it
// (score 0: untouched docs or zero sums).
constexpr uint64_t kZeroFillTheta = (uint64_t)0x80800000u << 32;

// theta[q] = k-th best key among the sample tiles' keys: k real documents
// score at least this, so it is a lower bound of the final k-th key.  A query
// with fewer than k sample keys (a sample reports no key for a slice without a
// positive sum) gets kZeroFillTheta on a non-negative index; otherwise it gets
// no threshold: theta = all ones (a NaN score: no REST key passes) and its list
// is marked overflowed, which sends it to the exact fallback stage.

//
// Sample keys carry GLOBAL doc ids (doc_offset + local), so the k-th key is
// the same on every shard; theta is then moved into this shard's frame: same
// score, tie doc L = global - doc_offset (docs <= L of that score pass),
// clamped to n_docs; L < 0 (the tie doc lies in an earlier shard) becomes
// "strictly higher scores only" = (score key + 1, any doc).
// The threshold by radix selection, one wave per query (no barriers; the
// sort-based form (topk_of) took 43 us per search, a fixed cost that is
// 7 % of an 8-way shard's batch): the k-th largest of the query's W * S
// sample keys, decided bit by bit from the top — the answer has a bit set iff
// at least `need` keys match its prefix with that bit set (need = k minus the
// keys already ranked above).  Keys in registers when the query has at most
// 1024 of them, re-read (L1) otherwise.
constexpr int kThetaR = 16;  // keys per lane held in registers

__global__ __launch_bounds__(256) void theta_wave_kernel(const uint64_t* __restrict__ all_keys,
                                                         int64_t W, int64_t Q, int64_t S,
                                                         int32_t k, uint64_t* __restrict__ theta,
                                                         int32_t* __restrict__ list_cnt,
                                                         int32_t C, int32_t nonneg,
                                                         int64_t doc_offset, int64_t n_docs) {
  const int64_t q = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (q >= Q) return;  // wave-uniform; no barriers
  const uint32_t lane = lane_id();
  const int64_t n = W * S;
  uint64_t t = 0ull;
  if (k > 0 && n >= k) {
    uint64_t prefix = 0ull;
    uint32_t need = (uint32_t)k;
    if (n <= 64 * kThetaR) {
      uint64_t key[kThetaR];
#pragma unroll
      for (int j = 0; j < kThetaR; ++j) {
        const int64_t i = (int64_t)j * 64 + lane;
        const int64_t w = i / S;
        key[j] = i < n ? all_keys[(w * Q + q) * S + (i - w * S)] : 0ull;
      }
      // score half first (32 steps on u32), then the doc half among the keys
      // of that score — only when more than one key holds it (ties)
      uint32_t hi = 0u;
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t hm = ~0u << bit, cand = hi | (1u << bit);
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < kThetaR; ++j) c += ((uint32_t)(key[j] >> 32) & hm) == cand;
        const uint32_t tot = wave_sum_u32(c);
        if (tot >= need) hi = cand;
        else need -= tot;
      }
      uint32_t ties = 0;
#pragma unroll
      for (int j = 0; j < kThetaR; ++j) ties += (uint32_t)(key[j] >> 32) == hi;
      uint32_t lo = 0u;
      if (wave_sum_u32(ties) == 1u) {  // the one key of that score
        uint32_t m = 0u;
#pragma unroll
        for (int j = 0; j < kThetaR; ++j) m = (uint32_t)(key[j] >> 32) == hi ? (uint32_t)key[j] : m;
        lo = wave_max_u32(m);
      } else {
        for (int bit = 31; bit >= 0; --bit) {
          const uint32_t hm = ~0u << bit, cand = lo | (1u << bit);
          uint32_t c = 0;
#pragma unroll
          for (int j = 0; j < kThetaR; ++j)
            c += (uint32_t)(key[j] >> 32) == hi && ((uint32_t)key[j] & hm) == cand;
          const uint32_t tot = wave_sum_u32(c);
          if (tot >= need) lo = cand;
          else need -= tot;
        }
      }
      prefix = ((uint64_t)hi << 32) | lo;
    } else {
      for (int bit = 63; bit >= 0; --bit) {
        const uint64_t hm = ~0ull << bit, cand = prefix | (1ull << bit);
        uint32_t c = 0;
        for (int64_t w = 0; w < W; ++w) {
          const uint64_t* kk = all_keys + (w * Q + q) * S;
          for (int64_t i = lane; i < S; i += 64) c += (kk[i] & hm) == cand;
        }
        const uint32_t tot = wave_sum_u32(c);
        if (tot >= need) prefix = cand;
        else need -= tot;
      }
    }
    t = prefix;
  }
  if (lane == 0) {
    if (t != 0ull) {
      const int64_t L = (int64_t)(0xFFFFFFFFu - (uint32_t)t) - doc_offset;
      if (L < 0)
        t = (t | 0xFFFFFFFFull) + 1ull;
      else
        t = (t & ~0xFFFFFFFFull) | (uint64_t)(0xFFFFFFFFu - (uint32_t)min(L, n_docs));
    }
    theta[q] = t != 0ull ? t : (nonneg ? kZeroFillTheta : ~0ull);
    if (t == 0ull && !nonneg) list_cnt[q] = C + 1;
  }
}


__device__ __forceinline__ int64_t stage_nq(const Stage& sg) {
  return sg.nq_dev ? (int64_t)*sg.nq_dev : (int64_t)sg.nq_host;
}

__global__ __launch_bounds__(kMergeNT) void merge_first_kernel(
    Stage sg, int32_t k, int64_t maxflag, int64_t doc_offset, int64_t n_docs, Workspace ws,
    int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  __shared__ int32_t s_nflag, s_cnt;
  __shared__ uint32_t zf_bits[2 * kMaxK / 32];
  const int64_t qi = blockIdx.x;
  if (qi >= stage_nq(sg)) return;
  const int64_t q = sg.qmap ? (int64_t)sg.qmap[qi] : qi;
  const int32_t cnt = sg.list ? sg.list_cnt[qi] : 0;
  if (cnt > sg.C) {  // the list overflowed: exact fallback stage
    if (threadIdx.x == 0) {
      ws.nflag[qi] = 0;
      sg.fb[atomicAdd(sg.fb_cnt, 1)] = (int32_t)q;
    }
    return;
  }
  const uint64_t* c = sg.cand + qi * sg.nt * kTileM;
  if (threadIdx.x == 0) s_nflag = 0;
  // theta (sampled stage): k sample candidates are >= it, so nothing below it
  // can reach the top-k; every list entry is above it
  topk_compact(SrcCat{c, sg.list ? sg.list + qi * sg.C : nullptr, sg.nt * kTileM},
               sg.nt * kTileM + cnt, k, sg.theta ? sg.theta[qi] : 0ull, keys, &s_cnt);
  if (sg.theta && sg.theta[qi] == kZeroFillTheta && cnt < k) {
    // the list holds every positive doc: complete it with the smallest doc ids
    // outside it (all < k + cnt), score 0; a shard holding fewer than k docs
    // leaves the rest as padding (key 0)
    const int span = k + cnt;
    for (int i = threadIdx.x; i < (span + 31) / 32; i += blockDim.x) zf_bits[i] = 0u;
    __syncthreads();
    for (int i = threadIdx.x; i < cnt; i += blockDim.x) {
      const uint32_t d = 0xFFFFFFFFu - (uint32_t)keys[i];
      if (d < (uint32_t)span) atomicOr(&zf_bits[d >> 5], 1u << (d & 31));
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      int filled = 0;
      for (int b0 = 0; b0 < span && filled < k - cnt; b0 += 64) {
        const int id = b0 + (int)threadIdx.x;
        const bool fr = id < span && id < n_docs && !((zf_bits[id >> 5] >> (id & 31)) & 1u);
        const uint64_t m = __ballot(fr);
        const int pos = filled + (int)__builtin_amdgcn_mbcnt_hi(
                                     (uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        if (fr && pos < k - cnt) keys[cnt + pos] = make_key(0.f, (uint32_t)id);
        filled += __popcll(m);
      }
    }
    __syncthreads();
  }
  const uint64_t theta = keys[k - 1];
  if (k > kTileM) {
    // A tile whose kTileM-th candidate beats theta may hold unreported docs
    // of the top-k: schedule it for an exact rescore (at most (k-1)/kTileM).
    for (int64_t j = threadIdx.x; j < sg.nt; j += blockDim.x) {
      if (c[j * kTileM + kTileM - 1] > theta) {
        const int i = atomicAdd(&s_nflag, 1);
        if (i < maxflag) ws.flag_tiles[qi * maxflag + i] = (int32_t)j;
      }
    }
  }
  __syncthreads();
  const int nf = s_nflag < maxflag ? s_nflag : (int)maxflag;
  if (threadIdx.x == 0) {
    ws.nflag[qi] = nf;
    if (nf > 0) {
      const int base = atomicAdd(&ws.counters[0], nf);
      atomicAdd(&ws.counters[3], nf);
      for (int i = 0; i < nf; ++i) ws.queue[base + i] = (int32_t)(qi * maxflag + i);
    }
  }
  if (nf == 0) write_result(keys, k, q, doc_offset, docs, scores);
}

__global__ __launch_bounds__(kMergeNT) void merge_final_kernel(
    Stage sg, int32_t k, int64_t maxflag, int64_t doc_offset, Workspace ws,
    int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  __shared__ uint32_t bits[kMaxFlagBits / 32];
  const int64_t qi = blockIdx.x;
  if (qi >= stage_nq(sg)) return;
  const int nf = ws.nflag[qi];
  if (nf == 0) return;
  const int64_t q = sg.qmap ? (int64_t)sg.qmap[qi] : qi;
  const int64_t nwords = (sg.nt + 31) >> 5;
  for (int64_t i = threadIdx.x; i < nwords; i += blockDim.x) bits[i] = 0;
  __syncthreads();
  if ((int)threadIdx.x < nf) {
    const int32_t j = ws.flag_tiles[qi * maxflag + threadIdx.x];
    atomicOr(&bits[j >> 5], 1u << (j & 31));
  }
  __syncthreads();
  const int32_t cnt = sg.list ? sg.list_cnt[qi] : 0;
  SrcFinal src{sg.cand + qi * sg.nt * kTileM, sg.list ? sg.list + qi * sg.C : nullptr,
               ws.cand2 + qi * maxflag * (int64_t)k, bits, sg.nt * kTileM, cnt};
  topk_of(src, sg.nt * kTileM + cnt + (int64_t)nf * k, k, keys);
  write_result(keys, k, q, doc_offset, docs, scores);
}

__global__ __launch_bounds__(kMergeNT) void merge_lists_kernel(
    const int32_t* __restrict__ in_docs, const float* __restrict__ in_scores, int64_t W,
    int64_t Q, int32_t k, int64_t rstride, int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  const int64_t q = blockIdx.x;
  topk_of(SrcLists{in_docs, in_scores, Q, q, k, rstride}, W * k, k, keys);
  write_result(keys, k, q, 0, docs, scores);
}

// Merge of W lists that are each sorted best first (bm25_search_finish_
// device's [Q, k] lists, padding last): one wave per query, the W list heads
// in lanes 0..W-1; each of the k steps takes the best head (wave max of the
// u64 key, as two u32 maxima) and advances that list.  A query's lists are
// staged in LDS first (W * k <= kMergeSortedCap keys); larger merges take
// merge_lists_kernel.  Keys are unique (global doc ids) except padding (0).
constexpr int kMergeSortedCap = 1024;  // keys per wave

__global__ __launch_bounds__(256) void merge_sorted_kernel(
    const int32_t* __restrict__ in_docs, const float* __restrict__ in_scores, int32_t W,
    int64_t Q, int32_t k, int64_t rstride, int32_t* __restrict__ docs,
    float* __restrict__ scores) {
  __shared__ uint64_t buf[4][kMergeSortedCap];
  const int wave = (int)(threadIdx.x >> 6);
  const int64_t q = (int64_t)blockIdx.x * 4 + wave;
  if (q >= Q) return;  // wave-uniform; no barriers
  uint64_t* kb = buf[wave];
  const uint32_t lane = lane_id();
  const int n = W * k;
  for (int i = (int)lane; i < n; i += 64) {
    const int w = i / k, j = i - w * k;
    const int64_t o = (int64_t)w * rstride + q * k + j;
    kb[i] = make_key(in_scores[o], (uint32_t)in_docs[o]);
  }
  int pos = 0;
  uint64_t head = ((int)lane < W) ? kb[lane * k] : 0ull;
  for (int j = 0; j < k; ++j) {
    const uint32_t hh = wave_max_u32((uint32_t)(head >> 32));
    const uint32_t hl = wave_max_u32((uint32_t)(head >> 32) == hh ? (uint32_t)head : 0u);
    const uint64_t best = ((uint64_t)hh << 32) | hl;
    if (lane == 0) {
      if (best == 0ull) {  // every list is down to its padding
        docs[q * k + j] = -1;
        scores[q * k + j] = __uint_as_float(0xFFFFFFFFu);
      } else {
        docs[q * k + j] = (int32_t)(0xFFFFFFFFu - (uint32_t)best);
        scores[q * k + j] = key_score(hh);
      }
    }
    if (best != 0ull && head == best) {
      ++pos;
      head = pos < k ? kb[lane * k + pos] : 0ull;
    }
  }
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
#ifdef BM25_S12
#define BM25_CASE12(call) case 12: call(12); break;
#else
#define BM25_CASE12(call)
#endif
#ifdef BM25_S12  // dev: 4096-doc tiles (timing experiments)
bool tile_shift_supported(int s) { return s == 10 || s == 11 || s == 12; }
#else
bool tile_shift_supported(int s) { return s == 10 || s == 11; }
#endif

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

hipError_t launch_count_tiles(const DevIndex& ix, const int32_t* d_indices, int64_t* d_cnt,
                              int32_t* d_err, hipStream_t stream) {
  if (ix.n_terms == 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((ix.n_terms + 3) / 4, 65536);
  hipLaunchKernelGGL(count_tiles_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, ix.indptr,
                     d_indices, ix.n_terms, ix.n_docs, ix.tile_shift, ix.ldoc, d_cnt, d_err);
  return hipGetLastError();
}

hipError_t launch_fill_tiles(const DevIndex& ix, const int32_t* d_indices, hipStream_t stream) {
  if (ix.n_terms == 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((ix.n_terms + 3) / 4, 65536);
  hipLaunchKernelGGL(fill_tiles_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, ix.indptr,
                     d_indices, ix.n_terms, ix.tile_shift, ix.tl_ptr, ix.tl_tile, ix.tl_start);
  return hipGetLastError();
}

// Sampling geometry: 1 tile in P is a sample tile reporting m keys (the best
// of each of m doc slices); the first (P, m) in the order P = BM25_SAMPLE_P
// (default 8), 4, 2 (powers of two), m = 1, 2, 4 whose sample — over the W
// doc shards searched together (global threshold) — yields >= 2k keys.
// Sample tiles come in groups of G = 8 consecutive tiles once the index has
// at least four such groups (G = 1, every P-th tile, below).  P = 1: no
// threshold — the exact top-4 path over every tile (small indices).  S =
// keys per query per shard.
SampleGeom sample_geom(int64_t ntiles, int k, int W) {
  const char* e = getenv("BM25_SAMPLE_P");
  const int pmax = e ? atoi(e) : 8;
  for (int P = 64; P >= 2; P >>= 1) {
    if (P > pmax || ntiles < 2 * P) continue;
    const int G = ntiles >= 4 * kSampleGroup * P ? kSampleGroup : 1;
    const int64_t nS = sample_count(ntiles, P, G);
    for (int m = 1; m <= kTileM; m <<= 1)
      if (nS * m * W >= 2 * (int64_t)k) return SampleGeom{P, m, nS * m, G};
  }
  return SampleGeom{1, 0, 0, 1};
}

// Every resident workgroup slot of the current device (a multiple of 8, one
// per XCD round), cached per (kernel, device).
template <int S, int PH, class K>
static int persistent_grid(K kernel, int block = 64 * kWaves) {
  static std::mutex mu;
  static std::map<std::pair<const void*, int>, int> cache;
  int dev = 0;
  hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_pair((const void*)kernel, dev);
  const auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int cus = 0, occ = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kernel, block, 0);
  const char* e = getenv("BM25_WG_PER_CU");
  if (e) occ = atoi(e);
  const int g = ((cus * (occ > 0 ? occ : 1) + 7) / 8) * 8;
  cache[key] = g;
  return g;
}

// The pipelined kernel serves queries of 1..64 terms (BM25_NO_PIPE=1 forces
// the plain one, which also serves longer queries).
static bool use_pipe(const DevIndex& ix, int64_t T) {
  static const bool off = getenv("BM25_NO_PIPE") != nullptr;
  return !off && T >= 1 && T <= kGroup && (ix.nnz + kPostingPad) * 4 < 0xFFFFFFF0ll;
}

// Tiles per band of the item order (BM25_BAND overrides, for tuning).
static int32_t band_tiles() {
  const char* e = getenv("BM25_BAND");
  const int v = e ? atoi(e) : kBand;
  return v >= 1 && v <= 4096 ? v : kBand;
}

// Item-claim geometry (BM25_CLAIM_CH / BM25_CLAIM_M override, for tuning).
static int32_t claim_ch() {
  const char* e = getenv("BM25_CLAIM_CH");
  const int v = e ? atoi(e) : kClaimCH;
  return v >= 1 && v <= 4096 ? v : kClaimCH;
}
static int32_t claim_m() {
  const char* e = getenv("BM25_CLAIM_M");
  const int v = e ? atoi(e) : 4;
  return v >= 1 && v <= kClaimM ? v : 4;
}

// Diagnostic builds (BM25_ABLATE, dev only): 1 = no adds, 4 = no selection,
// 5 = neither, 32 = s_memtime segment stamps of the REST kernel, printed to
// stderr per launch.
template <int S, int PH, bool QMAP, int DIAG, int SM = 1>
static void launch_pipe(const DevIndex& ix, const int32_t* q, int64_t T, const Stage& sg,
                        const Workspace& ws, hipStream_t st) {
  if constexpr (PH == kSample && SM == 1) {  // m keys per sample tile: a build per m
    if (sg.M == 2) {
      launch_pipe<S, PH, QMAP, DIAG, 2>(ix, q, T, sg, ws, st);
      return;
    }
    if (sg.M == kTileM) {
      launch_pipe<S, PH, QMAP, DIAG, kTileM>(ix, q, T, sg, ws, st);
      return;
    }
  }
  const int grid = persistent_grid<S, PH>(score_pipe_kernel<S, PH, QMAP, DIAG, SM>);
  int32_t* wctr = ws.wctr + (int64_t)sg.ctr_region * kWctrInts;
  if (!sg.ctr_zeroed) hipMemsetAsync(wctr, 0, sizeof(int32_t) * kWctrInts, st);
  uint64_t* stamps = nullptr;
  if (DIAG & 32) {
    static uint64_t* buf = nullptr;
    if (!buf) hipMalloc(&buf, sizeof(uint64_t) * 8 * grid * kWaves);
    hipMemsetAsync(buf, 0, sizeof(uint64_t) * 8 * grid * kWaves, st);
    stamps = buf;
  }
  hipLaunchKernelGGL((score_pipe_kernel<S, PH, QMAP, DIAG, SM>), dim3((unsigned)grid),
                     dim3(64 * kWaves), 0, st, args_of(ix), q, (int32_t)T, sg.P, sg.nq_host,
                     sg.nq_dev, sg.qmap, ws.theta, sg.cand_out, ws.list, ws.list_cnt, ws.list_cap,
                     wctr, claim_ch(), claim_m(), sg.cstride, sg.G, band_tiles(), stamps);
  if ((DIAG & 32) && PH == kRest) {
    std::vector<uint64_t> h(8 * grid * kWaves);
    hipStreamSynchronize(st);
    hipMemcpy(h.data(), stamps, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost);
    double tot[8] = {0};
    for (size_t i = 0; i < h.size(); ++i) tot[i % 8] += (double)h[i];
    double loop = 0;
    for (int k = 0; k < 6; ++k) loop += tot[k];
    fprintf(stderr, "stamps: items %.0f, per item:", tot[6]);
    for (int k = 0; k < 6; ++k) fprintf(stderr, " s%d=%.0f", k, tot[k] / tot[6]);
    fprintf(stderr, " | loop %.0f (s_memtime ticks per wave)\n", loop / tot[6]);
  }
}

// Band items claimed per claim of the band kernel (BM25_BAND_CLAIM overrides).
static int32_t band_claim() {
  const char* e = getenv("BM25_BAND_CLAIM");
  const int v = e ? atoi(e) : 1;
  return v >= 1 && v <= 64 ? v : 1;
}

// The band kernel serves SAMPLE and REST for queries of 1..8 terms
// (BM25_NO_BAND=1 forces the per-tile pipelined kernel).
static bool use_band(const DevIndex& ix, int64_t T) {
  static const bool off = getenv("BM25_NO_BAND") != nullptr;
  return !off && T >= 1 && T <= kBandT && (ix.nnz + kPostingPad) * 4 < 0xFFFFFFF0ll;
}

// The flat kernel replaces the band kernel's tile loop (BM25_FLAT=0: band).
static bool use_flat() {
  static const bool off = getenv("BM25_FLAT") && atoi(getenv("BM25_FLAT")) == 0;
  return !off;
}

// Tiles per flat-kernel item: 8, halved while the phase would give the
// resident waves fewer than BM25_ITEMS_PER_WAVE (8) items each — a small doc
// shard's SAMPLE pass has ~2 eight-tile items per wave, and the last wave's
// items set the pass time (BM25_FLAT_BW forces a width).
static int32_t flat_band(int64_t nt, int64_t nq, int grid) {
  static const int forced = getenv("BM25_FLAT_BW") ? atoi(getenv("BM25_FLAT_BW")) : 0;
  if (forced == 1 || forced == 2 || forced == 4 || forced == 8) return forced;
  static const int64_t per = getenv("BM25_ITEMS_PER_WAVE") ? atoi(getenv("BM25_ITEMS_PER_WAVE")) : 8;
  int32_t bw = 8;
  while (bw > 1 && ((nt + bw - 1) / bw) * nq < per * (int64_t)grid) bw >>= 1;
  return bw;
}

template <int S, int PH, int SM = 1>
static void launch_band(const DevIndex& ix, const int32_t* q, int64_t T, const Stage& sg,
                        const Workspace& ws, hipStream_t st) {
  if constexpr (PH == kSample && SM == 1) {  // m keys per sample tile: a build per m
    if (sg.M == 2) {
      launch_band<S, PH, 2>(ix, q, T, sg, ws, st);
      return;
    }
    if (sg.M == kTileM) {
      launch_band<S, PH, kTileM>(ix, q, T, sg, ws, st);
      return;
    }
  }
  int32_t* wctr = ws.wctr + (int64_t)sg.ctr_region * kWctrInts;
  if (!sg.ctr_zeroed) hipMemsetAsync(wctr, 0, sizeof(int32_t) * kWctrInts, st);
  // REST skips the sample tiles whose best key is below theta (m = 1 samples
  // in groups of one band: ws.cand holds this shard's sample keys)
  const bool skip = PH == kRest && sg.sample_keys != nullptr && sg.M == 1 && sg.G == kBandW;
  IndexArgs a = args_of(ix);
  a.seg = ws.seg;
  if (use_flat()) {
#define BM25_FLAT_LAUNCH(SPV)                                                                     \
  {                                                                                               \
    const int grid = persistent_grid<S, PH>(score_flat_kernel<S, PH, SM, SPV>, 64);               \
    const int64_t nt = PH == kSample ? sample_count(ix.ntiles, sg.P, sg.G) : ix.ntiles;          \
    hipLaunchKernelGGL((score_flat_kernel<S, PH, SM, SPV>), dim3((unsigned)grid), dim3(64), 0, st, \
                       a, q, (int32_t)T, sg.P, sg.G, sg.nq_host, ws.theta, sg.cand_out,           \
                       sg.cstride, ws.list, ws.list_cnt, ws.list_cap, wctr, band_claim(),         \
                       claim_m(), skip ? sg.sample_keys : nullptr, sg.sample_stride,              \
                       flat_band(nt, sg.nq_host, grid));                                          \
  }
    if (ix.sparse)
      BM25_FLAT_LAUNCH(true)
    else
      BM25_FLAT_LAUNCH(false)
#undef BM25_FLAT_LAUNCH
    return;
  }
  if (ix.sparse) {
    const int grid = persistent_grid<S, PH>(score_band_kernel<S, PH, SM, true>, 64 * kBandWaves);
    hipLaunchKernelGGL((score_band_kernel<S, PH, SM, true>), dim3((unsigned)grid),
                       dim3(64 * kBandWaves), 0, st, a, q, (int32_t)T, sg.P, sg.G, sg.nq_host,
                       ws.theta, sg.cand_out, sg.cstride, ws.list, ws.list_cnt, ws.list_cap,
                       wctr, band_claim(), claim_m(), skip ? sg.sample_keys : nullptr,
                       sg.sample_stride);
    return;
  }
  const int grid = persistent_grid<S, PH>(score_band_kernel<S, PH, SM, false>, 64 * kBandWaves);
  hipLaunchKernelGGL((score_band_kernel<S, PH, SM, false>), dim3((unsigned)grid),
                     dim3(64 * kBandWaves), 0, st, a, q, (int32_t)T, sg.P, sg.G, sg.nq_host, ws.theta,
                     sg.cand_out, sg.cstride, ws.list, ws.list_cnt, ws.list_cap, wctr,
                     band_claim(), claim_m(), skip ? sg.sample_keys : nullptr, sg.sample_stride);
}

// Sparse index, band kernel: the segment of every (band item lane = tile li,
// query term lt) of the batch, from the query terms' tile lists — one wave
// per (query, term position) walks its term's non-empty tiles (coalesced
// reads) and writes (start | len << 32) into seg[q][tile / 8][pos][tile % 8]
// (a term's entries of one band are one 64-B run); seg was zeroed (empty
// segments).
__global__ __launch_bounds__(256) void seg_table_kernel(IndexArgs a,
                                                        const int32_t* __restrict__ queries,
                                                        int64_t Q, int32_t T,
                                                        uint64_t* __restrict__ seg) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= Q * T) return;  // wave-uniform; no barriers
  const int64_t q = w / T;
  const int pos = (int)(w - q * T);
  const int32_t term = queries[q * T + pos];
  if (term < 0 || term >= a.V) return;
  const int64_t nbp = (a.ntiles + 7) >> 3;
  const int64_t b = a.tl_ptr[term], e = a.tl_ptr[term + 1];
  const int64_t ip = a.indptr[term];
  const uint32_t df = (uint32_t)(a.indptr[term + 1] - ip);
  uint64_t* row = seg + q * nbp * 64;
  for (int64_t i = b + lane_id(); i < e; i += 64) {
    const uint32_t tile = a.tl_tile[i];
    const uint32_t st = a.tl_start[i];
    const uint32_t nx = i + 1 < e ? a.tl_start[i + 1] : df;
    row[(int64_t)(tile >> 3) * 64 + pos * 8 + (tile & 7)] =
        (uint64_t)(uint32_t)(ip + st) | ((uint64_t)(nx - st) << 32);
  }
}

// Largest token id of a device-resident query batch (bm25_native.py:91,
// queries.max(initial=0)), for the opt-in check of bm25_max_token_device.
__global__ __launch_bounds__(256) void max_token_kernel(const int32_t* __restrict__ q, int64_t n,
                                                        int32_t* __restrict__ out) {
  int32_t m = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = max(m, q[i]);
  m = (int32_t)wave_max_u32((uint32_t)max(m, 0));  // ids >= 0 compare as unsigned
  if (lane_id() == 0 && m > 0) atomicMax(out, m);
}

hipError_t launch_max_token(const int32_t* d_queries, int64_t n, int32_t* d_out,
                            hipStream_t stream) {
  hipMemsetAsync(d_out, 0, sizeof(int32_t), stream);
  if (n > 0) {
    const int64_t blocks = std::min<int64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(max_token_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, d_queries,
                       n, d_out);
  }
  return hipGetLastError();
}

int64_t seg_entries(const DevIndex& ix, int64_t Q) {  // + 64 zero entries past the table
  return ix.sparse ? Q * ((ix.ntiles + 7) >> 3) * 64 + 64 : 0;
}

static void launch_seg_table(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T,
                             const Workspace& ws, hipStream_t st) {
  hipMemsetAsync(ws.seg, 0, sizeof(uint64_t) * seg_entries(ix, Q), st);
  const int64_t waves = Q * T;
  hipLaunchKernelGGL(seg_table_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st,
                     args_of(ix), q, Q, (int32_t)T, ws.seg);
}

template <int S, int PH>
static void launch_wave(const DevIndex& ix, const int32_t* q, int64_t T, const Stage& sg,
                        const Workspace& ws, hipStream_t st) {
  if constexpr (PH != kAll) {
    if (!sg.qmap && use_band(ix, T) &&
        ((ix.ntiles + kBandW - 1) / kBandW) * (int64_t)sg.nq_host < 0x7FFFFFFFll) {
      launch_band<S, PH>(ix, q, T, sg, ws, st);
      return;
    }
  }
  if (use_pipe(ix, T) && ix.ntiles * (int64_t)sg.nq_host < 0x7FFFFFFFll) {
    static const int diag = getenv("BM25_ABLATE") ? atoi(getenv("BM25_ABLATE")) : 0;
    if (sg.qmap)
      launch_pipe<S, PH, true, 0>(ix, q, T, sg, ws, st);
    else if (diag == 0)
      launch_pipe<S, PH, false, 0>(ix, q, T, sg, ws, st);
    else if (diag == 1)
      launch_pipe<S, PH, false, 1>(ix, q, T, sg, ws, st);
    else if (diag == 4)
      launch_pipe<S, PH, false, 4>(ix, q, T, sg, ws, st);
    else if (diag == 5)
      launch_pipe<S, PH, false, 5>(ix, q, T, sg, ws, st);

    else
      launch_pipe<S, PH, false, 32>(ix, q, T, sg, ws, st);
    return;
  }
  const int grid = persistent_grid<S, PH>(score_wave_kernel<S, PH>);
  hipLaunchKernelGGL((score_wave_kernel<S, PH>), dim3((unsigned)grid), dim3(64 * kWaves), 0, st,
                     args_of(ix), q, (int32_t)T, sg, ws.theta, sg.cand_out, ws.list, ws.list_cnt,
                     ws.list_cap);
}

// P > 1: the sampled search (its merge reads the list only: nt = 0);
// P = 1: the exact path over every tile.
static Stage main_stage(const DevIndex& ix, int64_t Q, int P, const Workspace& ws) {
  Stage sg{};
  sg.cand = ws.cand;
  sg.cand_out = ws.cand;
  sg.cstride = ix.ntiles * kTileM;
  sg.P = P;
  sg.G = 1;
  sg.nt = P > 1 ? 0 : ix.ntiles;
  sg.nq_host = (int32_t)Q;
  if (P > 1) {
    sg.theta = ws.theta;
    sg.list = ws.list;
    sg.list_cnt = ws.list_cnt;
    sg.C = ws.list_cap;
    sg.fb = ws.fb;
    sg.fb_cnt = ws.counters + 2;
  }
  return sg;
}

static Stage fallback_stage(const DevIndex& ix, int64_t Q, const Workspace& ws) {
  Stage sg{};
  sg.cand = ws.cand;
  sg.cand_out = ws.cand;
  sg.cstride = ix.ntiles * kTileM;
  sg.P = 1;
  sg.G = 1;
  sg.nt = ix.ntiles;
  sg.qmap = ws.fb;
  sg.nq_dev = ws.counters + 2;
  sg.nq_host = (int32_t)Q;
  return sg;
}

__global__ __launch_bounds__(256) void zero_search_kernel(uint64_t* __restrict__ keys, int64_t nk,
                                                          int32_t* __restrict__ wctr, int64_t nw,
                                                          int32_t* __restrict__ counters,
                                                          int32_t* __restrict__ list_cnt, int64_t Q) {
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
  for (int64_t i = i0; i < nk; i += st) keys[i] = 0ull;
  for (int64_t i = i0; i < nw; i += st) wctr[i] = 0;
  for (int64_t i = i0; i < Q; i += st) list_cnt[i] = 0;
  if (i0 < 4) counters[i0] = 0;
}

// SAMPLE pass: each query's S keys into keys[Q][S] (zero-padded); a copy
// stays in ws.cand for the REST pass's sample-tile skip.
template <int S_>
static void sample_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T,
                     const SampleGeom& g, uint64_t* keys, const Workspace& ws, hipStream_t st) {
  // one launch zeroes everything the search counts into: the sample keys, the
  // claim counters of SAMPLE, REST and the fallback, the rescore/fallback
  // counters and the list counts (each was a memset launch: ~5 us apiece)
  hipLaunchKernelGGL(zero_search_kernel, dim3(64), dim3(256), 0, st, keys, Q * g.S, ws.wctr,
                     (int64_t)kWctrRegions * kWctrInts, ws.counters, ws.list_cnt, Q);
  if (ix.sparse && use_band(ix, T)) launch_seg_table(ix, q, Q, T, ws, st);  // SAMPLE + REST
  Stage sg = main_stage(ix, Q, g.P, ws);
  sg.ctr_region = 0;
  sg.ctr_zeroed = true;
  sg.M = g.m;
  sg.G = g.G;
  sg.cand_out = keys;
  sg.cstride = g.S;
  launch_wave<S_, kSample>(ix, q, T, sg, ws, st);
  if (keys != ws.cand)
    hipMemcpyAsync(ws.cand, keys, sizeof(uint64_t) * Q * g.S, hipMemcpyDeviceToDevice, st);
}

// theta from the W shards' sample keys [W][Q][S], then the REST pass (or, P =
// 1, the exact pass over every tile).
template <int S_>
static void finish_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int k,
                     const SampleGeom& g, int W, const uint64_t* all_keys, const Workspace& ws,
                     hipStream_t st) {
  Stage sg = main_stage(ix, Q, g.P, ws);
  if (g.P == 1) {  // no sample pass ran: nothing was zeroed
    hipMemsetAsync(ws.counters, 0, 4 * sizeof(int32_t), st);
    sg.ctr_region = 2;
    sg.ctr_zeroed = false;
    launch_wave<S_, kAll>(ix, q, T, sg, ws, st);
    return;
  }
  sg.ctr_region = 1;  // counters, list counts and claim counters: zeroed by sample_s
  sg.ctr_zeroed = true;
  sg.M = g.m;
  sg.G = g.G;
  sg.sample_keys = ws.cand;  // launch_sample left this shard's keys there
  sg.sample_stride = g.S;
  hipLaunchKernelGGL(theta_wave_kernel, dim3((unsigned)((Q + 3) / 4)), dim3(256), 0, st, all_keys,
                     (int64_t)W, Q, g.S, (int32_t)k, ws.theta, ws.list_cnt, ws.list_cap,
                     ix.nonneg ? 1 : 0, ix.doc_offset, ix.n_docs);
  launch_wave<S_, kRest>(ix, q, T, sg, ws, st);
}

template <int S_>
static void select_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int k, int P,
                     const Workspace& ws, int32_t* docs, float* scores, hipStream_t st);

#define BM25_SHIFT_DISPATCH(call)                        \
  switch (ix.tile_shift) {                               \
    case 10: call(10); break;                            \
    case 11: call(11); break;                            \
    BM25_CASE12(call)                                    \
    default: return hipErrorInvalidValue;                \
  }

hipError_t launch_sample(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                         const SampleGeom& g, uint64_t* keys, const Workspace& ws,
                         hipStream_t stream) {
  if (Q == 0 || g.P == 1) return hipSuccess;
  if (ix.ntiles == 0) {  // an empty doc shard contributes no keys
    hipMemsetAsync(keys, 0, sizeof(uint64_t) * Q * g.S, stream);
    return hipGetLastError();
  }
#define CALL(s) sample_s<s>(ix, d_queries, Q, T, g, keys, ws, stream)
  BM25_SHIFT_DISPATCH(CALL)
#undef CALL
  return hipGetLastError();
}

hipError_t launch_finish(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                         int k, const SampleGeom& g, int W, const uint64_t* all_keys,
                         const Workspace& ws, hipStream_t stream) {
  if (Q == 0 || ix.ntiles == 0) return hipSuccess;
#define CALL(s) finish_s<s>(ix, d_queries, Q, T, k, g, W, all_keys, ws, stream)
  BM25_SHIFT_DISPATCH(CALL)
#undef CALL
  return hipGetLastError();
}

hipError_t launch_score(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                        int k, const Workspace& ws, hipStream_t stream) {
  const SampleGeom g = sample_geom(ix.ntiles, k, 1);
  hipError_t e = launch_sample(ix, d_queries, Q, T, g, ws.cand, ws, stream);
  if (e != hipSuccess) return e;
  return launch_finish(ix, d_queries, Q, T, k, g, 1, ws.cand, ws, stream);
}

template <int S>
static void select_stage(const DevIndex& ix, const int32_t* q, int64_t T, int k, const Stage& sg,
                         const Workspace& ws, int32_t* docs, float* scores, hipStream_t st) {
  const int64_t maxflag = maxflag_for(k, sg.nt);
  hipLaunchKernelGGL(merge_first_kernel, dim3((unsigned)sg.nq_host), dim3(kMergeNT), 0, st, sg,
                     (int32_t)k, maxflag, ix.doc_offset, ix.n_docs, ws, docs, scores);
  if (k > kTileM && sg.nt > 0) {  // tiles with exact top-4 candidates may need a rescore
    hipLaunchKernelGGL(rescore_kernel<S>, dim3(256), dim3(kRescoreNT), 0, st, args_of(ix), q,
                       (int32_t)T, (int32_t)k, maxflag, sg, ws);
    hipLaunchKernelGGL(merge_final_kernel, dim3((unsigned)sg.nq_host), dim3(kMergeNT), 0, st, sg,
                       (int32_t)k, maxflag, ix.doc_offset, ws, docs, scores);
  }
}

template <int S_>
static void select_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int k, int P,
                     const Workspace& ws, int32_t* docs, float* scores, hipStream_t st) {
  select_stage<S_>(ix, q, T, k, main_stage(ix, Q, P, ws), ws, docs, scores, st);
  if (P == 1) return;
  // queries whose list overflowed: exact pass over every tile (usually none;
  // the kernels read their count on the device and exit at once)
  hipMemsetAsync(ws.counters, 0, 2 * sizeof(int32_t), st);
  Stage fb = fallback_stage(ix, Q, ws);
  fb.ctr_region = 2;  // unused by the sampled search: zeroed by sample_s
  fb.ctr_zeroed = true;
  launch_wave<S_, kAll>(ix, q, T, fb, ws, st);
  select_stage<S_>(ix, q, T, k, fb, ws, docs, scores, st);
}

hipError_t launch_select(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                         int k, int P, const Workspace& ws, int32_t* d_docs, float* d_scores,
                         hipStream_t stream) {
  if (Q == 0 || k == 0) return hipSuccess;
  if (ix.ntiles == 0) {  // an empty doc shard: an all-padding list (doc -1, score bits ~0)
    hipMemsetAsync(d_docs, 0xFF, sizeof(int32_t) * Q * k, stream);
    hipMemsetAsync(d_scores, 0xFF, sizeof(float) * Q * k, stream);
    return hipGetLastError();
  }
#define CALL(s) select_s<s>(ix, d_queries, Q, T, k, P, ws, d_docs, d_scores, stream)
  BM25_SHIFT_DISPATCH(CALL)
#undef CALL
  return hipGetLastError();
}

hipError_t launch_scores_dense(const DevIndex& ix, const int32_t* d_query, int64_t T,
                               float* d_out, hipStream_t stream) {
  if (ix.ntiles == 0) return hipSuccess;
  const dim3 grid((unsigned)ix.ntiles);
  switch (ix.tile_shift) {
    case 10: hipLaunchKernelGGL(scores_dense_kernel<10>, grid, dim3(64), 0, stream, args_of(ix), d_query, (int32_t)T, d_out); break;
#ifdef BM25_S12
    case 12: hipLaunchKernelGGL(scores_dense_kernel<12>, grid, dim3(64), 0, stream, args_of(ix), d_query, (int32_t)T, d_out); break;
#endif
    case 11: hipLaunchKernelGGL(scores_dense_kernel<11>, grid, dim3(64), 0, stream, args_of(ix), d_query, (int32_t)T, d_out); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_merge_lists(const int32_t* d_docs, const float* d_scores, int64_t W,
                              int64_t Q, int k, int64_t rank_stride, bool sorted,
                              int32_t* d_out_docs, float* d_out_scores, hipStream_t stream) {
  if (Q == 0 || k == 0) return hipSuccess;
  if (sorted && W * k <= kMergeSortedCap && W <= 64) {
    hipLaunchKernelGGL(merge_sorted_kernel, dim3((unsigned)((Q + 3) / 4)), dim3(256), 0, stream,
                       d_docs, d_scores, (int32_t)W, Q, (int32_t)k, rank_stride, d_out_docs,
                       d_out_scores);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(merge_lists_kernel, dim3((unsigned)Q), dim3(kMergeNT), 0, stream, d_docs,
                     d_scores, W, Q, (int32_t)k, rank_stride, d_out_docs, d_out_scores);
  return hipGetLastError();
}

}  // namespace bm25mi
