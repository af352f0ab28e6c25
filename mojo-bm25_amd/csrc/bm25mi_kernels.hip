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

constexpr int kJ = 8;       // posting rows (64 postings each) in flight per wave (add_group)
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
  const uint64_t* seg;      // sparse + flat kernel: this search's segment table
  int64_t seg_zero;         // ... index of a zero entry past it
  const uint16_t* bmax;     // dense, non-negative index: f16 upper bound of each (term,
                            // tile)'s largest score ([V][ntiles]; null: no tile bounds)
};

static IndexArgs args_of(const DevIndex& ix) {
  return IndexArgs{ix.indptr, ix.rel, ix.ldoc, ix.val, ix.n_terms, ix.ntiles, ix.n_docs,
                   ix.nnz, ix.doc_offset, ix.nonneg ? 1 : 0, ix.sparse ? 1 : 0, ix.tl_ptr,
                   ix.tl_tile, ix.tl_start, nullptr, 0, ix.opt.tile_bound ? ix.bmax : nullptr};
}

// Segment bounds [r0, r1) (relative to indptr[term]) of a valid term in a
// tile.  Sparse: a binary search of the term's tile list (the cold paths; the
// flat kernel reads a per-search table instead, seg_table_kernel).
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
  uint64_t* cand_mirror;        // SAMPLE (flat, m = 1): a second copy of cand_out's keys (or null)
  int64_t sample_stride;
  const int32_t* qmap;       // stage query -> batch row (null: identity)
  const int32_t* nq_dev;     // stage queries, on the device (null: nq_host)
  int32_t nq_host;           // stage queries (host bound)
  int32_t* fb;               // overflowed queries are appended here
  int32_t* fb_cnt;
  int32_t ctr_region;        // claim counters of the launch: ws.wctr + region * kWctrInts
                             // (zero at launch: each flat launch leaves its region zeroed)
  bool remap;                // merges: qmap gives the batch row of every array (the
                             // main stage's queries left to the block merge)
  bool unsorted;             // merge_fast: a doc shard's list for the W-way merge — its
                             // keys >= the k-th, in no order (padding last): no sort
  bool split;                // REST: over split items (ws.sub, built by bound_keys_kernel)
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

// Sum over each group of 2^TL consecutive lanes (a flat-kernel tile's term
// lanes), every lane of the group getting it: DPP inside 16-lane rows (no LDS
// round trip, unlike __shfl_xor's ds_bpermute), shuffles above.
template <int TL>
__device__ __forceinline__ uint32_t seg_sum_u32(uint32_t v) {
  if (TL >= 1) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
  if (TL >= 2) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
  if (TL >= 3) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  if (TL >= 4) v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  if (TL >= 5) v += (uint32_t)__shfl_xor((int)v, 16, 64);
  if (TL >= 6) v += (uint32_t)__shfl_xor((int)v, 32, 64);
  return v;
}
template <int TL>
__device__ __forceinline__ float seg_sum_f32(float v) {
  if (TL >= 1) v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
  if (TL >= 2) v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));
  if (TL >= 3) v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x141, 0xF, 0xF, false));
  if (TL >= 4) v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x140, 0xF, 0xF, false));
  if (TL >= 5) v += __shfl_xor(v, 16, 64);
  if (TL >= 6) v += __shfl_xor(v, 32, 64);
  return v;
}

// Bitwise OR over the 64 lanes (DPP inside rows, then SGPRs); AND as ~OR(~x).
__device__ __forceinline__ uint32_t wave_or_u32(uint32_t v) {
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad [1,0,3,2]
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad [2,3,0,1]
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  v |= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x140, 0xF, 0xF, false);  // row_mirror
  return (uint32_t)__builtin_amdgcn_readlane((int)v, 0) | (uint32_t)__builtin_amdgcn_readlane((int)v, 16) |
         (uint32_t)__builtin_amdgcn_readlane((int)v, 32) | (uint32_t)__builtin_amdgcn_readlane((int)v, 48);
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
        if (live) lds_add(acc + (dl[j] >> 2), v[j]);
      } else {
        for (int sc = sf[j]; sc <= sl[j]; ++sc)
          if (live && ts[j] == sc) lds_add(acc + (dl[j] >> 2), v[j]);
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

#define BM25_ZA(o) "ds_write_addtid_b32 %2 offset:" #o "\n"
template <int S>
__device__ __forceinline__ void zero_acc(float* acc) {
  if constexpr (S == 12) {  // (variant builds: 4096-doc tiles) as below, 64 stores
    const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)acc;
    uint32_t m0_saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 1\n"
                 BM25_ZA(0) BM25_ZA(256) BM25_ZA(512) BM25_ZA(768) BM25_ZA(1024) BM25_ZA(1280)
                 BM25_ZA(1536) BM25_ZA(1792) BM25_ZA(2048) BM25_ZA(2304) BM25_ZA(2560) BM25_ZA(2816)
                 BM25_ZA(3072) BM25_ZA(3328) BM25_ZA(3584) BM25_ZA(3840) BM25_ZA(4096) BM25_ZA(4352)
                 BM25_ZA(4608) BM25_ZA(4864) BM25_ZA(5120) BM25_ZA(5376) BM25_ZA(5632) BM25_ZA(5888)
                 BM25_ZA(6144) BM25_ZA(6400) BM25_ZA(6656) BM25_ZA(6912) BM25_ZA(7168) BM25_ZA(7424)
                 BM25_ZA(7680) BM25_ZA(7936) BM25_ZA(8192) BM25_ZA(8448) BM25_ZA(8704) BM25_ZA(8960)
                 BM25_ZA(9216) BM25_ZA(9472) BM25_ZA(9728) BM25_ZA(9984) BM25_ZA(10240) BM25_ZA(10496)
                 BM25_ZA(10752) BM25_ZA(11008) BM25_ZA(11264) BM25_ZA(11520) BM25_ZA(11776)
                 BM25_ZA(12032) BM25_ZA(12288) BM25_ZA(12544) BM25_ZA(12800) BM25_ZA(13056)
                 BM25_ZA(13312) BM25_ZA(13568) BM25_ZA(13824) BM25_ZA(14080) BM25_ZA(14336)
                 BM25_ZA(14592) BM25_ZA(14848) BM25_ZA(15104) BM25_ZA(15360) BM25_ZA(15616)
                 BM25_ZA(15872) BM25_ZA(16128)
                 "s_mov_b32 m0, %0\n\ts_nop 1"
                 : "=&s"(m0_saved)
                 : "s"(la), "v"(0.f)
                 : "memory");
    return;
  }
  if constexpr (S == 11) {
    // ds_write_addtid_b32 stores lane l at M0 + offset + 4 l: no address VGPR
    // to move, 2 cycles per 256 B (128 B/clk/CU, vs ~79 for ds_write_b128);
    // clearing the tile is a large part of the flat kernel's LDS time
    const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) float*)acc;
    // M0 is the compiler's (it sets it for its own lane-select uses): saved
    // and restored here.  An M0 write needs a wait state before an
    // instruction reads M0 (without it the first store used a stale M0).
    //
    // Why stores the compiler cannot see are safe here: the LDS executes one
    // wave's LDS instructions in issue order (reads, writes and atomics
    // alike; lgkmcnt only tracks when their results come back), and an LDS
    // write has no result to wait for.  So (1) every LDS read the compiler
    // issued before this block — the epilogue's reads of the tile — reads its
    // data before these stores overwrite it, whether or not its lgkmcnt wait
    // has retired yet, and its returned value is unaffected; (2) every LDS
    // access issued after the block (the next tile's row reads and writes)
    // executes after all 32 stores, so it sees the zeros.  The "memory"
    // clobber keeps the compiler from moving its own LDS accesses across the
    // block.  Nothing else writes this wave's slice: the accumulator is
    // wave-private (no other wave, no barrier).
    uint32_t m0_saved;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 1\n"
                 BM25_ZA(0) BM25_ZA(256) BM25_ZA(512) BM25_ZA(768) BM25_ZA(1024) BM25_ZA(1280)
                 BM25_ZA(1536) BM25_ZA(1792) BM25_ZA(2048) BM25_ZA(2304) BM25_ZA(2560) BM25_ZA(2816)
                 BM25_ZA(3072) BM25_ZA(3328) BM25_ZA(3584) BM25_ZA(3840) BM25_ZA(4096) BM25_ZA(4352)
                 BM25_ZA(4608) BM25_ZA(4864) BM25_ZA(5120) BM25_ZA(5376) BM25_ZA(5632) BM25_ZA(5888)
                 BM25_ZA(6144) BM25_ZA(6400) BM25_ZA(6656) BM25_ZA(6912) BM25_ZA(7168) BM25_ZA(7424)
                 BM25_ZA(7680) BM25_ZA(7936)
                 "s_mov_b32 m0, %0\n\ts_nop 1"
                 : "=&s"(m0_saved)
                 : "s"(la), "v"(0.f)
                 : "memory");
    return;
  }
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
  zero_acc<S>(acc);  // (LDS order: after every read above)
}

// The large-k list path's REST tiles: as emit_rest, but a tile's keys go to
// its own slot of Cb keys (slot_n: how many it has, possibly more than Cb) at
// positions counted inside the tile, so the common case takes no atomic — a
// returning atomic per chunk stalls the wave for the device-scope round trip,
// and at k = 10 000 most tiles list a few keys.  Keys past the slot go to the
// query's overflow list (capacity Co, count ovf_cnt: one atomic per such
// chunk).  slot_pack_kernel (bm25mi_large.hip) gathers slots and overflow
// into the query's list.
template <int S>
__device__ __forceinline__ void emit_rest_slot(float* acc, int64_t tile, int64_t n_docs,
                                               uint64_t theta, uint64_t* __restrict__ slot,
                                               int32_t Cb, int32_t* __restrict__ slot_n,
                                               uint64_t* __restrict__ ovf,
                                               int32_t* __restrict__ ovf_cnt, int32_t Co) {
  constexpr int D = 1 << S;
  float4* a4 = reinterpret_cast<float4*>(acc);
  const uint32_t lane = lane_id();
  const float th = key_score((uint32_t)(theta >> 32));
  const int64_t base = tile << S;
  const int lim = (int)max<int64_t>(-1, min<int64_t>(D, n_docs - base));
  const int tie = (int)max<int64_t>(
      -1, min<int64_t>(D, (int64_t)(0xFFFFFFFFu - (uint32_t)theta) - base + 1));
  int32_t n = 0;  // the tile's keys so far (wave-uniform)
#pragma unroll 1
  for (int j0 = 0; j0 < D / 256; j0 += 2) {
    const float4 f0 = a4[j0 * 64 + lane], f1 = a4[(j0 + 1) * 64 + lane];
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
    if (__ballot(c > 0) == 0) continue;
    const uint32_t incl = wave_incl_scan((uint32_t)c);
    const int32_t tot = (int32_t)__builtin_amdgcn_readlane(incl, 63);
    int pos = n + (int)incl - c;
    const int32_t past = max(n, Cb);  // the first position of this chunk beyond the slot
    int obase = 0;
    if (n + tot > past) {  // (uniform) rare: the slot is full
      if (lane == 0) obase = atomicAdd(ovf_cnt, n + tot - past);
      obase = __shfl(obase, 0, 64) - past;  // overflow index = obase + position
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int d = (int)entry_doc(4 * j0 + e, lane);
      const bool pass = (d < lim) & ((fe[e] > th) | ((fe[e] == th) & (d < tie)));
      if (pass) {
        const uint64_t key = ((uint64_t)score_key(fe[e]) << 32) |
                             (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + d));
        if (pos < Cb) slot[pos] = key;
        else if (obase + pos < Co) ovf[obase + pos] = key;
        ++pos;
      }
    }
    n += tot;
  }
  if (n > 0 && lane == 0) *slot_n = n;
  zero_acc<S>(acc);  // (LDS order: after every read above)
}

// The large-k list path's REST tiles with a crossing list: the row loop has
// recorded (xl, n of them) the slot of a document each time one of its adds
// left its sum at or above theta's score — a document more than once when it
// gets postings after crossing — so only those are tested and keyed, into the
// tile's slot as emit_rest_slot does, instead of a pass over the tile's 2048
// accumulators.  Each entry takes its accumulator by an LDS exchange with -1
// (sums are >= 0 on a non-negative index): only a document's first entry
// gets its sum, the others read -1 and pass nothing.
constexpr int kCrossCap = 256;  // crossing-list entries per wave (512 B of LDS)
template <int S>
__device__ __forceinline__ void emit_cross(float* acc, const uint16_t* xl, int32_t nx,
                                           int64_t tile, int64_t n_docs, uint64_t theta,
                                           uint64_t* __restrict__ slot, int32_t Cb,
                                           int32_t* __restrict__ slot_n,
                                           uint64_t* __restrict__ ovf,
                                           int32_t* __restrict__ ovf_cnt, int32_t Co) {
  constexpr int D = 1 << S;
  const uint32_t lane = lane_id();
  const float th = key_score((uint32_t)(theta >> 32));
  const int64_t base = tile << S;
  const int lim = (int)max<int64_t>(-1, min<int64_t>(D, n_docs - base));
  const int tie = (int)max<int64_t>(
      -1, min<int64_t>(D, (int64_t)(0xFFFFFFFFu - (uint32_t)theta) - base + 1));
  int32_t n = 0;
  for (int32_t i0 = 0; i0 < nx; i0 += 64) {
    const int32_t i = i0 + (int32_t)lane;
    const uint32_t off = i < nx ? (uint32_t)xl[i] : 0u;
    const int d = (int)(off >> 2);
    const float f = i < nx ? atomicExch(&acc[d], -1.0f) : -1.0f;  // (first entry: the sum)
    const bool pass = i < nx && f >= 0.f && d < lim && ((f > th) | ((f == th) & (d < tie)));
    const uint64_t m = __ballot(pass);
    if (m == 0ull) continue;
    const int32_t tot = (int32_t)__popcll(m);
    const int pos = n + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                     __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const int32_t past = max(n, Cb);
    int obase = 0;
    if (n + tot > past) {  // (uniform) rare: the slot is full
      if (lane == 0) obase = atomicAdd(ovf_cnt, n + tot - past);
      obase = __shfl(obase, 0, 64) - past;
    }
    if (pass) {
      const uint64_t key = ((uint64_t)score_key(f) << 32) |
                           (uint64_t)(0xFFFFFFFFu - (uint32_t)(base + d));
      if (pos < Cb) slot[pos] = key;
      else if (obase + pos < Co) ovf[obase + pos] = key;
    }
    n += tot;
  }
  if (n > 0 && lane == 0) *slot_n = n;
  zero_acc<S>(acc);  // (LDS order: after every read above)
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
// The flat kernel's row loads as STRUCTURED buffer loads: records of one
// lane's pair (4 B of ldoc, 8 B of val), the record index in a VGPR, the
// row's first pair as soffset (outside the range check).  One clamped index
// then serves both loads: lanes past the row's last valid one reload that
// lane's pair, so a short segment's row touches no cache line of its
// neighbours (the struct form has no builtin: the intrinsic by name).
typedef uint32_t bm25_v2u __attribute__((ext_vector_type(2)));
__device__ uint32_t bm25_sload_b32(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset,
                                   int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.i32");
__device__ bm25_v2u bm25_sload_b64(__amdgpu_buffer_rsrc_t r, int vindex, int voffset, int soffset,
                                   int aux) __asm("llvm.amdgcn.struct.ptr.buffer.load.v2i32");

__device__ __forceinline__ PostingRsrc posting_rsrc_pairs(const IndexArgs& a) {
  PostingRsrc r;
  // num_records = whole pairs (a row's clamped index stays below its row's
  // last posting, so below this); stride 4 B (two u16 slots) / 8 B (two f32)
  const int np2 = (int)((a.nnz + kPostingPad) >> 1);
  r.ldoc = __builtin_amdgcn_make_buffer_rsrc((void*)a.ldoc, 4, np2, 0x00020000);
  r.val = __builtin_amdgcn_make_buffer_rsrc((void*)a.val, 8, np2, 0x00020000);
  return r;
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

// M keys per tile on a non-negative index (the flat kernel's SAMPLE epilogue,
// M > 1): each slice's best sum (a float max: sums >= 0 compare as their bit
// patterns), keyed with the slice's last document — a key <= its best
// document's own, so k keys still bound the k-th best from below, as
// SM == 1's running maximum.  One slice at a time, no second read: a few
// registers live (best_dense holds 2 M across the tile).
template <int S, int M>
__device__ __forceinline__ void best_slices_pos(float* acc, int64_t tile, int64_t n_docs,
                                                uint32_t idoff, uint64_t* __restrict__ out) {
  constexpr int per = (1 << S) / 256 / M;  // float4 groups per lane and slice
  static_assert(per >= 1, "a slice holds at least one float4 per lane");
  const float4* a4 = reinterpret_cast<const float4*>(acc);
  const uint32_t lane = lane_id();
  const int64_t base = tile << S;
#pragma unroll
  for (int i = 0; i < M; ++i) {
    float m = 0.f;
#pragma unroll
    for (int jj = 0; jj < per; ++jj) {
      const float4 f = a4[(i * per + jj) * 64 + lane];
      m = fmaxf(m, fmaxf(fmaxf(f.x, f.y), fmaxf(f.z, f.w)));
    }
    const uint32_t wm = wave_max_u32(__float_as_uint(m));
    const int64_t last = min<int64_t>(base + (int64_t)(i + 1) * per * 256 - 1, n_docs - 1);
    const uint64_t key = wm == 0u ? 0ull
                         : ((uint64_t)score_key(__uint_as_float(wm)) << 32) |
                               (uint64_t)(0xFFFFFFFFu - (uint32_t)last - idoff);
    if (lane == (uint32_t)i) out[i] = key;
  }
  zero_acc<S>(acc);  // (LDS order: after every read above)
}

// One key per tile, positive sums only (the flat kernel's SAMPLE epilogue):
// the tile's best score by a float max over each lane's entries (sums >= 0
// compare as their bit patterns), then the smallest doc holding it from a
// second read; the accumulators are cleared.  Same key as best_dense<S, 1,
// true>, about half its VALU work.
template <int S>
__device__ __forceinline__ void best1_pos(float* acc, int64_t tile, uint32_t idoff,
                                          uint64_t* __restrict__ out, uint64_t* mirror) {
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
  if (lane == 1 && mirror) *mirror = key;
}
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
// ===========================================================================
// Flat score kernel (queries of 1..64 terms; SAMPLE, REST and ALL).
// DESIGN.md §4.
//
// Items: (query, band of up to BW consecutive phase tiles), claimed per XCD.
// An item's 64 lanes describe its (tile, term) posting segments, lane =
// tile * 2^TL + term: TL = 3 (T <= 8, up to 8 tiles per item), 4 (T <= 16,
// 4 tiles), 5 (T <= 32, 2 tiles), 6 (T <= 64, 1 tile).  The wave streams the
// posting rows of all its items as ONE sequence that ignores tile and item
// boundaries:
//   * an item's rows (double rows, each inside one (tile, term) segment;
//     tile-major, query-term order inside a tile) are numbered once per item
//     by a scan over its 64 segments; a CHUNK of up to 64 rows is one table,
//     lane r = row r (flat_chunk: a binary search of the scan);
//   * a ring of kFR rows is in flight: the step that adds row r issues row
//     r + kFR into the registers row r freed, so loads never pause at a tile
//     or item edge and every step issues the same loads (static vmcnt);
//   * a row of another tile than the accumulator's runs that tile's epilogue
//     (REST: the keys >= theta, or a plain clear when no add reached theta;
//     SAMPLE: the tile's best key per slice; ALL: the tile's exact top-4).
// Each doc's adds stay in query-term order (bm25_native.py:152).
// ===========================================================================
// wavefronts per workgroup of the one-wave-per-query kernels (theta_wave,
// merge_fast, merge_sorted); measured: one-wave workgroups change nothing
// (profiles/r04/rejected/qw1_*)
#ifndef BM25_QW
#define BM25_QW 4
#endif
constexpr int kQW = BM25_QW;
#ifndef BM25_FR    // rows in flight (ring slots): REST / ALL, SAMPLE
#define BM25_FR 10
#endif
#ifndef BM25_FR_S
#define BM25_FR_S 8
#endif

#ifndef BM25_FLAT_WPE
#define BM25_FLAT_WPE 5
#endif

#ifndef BM25_CLAMP  // row loads of idle lanes kept inside the row's valid lanes: 2 by
#define BM25_CLAMP 2  // a record index (one VALU min), 1 by byte offsets, 0 not at all
#endif

#ifndef BM25_TRACE  // dev variant builds: per-wave start / end clocks of the REST pass
#define BM25_TRACE 0
#endif
#if BM25_TRACE
constexpr int kTraceWaves = 1 << 14;
__device__ uint64_t g_bm25_trace[4 * kTraceWaves];  // (start, end, items, rows) per wave
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

struct FlatCur {    // XCD-relative item ordinal, its claim's end, first phase tile, stage
  int32_t rit, end, b, q, qb, bw;  // query, batch row, tiles
};

struct FlatDesc {   // lane tile * 2^TL + term: the term's segment in the tile (raw; r1 == r0: none)
  uint32_t ip, r0, r1;
  uint32_t aux;     // REST, one of (the launch never asks for both):
                    //   tile bounds: f16 bits of an upper bound of the term's scores in
                    //     the tile (one step above bmax; 0 outside the item)
                    //   sample skip: score-key half of the tile's best sample key
};

// f16 bits (of build_bmax_kernel's table) -> float.
__device__ __forceinline__ float f16_bits_to_float(uint16_t h) {
  _Float16 x;
  __builtin_memcpy(&x, &h, 2);
  return (float)x;
}

// Row word of the process side: the row's valid positions [lo, hi) of its
// 128 (position p = lane p / 2, slot p % 2) as lane ranges — slot 0: lanes
// [lo, lo + n0), slot 1: lanes [0, n1) — and whether the row starts a tile
// (and which tile of its item).
constexpr uint32_t kRowNewTile = 1u << 17;
constexpr uint32_t kRowParity = 1u << 24;    // the item's context slot (ctxV lanes 4 * parity ..)
constexpr uint32_t kRowDead = 1u << 25;      // past the wave's last item
__device__ __forceinline__ uint32_t row_lo(uint32_t w) { return w & 1u; }
__device__ __forceinline__ uint32_t row_n0(uint32_t w) { return (w >> 1) & 0xFFu; }
__device__ __forceinline__ uint32_t row_n1(uint32_t w) { return (w >> 9) & 0xFFu; }
__device__ __forceinline__ uint32_t row_tile(uint32_t w) { return (w >> 18) & 0x3Fu; }

struct FlatTab {    // one chunk of an item's rows: lane r = row j0 + r
  uint32_t base;    // ldoc byte offset of the row's first pair (2 x an even posting index; 0: dead row)
  uint32_t w;       // row word (above); 0: padding row
  uint32_t last;    // (uniform) tile index of the chunk's row 63 (the next chunk's predecessor)
};

struct FlatCtx {    // the item the accumulator's tile belongs to
  int32_t q, b;
  uint64_t th;
};

// Rows [j0, j0 + 64) of an item whose segment lane s holds segment
// [sb, sb + sl), rows [excl, incl) of the item; prev = tile index of row
// j0 - 1 (kNoTile at the item's first chunk: its first row starts a tile);
// par = the item's context slot.
constexpr uint32_t kNoTile = 0xFFFFFFFFu;
template <int TL>
__device__ __forceinline__ FlatTab flat_chunk(uint32_t sb, uint32_t sl, uint32_t incl,
                                              uint32_t excl, uint32_t total, uint32_t j0,
                                              uint32_t prev, uint32_t par) {
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
  t.base = (in && l != 0u) ? ((b & ~1u) + 128u * k) * 2u : 0u;
  // row positions p of the segment: p + base in [b, b + l)
  const uint32_t rlo = k == 0u ? (b & 1u) : 0u;
  const uint32_t rhi = min(128u, (b & 1u) + l - 128u * k);
  // slot 0 of lane l holds position 2l: valid for lanes [rlo, ceil(rhi / 2));
  // slot 1 holds 2l + 1: lanes [0, floor(rhi / 2))
  const uint32_t masks = (in && l != 0u) ? (rlo | ((((rhi + 1u) >> 1) - rlo) << 1) | ((rhi >> 1) << 9))
                                         : 0u;
  const uint32_t tile = (uint32_t)pos >> TL;
  uint32_t tp = (uint32_t)__shfl_up((int)tile, 1, 64);
  if (lane == 0u) tp = prev;
  // bits 26-31: the row's last lane with a valid slot (top - 1; 0 for empty rows)
  const uint32_t top1 = masks != 0u ? (((rhi + 1u) >> 1) - 1u) : 0u;
  t.w = masks | ((in && tile != tp) ? kRowNewTile : 0u) | (tile << 18) | (par ? kRowParity : 0u) |
        (top1 << 26);
  t.last = lane_u32(tile, 63);
  return t;
}

// Term lanes (log2) of a query width T in 1..64.
__host__ __device__ inline int flat_tl(int64_t T) {
  return T <= 8 ? 3 : (T <= 16 ? 4 : (T <= 32 ? 5 : 6));
}

template <int S, int PH, int SM, bool SP, int TL>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(BM25_FLAT_WPE, BM25_FLAT_WPE))) void score_flat_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, int32_t P, int32_t G,
    int32_t nq_host, const int32_t* __restrict__ nq_dev, const int32_t* __restrict__ qmap,
    const uint64_t* __restrict__ theta, uint64_t* __restrict__ cand, int64_t cstride,
    uint64_t* __restrict__ list, int32_t* __restrict__ list_cnt, int32_t C,
    int32_t* __restrict__ wctr, int32_t claim_ch, int32_t claim_m,
    const uint64_t* __restrict__ skeys, int64_t sstride, int32_t BW, uint64_t* mirror,
    int32_t* __restrict__ stats, int32_t* __restrict__ slot_cnt,
    const uint32_t* __restrict__ sub, const int32_t* __restrict__ sub_ipb) {
  constexpr int D = 1 << S;
  // REST over split items (SM == kSplitM): the per-search table `sub` gives
  // each of a band's *sub_ipb items its query, first tile and width — a heavy
  // query's band in 2..8 sub-items (bound_keys_kernel builds it), so the last
  // items a wave claims are short and the waves end together
  constexpr bool kSplit = PH == kRest && SM == kSplitM;
  constexpr int kFR = PH == kSample ? BM25_FR_S : BM25_FR;  // ring slots (>= 2)
  constexpr uint32_t TT = 1u << TL;                          // term lanes per tile
  constexpr uint32_t kTileMask = (64u >> TL) - 1u;           // tile of a segment lane
  __shared__ __attribute__((aligned(16))) float acc[D + 64];
  // the large-k list path's REST: the tile's crossing list (emit_cross)
  constexpr bool kCross = PH == kRest && SM == kLargeM;
  __shared__ uint16_t xl[kCross ? kCrossCap : 1];
  const uint32_t lane = lane_id();
  // byte offset of this lane's trash slot: it holds -inf, so a masked lane
  // needs no masked score (-inf + any finite score = -inf) and never raises
  // the tile's running maximum
  const uint32_t trash = ((uint32_t)D + lane) * 4u;
  // stage queries: the fallback stage (ALL) reads its count on the device
  const int32_t nq = (PH == kAll && nq_dev) ? uniform(*nq_dev) : nq_host;
  const int32_t nt = PH == kSample ? (int32_t)sample_count(a.ntiles, P, G) : (int32_t)a.ntiles;
  const int32_t nb = (nt + BW - 1) / BW;  // items: (query, BW consecutive phase tiles)
  const int32_t ipb = kSplit ? uniform(*sub_ipb) : nq;  // items per band
  const int64_t nitems = (int64_t)nb * ipb;
  const int64_t per = (nitems + 7) >> 3;
  const int grp = (int)(blockIdx.x & 7);
  const uint32_t lo = (uint32_t)(grp * per);
  const int32_t ngi = (int32_t)max<int64_t>(0, min<int64_t>(nitems, lo + per) - lo);
  if (ngi == 0) return;  // wave-uniform; no barriers in this kernel (no claims made)
  const int32_t cm = (int32_t)(blockIdx.x >> 3) % claim_m;
  int32_t* ctr = wctr + (grp * kClaimM + cm) * kCtrStride;
  // the last of the waves sharing a claim counter to finish resets it (and its
  // finished count, on a line of its own) for the next launch on the region:
  // no zeroing launch per search, and ~150 arrivals per count, not the grid's
  auto finish = [&]() {
    const int32_t g8 = (int32_t)(gridDim.x >> 3);
    const int32_t sharers = g8 / claim_m + (cm < g8 % claim_m ? 1 : 0);
    int32_t old = 0;
    if (lane == 0) old = atomicAdd(ctr + kDoneOff, 1);
    if (uniform(old) == sharers - 1 && lane == 0) {
      ctr[0] = 0;
      ctr[kDoneOff] = 0;
    }
  };
#if BM25_CLAMP == 2
  const PostingRsrc pr = posting_rsrc_pairs(a);
#else
  const PostingRsrc pr = posting_rsrc(a);
#endif
#if BM25_TRACE
  const uint64_t tr_t0 = wall_clock64();
  uint32_t tr_items = 0, tr_rows = 0;
#endif
  const uint32_t lt = lane & (TT - 1u), li = lane >> TL;  // segment lane: tile li, term lt
  const int64_t nbp = (a.ntiles + 7) >> 3;                // 8-tile groups of the sparse seg rows

  // split items: ordinal -> (band, table entry: query | first tile << 20 |
  // tiles << 26)
  auto dec = [&](FlatCur& c, uint32_t it) {
    const uint32_t band = it / (uint32_t)ipb;
    const uint32_t e = uniform((int)sub[it - band * (uint32_t)ipb]);
    c.q = (int32_t)(e & 0xFFFFFu);
    c.qb = c.q;
    c.b = (int32_t)(band * (uint32_t)BW + ((e >> 20) & 63u));
    c.bw = min((int32_t)(e >> 26), nt - c.b);
  };
  // ---- items: claims, terms -> segment descriptors
  auto claim = [&]() -> int32_t {
    int32_t v = 0;
    if (lane == 0) v = atomicAdd(ctr, 1);
    return v;
  };
  int32_t pending = claim();
  // batch row of a stage query (ALL: the fallback stage's qmap)
  auto batch_row = [&](int32_t q) -> int32_t {
    return (PH == kAll && qmap) ? uniform(qmap[q]) : q;
  };
  auto next = [&](FlatCur c) -> FlatCur {
    if (c.rit >= ngi) return c;
    if (c.rit + 1 < c.end) {
      ++c.rit;
      if constexpr (kSplit) {
        dec(c, lo + (uint32_t)c.rit);
        return c;
      }
      if (++c.q == nq) {
        c.q = 0;
        c.b += BW;
        c.bw = min(BW, nt - c.b);
      }
      c.qb = batch_row(c.q);
      return c;
    }
    const int64_t bb = ((int64_t)uniform(pending) * claim_m + cm) * claim_ch;
    if (bb >= ngi) {
      c.rit = c.end = ngi;
      return c;
    }
    pending = claim();
    FlatCur n;
    n.rit = (int32_t)bb;
    n.end = (int32_t)min<int64_t>(ngi, bb + claim_ch);
    const uint32_t it = lo + (uint32_t)bb;
    if constexpr (kSplit) {
      dec(n, it);
      return n;
    }
    const uint32_t band = it / (uint32_t)nq;
    n.q = (int32_t)(it - band * (uint32_t)nq);
    n.qb = batch_row(n.q);
    n.b = (int32_t)band * BW;
    n.bw = min(BW, nt - n.b);
    return n;
  };
  auto terms_of = [&](const FlatCur& c) -> int32_t {
    return queries[(int64_t)c.qb * T + (int)min(lt, (uint32_t)(T - 1))];
  };
  // REST: sample tiles (groups of G = kSampleGroup tiles, one group per G * P)
  // whose best sample key is below theta are skipped
  const bool skipping = PH == kRest && skeys != nullptr && G == kSampleGroup && a.bmax == nullptr;
  const uint32_t lgG = (uint32_t)__builtin_ctz((unsigned)G), lgP = (uint32_t)__builtin_ctz((unsigned)P);
  // an item's segment descriptors (4 VGPRs: a lane outside the item reads its
  // r1 from r0's address, so r1 - r0 = 0 needs no flag; the sample-tile test
  // is redone from the item cursor at enter_item)
  auto load_bdesc = [&](const FlatCur& c, int32_t tm) -> FlatDesc {
    FlatDesc d;
    const int32_t term = tm;
    const bool ok = (int)lt < T && (int)li < c.bw && term >= 0 && term < a.V;
    const int64_t tt = ok ? term : 0;
    const int64_t tile = ok ? (int64_t)tile_of32<PH>((uint32_t)(c.b + li), (uint32_t)P,
                                                      (uint32_t)G)
                            : 0;
    if constexpr (SP) {  // outside the item: the zero entry past the table
      const uint64_t e = a.seg[ok ? ((int64_t)c.qb * nbp + (tile >> 3)) * (8 * TT) + lt * 8 + (tile & 7)
                                  : a.seg_zero];
      d.ip = 0u;
      d.r0 = (uint32_t)e;
      d.r1 = (uint32_t)e + (uint32_t)(e >> 32);
    } else {
      const uint32_t* r = a.rel + tt * (a.ntiles + 1) + tile;
      d.ip = (uint32_t)a.indptr[tt];
      d.r0 = r[0];
      d.r1 = *(ok ? r + 1 : r);
    }
    d.aux = 0u;
    if (PH == kRest && a.bmax != nullptr) {  // > the term's largest score in the tile: one
      // f16 step above its rounded-down maximum
      if (ok) d.aux = (uint32_t)a.bmax[tt * bmax_stride(a.ntiles) + tile] + 1u;
    } else if (skipping) {  // the score-key half of this tile's best sample key
      // G and P are powers of two (sample_geom): shifts, no integer division
      const uint32_t t32 = (uint32_t)tile;
      const int64_t si = (int64_t)(((t32 >> (lgG + lgP)) << lgG) | (t32 & (uint32_t)(G - 1)));
      d.aux = reinterpret_cast<const uint32_t*>(skeys)[2 * ((int64_t)c.q * sstride +
                                                              min<int64_t>(si, sstride - 1)) + 1];
    }
    return d;
  };
  auto th_positive = [&](uint64_t th) -> bool {
    return (uint32_t)(th >> 32) > score_key(0.f);
  };

  uint32_t nbound = 0;  // REST: (query, tile) pairs this lane's tiles skipped by their bound
  // ... and the postings of this lane's skipped segments.  Both only in the
  // REST build of the count_skips option (SM == 2): the two live registers
  // cost the pass 13 % on an 8-way doc shard (profiles/r05/counters)
  constexpr bool kCountPost = PH == kRest && SM == 2;
  uint32_t npost = 0;
  // ---- the issue side's item: its segments (lane s = tile * TT + term) and
  // row numbering; the item prefetch pipeline one and two items ahead
  uint32_t iSb = 0, iSl = 0, iIncl = 0, iExcl = 0;
  uint32_t iTotal = 0, iR = 0, iJ0 = 0, iPrev = kNoTile, iCur = 0;
  int32_t ctxV = 0, iPar = 0;  // iPar: the context slot the next item takes
  FlatCur nx, nx2;
  FlatDesc dN;
  uint64_t thN = 0ull;
  int32_t tmN2 = 0;
  // enter item nx (descriptors dN) on the issue side; advance the prefetch
  auto enter_item = [&]() {
#if BM25_TRACE
    ++tr_items;
#endif
    const bool th_pos = PH == kRest && th_positive(thN);
    const uint32_t t32 = (uint32_t)nx.b + li;  // REST: phase tile = tile
    const bool smp = skipping && ((t32 >> lgG) & (uint32_t)(P - 1)) == 0u;
    bool skip = smp && th_pos && dN.aux < (uint32_t)(thN >> 32);
    if constexpr (PH == kRest) {
      // tile bound: no doc of the tile can reach theta when the sum of its
      // query terms' largest scores in the tile (every term lane of the tile,
      // duplicates included) is below theta's score.  fp32 addition is
      // monotone, so the query-order sum of a doc's scores is at most the sum
      // of these maxima; the 1e-4 margin covers this tree-order sum's own
      // rounding.  The tile runs no rows and no epilogue.
      if (a.bmax != nullptr && th_pos) {
        const float ub = seg_sum_f32<TL>(f16_bits_to_float((uint16_t)dN.aux));
        const bool cut = ub * 1.0001f < key_score((uint32_t)(thN >> 32));
        // ... the tile's postings (lanes outside the item hold r1 == r0), counted
        // with the pair by the tile's first term lane (the count_skips build)
        const uint32_t tp = kCountPost ? seg_sum_u32<TL>(dN.r1 - dN.r0) : 0u;
        if (kCountPost && cut && !skip && lt == 0u && (int)li < nx.bw) {
          ++nbound;
          npost += tp;
        }
        skip = skip || cut;
      }
    }
    iSb = dN.ip + dN.r0;
    iSl = skip ? 0u : dN.r1 - dN.r0;
    uint32_t nr = iSl == 0u ? 0u : ((iSb & 1u) + iSl + 127u) >> 7;
    // every tile of the item runs its epilogue (one row, possibly empty, in
    // each tile): ALL, and REST without a positive threshold
    if ((PH == kAll || (PH == kRest && !th_pos)) && lt == 0u && (int)li < nx.bw)
      nr = max(nr, 1u);
    if constexpr (PH == kSample) {
      // a sample tile of the item without any posting row runs no epilogue:
      // its keys are written here (0: no positive sum)
      const uint32_t tr = seg_sum_u32<TL>(nr);
      if (lt == 0u && (int)li < nx.bw && tr == 0u) {
        uint64_t* out = cand + (int64_t)nx.q * cstride + (int64_t)(nx.b + (int32_t)li) * SM;
#pragma unroll
        for (int i = 0; i < SM; ++i) out[i] = 0ull;
        if (SM == 1 && mirror) mirror[out - cand] = 0ull;
      }
    }
    iIncl = scan64(nr);
    iExcl = iIncl - nr;
    iTotal = lane_u32(iIncl, 63);
    uint32_t R = max(iTotal, (uint32_t)kFR);
    if ((R & 63u) != 0u && (R & 63u) < (uint32_t)kFR) R += (uint32_t)kFR - (R & 63u);
    iR = R;
    iJ0 = 0;
    iPrev = kNoTile;  // the item's first row starts a tile
    // the item's context for the process side: lanes 4 * parity + (q, b,
    // theta lo, theta hi) of ctxV (items hold >= kFR rows, so at most two are
    // between the process and the issue side)
    {
      const int32_t c4 = (int32_t)lane - 4 * iPar;
      ctxV = c4 == 0 ? nx.q : c4 == 1 ? nx.b : c4 == 2 ? (int32_t)(uint32_t)thN
           : c4 == 3 ? (int32_t)(uint32_t)(thN >> 32) : ctxV;
    }
    iCur = (uint32_t)iPar;
    iPar ^= 1;
    // prefetch: descriptors of the item after, terms of the one after that
    FlatCur nx3 = next(nx2);
    dN = load_bdesc(nx2, tmN2);
    thN = PH == kRest ? theta[nx2.q] : 0ull;
    tmN2 = terms_of(nx3);
    nx = nx2;
    nx2 = nx3;
  };

  FlatCur c0;
  c0.rit = -1;
  c0.end = 0;
  c0.b = c0.q = c0.qb = 0;
  c0.bw = 1;
  nx = next(c0);
  if (nx.rit >= ngi) {
    // (its claim returned: next() read it, so the count is final)
    finish();
    return;
  }
  dN = load_bdesc(nx, terms_of(nx));
  thN = PH == kRest ? theta[nx.q] : 0ull;
  nx2 = next(nx);
  tmN2 = terms_of(nx2);
  for (int j = 0; j < D / 256; ++j)
    reinterpret_cast<float4*>(acc)[j * 64 + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
  acc[D + lane] = -__builtin_inff();

  // issue table: the chunk the next issued row comes from
  bool items_left = true;
  FlatTab tI;
  uint32_t nI = 0, il = 0;
  auto next_chunk = [&]() {  // tI <- the chunk after it (or the dead tail)
    if (iJ0 + 64u < iR) {
      iJ0 += 64u;
      iPrev = tI.last;
    } else if (items_left && nx.rit < ngi) {
      enter_item();
    } else {
      items_left = false;
      tI.base = 0u;
      tI.w = kRowDead;
      nI = 0x7FFFFFFFu;
      il = 0;
      return;
    }
    tI = flat_chunk<TL>(iSb, iSl, iIncl, iExcl, iTotal, iJ0, iPrev, iCur);
    nI = min(64u, iR - iJ0);
    il = 0;
  };
  enter_item();
  tI = flat_chunk<TL>(iSb, iSl, iIncl, iExcl, iTotal, 0u, iPrev, iCur);
  nI = min(64u, iR);
  il = 0;

  // ring: slot s holds the raw loads and the row word of rows r == s (mod kFR)
  uint32_t ldR[kFR], wR[kFR];
  float v0R[kFR], v1R[kFR];
  auto issue = [&](int s) {
    if (il == nI) next_chunk();
    const uint32_t base = lane_u32(tI.base, (int)il);
    wR[s] = lane_u32(tI.w, (int)il);
#if BM25_CLAMP == 2
    const int li2 = (int)min(lane, wR[s] >> 26);  // (row word bits 26-31: top - 1)
    ldR[s] = bm25_sload_b32(pr.ldoc, li2, 0, (int)base, 0);
    const bm25_v2u v = bm25_sload_b64(pr.val, li2, 0, (int)(base * 2u), 0);
    v0R[s] = __uint_as_float(v[0]);
    v1R[s] = __uint_as_float(v[1]);
#else
#if BM25_CLAMP
    // lanes past the row's last valid one load that lane's pair again: the
    // row touches no cache line beyond its segment's (a short segment's row
    // would otherwise pull in 768 B of other segments' postings)
    const uint32_t wv = wR[s];
    const uint32_t top = max(row_lo(wv) + row_n0(wv), row_n1(wv));
    const uint32_t t4 = (top > 0u ? top - 1u : 0u) * 4u;
    const uint32_t lo4 = min(lane * 4u, t4), lo8 = min(lane * 8u, 2u * t4);
#else
    const uint32_t lo4 = lane * 4u, lo8 = lane * 8u;
#endif
    ldR[s] = __builtin_amdgcn_raw_buffer_load_b32(pr.ldoc, (int)lo4, (int)base, 0);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(pr.val, (int)lo8, (int)(base * 2u), 0);
    v0R[s] = __uint_as_float((uint32_t)v[0]);
    v1R[s] = __uint_as_float((uint32_t)v[1]);
#endif
    ++il;
  };
#pragma unroll
  for (int s = 0; s < kFR; ++s) issue(s);  // the first chunk holds >= kFR rows

  // process side
  FlatCtx ctxE{0, 0, 0ull};
  uint32_t curTi = kNoTile;  // the accumulator's tile (index in item ctxE), kNoTile: none
  // REST and SAMPLE: the running maximum of the tile's sums (each doc's
  // running sums only grow on a non-negative index, so it is the tile's best
  // sum; REST: the tile holds a key >= theta only if this reaches theta's score)
  float hmax = 0.f;
  bool done = false;
  // kCross: theta's score for the tile's query, and the tile's crossings
  // (past kCrossCap, or a threshold that is not positive: the epilogue scans
  // the whole tile)
  float thS = 0.f;
  int32_t ncross = 0;

  auto epilogue = [&]() {
    const int32_t ti = ctxE.b + (int32_t)curTi;
    const int64_t tile = tile_of32<PH>((uint32_t)ti, (uint32_t)P, (uint32_t)G);
    if constexpr (kCross) {  // the large-k list path: per-tile slots
      const int64_t si = (int64_t)ctxE.q * a.ntiles + tile;
      if (ncross == 0)
        zero_acc<S>(acc);
      else if (ncross <= kCrossCap)
        emit_cross<S>(acc, xl, ncross, tile, a.n_docs, ctxE.th, cand + si * cstride,
                      (int32_t)cstride, slot_cnt + si, list + (int64_t)ctxE.q * C,
                      list_cnt + ctxE.q, C);
      else
        emit_rest_slot<S>(acc, tile, a.n_docs, ctxE.th, cand + si * cstride, (int32_t)cstride,
                          slot_cnt + si, list + (int64_t)ctxE.q * C, list_cnt + ctxE.q, C);
    } else if constexpr (PH == kRest) {
      const bool flagged = a.nonneg && th_positive(ctxE.th);
      if (flagged && __ballot(hmax >= key_score((uint32_t)(ctxE.th >> 32))) == 0) {
        zero_acc<S>(acc);
      } else {
        emit_rest<S>(acc, tile, a.n_docs, ctxE.th, list + (int64_t)ctxE.q * C,
                     list_cnt + ctxE.q, C);
      }
      hmax = 0.f;
    } else if constexpr (PH == kAll) {
      select_top_lds<S>(acc, tile, a.n_docs, kTileM, cand + (int64_t)ctxE.q * cstride + tile * kTileM);
    } else {
      uint64_t* out = cand + (int64_t)ctxE.q * cstride + (int64_t)ti * SM;
      if constexpr (SM == 1) {
        if (a.nonneg) {
          // running sums only grow on a non-negative index: the tile's best
          // sum is the running maximum, no pass over the accumulator.  Its
          // key takes the tile's last doc (a key <= the best doc's own), so
          // k real keys still reach theta
          const uint32_t wm = wave_max_u32(__float_as_uint(hmax));
          const uint32_t last = (uint32_t)min<int64_t>((tile << S) + D - 1, a.n_docs - 1);
          const uint64_t key = wm == 0u ? 0ull
                               : ((uint64_t)score_key(__uint_as_float(wm)) << 32) |
                                     (uint64_t)(0xFFFFFFFFu - last - (uint32_t)a.doc_offset);
          zero_acc<S>(acc);
          if (lane == 0) *out = key;
          if (lane == 1 && mirror) mirror[out - cand] = key;
          hmax = 0.f;
        } else {
          best1_pos<S>(acc, tile, (uint32_t)a.doc_offset, out, mirror ? mirror + (out - cand) : nullptr);
        }
      } else if (SM == kLargeM || a.nonneg) {  // (the large-k list path: non-negative only)
        best_slices_pos<S, SM>(acc, tile, a.n_docs, (uint32_t)a.doc_offset, out);
      } else {
        best_dense<S, SM, true>(acc, tile, a.n_docs, (uint32_t)a.doc_offset, out);
      }
    }
  };

  // the current row (its slot already consumed): masked slot byte offsets
  // and scores, the accumulator values read one step early, its row word
  uint32_t sc0, sc1, wC;
  float ac0, ac1, xc0, xc1;
  auto lds_at = [&](uint32_t off) -> float& {
    return *reinterpret_cast<float*>(reinterpret_cast<char*>(acc) + off);
  };
  auto prepare = [&](int s) {  // the row of slot s
    wC = wR[s];
    const bool m0 = lane - row_lo(wC) < row_n0(wC), m1 = lane < row_n1(wC);
    sc0 = m0 ? (ldR[s] & 0xFFFFu) : trash;
    sc1 = m1 ? (ldR[s] >> 16) : trash;
    ac0 = v0R[s];  // masked lanes: a finite score of another posting, added to -inf
    ac1 = v1R[s];
    xc0 = lds_at(sc0);
    xc1 = lds_at(sc1);
  };
  prepare(0);

  // step of ring slot s: row r (prepared) is added, row r + kFR goes into slot
  // s (consumed by the previous step), row r + 1 is prepared from slot s + 1
  auto step = [&](int s) {
    issue(s);
    if (wC & kRowNewTile) {
      if (curTi != kNoTile) epilogue();
      curTi = row_tile(wC) & kTileMask;
      const int32_t pPar = (wC & kRowParity) ? 1 : 0;
      ctxE.q = __builtin_amdgcn_readlane(ctxV, 4 * pPar);
      ctxE.b = __builtin_amdgcn_readlane(ctxV, 4 * pPar + 1);
      ctxE.th = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane(ctxV, 4 * pPar + 3) << 32) |
                (uint32_t)__builtin_amdgcn_readlane(ctxV, 4 * pPar + 2);
      // read before the epilogue cleared the accumulator (trash lanes keep -inf)
      xc0 = sc0 == trash ? xc0 : 0.f;
      xc1 = sc1 == trash ? xc1 : 0.f;
      if constexpr (kCross) {
        thS = key_score((uint32_t)(ctxE.th >> 32));
        ncross = th_positive(ctxE.th) ? 0 : kCrossCap + 1;
      }
    }
    const float y0 = xc0 + ac0, y1 = xc1 + ac1;
    lds_at(sc0) = y0;
    lds_at(sc1) = y1;
    if constexpr (kCross) {  // a doc whose sum is at or above theta's score (trash lanes: -inf);
      // one compare per slot: a doc that is already above records again, and
      // emit_cross keeps its first entry
      const uint64_t m0 = __ballot(y0 >= thS);
      const uint64_t m1 = __ballot(y1 >= thS);
      if ((m0 | m1) != 0ull) {
        const int32_t n0 = (int32_t)__popcll(m0), n1 = (int32_t)__popcll(m1);
        if (ncross + n0 + n1 <= kCrossCap) {
          const uint32_t b0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
          const uint32_t b1 = __builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
          if ((m0 >> lane) & 1ull) xl[ncross + (int32_t)b0] = (uint16_t)sc0;
          if ((m1 >> lane) & 1ull) xl[ncross + n0 + (int32_t)b1] = (uint16_t)sc1;
        }
        ncross += n0 + n1;
      }
    } else if (PH == kRest || (PH == kSample && SM == 1)) {
      hmax = fmaxf(hmax, fmaxf(y0, y1));
    }
    done = (wC & kRowDead) != 0u;  // (rows past the last item add nothing)
    prepare((s + 1) % kFR);
  };

  while (!done) {
#pragma unroll
    for (int s = 0; s < kFR; ++s) step(s);
#if BM25_TRACE
    tr_rows += kFR;
#endif
  }
#if BM25_TRACE
  if (PH == kRest && lane == 0 && blockIdx.x < kTraceWaves) {
    uint64_t* tr = g_bm25_trace + 4 * blockIdx.x;
    tr[0] = tr_t0;
    tr[1] = wall_clock64();
    tr[2] = tr_items;
    tr[3] = tr_rows;
  }
#endif
  if (curTi != kNoTile) epilogue();
  if (kCountPost && stats != nullptr) {  // bound-skipped tiles and postings of this wave
    const uint32_t nb = wave_sum_u32(nbound);
    if (lane == 0 && nb != 0u) atomicAdd(stats, (int32_t)nb);
    // stats + 1 .. + 2: a u64 count (Workspace::counters[6..7], 8-B aligned)
    const uint32_t np = wave_sum_u32(npost);
    if (lane == 0 && np != 0u)
      atomicAdd(reinterpret_cast<unsigned long long*>(stats + 1), (unsigned long long)np);
  }
  // every claim of this wave has returned (the last one, read by next(), ran
  // out of items) before it counts itself finished
  finish();
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

// Exact top-k (k keys, zero-padded) of one tile of query q into out: wave 0
// accumulates, the workgroup sorts the 2^S keys (acc: 2^S floats, keys: 2^S
// u64, both LDS).
template <int S>
__device__ void rescore_tile(const IndexArgs& a, const int32_t* __restrict__ queries, int32_t T,
                             int32_t k, int64_t q, int64_t tile, uint64_t* out, float* acc,
                             uint64_t* keys) {
  constexpr int D = 1 << S;
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
  for (int i = threadIdx.x; i < k; i += blockDim.x) out[i] = i < D ? keys[i] : 0ull;
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
    rescore_tile<S>(a, queries, T, k, q, tile, ws.cand2 + (int64_t)code * k, acc, keys);
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

// Dense per-doc scores of G queries at once (the large-k path,
// bm25mi_large.hip): one wave per (tile, query), the whole tile stored to
// out[g * stride + doc] (stride = ntiles << S: docs past n_docs hold 0).
template <int S>
__global__ __launch_bounds__(64) void scores_batch_kernel(IndexArgs a,
                                                          const int32_t* __restrict__ queries,
                                                          int32_t T, int64_t stride,
                                                          float* __restrict__ out) {
  constexpr int D = 1 << S, E = D / 64;
  __shared__ __attribute__((aligned(16))) float acc[D];
  const int64_t tile = blockIdx.x, g = blockIdx.y;
  zero_acc<S>(acc);
  add_item<S>(a, tile, queries + g * T, T, acc);
  float fv[E];
  take_entries<S>(acc, fv);
  float* row = out + g * stride + (tile << S);
  const uint32_t lane = lane_id();
#pragma unroll
  for (int j = 0; j < E / 4; ++j)  // docs 256 j + 4 lane + (0..3) of the tile
    *reinterpret_cast<float4*>(row + entry_doc(4 * j, lane)) =
        make_float4(fv[4 * j], fv[4 * j + 1], fv[4 * j + 2], fv[4 * j + 3]);
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
      ldoc[p] = (uint16_t)(((uint32_t)d & mask) << 2);  // LDS byte offset of the doc's slot
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

// Tile bounds (dense segment table, non-negative index): bmax[t][j] = term
// t's largest score in tile j as f16 bits rounded down (rows of
// bmax_stride(ntiles) entries, zero past the last tile; 0: no posting there;
// 65504 past f16's range), one block per term (coalesced over its tiles), the
// segments from the rel table.  The value is <= the real maximum (a lower
// bound: bound_keys_kernel) and the next f16 up is > it (an upper bound: the
// REST pass's tile skip, inf past the range).
__global__ __launch_bounds__(256) void build_bmax_kernel(const int64_t* __restrict__ indptr,
                                                         const uint32_t* __restrict__ rel,
                                                         const float* __restrict__ val, int64_t V,
                                                         int64_t ntiles,
                                                         uint16_t* __restrict__ bmax) {
  const int64_t bs = bmax_stride(ntiles);
  for (int64_t t = blockIdx.x; t < V; t += gridDim.x) {
    const int64_t ip = indptr[t];
    const uint32_t* r = rel + t * (ntiles + 1);
    for (int64_t j = ntiles + threadIdx.x; j < bs; j += blockDim.x) bmax[t * bs + j] = 0;
    for (int64_t j = threadIdx.x; j < ntiles; j += blockDim.x) {
      float m = 0.f;
      for (int64_t p = ip + r[j]; p < ip + r[j + 1]; ++p) m = fmaxf(m, val[p]);
      _Float16 h = (_Float16)m;  // round to nearest, then down to <= m
      uint16_t u;
      __builtin_memcpy(&u, &h, 2);
      if ((float)h > m) --u;  // (inf past the range becomes 65504)
      bmax[t * bs + j] = u;
    }
  }
}

// Pooled tile bounds (DevIndex::bpool / wbpool): each group of kPool
// consecutive entries of a row -> its max (f16 bits of values >= 0 order as
// integers); groups past the input row are 0.  Once per index / world table.
__global__ __launch_bounds__(256) void pool_bounds_kernel(const uint16_t* __restrict__ in,
                                                          int64_t rows, int64_t in_stride,
                                                          uint16_t* __restrict__ out,
                                                          int64_t out_stride) {
  const int64_t n = rows * out_stride;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / out_stride, g = e - r * out_stride;
    uint16_t m = 0;
    for (int64_t j = g * kPool; j < min<int64_t>((g + 1) * kPool, in_stride); ++j)
      m = max(m, in[r * in_stride + j]);
    out[e] = m;
  }
}

// Tile-bound threshold keys (search_geom's P = 0), one workgroup per query:
// for every tile j, lb_j = the largest of its query terms' tile maxima (bmax,
// rounded down).  A document of the tile that holds such a maximum scores at
// least lb_j — its sum includes that term's score, and fp32 additions of
// non-negative values never decrease — so the key (lb_j, the tile's LAST
// doc) is <= that document's own key, and the tiles' keys belong to distinct
// documents.  The k-th best of them is thus a lower bound of the k-th best
// key, like the SAMPLE pass's keys, with no posting scored.  Writes this
// shard's best S keys of every query (global doc ids; 0: fewer positive
// tiles).  LDS: the tiles' lb_j as f16 bits (ordered as integers: all >= 0).
// The four waves read the bmax rows (T <= kBoundMaxTerms = 16 loads per tile
// in flight, coalesced over consecutive tiles: T * ntiles * 2 B per query);
// wave 0 then selects and writes from LDS.
constexpr int kBoundNT = 256;

// The k-th largest of the block's u16 values (lbq: four per u64 group, nq4
// groups, zero padding) and its rank among the values equal to it (need):
// two 8-bit radix passes, each an LDS histogram of the digit (high byte, then
// the low byte of the values in the chosen high bin) and one wave's scan of
// it from the top bin down — four barriers, where a bit-by-bit selection
// takes sixteen.  k >= 1; every thread returns the same (v, need).
__device__ __forceinline__ void block_kth_u16(const uint64_t* lbq, int32_t nq4, uint32_t k,
                                              uint32_t* hist, uint32_t* sh, uint32_t& v,
                                              uint32_t& need) {
  const uint32_t lane = lane_id();
  uint32_t hi = 0u, nd = k;
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    for (int i = (int)threadIdx.x; i < 256; i += kBoundNT) hist[i] = 0u;
    __syncthreads();
    for (int32_t g = (int32_t)threadIdx.x; g < nq4; g += kBoundNT) {
      const uint64_t x = lbq[g];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const uint32_t val = (uint32_t)(x >> (16 * u)) & 0xFFFFu;
        if (pass == 0) atomicAdd(&hist[val >> 8], 1u);
        else if ((val >> 8) == hi) atomicAdd(&hist[val & 255u], 1u);
      }
    }
    __syncthreads();
    if (threadIdx.x < 64) {
      // lane l holds bins 255 - 4l .. 252 - 4l (from the top)
      uint32_t c[4], t = 0u;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        c[j] = hist[255 - 4 * (int)lane - j];
        t += c[j];
      }
      uint32_t above = wave_incl_scan(t) - t;  // values in the bins above this lane's
      uint32_t bin1 = 0u, rk = 0u;              // (bin + 1, rank in it) of the k-th value
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        if (above < nd && nd <= above + c[j]) {
          bin1 = 256u - 4u * lane - (uint32_t)j;
          rk = nd - above;
        }
        above += c[j];
      }
      bin1 = wave_max_u32(bin1);
      rk = wave_max_u32(rk);
      if (lane == 0) {
        sh[0] = bin1;
        sh[1] = rk;
      }
    }
    __syncthreads();
    const uint32_t b = sh[0] - 1u;  // (fewer than k values cannot happen: padding counts)
    nd = sh[1];
    hi = pass == 0 ? b : hi;
    v = pass == 0 ? (b << 8) : (v | b);
    __syncthreads();  // (hist and sh are rewritten by the next pass)
  }
  need = nd;
}

// The REST pass's split-item table (score_flat_kernel, SM == kSplitM), built
// by the threshold blocks of one search: each block stores its query's weight
// (the postings of its distinct terms in this index); the last block to
// finish (a device-scope counter, reset for the next search) splits each
// query's band into f(q) sub-items of bwmax / f(q) tiles — f(q) the power of
// two >= weight / (1.25 x the batch's mean weight), at most bwmax — and lays
// them out in query order: entry = q | first tile << 20 | tiles << 26, and
// *sub_ipb = the items per band.  The heavy queries' items shrink to about
// the mean, so the last items the waves claim end close together.
__device__ void split_table(const IndexArgs& a, const int32_t* __restrict__ queries, int32_t T,
                            int64_t q, int32_t nq, int32_t bwmax, uint32_t* __restrict__ qw,
                            uint32_t* __restrict__ sub, int32_t* __restrict__ sub_ipb,
                            int32_t* __restrict__ sub_done, uint32_t* sh /* >= 2 + kBoundNT / 64 */) {
  __shared__ int32_t s_last;
  if (threadIdx.x == 0) {
    const int32_t* qt = queries + q * T;
    uint64_t w = 0;
    for (int i = 0; i < T; ++i) {
      const int32_t t = qt[i];
      bool dup = t < 0 || (int64_t)t >= a.V;
      for (int j = 0; j < i && !dup; ++j) dup = qt[j] == t;
      if (!dup) w += (uint64_t)(a.indptr[t + 1] - a.indptr[t]);
    }
    qw[q] = (uint32_t)min<uint64_t>(w, 0xFFFFFFFFull);
    __threadfence();
    s_last = atomicAdd(sub_done, 1) == nq - 1;
  }
  __syncthreads();
  if (!s_last) return;
  __threadfence();  // every block's weight is visible past the counter
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  // the batch's mean weight
  uint64_t tw = 0;
  for (int32_t i = (int32_t)threadIdx.x; i < nq; i += kBoundNT) tw += __hip_atomic_load(qw + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  uint32_t tw32 = (uint32_t)min<uint64_t>(tw, 0xFFFFFFFFull);
  tw32 = wave_sum_u32(tw32);  // (a u32 sum of the batch: saturates only past 4 G postings)
  if (lane == 0) sh[2 + wv] = tw32;
  __syncthreads();
  uint64_t tot = 0;
#pragma unroll
  for (int i = 0; i < kBoundNT / 64; ++i) tot += sh[2 + i];
  const double lim = 1.25 * (double)tot / (double)nq;  // f = 1 up to 1.25 x the mean
  // f(q) per query (thread t: queries t * per .. ), then a block scan of the counts
  const int32_t per = (nq + kBoundNT - 1) / kBoundNT;
  const int32_t q0 = (int32_t)threadIdx.x * per;
  uint32_t fsum = 0u;
  for (int32_t i = q0; i < min(nq, q0 + per); ++i) {
    const double w = (double)__hip_atomic_load(qw + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t f = 1u;
    while ((int32_t)f < bwmax && w > lim * (double)f) f <<= 1;
    fsum += f;
  }
  const uint32_t incl = wave_incl_scan(fsum);
  __syncthreads();  // (sh[2..] reused)
  if (lane == 63) sh[2 + wv] = incl;
  __syncthreads();
  uint32_t base = incl - fsum;
  for (int i = 0; i < (int)wv; ++i) base += sh[2 + i];
  for (int32_t i = q0; i < min(nq, q0 + per); ++i) {
    const double w = (double)__hip_atomic_load(qw + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t f = 1u;
    while ((int32_t)f < bwmax && w > lim * (double)f) f <<= 1;
    const uint32_t width = (uint32_t)bwmax / f;
    for (uint32_t j = 0; j < f; ++j) sub[base + j] = (uint32_t)i | ((j * width) << 20) | (width << 26);
    base += f;
  }
  if (threadIdx.x == kBoundNT - 1) {
    *sub_ipb = (int32_t)base;  // (the last thread's end: every query's count)
    *sub_done = 0;
  }
}

// lb of every tile group of a query into lbq: the packed u16 maxima of its
// terms' bmax rows (v_pk_max_u16), GPI groups per thread per round with all
// their TMAX x GPI row loads issued before any is used.
typedef unsigned short bm25_us4 __attribute__((ext_vector_type(4)));
template <int TMAX, int GPI>
__device__ __forceinline__ void bound_rows(const IndexArgs& a, const uint16_t* __restrict__ bmax,
                                           const int32_t* __restrict__ qt, int32_t T, int64_t bs,
                                           int32_t gpr, int32_t nq4, int64_t rrank, bool world,
                                           uint64_t* lbq) {
  const uint64_t* row[TMAX];
  bool has[TMAX];
#pragma unroll
  for (int i = 0; i < TMAX; ++i) {
    const int32_t t = i < T ? __builtin_amdgcn_readfirstlane(qt[i]) : -1;
    has[i] = t >= 0 && (int64_t)t < a.V;
    row[i] = reinterpret_cast<const uint64_t*>(bmax + (has[i] ? (int64_t)t * bs : 0));
  }
  for (int32_t g0 = (int32_t)threadIdx.x; g0 < nq4; g0 += GPI * kBoundNT) {
    int64_t o[GPI];
#pragma unroll
    for (int j = 0; j < GPI; ++j) {
      const int32_t g = g0 + j * kBoundNT;
      const int32_t w = world ? g / gpr : 0;
      o[j] = g < nq4 ? (int64_t)w * rrank + (g - w * gpr) : -1;
    }
    // every load unconditional at a valid address (a term slot without a term
    // reads row 0, a group past the last reads group 0) and masked after it:
    // a guarded load compiles to a branch with a wait of its own — one memory
    // round trip per load
    uint64_t v[GPI][TMAX];
#pragma unroll
    for (int j = 0; j < GPI; ++j)
#pragma unroll
      for (int i = 0; i < TMAX; ++i) v[j][i] = row[i][o[j] >= 0 ? o[j] : 0];
#pragma unroll
    for (int j = 0; j < GPI; ++j)
#pragma unroll
      for (int i = 0; i < TMAX; ++i) v[j][i] = (has[i] && o[j] >= 0) ? v[j][i] : 0ull;
#pragma unroll
    for (int j = 0; j < GPI; ++j) {
      bm25_us4 m = {0, 0, 0, 0};
#pragma unroll
      for (int i = 0; i < TMAX; ++i) {
        bm25_us4 x;
        __builtin_memcpy(&x, &v[j][i], 8);
        m = __builtin_elementwise_max(m, x);
      }
      if (o[j] >= 0) {
        uint64_t mm;
        __builtin_memcpy(&mm, &m, 8);
        lbq[g0 + j * kBoundNT] = mm;
      }
    }
  }
}

__global__ __launch_bounds__(kBoundNT) void bound_keys_kernel(IndexArgs a,
                                                              const uint16_t* __restrict__ bmax,
                                                              const int32_t* __restrict__ queries,
                                                              int32_t T, int32_t S_log2, int64_t S,
                                                              uint64_t* __restrict__ keys,
                                                              uint64_t* __restrict__ theta,
                                                              int32_t* __restrict__ list_cnt,
                                                              int32_t* __restrict__ counters,
                                                              int32_t nranks, int64_t wstride,
                                                              uint32_t* __restrict__ qw,
                                                              uint32_t* __restrict__ sub,
                                                              int32_t* __restrict__ sub_ipb,
                                                              int32_t* __restrict__ sub_done,
                                                              int32_t nq, int32_t bwmax) {
  extern __shared__ uint64_t lbq[];  // lb_j as u16, four tiles per u64 (zero past the last)
  const int64_t q = blockIdx.x;
  // world bounds (nranks > 0, theta mode): the rows of every shard, [nranks][V]
  // [wstride] — the groups of shard w follow those of shard w - 1 (a shard's
  // zero padding holds no positive tile); otherwise this index's [V][bs]
  // (theta mode: wstride > 0 without world = the pooled table's row stride —
  // its groups take the tiles' place, launch_score)
  const bool world = nranks > 0;
  const int64_t bs = wstride > 0 ? wstride : bmax_stride(a.ntiles);  // a row holds whole groups
  const int32_t gpr = (int32_t)(bs >> 2);                              // u64 groups per row
  const int32_t nq4 = world ? nranks * gpr : gpr;
  const int64_t rrank = world ? a.V * (bs >> 2) : 0;             // u64 between two shards' rows
  // the query's terms (T <= kBoundMaxTerms, launch_sample checks), loaded at uniform
  // addresses with every lane active; padding and ids >= V: none
  const int32_t* qt = queries + q * T;
  if (T <= 8)  // (the common width: four groups per round, 32 loads in flight)
    bound_rows<8, 4>(a, bmax, qt, T, bs, gpr, nq4, rrank, world, lbq);
  else
    bound_rows<kBoundMaxTerms, 2>(a, bmax, qt, T, bs, gpr, nq4, rrank, world, lbq);
  __syncthreads();
  const uint32_t lane = lane_id(), wv = threadIdx.x >> 6;
  if (theta != nullptr) {
    // a single-index search (theta != null, S = k): theta itself — the k-th
    // key in this index's own doc frame — and the resets theta_wave_kernel
    // would do (list count, search counters); no key list
    if (blockIdx.x == 0 && threadIdx.x < kCounters) counters[threadIdx.x] = 0;
    __shared__ uint32_t hist[256], sh[2];
    uint32_t vk = 0u, needk = 0u;
    block_kth_u16(lbq, nq4, (uint32_t)S, hist, sh, vk, needk);
    if (threadIdx.x == 0) {
      if (vk == 0u) {  // fewer than k positive tiles: every positive doc + zero fill
        theta[q] = (uint64_t)0x80800000u << 32;  // kZeroFillTheta
      } else {
        // the weakest key at the k-th bound's score: k tiles hold a document
        // scoring at least vk, so k keys are >= it (the tie's doc does not
        // tighten it: a doc scoring exactly an f16 value is rare)
        _Float16 h;
        const uint16_t xb = (uint16_t)vk;
        __builtin_memcpy(&h, &xb, 2);
        theta[q] = (uint64_t)score_key((float)h) << 32;
      }
      list_cnt[q] = 0;
    }
    if (sub != nullptr) split_table(a, queries, T, q, nq, bwmax, qw, sub, sub_ipb, sub_done, hist);
    return;
  }
  // the S-th largest lb and how many of the tiles at it are kept
  __shared__ uint32_t hist[256], sh[2];
  uint32_t v = 0u, need = 0u;
  block_kth_u16(lbq, nq4, (uint32_t)S, hist, sh, v, need);
  // fewer than k positive tiles (v = 0): every positive one, zeros after it.
  // Otherwise the tiles above v and the first `need` tiles at v (lowest tile
  // first: their keys are the larger ones), compacted in tile order: rounds
  // of 256 groups, a thread's four tiles in order, then the threads in order
  // (a scan inside each wave, the waves' totals through LDS).
  __shared__ uint32_t wsc[2][kBoundNT / 64];
  uint32_t eq_seen = 0u, kept = 0u;
  uint64_t* out = keys + q * S;
  for (int32_t g0 = 0; g0 < nq4; g0 += kBoundNT) {
    const int32_t g = g0 + (int32_t)threadIdx.x;
    const uint64_t x = g < nq4 ? lbq[g] : 0ull;
    uint32_t ne = 0u;
#pragma unroll
    for (int u = 0; u < 4; ++u) ne += v != 0u && ((uint32_t)(x >> (16 * u)) & 0xFFFFu) == v;
    const uint32_t ie = wave_incl_scan(ne);
    if (lane == 63) wsc[0][wv] = ie;
    __syncthreads();
    uint32_t ebase = eq_seen, etot = 0u;
#pragma unroll
    for (int w = 0; w < kBoundNT / 64; ++w) {
      ebase += w < (int)wv ? wsc[0][w] : 0u;
      etot += wsc[0][w];
    }
    uint32_t er = ebase + ie - ne;  // ties before this thread's first tile
    uint32_t keep4 = 0u, nk = 0u;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint32_t xu = (uint32_t)(x >> (16 * u)) & 0xFFFFu;
      const bool eq = v != 0u && xu == v;
      const bool keep = xu > v || (eq && er < need);
      er += eq ? 1u : 0u;
      keep4 |= keep ? (1u << u) : 0u;
      nk += keep ? 1u : 0u;
    }
    const uint32_t ik = wave_incl_scan(nk);
    if (lane == 63) wsc[1][wv] = ik;
    __syncthreads();
    uint32_t kbase = kept, ktot = 0u;
#pragma unroll
    for (int w = 0; w < kBoundNT / 64; ++w) {
      kbase += w < (int)wv ? wsc[1][w] : 0u;
      ktot += wsc[1][w];
    }
    uint32_t pos = kbase + ik - nk;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if ((keep4 >> u) & 1u) {
        if ((int64_t)pos < S) {
          const int64_t j = 4 * (int64_t)g + u;
          const int64_t last = min((j + 1) << S_log2, a.n_docs) - 1 + a.doc_offset;
          _Float16 h;
          const uint16_t xb = (uint16_t)(x >> (16 * u));
          __builtin_memcpy(&h, &xb, 2);
          out[pos] = ((uint64_t)score_key((float)h) << 32) | (uint64_t)(0xFFFFFFFFu - (uint32_t)last);
        }
        ++pos;
      }
    }
    eq_seen += etot;
    kept += ktot;
    __syncthreads();  // (wsc is rewritten by the next round)
  }
  for (int64_t p = (int64_t)kept + threadIdx.x; p < S; p += kBoundNT) out[p] = 0ull;
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
 ldoc[p] = (uint16_t)(((uint32_t)d & mask) << 2);
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
// Workgroups of the fallback stage's launches (its queries are counted on the
// device and are usually none; the launches must stay cheap).
constexpr int kFallbackBlocks = 64;
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

__global__ __launch_bounds__(64 * kQW) void theta_wave_kernel(const uint64_t* __restrict__ all_keys,
                                                         int64_t W, int64_t Q, int64_t S,
                                                         int32_t k, uint64_t* __restrict__ theta,
                                                         int32_t* __restrict__ list_cnt,
                                                         int32_t C, int32_t nonneg,
                                                         int64_t doc_offset, int64_t n_docs,
                                                         int32_t* __restrict__ counters) {
  // between the SAMPLE and the REST pass, this launch also resets what the
  // rest of the search counts into (no zeroing launch per search): the list
  // counts and the rescore / fallback / block-merge counters (the flat
  // kernel's claim counters reset themselves)
  if (blockIdx.x == 0 && threadIdx.x < kCounters) counters[threadIdx.x] = 0;
  const int64_t q = (int64_t)blockIdx.x * kQW + (threadIdx.x >> 6);
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
      for (int j = 0; j < kThetaR; ++j) {  // (32-bit division: n <= 1024)
        const uint32_t i = (uint32_t)j * 64u + lane;
        const uint32_t w = i / (uint32_t)S;
        // (unconditional load at a valid index, masked after: a guarded load
        // is a branch with a memory wait of its own)
        const uint32_t ic = i < (uint32_t)n ? i : 0u, wc = ic / (uint32_t)S;
        const uint64_t x = all_keys[((int64_t)wc * Q + q) * S + (ic - wc * (uint32_t)S)];
        key[j] = i < (uint32_t)n ? x : 0ull;
      }
      // fewer than k real keys: the k-th is a zero key (no threshold)
      uint32_t nz = 0u, om = 0u, nm = 0u;
#pragma unroll
      for (int j = 0; j < kThetaR; ++j)
        if (key[j] != 0ull) {
          ++nz;
          om |= (uint32_t)(key[j] >> 32);
          nm |= ~(uint32_t)(key[j] >> 32);
        }
      if (wave_sum_u32(nz) >= (uint32_t)k) {
        // score half first, then the doc half among the keys of that score —
        // only when more than one key holds it (ties).  The k-th key is a real
        // key: bits no real key sets stay 0, bits every real key sets are 1,
        // and only the others take a counting step (tile-bound keys carry
        // f16-valued scores: 13 mantissa bits are never set)
        om = wave_or_u32(om);
        const uint32_t am = ~wave_or_u32(nm);
        uint32_t hi = 0u;
        for (int bit = 31; bit >= 0; --bit) {
          const uint32_t b1 = 1u << bit;
          if (!(om & b1)) continue;  // (uniform)
          if (am & b1) { hi |= b1; continue; }
          const uint32_t hm = ~0u << bit, cand = hi | b1;
          uint32_t c = 0;
#pragma unroll
          for (int j = 0; j < kThetaR; ++j) c += ((uint32_t)(key[j] >> 32) & hm) == cand;
          const uint32_t tot = wave_sum_u32(c);
          if (tot >= need) hi = cand;
          else need -= tot;
        }
        uint32_t ties = 0, ol = 0u, nl = 0u;
#pragma unroll
        for (int j = 0; j < kThetaR; ++j)
          if ((uint32_t)(key[j] >> 32) == hi) {
            ++ties;
            ol |= (uint32_t)key[j];
            nl |= ~(uint32_t)key[j];
          }
        uint32_t lo = 0u;
        if (wave_sum_u32(ties) == 1u) {  // the one key of that score
          uint32_t m = 0u;
#pragma unroll
          for (int j = 0; j < kThetaR; ++j) m = (uint32_t)(key[j] >> 32) == hi ? (uint32_t)key[j] : m;
          lo = wave_max_u32(m);
        } else {
          ol = wave_or_u32(ol);
          const uint32_t al = ~wave_or_u32(nl);
          for (int bit = 31; bit >= 0; --bit) {
            const uint32_t b1 = 1u << bit;
            if (!(ol & b1)) continue;
            if (al & b1) { lo |= b1; continue; }
            const uint32_t hm = ~0u << bit, cand = lo | b1;
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
      }
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
    list_cnt[q] = (t == 0ull && !nonneg) ? C + 1 : 0;
  }
}


__device__ __forceinline__ int64_t stage_nq(const Stage& sg) {
  return sg.nq_dev ? (int64_t)*sg.nq_dev : (int64_t)sg.nq_host;
}

// One query of merge_first_kernel (the block's shared arrays passed in).
__device__ void merge_first_one(const Stage& sg, int32_t k, int64_t maxflag, int64_t doc_offset,
                                int64_t n_docs, const Workspace& ws, int32_t* __restrict__ docs,
                                float* __restrict__ scores, int64_t qi, uint64_t* keys,
                                int32_t& s_nflag, int32_t* s_cnt, uint32_t* zf_bits) {
  const int64_t q = (sg.qmap && !sg.remap) ? (int64_t)sg.qmap[qi] : qi;
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
               sg.nt * kTileM + cnt, k, sg.theta ? sg.theta[qi] : 0ull, keys, s_cnt);
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

// One block per stage query, or (the fallback stage, whose query count is
// read on the device and usually 0) a few blocks looping over them.
__global__ __launch_bounds__(kMergeNT) void merge_first_kernel(
    Stage sg, int32_t k, int64_t maxflag, int64_t doc_offset, int64_t n_docs, Workspace ws,
    int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  __shared__ int32_t s_nflag, s_cnt;
  __shared__ uint32_t zf_bits[2 * kMaxK / 32];
  const int64_t nq = stage_nq(sg);
  for (int64_t i = blockIdx.x; i < nq; i += gridDim.x) {
    __syncthreads();  // the previous query's shared state is consumed
    merge_first_one(sg, k, maxflag, doc_offset, n_docs, ws, docs, scores,
                    sg.remap ? (int64_t)sg.qmap[i] : i, keys, s_nflag, &s_cnt, zf_bits);
  }
}

// Main stage of a sampled search, one wavefront per query (no barriers): the
// query's list — every key >= theta of the non-sample tiles, ~P k keys —
// is held in registers (kFastR per lane), the k-th largest key is found by a
// radix selection (score half, then the doc half only among keys of that
// score), the <= k keys at or above it are sorted in the wave's LDS slice
// (bitonic) and written out.  Queries this cannot serve — an overflowed list
// (the exact fallback stage, as merge_first), a list longer than 64 kFastR,
// a zero-fill threshold with fewer than k keys — are queued for
// merge_first_kernel (ws.slow).  Replaces the block-per-query sort of the
// whole list (merge_first: 1024 threads, ~55 barrier-separated bitonic stages
// over the padded list) for the common case.
// ---- register bitonic sort of a wave's keys (R per lane, element j * 64 +
// lane), best (largest) first.  Partners in other lanes come over DPP
// (xor 1, 2: quad permutes), ds_swizzle (xor 4 .. 16, within 32 lanes) or
// ds_bpermute (xor 32): no LDS memory round trips and no fences, where the
// LDS bitonic of wave_sort_write waits on two LDS reads per step.
template <int X>
__device__ __forceinline__ uint32_t lane_xor32(uint32_t v) {
  if constexpr (X == 1) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  else if constexpr (X == 2) return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  else if constexpr (X < 32) return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (X << 10));
  else return (uint32_t)__shfl_xor((int)v, X, 64);
}
template <int X>
__device__ __forceinline__ uint64_t lane_xor64(uint64_t v) {
  return ((uint64_t)lane_xor32<X>((uint32_t)(v >> 32)) << 32) | lane_xor32<X>((uint32_t)v);
}
// One compare-exchange step (block size SZ, partner distance ST) of the
// bitonic network over 64 R elements, sorting descending.
template <int R, int SZ, int ST>
__device__ __forceinline__ void bitonic_step(uint64_t (&k)[R], uint32_t lane) {
  if constexpr (ST >= 64) {
    constexpr int js = ST / 64;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      if ((j & js) == 0) {
        const bool desc = ((j * 64) & SZ) == 0;  // (SZ >= 128: uniform per register)
        const uint64_t a = k[j], b = k[j | js];
        const bool sw = desc ? (a < b) : (a > b);
        k[j] = sw ? b : a;
        k[j | js] = sw ? a : b;
      }
    }
  } else {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const uint64_t p = lane_xor64<ST>(k[j]);
      const bool desc = (((uint32_t)j * 64u + lane) & (uint32_t)SZ) == 0u;
      const bool low = (lane & (uint32_t)ST) == 0u;
      const bool mx = low == desc;
      k[j] = mx ? (k[j] > p ? k[j] : p) : (k[j] < p ? k[j] : p);
    }
  }
}
template <int R, int SZ, int ST>
__device__ __forceinline__ void bitonic_merge(uint64_t (&k)[R], uint32_t lane) {
  bitonic_step<R, SZ, ST>(k, lane);
  if constexpr (ST > 1) bitonic_merge<R, SZ, ST / 2>(k, lane);
}
template <int R, int SZ>
__device__ __forceinline__ void bitonic_sizes(uint64_t (&k)[R], uint32_t lane) {
  bitonic_merge<R, SZ, SZ / 2>(k, lane);
  if constexpr (SZ < 64 * R) bitonic_sizes<R, SZ * 2>(k, lane);
}
template <int R>
__device__ __forceinline__ void wave_sort_regs(uint64_t (&k)[R]) {
  bitonic_sizes<R, 2>(k, (uint32_t)lane_id());
}

// keys[0, n) of a wave's LDS slice (n <= 64 R), sorted best first in
// registers; the first k written as docs / scores of row q (past n: doc -1,
// score bits ~0).  Every key is read before any output is written.
template <int R>
__device__ __forceinline__ void regs_sort_write(const uint64_t* keys, uint32_t n, int32_t k,
                                                int64_t doc_offset, int64_t q,
                                                int32_t* __restrict__ docs,
                                                float* __restrict__ scores) {
  const uint32_t lane = lane_id();
  uint64_t key[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t i = (uint32_t)j * 64u + lane;
    const uint64_t x = keys[i < n ? i : 0u];  // (unconditional read, masked)
    key[j] = i < n ? x : 0ull;
  }
  wave_sort_regs<R>(key);
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int i = j * 64 + (int)lane;
    if (i < k) {
      const uint64_t x = key[j];
      if (x == 0ull) {  // padding (a shard holding fewer than k keys)
        docs[q * k + i] = -1;
        scores[q * k + i] = __uint_as_float(0xFFFFFFFFu);
      } else {
        docs[q * k + i] = (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)x) + doc_offset);
        scores[q * k + i] = key_score((uint32_t)(x >> 32));
      }
    }
  }
  // k > 64 R (n <= 64 R): the rest is padding
  for (int i = 64 * R + (int)lane; i < k; i += 64) {
    docs[q * k + i] = -1;
    scores[q * k + i] = __uint_as_float(0xFFFFFFFFu);
  }
}

// n keys in the wave's LDS slice -> sorted and written: registers for n <=
// 64 MAXR, the LDS bitonic above that.
__device__ __forceinline__ void wave_sort_write(uint64_t* keys, uint32_t n, int m, int32_t k,
                                                int64_t doc_offset, int64_t q,
                                                int32_t* __restrict__ docs,
                                                float* __restrict__ scores);
template <int MAXR = 4>
__device__ __forceinline__ void sort_write_any(uint64_t* keys, uint32_t n, int32_t k,
                                               int64_t doc_offset, int64_t q,
                                               int32_t* __restrict__ docs,
                                               float* __restrict__ scores) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  if (n <= 128u)
    regs_sort_write<2>(keys, n, k, doc_offset, q, docs, scores);
  else if (MAXR >= 4 && n <= 256u)
    regs_sort_write<4>(keys, n, k, doc_offset, q, docs, scores);
  else if (MAXR >= 8 && n <= 512u)
    regs_sort_write<MAXR >= 8 ? 8 : 2>(keys, n, k, doc_offset, q, docs, scores);
  else
    wave_sort_write(keys, n, next_pow2((int64_t)n), k, doc_offset, q, docs, scores);
}

constexpr int kFastR = 32;      // list keys per lane held in registers
// lists longer than this at k <= 128 go to merge_tail_kernel's block merge
// (block_long_merge: 1024 threads load them in one round)
#ifndef BM25_BLOCK_LONG
#define BM25_BLOCK_LONG 512
#endif
constexpr int kBlockLongMin = BM25_BLOCK_LONG;
constexpr int kFastMaxK = 1024; // largest k served (LDS: k keys per wave)

__device__ __forceinline__ void wave_sort_write(uint64_t* keys, uint32_t n, int m, int32_t k,
                                                int64_t doc_offset, int64_t q,
                                                int32_t* __restrict__ docs,
                                                float* __restrict__ scores);

template <int R>
__device__ __forceinline__ uint64_t wave_kth_key(const uint64_t (&key)[R], int32_t k, uint32_t& n);

// The body of merge_fast_kernel for a list held in R keys per lane.
template <int R>
__device__ __forceinline__ void fast_merge_one(const Stage& sg, int32_t k, int64_t doc_offset,
                                               int64_t q, int32_t cnt, uint64_t th,
                                               uint64_t* keys, int32_t* __restrict__ docs,
                                               float* __restrict__ scores) {
  const uint32_t lane = lane_id();
  const uint64_t* lst = sg.list + q * (int64_t)sg.C;
  uint64_t key[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int i = j * 64 + (int)lane;
    const uint64_t y = lst[i < cnt ? i : 0];  // (unconditional load, masked: a guarded
    const uint64_t x = i < cnt ? y : 0ull;    // load waits for memory on its own)
    key[j] = x >= th ? x : 0ull;  // (every list key is >= theta; key 0 = empty)
  }
  uint32_t n = 0;
  if (sg.unsorted) {
    // a doc shard's list for the W-way merge, which sorts: its best k keys
    // (all of them when there are at most k) go out in no particular order —
    // the k-th key selected in registers, no sort — padding after them
    const uint64_t kth = wave_kth_key<R>(key, k, n);  // (0: every key kept)
    uint32_t base = 0u;
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const bool keep = key[j] != 0ull && key[j] >= kth;
      const uint64_t b = __ballot(keep);
      if (keep) {
        const uint32_t i = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
        docs[q * k + i] = (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)key[j]) + doc_offset);
        scores[q * k + i] = key_score((uint32_t)(key[j] >> 32));
      }
      base += (uint32_t)__popcll(b);
    }
    for (int i = (int)base + (int)lane; i < k; i += 64) {
      docs[q * k + i] = -1;
      scores[q * k + i] = __uint_as_float(0xFFFFFFFFu);
    }
    return;
  }
  if (R == 8 && k <= 128) {  // (also at R = 16 the kernel spills)
    // a longer list: a provisional threshold t1 from a sample (the list's
    // first 128 keys, sorted in registers: the sample key at the rank where
    // ~1.5 k of the list's keys are expected at or above it); when k to 256
    // keys reach t1 — they hold the top k — those are compacted into LDS and
    // sorted; otherwise the exact selection below
    uint64_t smp[2] = {key[0], key[1]};
    wave_sort_regs<2>(smp);
    const int r = min(127, max(0, (int)((3u * (uint32_t)k * 64u) / (uint32_t)cnt)));
    const uint64_t t1 = __shfl(r >= 64 ? smp[1] : smp[0], r & 63, 64);  // (no dynamic index)
    uint32_t c = 0u;
#pragma unroll
    for (int j = 0; j < R; ++j) c += key[j] != 0ull && key[j] >= t1;
    c = wave_sum_u32(c);
    if (t1 != 0ull && c >= (uint32_t)k && c <= 256u) {
      uint32_t base = 0u;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        const bool keep = key[j] != 0ull && key[j] >= t1;
        const uint64_t b = __ballot(keep);
        if (keep)
          keys[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] = key[j];
        base += (uint32_t)__popcll(b);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      regs_sort_write<4>(keys, base, k, doc_offset, q, docs, scores);
      return;
    }
  }
  if (R <= 4) {
    // a list of <= 256 keys: sorted whole in registers, its first k written
    // (no selection; a shard's unsorted list may be sorted too)
    wave_sort_regs<R>(key);
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int i = j * 64 + (int)lane;
      if (i < k) {
        const uint64_t x = key[j];
        docs[q * k + i] = x == 0ull ? -1 : (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)x) + doc_offset);
        scores[q * k + i] = x == 0ull ? __uint_as_float(0xFFFFFFFFu) : key_score((uint32_t)(x >> 32));
      }
    }
    for (int i = 64 * R + (int)lane; i < k; i += 64) {
      docs[q * k + i] = -1;
      scores[q * k + i] = __uint_as_float(0xFFFFFFFFu);
    }
    return;
  }
  const uint64_t kth = wave_kth_key<R>(key, k, n);
  // the n kept keys (>= kth; unique: doc ids differ) -> LDS, sorted best first
  uint32_t base = 0u;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const bool keep = key[j] != 0ull && key[j] >= kth;
    const uint64_t b = __ballot(keep);
    if (keep)
      keys[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                            __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] = key[j];
    base += (uint32_t)__popcll(b);
  }
  sort_write_any(keys, n, k, doc_offset, q, docs, scores);
}

// The k-th largest of a wave's keys held R per lane (key 0 = empty; keys
// unique otherwise) by a radix selection: the score half bit by bit, then the
// doc half only among the keys of that score.  Returns 0 when there are at
// most k keys (all of them are kept); n = the keys kept (min(count, k)).
template <int R>
__device__ __forceinline__ uint64_t wave_kth_key(const uint64_t (&key)[R], int32_t k, uint32_t& n) {
  uint64_t kth = 0ull;
  n = 0;
#pragma unroll
  for (int j = 0; j < R; ++j) n += key[j] != 0ull;
  n = wave_sum_u32(n);
  if (n > (uint32_t)k) {
    // bits no real key sets stay 0 and bits every real key sets are 1 in the
    // answer (the k-th key is a real key): only the bits that differ need a
    // counting step (f16-valued scores leave 13 mantissa bits unused)
    uint32_t om = 0u, nm = 0u;  // OR and NOR-complement (~AND) over the real keys
#pragma unroll
    for (int j = 0; j < R; ++j)
      if (key[j] != 0ull) {
        om |= (uint32_t)(key[j] >> 32);
        nm |= ~(uint32_t)(key[j] >> 32);
      }
    om = wave_or_u32(om);
    const uint32_t am = ~wave_or_u32(nm);
    uint32_t need = (uint32_t)k, hi = 0u;
    for (int bit = 31; bit >= 0; --bit) {
      const uint32_t b1 = 1u << bit;
      if (!(om & b1)) continue;         // (uniform)
      if (am & b1) { hi |= b1; continue; }
      const uint32_t hm = ~0u << bit, cand = hi | b1;
      uint32_t c = 0;
#pragma unroll
      for (int j = 0; j < R; ++j) c += ((uint32_t)(key[j] >> 32) & hm) == cand;
      const uint32_t tot = wave_sum_u32(c);
      if (tot >= need) hi = cand;
      else need -= tot;
    }
    // need = rank of the answer among the keys of score hi
    uint32_t ties = 0, ol = 0u, nl = 0u;
#pragma unroll
    for (int j = 0; j < R; ++j)
      if ((uint32_t)(key[j] >> 32) == hi) {
        ++ties;
        ol |= (uint32_t)key[j];
        nl |= ~(uint32_t)key[j];
      }
    uint32_t lo = 0u;
    if (wave_sum_u32(ties) > 1u) {
      ol = wave_or_u32(ol);
      const uint32_t al = ~wave_or_u32(nl);
      for (int bit = 31; bit >= 0; --bit) {
        const uint32_t b1 = 1u << bit;
        if (!(ol & b1)) continue;
        if (al & b1) { lo |= b1; continue; }
        const uint32_t hm = ~0u << bit, cand = lo | b1;
        uint32_t c = 0;
#pragma unroll
        for (int j = 0; j < R; ++j)
          c += ((uint32_t)(key[j] >> 32) == hi) & (((uint32_t)key[j] & hm) == cand);
        const uint32_t tot = wave_sum_u32(c);
        if (tot >= need) lo = cand;
        else need -= tot;
      }
    } else {
      uint32_t m = 0u;
#pragma unroll
      for (int j = 0; j < R; ++j) m = (uint32_t)(key[j] >> 32) == hi ? (uint32_t)key[j] : m;
      lo = wave_max_u32(m);
    }
    kth = ((uint64_t)hi << 32) | lo;
    n = (uint32_t)k;
  }
  return kth;
}

// The n keys in keys[0, n) (the wave's LDS slice, m = next_pow2 >= n) ->
// sorted best first; the first k written as docs / scores of row q
// (padding past n: doc -1, score bits ~0).
__device__ __forceinline__ void wave_sort_write(uint64_t* keys, uint32_t n, int m, int32_t k,
                                                int64_t doc_offset, int64_t q,
                                                int32_t* __restrict__ docs,
                                                float* __restrict__ scores) {
  const uint32_t lane = lane_id();
  for (int i = (int)n + (int)lane; i < m; i += 64) keys[i] = 0ull;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  for (int size = 2; size <= m; size <<= 1) {
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      const int ls = __builtin_ctz((unsigned)stride);
      for (int i = (int)lane; i < (m >> 1); i += 64) {
        const int a = ((i >> ls) << (ls + 1)) + (i & (stride - 1)), b2 = a + stride;
        const bool desc = (a & size) == 0;
        const uint64_t x = keys[a], y = keys[b2];
        if ((x < y) == desc) {
          keys[a] = y;
          keys[b2] = x;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    }
  }
  for (int i = (int)lane; i < k; i += 64) {
    const uint64_t x = i < m ? keys[i] : 0ull;
    if (x == 0ull) {  // padding (a shard holding fewer than k keys)
      docs[q * k + i] = -1;
      scores[q * k + i] = __uint_as_float(0xFFFFFFFFu);
    } else {
      docs[q * k + i] = (int32_t)((int64_t)(0xFFFFFFFFu - (uint32_t)x) + doc_offset);
      scores[q * k + i] = key_score((uint32_t)(x >> 32));
    }
  }
}

// A list longer than the registers hold (64 kFastR < cnt <= C: a query
// whose threshold sits far below its k-th key), one wave: the k-th largest
// score half by a radix selection over the list in memory (four 8-bit
// digits, a wave-private LDS histogram), then the keys above that score and
// all keys at it compacted into the wave's LDS slice and sorted.  Returns
// false (nothing written) when score ties make that more than kFastMaxK
// keys: the block merge takes the query.
template <int R>
__device__ __forceinline__ void lds_merge_one(uint64_t* kb, uint32_t cnt, int32_t k,
                                              int64_t doc_offset, int64_t q,
                                              int32_t* __restrict__ docs,
                                              float* __restrict__ scores);

// First attempt for a long list: a provisional threshold from a sample of it
// (every s-th key, <= 1024 in registers: the ceil(2k / s)-th best sample key,
// expected ~2k list keys at or above it), one pass compacting the keys at or
// above it into the wave's LDS slice, then the exact merge of those.  Valid
// whenever they are at least k (the top k are among them) and fit the slice;
// otherwise it returns false and the digit passes below run.
__device__ bool long_merge_sampled(const Stage& sg, int32_t k, int64_t doc_offset, int64_t q,
                                   int32_t cnt, uint64_t* keys, int32_t* __restrict__ docs,
                                   float* __restrict__ scores) {
  const uint32_t lane = lane_id();
  const uint64_t* lst = sg.list + q * (int64_t)sg.C;
  constexpr int RS = 16;
  const int s = (cnt + 64 * RS - 1) / (64 * RS);  // sample stride
  uint64_t smp[RS];
#pragma unroll
  for (int j = 0; j < RS; ++j) {
    const int64_t i = (int64_t)(j * 64 + (int)lane) * s;
    const uint64_t y = lst[i < cnt ? i : 0];
    smp[j] = i < cnt ? y : 0ull;
  }
  const int32_t want = min((2 * k + s - 1) / s, 64 * RS);
  uint32_t nk = 0;
  const uint64_t t1 = wave_kth_key<RS>(smp, want, nk);  // (0: the sample holds fewer)
  uint32_t base = 0u;
  for (int i0 = 0; i0 < cnt; i0 += 8 * 64) {
    uint64_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 64 + (int)lane;
      const uint64_t y = lst[i < cnt ? i : 0];
      x[u] = i < cnt ? y : 0ull;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool keep = x[u] != 0ull && x[u] >= t1;
      const uint64_t b = __ballot(keep);
      const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
      if (keep && pos < (uint32_t)kFastMaxK) keys[pos] = x[u];
      base += (uint32_t)__popcll(b);
    }
  }
  if (base < (uint32_t)k || base > (uint32_t)kFastMaxK) return false;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  const uint32_t nj = (base + 63u) >> 6;
  if (nj <= 4u)
    lds_merge_one<4>(keys, base, k, doc_offset, q, docs, scores);
  else if (nj <= 8u)
    lds_merge_one<8>(keys, base, k, doc_offset, q, docs, scores);
  else
    lds_merge_one<16>(keys, base, k, doc_offset, q, docs, scores);
  return true;
}

__device__ bool long_merge_one(const Stage& sg, int32_t k, int64_t doc_offset, int64_t q,
                               int32_t cnt, uint64_t* keys, uint32_t* h,
                               int32_t* __restrict__ docs, float* __restrict__ scores) {
  if (long_merge_sampled(sg, k, doc_offset, q, cnt, keys, docs, scores)) return true;
  const uint32_t lane = lane_id();
  const uint64_t* lst = sg.list + q * (int64_t)sg.C;
  uint32_t prefix = 0u, need = (uint32_t)k;
  for (int shift = 24; shift >= 0; shift -= 8) {
    for (int b = (int)lane; b < 256; b += 64) h[b] = 0u;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    const int hs = shift + 8;
    // 8 loads in flight per lane; the lanes that share the first pending
    // lane's digit (most of them: one exponent range) add once
    for (int i0 = 0; i0 < cnt; i0 += 8 * 64) {
      uint32_t x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 64 + (int)lane;
        const uint64_t y = lst[i < cnt ? i : 0];
        x[u] = i < cnt ? (uint32_t)(y >> 32) : 0u;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int i = i0 + u * 64 + (int)lane;
        bool pend = i < cnt && (hs >= 32 || (x[u] >> hs) == (prefix >> hs));
        const uint32_t dig = (x[u] >> shift) & 255u;
        const uint64_t m = __ballot(pend);
        if (m != 0ull) {  // wave-uniform
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
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    uint32_t c[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) c[j] = h[4 * lane + j];
    const uint32_t t = c[0] + c[1] + c[2] + c[3];
    uint32_t incl = t;  // inclusive scan over the lanes
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)incl, o, 64);
      if ((int)lane >= o) incl += y;
    }
    const uint32_t tot = (uint32_t)__shfl((int)incl, 63, 64);
    uint32_t above = tot - incl;  // keys in the bins of the higher lanes
    uint32_t d1 = 0u, pneed = 0u;  // (digit + 1, rank in its bin) of the one lane holding it
#pragma unroll
    for (int j = 3; j >= 0; --j) {
      if (above < need && need <= above + c[j]) {
        d1 = 4u * lane + (uint32_t)j + 1u;
        pneed = need - above;
      }
      above += c[j];
    }
    d1 = wave_max_u32(d1);
    pneed = wave_max_u32(pneed);
    if (d1 == 0u) return false;  // (cannot happen: need <= the keys of the prefix)
    prefix |= (d1 - 1u) << shift;
    need = pneed;
  }
  // every key of score >= the k-th key's score (the sort below orders them)
  uint32_t base = 0u;
  for (int i0 = 0; i0 < cnt; i0 += 8 * 64) {
    uint64_t x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = i0 + u * 64 + (int)lane;
      const uint64_t y = lst[i < cnt ? i : 0];
      x[u] = i < cnt ? y : 0ull;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool keep = x[u] != 0ull && (uint32_t)(x[u] >> 32) >= prefix;
      const uint64_t b = __ballot(keep);
      const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
      if (keep && pos < (uint32_t)kFastMaxK) keys[pos] = x[u];
      base += (uint32_t)__popcll(b);
    }
  }
  if (base > (uint32_t)kFastMaxK) return false;
  wave_sort_write(keys, base, next_pow2(base > 1u ? (int)base : 2), k, doc_offset, q, docs, scores);
  return true;
}

__global__ __launch_bounds__(64 * kQW) void merge_fast_kernel(Stage sg, int32_t k, int64_t doc_offset,
                                                         Workspace ws, int32_t* __restrict__ docs,
                                                         float* __restrict__ scores) {
  __shared__ uint64_t sk[kQW][kFastMaxK];
  __shared__ uint32_t hist[kQW][256];
  const int64_t q = (int64_t)blockIdx.x * kQW + (threadIdx.x >> 6);
  if (q >= sg.nq_host) return;  // wave-uniform; no barriers in this kernel
  const uint32_t lane = lane_id();
  uint64_t* keys = sk[threadIdx.x >> 6];
  const int32_t cnt = sg.list_cnt[q];
  const uint64_t th = sg.theta[q];
  if (cnt > sg.C) {  // overflowed: exact fallback stage
    if (lane == 0) {
      ws.nflag[q] = 0;
      sg.fb[atomicAdd(sg.fb_cnt, 1)] = (int32_t)q;
    }
    return;
  }
  // a list of more than kBlockLongMin = 512 keys at k <= 128 (a few queries
  // whose threshold sits far below their k-th key): merge_tail_kernel's block
  // merge, whose 1024 threads load it in one round (block_long_merge); one
  // wave alone kept the whole merge waiting ~20 us for such a query (config
  // 3: merge_fast 15.5 -> 11.2 us with 512 in place of 1024, the tail alike)
  // (a doc shard's unsorted list of <= 1024 keys stays here: its best k are
  // selected in registers, no sort — faster than the block merge's sorts)
  const bool block_long = (cnt > 1024 || (cnt > kBlockLongMin && !sg.unsorted)) && k <= 128 &&
                          th != kZeroFillTheta;
  if (!block_long && cnt > 64 * kFastR &&
      long_merge_one(sg, k, doc_offset, q, cnt, keys, hist[threadIdx.x >> 6], docs, scores))
    return;
  if (block_long || cnt > 64 * kFastR || (th == kZeroFillTheta && cnt < k)) {
    if (lane == 0) ws.slow[atomicAdd(ws.counters + 4, 1)] = (int32_t)q;
    return;
  }
  // the fewest register slots that hold the list: 4, 8, 16 or 32 keys per lane
  const int32_t nj = (cnt + 63) >> 6;
  if (nj <= 4)
    fast_merge_one<4>(sg, k, doc_offset, q, cnt, th, keys, docs, scores);
  else if (nj <= 8)
    fast_merge_one<8>(sg, k, doc_offset, q, cnt, th, keys, docs, scores);
  else if (nj <= 16)
    fast_merge_one<16>(sg, k, doc_offset, q, cnt, th, keys, docs, scores);
  else
    fast_merge_one<kFastR>(sg, k, doc_offset, q, cnt, th, keys, docs, scores);
}

__device__ void merge_final_one(const Stage& sg, int32_t k, int64_t maxflag, int64_t doc_offset,
                                const Workspace& ws, int32_t* __restrict__ docs,
                                float* __restrict__ scores, int64_t qi, uint64_t* keys,
                                uint32_t* bits) {
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

__global__ __launch_bounds__(kMergeNT) void merge_final_kernel(
    Stage sg, int32_t k, int64_t maxflag, int64_t doc_offset, Workspace ws,
    int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  __shared__ uint32_t bits[kMaxFlagBits / 32];
  const int64_t nq = stage_nq(sg);
  for (int64_t qi = blockIdx.x; qi < nq; qi += gridDim.x) {
    __syncthreads();
    merge_final_one(sg, k, maxflag, doc_offset, ws, docs, scores, qi, keys, bits);
  }
}

// A long list (1024 < cnt <= kMergeP keys, k <= 128, a threshold other than
// zero fill) with the whole block: every thread loads its <= 8 keys in one
// round; wave 0 sorts a 256-key sample of the list (its first 256 keys) in
// registers and takes as provisional threshold t1 the sample key at the rank
// where ~1.5 k of the list's keys are expected at or above it; when k to 256
// keys reach t1 (they hold the top k) they are compacted into LDS and wave 0
// sorts and writes them.  Returns false (nothing written; uniform) otherwise:
// the caller's block merge takes the query.
constexpr int kLongPT = kMergeP / kMergeNT;  // keys per thread
__device__ bool block_long_merge(const Stage& sg, int32_t k, int64_t doc_offset, int64_t q,
                                 uint64_t* keys, int32_t* s_cnt, uint64_t* s_t1,
                                 int32_t* __restrict__ docs, float* __restrict__ scores) {
  const int32_t cnt = sg.list_cnt[q];
  const uint64_t th = sg.theta[q];
  if (cnt <= kBlockLongMin || cnt > kMergeP || k > 128 || th == kZeroFillTheta) return false;
  const uint64_t* lst = sg.list + q * (int64_t)sg.C;
  const uint32_t lane = lane_id();
  uint64_t x[kLongPT];
#pragma unroll
  for (int i = 0; i < kLongPT; ++i) {
    const int e = i * kMergeNT + (int)threadIdx.x;
    const uint64_t y = lst[e < cnt ? e : 0];  // (unconditional load, masked)
    const uint64_t v = e < cnt ? y : 0ull;
    x[i] = v >= th ? v : 0ull;
  }
  if (threadIdx.x < 64) {
    uint64_t smp[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint64_t v = lst[j * 64 + (int)lane];  // (cnt > 1024: all in the list)
      smp[j] = v >= th ? v : 0ull;
    }
    wave_sort_regs<4>(smp);
    const int r = min(255, (int)((3u * (uint32_t)k * 128u) / (uint32_t)cnt));
    const uint64_t a0 = r < 128 ? smp[0] : smp[2], a1 = r < 128 ? smp[1] : smp[3];
    const uint64_t t1 = __shfl((r & 64) ? a1 : a0, r & 63, 64);  // (no dynamic index)
    if (lane == 0) {
      *s_t1 = t1;
      *s_cnt = 0;
    }
  }
  __syncthreads();
  const uint64_t t1 = *s_t1;
  uint32_t c = 0u;
#pragma unroll
  for (int i = 0; i < kLongPT; ++i) c += x[i] != 0ull && x[i] >= t1;
  c = wave_sum_u32(c);
  if (lane == 0 && c) atomicAdd(s_cnt, (int32_t)c);
  __syncthreads();
  const int32_t tot = *s_cnt;
  __syncthreads();  // (s_cnt is reset below)
  if (t1 == 0ull || tot < k || tot > 256) return false;
  if (threadIdx.x == 0) *s_cnt = 0;
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kLongPT; ++i) {
    const bool keep = x[i] != 0ull && x[i] >= t1;
    const uint64_t m = __ballot(keep);
    int base = 0;
    if (lane == 0 && m) base = atomicAdd(s_cnt, (int)__popcll(m));
    base = __shfl(base, 0, 64);
    if (keep)
      keys[base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                                                 __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u))] = x[i];
  }
  __syncthreads();
  if (threadIdx.x < 64) regs_sort_write<4>(keys, (uint32_t)tot, k, doc_offset, q, docs, scores);
  __syncthreads();  // (keys are reused by the block's next query)
  return true;
}

// The tail of a sampled search, one launch whose queries are counted on the
// device (usually none): (1) the queries merge_fast_kernel left (lists longer
// than it holds, zero-fill thresholds), merged as merge_first does; (2) the
// fallback stage's queries (overflowed lists, re-scored over every tile by
// the exact pass), each workgroup taking a whole query through merge_first,
// the exact rescore of its flagged tiles and merge_final.  One launch in place
// of four (each ~4.5 us even when it has nothing to do).
template <int S>
__global__ __launch_bounds__(kMergeNT) void merge_tail_kernel(
    IndexArgs a, const int32_t* __restrict__ queries, int32_t T, Stage sl, Stage fb, int32_t k,
    int64_t maxflag, Workspace ws, int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  __shared__ __attribute__((aligned(16))) float acc[1 << S];
  __shared__ uint32_t bits[kMaxFlagBits / 32];
  __shared__ int32_t s_nflag, s_cnt;
  __shared__ uint32_t zf_bits[2 * kMaxK / 32];
  static_assert((1 << S) <= kMergeP, "rescore keys live in the merge buffer");
  if (blockIdx.x == 0 && threadIdx.x == 0 && ws.report != nullptr) {
    // the search's overflow, for the host's choice of the next threshold
    // source (bound_ok): the count, then the sequence number that marks it valid
    __hip_atomic_store(ws.report, (int32_t)stage_nq(fb), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(ws.report + 1, ws.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __shared__ uint64_t s_t1;
  const int64_t ns = stage_nq(sl);
  for (int64_t i = blockIdx.x; i < ns; i += gridDim.x) {
    __syncthreads();
    const int64_t qi = (int64_t)sl.qmap[i];
    if (block_long_merge(sl, k, a.doc_offset, qi, keys, &s_cnt, &s_t1, docs, scores)) continue;
    merge_first_one(sl, k, maxflag, a.doc_offset, a.n_docs, ws, docs, scores, qi, keys, s_nflag,
                    &s_cnt, zf_bits);
  }
  const int64_t nf = stage_nq(fb);
  for (int64_t qi = blockIdx.x; qi < nf; qi += gridDim.x) {
    __syncthreads();
    merge_first_one(fb, k, maxflag, a.doc_offset, a.n_docs, ws, docs, scores, qi, keys, s_nflag,
                    &s_cnt, zf_bits);
    __syncthreads();
    const int nfl = ws.nflag[qi];  // (written by thread 0 above)
    if (nfl == 0) continue;
    const int64_t q = (int64_t)fb.qmap[qi];
    for (int i = 0; i < nfl; ++i) {
      const int64_t code = qi * maxflag + i;
      __syncthreads();
      rescore_tile<S>(a, queries, T, k, q, (int64_t)ws.flag_tiles[code],
                      ws.cand2 + code * k, acc, keys);
    }
    __syncthreads();
    merge_final_one(fb, k, maxflag, a.doc_offset, ws, docs, scores, qi, keys, bits);
  }
}

__global__ __launch_bounds__(kMergeNT) void merge_lists_kernel(
    const int32_t* __restrict__ in_docs, const float* __restrict__ in_scores, int64_t W,
    int64_t Q, int32_t k, int64_t rstride, int32_t* __restrict__ docs, float* __restrict__ scores) {
  __shared__ uint64_t keys[kMergeP];
  const int64_t q = blockIdx.x;
  topk_of(SrcLists{in_docs, in_scores, Q, q, k, rstride}, W * k, k, keys);
  write_result(keys, k, q, 0, docs, scores);
}

// Merge of W per-rank [Q, k] lists (bm25_search_finish_device's, padding
// last): one wave per query holds the W * k keys in registers (16 per lane,
// all loads in flight), selects the k-th largest key (wave_kth_key) and
// sorts the k keys at or above it in its LDS slice — a handful of reduction
// steps instead of k dependent head-advance steps (33 us at W = 8, k = 100).
// W * k <= kMergeSortedCap; larger merges take merge_lists_kernel.  Keys are
// unique (global doc ids) except padding (0).
constexpr int kMergeSortedCap = 1024;  // keys per wave

// The cnt keys in the wave's LDS slice -> the best k of them, sorted and
// written (global doc ids: no offset).  Every key is read into registers
// before the slice is rewritten (one wave: its LDS operations keep order).
template <int R>
__device__ __forceinline__ void lds_merge_one(uint64_t* kb, uint32_t cnt, int32_t k,
                                              int64_t doc_offset, int64_t q,
                                              int32_t* __restrict__ docs,
                                              float* __restrict__ scores) {
  const uint32_t lane = lane_id();
  uint64_t key[R];
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const uint32_t i = (uint32_t)j * 64u + lane;
    const uint64_t y = kb[i < cnt ? i : 0u];
    key[j] = i < cnt ? y : 0ull;
  }
  uint32_t kept = 0;
  const uint64_t kth = wave_kth_key<R>(key, k, kept);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  uint32_t base = 0u;
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const bool keep = key[j] != 0ull && key[j] >= kth;
    const uint64_t b = __ballot(keep);
    if (keep)
      kb[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                          __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] = key[j];
    base += (uint32_t)__popcll(b);
  }
  // (the LDS bitonic: the register sort here would make merge_fast_kernel,
  // which inlines this for long lists, spill)
  wave_sort_write(kb, kept, next_pow2(kept > 1u ? kept : 2u), k, doc_offset, q, docs, scores);
}

__global__ __launch_bounds__(64 * kQW) void merge_sorted_kernel(
    const int32_t* __restrict__ in_docs, const float* __restrict__ in_scores, int32_t W,
    int64_t Q, int32_t k, int64_t rstride, int32_t* __restrict__ docs,
    float* __restrict__ scores) {
  __shared__ uint64_t buf[kQW][kMergeSortedCap];
  const int wave = (int)(threadIdx.x >> 6);
  const int64_t q = (int64_t)blockIdx.x * kQW + wave;
  if (q >= Q) return;  // wave-uniform; no barriers
  uint64_t* kb = buf[wave];
  const uint32_t lane = lane_id();
  // the lists' real keys (most slots are padding: the world holds ~2-3 k keys
  // >= theta) compacted into the wave's LDS slice: columns of 64 keys over
  // the ranks' lists (rank-major), eight columns' loads in flight at a time
  // (W = 8, k = 100: all sixteen columns in two rounds), each load
  // unconditional at a valid address and masked after it — a guarded load is
  // a branch with a memory wait of its own; no index division
  uint32_t cnt = 0u;
  const int nc = (k + 63) >> 6;
  const int ncol = W * nc;
  int cw = 0, cc = 0;  // (rank, column) of the round's first column
  for (int b0 = 0; b0 < ncol; b0 += 8) {
    float sv[8];
    int32_t dv[8];
    int w = cw, c = cc;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int j = c * 64 + (int)lane;
      const bool in = b0 + u < ncol && j < k;
      const int64_t off = in ? (int64_t)w * rstride + q * k + j : q * k;
      const float sy = in_scores[off];
      const int32_t dy = in_docs[off];
      sv[u] = in ? sy : 0.f;
      dv[u] = in ? dy : -1;
      if (++c == nc) {
        c = 0;
        ++w;
      }
    }
    cw = w;
    cc = c;
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const bool nz = dv[u] >= 0;  // (padding: doc -1)
      const uint64_t b = __ballot(nz);
      if (nz)
        kb[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                           __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] =
            make_key(sv[u], (uint32_t)dv[u]);
      cnt += (uint32_t)__popcll(b);
    }
  }
  // <= 512 keys: sorted whole in registers, the first k written; more: the
  // k-th key selected first, the keys at or above it sorted
  if (k <= 128 && cnt > 256u) {
    // a long merge at k <= 128 (W = 8, k = 100: up to 800 keys): a provisional
    // threshold t1 from 128 keys sampled at a stride over the list (sorted in
    // registers: the sample key at the rank where ~2 k keys are expected at or
    // above it); when k to 512 keys reach t1 — they hold the top k — those
    // are compacted and sorted in registers, not the whole list.  (The kernel
    // waits for its slowest query; a debug build counted no miss of this
    // window over a W = 8 batch.)
    uint64_t smp[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) smp[j] = kb[(((uint32_t)j * 64u + lane) * cnt) >> 7];
    wave_sort_regs<2>(smp);
    const int r = min(127, max(0, (int)((4u * (uint32_t)k * 64u) / cnt)));
    const uint64_t t1 = __shfl(r >= 64 ? smp[1] : smp[0], r & 63, 64);
    uint64_t key[kMergeSortedCap / 64];
    uint32_t c = 0u;
#pragma unroll
    for (int j = 0; j < kMergeSortedCap / 64; ++j) {
      const uint32_t i = (uint32_t)j * 64u + lane;
      const uint64_t y = kb[i < cnt ? i : 0u];
      key[j] = i < cnt ? y : 0ull;
      c += key[j] != 0ull && key[j] >= t1;
    }
    c = wave_sum_u32(c);
    if (t1 != 0ull && c >= (uint32_t)k && c <= 512u) {
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      uint32_t base = 0u;
#pragma unroll
      for (int j = 0; j < kMergeSortedCap / 64; ++j) {
        const bool keep = key[j] != 0ull && key[j] >= t1;
        const uint64_t b = __ballot(keep);
        if (keep)
          kb[base + __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32),
                                              __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u))] = key[j];
        base += (uint32_t)__popcll(b);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      if (base <= 256u)
        regs_sort_write<4>(kb, base, k, 0, q, docs, scores);
      else
        regs_sort_write<8>(kb, base, k, 0, q, docs, scores);
      return;
    }
  }

  if (cnt <= 512u) {
    sort_write_any<8>(kb, cnt, k, 0, q, docs, scores);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  lds_merge_one<kMergeSortedCap / 64>(kb, cnt, k, 0, q, docs, scores);
}

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
// Tile shift of this build (BM25_TILE_SHIFT: 11 = 2048-doc tiles, the product;
// 12 = 4096-doc tiles, a variant build for scripts/variant_lib_time.py).
#ifndef BM25_TILE_SHIFT
#define BM25_TILE_SHIFT 11
#endif
static_assert(BM25_TILE_SHIFT == 11 || BM25_TILE_SHIFT == 12, "2048- or 4096-doc tiles");
bool tile_shift_supported(int s) { return s == BM25_TILE_SHIFT; }
int build_tile_shift() { return BM25_TILE_SHIFT; }

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

hipError_t launch_pool_bounds(const uint16_t* in, int64_t rows, int64_t in_stride, uint16_t* out,
                              int64_t out_stride, hipStream_t stream) {
  if (rows <= 0 || out_stride <= 0) return hipSuccess;
  const int64_t n = rows * out_stride;
  const unsigned blocks = (unsigned)std::min<int64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(pool_bounds_kernel, dim3(blocks), dim3(256), 0, stream, in, rows, in_stride,
                     out, out_stride);
  return hipGetLastError();
}

hipError_t launch_build_bmax(const DevIndex& ix, hipStream_t stream) {
  if (ix.n_terms == 0 || ix.ntiles == 0 || !ix.bmax || ix.sparse) return hipSuccess;
  const int64_t blocks = std::min<int64_t>(ix.n_terms, 65536);
  hipLaunchKernelGGL(build_bmax_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, ix.indptr,
                     ix.rel, ix.val, ix.n_terms, ix.ntiles, ix.bmax);
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
// of each of m doc slices); the first (P, m) in the order P = pmax (the
// handle's sample_p option, default 8), pmax / 2, ... 2 (powers of two), m =
// 1, 2, 4 whose sample — over the W doc shards searched together (global
// threshold) — yields >= 2k keys.  Sample tiles come in groups of G = 8
// consecutive tiles once the index has at least four such groups (G = 1,
// every P-th tile, below).  P = 1: no threshold — the exact top-4 path over
// every tile (small indices).  S = keys per query per shard.
SampleGeom sample_geom(int64_t ntiles, int k, int W, int pmax) {
  for (int P = 64; P >= 2; P >>= 1) {
    if (P > pmax || ntiles < 2 * P) continue;
    const int G = ntiles >= 4 * kSampleGroup * P ? kSampleGroup : 1;
    const int64_t nS = sample_count(ntiles, P, G);
    for (int m = 1; m <= kTileM; m <<= 1)
      if (nS * m * W >= 2 * (int64_t)k) return SampleGeom{P, m, nS * m, G};
  }
  return SampleGeom{1, 0, 0, 1};
}

// Tile-bound keys (P = 0) need the tile bounds (a dense, non-negative index
// with its bmax table; an empty shard contributes no keys either way), at
// most kBoundMaxTiles tiles, a collection of at least kBoundTilesPerK * k
// tiles — one key per tile, and the k-th best single-term maximum is only a
// tight threshold while k is a small share of the tiles (at k ~ tiles / 2
// every query's list overflows) — and queries of at most kBoundMaxTerms
// terms: a longer query's sum of many terms lies further above its largest
// single-term score (16-term queries at config 3: 5.00 ms with tile-bound
// keys, 5.31 sampled).
// Otherwise the SAMPLE pass (sample_geom), whose sample tiles report up to
// 4 real sums each; sample_p = 1 keeps asking for the exact pass.  The key
// width S is the sampled geometry's either way (so bm25_sample_width needs no
// T): any set of such keys of distinct documents gives a valid theta (the
// k-th best of them), and each shard's best S (W * S >= 2k) are the world's
// k best unless a shard holds more than S of them.
SampleGeom search_geom(const DevIndex& ix, int64_t ntiles, int k, int W, int64_t T) {
  const SampleGeom g = sample_geom(ntiles, k, W, ix.opt.sample_p);
  const bool bounds = ix.ntiles == 0 || (ix.bmax != nullptr && ix.nonneg && !ix.sparse);
  if (g.P > 1 && ix.opt.theta_bound && !ix.bound_weak && bounds && k >= 1 && T >= 1 &&
      T <= kBoundMaxTerms &&
      ntiles <= kBoundMaxTiles && ntiles * std::max(W, 1) >= kBoundTilesPerK * (int64_t)k)
    return SampleGeom{0, 1, g.S, 1};
  return g;
}

SampleGeom shard_geom_world(const DevIndex& ix, int k, int64_t T, bool world) {
  if (world && ix.wbmax != nullptr) {
    const SampleGeom g = search_geom(ix, ix.wtiles, k, 1, T);
    if (g.P == 0) return g;
  }
  return search_geom(ix, ix.ntiles, k, 1, T);
}

// Every resident workgroup slot of the current device (a multiple of 8, one
// per XCD round), cached per (kernel, device).
template <class K>
static int persistent_grid(K kernel, int block) {
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
  const int g = ((cus * (occ > 0 ? occ : 1) + 7) / 8) * 8;
  cache[key] = g;
  return g;
}

// The flat kernel serves queries of 1..64 terms over posting arrays that a
// buffer resource addresses (32-bit byte offsets: < 2^30 postings) and item
// ordinals of 32 bits; everything else — and every phase when the handle's
// `flat` option is 0 — takes score_wave_kernel.
static bool use_flat(const DevIndex& ix, int64_t T, int64_t Q) {
  return ix.opt.flat && T >= 1 && T <= 64 && (ix.nnz + kPostingPad) * 4 < 0xFFFFFFF0ll &&
         ix.ntiles * Q < 0x7FFFFFFFll;
}

// Tiles per flat-kernel item: the most the term lanes allow (64 / 2^TL),
// halved while the phase would give the resident waves fewer than
// `items_per_wave` items each — a small doc shard's SAMPLE pass has ~2
// eight-tile items per wave, and the last wave's items set the pass time.
// The fallback stage (a few queries, counted on the device) uses 1-tile items.
static int32_t flat_band(const SearchOpts& o, int64_t nt, int64_t nq, int grid, int bwmax,
                         bool fallback) {
  if (o.flat_bw > 0) return std::min(o.flat_bw, bwmax);
  if (fallback) return 1;
  int32_t bw = bwmax;
  while (bw > 1 && ((nt + bw - 1) / bw) * nq < (int64_t)o.items_per_wave * grid) bw >>= 1;
  return bw;
}

int flat_term_lanes(int64_t T) { return 1 << flat_tl(T); }

template <int S, int PH, int SM, int TL>
static void launch_flat(const DevIndex& ix, const int32_t* q, int64_t T, int64_t Qb,
                        const Stage& sg, const Workspace& ws, hipStream_t st) {
  int32_t* wctr = ws.wctr + (int64_t)sg.ctr_region * kWctrInts;
  // REST of the large-k list path (SM == kLargeM): keys into per-tile slots
  // (ws.slots, ws.slot_cap keys each, counts ws.slot_cnt), the overflow into ws.list
  constexpr bool kSlots = PH == kRest && SM == kLargeM;
  // REST skips the sample tiles whose best key is below theta (m = 1 samples
  // in groups of 8 tiles: ws.cand holds this shard's sample keys)
  const bool skip = PH == kRest && sg.sample_keys != nullptr && sg.M == 1 && sg.G == kSampleGroup;
  IndexArgs a = args_of(ix);
  // one descriptor field: the sample keys' skip or the tile bounds; and the
  // bounds only at 8 term lanes (16 lanes: 4-tile items whose 16 bmax rows cost
  // more than the few tiles they skip — 5.45 vs 5.00 ms, 16-term queries)
  if (skip || TL > 3) a.bmax = nullptr;
  a.seg = ws.seg;
  a.seg_zero = Qb * ((ix.ntiles + 7) >> 3) * 8 * (1 << TL);
  const int64_t nt = PH == kSample ? sample_count(ix.ntiles, sg.P, sg.G) : ix.ntiles;
  auto go = [&](auto kern) {
    int grid = persistent_grid(kern, 64);
    // grid_pct < 100: leave resident slots to another stream's kernels (whole
    // XCD rounds: the item ranges are split over blockIdx % 8)
    if (ix.opt.grid_pct < 100) grid = std::max(8, grid * ix.opt.grid_pct / 100 / 8 * 8);
    if (sg.nq_dev) grid = std::min(grid, 8 * kFallbackBlocks);  // fallback: usually no queries
    // every claim counter of an XCD range needs a wave: counter cm is served
    // by the workgroups with (blockIdx / 8) % claim_m == cm
    const int claim_m = std::max(1, std::min(ix.opt.claim_m, grid / 8));
    // (split items: the table was built for bands of 64 >> TL tiles)
    const int bw = SM == kSplitM ? (64 >> TL)
                                 : flat_band(ix.opt, nt, sg.nq_host, grid, 64 >> TL, sg.nq_dev != nullptr);
    ix.disp.kernels |= PH == kSample ? kKFlatSample : (PH == kRest ? kKFlatRest : kKFlatAll);
    if (PH == kRest && SM == 2) ix.disp.kernels |= kKCountSkips;
    ix.disp.term_lanes = 1 << TL;
    ix.disp.band_tiles[PH] = bw;
    hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(64), 0, st, a, q, (int32_t)T, sg.P,
                       sg.G, sg.nq_host, sg.nq_dev, sg.qmap, ws.theta,
                       kSlots ? ws.slots : sg.cand_out, kSlots ? (int64_t)ws.slot_cap : sg.cstride,
                       ws.list, ws.list_cnt, ws.list_cap, wctr, ix.opt.claim_ch, claim_m,
                       skip ? sg.sample_keys : nullptr, sg.sample_stride, bw,
                       PH == kSample && SM == 1 ? sg.cand_mirror : nullptr,
                       PH == kRest ? ws.counters + 5 : nullptr, kSlots ? ws.slot_cnt : nullptr,
                       SM == kSplitM ? ws.sub : nullptr, SM == kSplitM ? ws.sub_ipb : nullptr);
  };
  if (ix.sparse)
    go(score_flat_kernel<S, PH, SM, true, TL>);
  else
    go(score_flat_kernel<S, PH, SM, false, TL>);
}

template <int S, int PH, int SM>
static void launch_flat_tl(const DevIndex& ix, const int32_t* q, int64_t T, int64_t Qb,
                           const Stage& sg, const Workspace& ws, hipStream_t st) {
  switch (flat_tl(T)) {
    case 3: launch_flat<S, PH, SM, 3>(ix, q, T, Qb, sg, ws, st); break;
    case 4: launch_flat<S, PH, SM, 4>(ix, q, T, Qb, sg, ws, st); break;
    case 5: launch_flat<S, PH, SM, 5>(ix, q, T, Qb, sg, ws, st); break;
    default: launch_flat<S, PH, SM, 6>(ix, q, T, Qb, sg, ws, st); break;
  }
}

// One score phase of a search over the batch of Qb queries (the stage may
// cover a subset: the fallback stage's qmap).
template <int S, int PH>
static void launch_phase(const DevIndex& ix, const int32_t* q, int64_t T, int64_t Qb,
                         const Stage& sg, const Workspace& ws, hipStream_t st) {
  if (use_flat(ix, T, Qb)) {
    if constexpr (PH == kSample) {  // m keys per sample tile: a build per m
      if (sg.M == 2) return launch_flat_tl<S, PH, 2>(ix, q, T, Qb, sg, ws, st);
      if (sg.M == kTileM) return launch_flat_tl<S, PH, kTileM>(ix, q, T, Qb, sg, ws, st);
      if (sg.M == kLargeM) return launch_flat_tl<S, PH, kLargeM>(ix, q, T, Qb, sg, ws, st);
    }
    if constexpr (PH == kRest) {
      if (sg.M == kLargeM && ws.slots != nullptr)  // the large-k list path's slots
        return launch_flat_tl<S, PH, kLargeM>(ix, q, T, Qb, sg, ws, st);
      if (ix.opt.count_skips)  // the build that counts the skipped postings
        return launch_flat_tl<S, PH, 2>(ix, q, T, Qb, sg, ws, st);
      if (sg.split && ws.sub != nullptr && flat_tl(T) == 3)  // split items (8-tile bands)
        return launch_flat_tl<S, PH, kSplitM>(ix, q, T, Qb, sg, ws, st);
    }
    return launch_flat_tl<S, PH, 1>(ix, q, T, Qb, sg, ws, st);
  }
  int32_t* wctr = ws.wctr + (int64_t)sg.ctr_region * kWctrInts;
  (void)wctr;
  ix.disp.kernels |= PH == kSample ? kKWaveSample : (PH == kRest ? kKWaveRest : kKWaveAll);
  int grid = persistent_grid(score_wave_kernel<S, PH>, 64 * kWaves);
  if (sg.nq_dev) grid = std::min(grid, 8 * kFallbackBlocks);
  hipLaunchKernelGGL((score_wave_kernel<S, PH>), dim3((unsigned)grid), dim3(64 * kWaves), 0, st,
                     args_of(ix), q, (int32_t)T, sg, ws.theta, sg.cand_out, ws.list, ws.list_cnt,
                     ws.list_cap);
}

// Sparse index: the segment of every (query, term position, tile) the flat
// kernel reads, from the query terms' tile lists — one wave per (query, term
// position) walks its term's non-empty tiles (coalesced reads) and writes
// (start | len << 32) into seg[q][tile / 8][pos][tile % 8] (TT term slots per
// 8-tile group: a term's entries of one group are one 64-B run); seg was
// zeroed (empty segments).
__global__ __launch_bounds__(256) void seg_table_kernel(IndexArgs a,
                                                        const int32_t* __restrict__ queries,
                                                        int64_t Q, int32_t T, int32_t TT,
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
  uint64_t* row = seg + q * nbp * 8 * TT;
  for (int64_t i = b + lane_id(); i < e; i += 64) {
    const uint32_t tile = a.tl_tile[i];
    const uint32_t st = a.tl_start[i];
    const uint32_t nx = i + 1 < e ? a.tl_start[i + 1] : df;
    row[(int64_t)(tile >> 3) * 8 * TT + pos * 8 + (tile & 7)] =
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

// u64 entries of the per-search segment table (+ 64 zero entries past it).
int64_t seg_entries(const DevIndex& ix, int64_t Q, int64_t T) {
  if (!ix.sparse || !use_flat(ix, T, Q)) return 0;
  return Q * ((ix.ntiles + 7) >> 3) * 8 * flat_term_lanes(T) + 64;
}

static void launch_seg_table(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T,
                             const Workspace& ws, hipStream_t st) {
  hipMemsetAsync(ws.seg, 0, sizeof(uint64_t) * seg_entries(ix, Q, T), st);
  const int64_t waves = Q * T;
  hipLaunchKernelGGL(seg_table_kernel, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st,
                     args_of(ix), q, Q, (int32_t)T, (int32_t)flat_term_lanes(T), ws.seg);
}

// P != 1: the thresholded search (sampled, or tile-bound keys at P = 0; its
// merge reads the list only: nt = 0); P = 1: the exact path over every tile.
static Stage main_stage(const DevIndex& ix, int64_t Q, int P, const Workspace& ws) {
  Stage sg{};
  sg.cand = ws.cand;
  sg.cand_out = ws.cand;
  sg.cstride = ix.ntiles * kTileM;
  sg.P = P;
  sg.G = 1;
  sg.nt = P != 1 ? 0 : ix.ntiles;
  sg.nq_host = (int32_t)Q;
  if (P != 1) {
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

// SAMPLE pass: each query's S keys into keys[Q][S] (zero-padded); the flat
// kernel also writes a copy (m = 1) into ws.cand for the REST pass's
// sample-tile skip — the caller's buffer may change before launch_finish.
template <int S_>
static void sample_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T,
                     const SampleGeom& g, uint64_t* keys, const Workspace& ws, hipStream_t st) {
  // the SAMPLE pass writes a key (0: no positive sum) for every sample tile
  // of every query; only a shard with fewer sample tiles than the widest
  // shard leaves padding to clear.  Counters: theta_wave_kernel resets them.
  if (sample_count(ix.ntiles, g.P, g.G) * g.m < g.S)
    hipMemsetAsync(keys, 0, sizeof(uint64_t) * Q * g.S, st);
  if (seg_entries(ix, Q, T) > 0) launch_seg_table(ix, q, Q, T, ws, st);  // SAMPLE + REST + fallback
  Stage sg = main_stage(ix, Q, g.P, ws);
  sg.ctr_region = 0;
  sg.M = g.m;
  sg.G = g.G;
  sg.cand_out = keys;
  sg.cand_mirror = keys != ws.cand ? ws.cand : nullptr;
  sg.cstride = g.S;
  launch_phase<S_, kSample>(ix, q, T, Q, sg, ws, st);
}

// theta from the W shards' sample keys [W][Q][S], then the REST pass (or, P =
// 1, the exact pass over every tile).
template <int S_>
static void finish_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int k,
                     const SampleGeom& g, int W, const uint64_t* all_keys, const Workspace& ws,
                     hipStream_t st, bool theta_ready = false, hipStream_t st_rest = nullptr,
                     hipEvent_t join = nullptr, hipEvent_t rest_timing = nullptr,
                     bool split = false) {
  Stage sg = main_stage(ix, Q, g.P, ws);
  sg.split = split;
  // the score pass's stream: after everything enqueued on st so far
  auto to_rest = [&]() -> hipStream_t {
    if (st_rest == nullptr || st_rest == st || join == nullptr) {
      if (rest_timing) hipEventRecord(rest_timing, st);
      return st;
    }
    hipEventRecord(join, st);
    hipStreamWaitEvent(st_rest, join, 0);
    if (rest_timing) hipEventRecord(rest_timing, st_rest);
    return st_rest;
  };
  if (g.P == 1) {  // no sample pass ran: nothing was zeroed, no segment table built
    hipMemsetAsync(ws.counters, 0, kCounters * sizeof(int32_t), st);
    if (seg_entries(ix, Q, T) > 0) launch_seg_table(ix, q, Q, T, ws, st);
    sg.ctr_region = 2;
    launch_phase<S_, kAll>(ix, q, T, Q, sg, ws, to_rest());
    return;
  }
  sg.ctr_region = 1;  // counters and list counts: reset by theta_wave_kernel
  sg.M = g.m;
  sg.G = g.G;
  if (g.P > 1) {  // the sample tiles' keys: launch_sample left this shard's copy there
    sg.sample_keys = ws.cand;
    sg.sample_stride = g.S;
  }
  if (!theta_ready)
    hipLaunchKernelGGL(theta_wave_kernel, dim3((unsigned)((Q + kQW - 1) / kQW)), dim3(64 * kQW), 0, st,
                       all_keys, (int64_t)W, Q, g.S, (int32_t)k, ws.theta, ws.list_cnt,
                       ws.list_cap, ix.nonneg ? 1 : 0, ix.doc_offset, ix.n_docs, ws.counters);
  launch_phase<S_, kRest>(ix, q, T, Q, sg, ws, to_rest());
}

#define BM25_SHIFT_DISPATCH(call)                        \
  switch (ix.tile_shift) {                               \
    case BM25_TILE_SHIFT: call(BM25_TILE_SHIFT); break;    \
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
  if (g.P == 0) {  // tile-bound keys: no posting is scored before REST
    if (ix.bmax == nullptr || ix.ntiles > kBoundMaxTiles || Q > 0x7FFFFFFF || T > kBoundMaxTerms)
      return hipErrorInvalidValue;
    if (seg_entries(ix, Q, T) > 0) launch_seg_table(ix, d_queries, Q, T, ws, stream);
    ix.disp.kernels |= kKBound;
    hipLaunchKernelGGL(bound_keys_kernel, dim3((unsigned)Q), dim3(kBoundNT),
                       (size_t)(bmax_stride(ix.ntiles) * 2), stream, args_of(ix), ix.bmax,
                       d_queries, (int32_t)T, ix.tile_shift, g.S, keys, (uint64_t*)nullptr,
                       (int32_t*)nullptr, (int32_t*)nullptr, 0, (int64_t)0, (uint32_t*)nullptr,
                       (uint32_t*)nullptr, (int32_t*)nullptr, (int32_t*)nullptr, 0, 0);
    return hipGetLastError();
  }
#define CALL(s) sample_s<s>(ix, d_queries, Q, T, g, keys, ws, stream)
  BM25_SHIFT_DISPATCH(CALL)
#undef CALL
  return hipGetLastError();
}

hipError_t launch_finish(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                         int k, const SampleGeom& g, int W, const uint64_t* all_keys,
                         const Workspace& ws, hipStream_t stream, hipStream_t rest_stream,
                         hipEvent_t join, hipEvent_t rest_timing) {
  if (Q == 0 || ix.ntiles == 0) {
    if (rest_stream && rest_stream != stream && join) {  // (the caller's order still holds)
      hipEventRecord(join, stream);
      hipStreamWaitEvent(rest_stream, join, 0);
    }
    if (rest_timing) hipEventRecord(rest_timing, rest_stream ? rest_stream : stream);
    return hipGetLastError();
  }
#define CALL(s) finish_s<s>(ix, d_queries, Q, T, k, g, W, all_keys, ws, stream, false, \
                            rest_stream, join, rest_timing)
  BM25_SHIFT_DISPATCH(CALL)
#undef CALL
  return hipGetLastError();
}

// The large-k list path's score passes (bm25mi_large.hip): a SAMPLE pass with
// kLargeM keys per sample tile (the best of each 256-doc slice) into
// keys[Q][g.S], then a REST pass that appends every key >= ws.theta[q] to
// ws.list (capacity ws.list_cap, counts ws.list_cnt: the caller's buffers).
hipError_t launch_sample_large(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                               const SampleGeom& g, uint64_t* keys, const Workspace& ws,
                               hipStream_t stream) {
  if (Q == 0 || ix.ntiles == 0) return hipSuccess;
  if (g.m != kLargeM || g.P < 2 || !use_flat(ix, T, Q)) return hipErrorInvalidValue;
  if (sample_count(ix.ntiles, g.P, g.G) * g.m < g.S)
    hipMemsetAsync(keys, 0, sizeof(uint64_t) * Q * g.S, stream);
  if (seg_entries(ix, Q, T) > 0) launch_seg_table(ix, d_queries, Q, T, ws, stream);
  Stage sg = main_stage(ix, Q, g.P, ws);
  sg.ctr_region = 0;
  sg.M = g.m;
  sg.G = g.G;
  sg.cand_out = keys;
  sg.cstride = g.S;
#define CALL(s_) launch_phase<s_, kSample>(ix, d_queries, T, Q, sg, ws, stream)
  BM25_SHIFT_DISPATCH(CALL)
#undef CALL
  return hipGetLastError();
}

hipError_t launch_rest_lists(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                             const SampleGeom& g, const Workspace& ws, hipStream_t stream) {
  if (Q == 0 || ix.ntiles == 0) return hipSuccess;
  if (!use_flat(ix, T, Q)) return hipErrorInvalidValue;
  Stage sg = main_stage(ix, Q, g.P, ws);
  sg.ctr_region = 1;
  sg.M = g.m;
  sg.G = g.G;
#define CALL(s_) launch_phase<s_, kRest>(ix, d_queries, T, Q, sg, ws, stream)
  BM25_SHIFT_DISPATCH(CALL)
#undef CALL
  return hipGetLastError();
}

bool large_list_supported(const DevIndex& ix, int64_t T, int64_t Q) {
  return ix.nonneg && use_flat(ix, T, Q);
}

hipError_t launch_score(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                        int k, const Workspace& ws, hipStream_t stream, bool world) {
  world = world && ix.wbmax != nullptr;
  // a shard with world bounds sizes its threshold geometry by the collection
  // (shard_geom_world: its own geometry where the world's tile bounds do not
  // serve — the shard's own k-th key is a valid, looser threshold)
  const SampleGeom g = shard_geom_world(ix, k, T, world);
  world = world && g.P == 0;
  const int64_t ntg = world ? ix.wtiles : ix.ntiles;
  // split REST items where the waves get few items each (a doc shard of a
  // few GPUs' collection: ~16 at W = 8): the heavy queries' last items set
  // when the pass ends
  static int cus = 0;
  if (cus == 0 && hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ix.device) != hipSuccess)
    cus = 256;
  const bool split = ix.opt.rest_split && ws.sub != nullptr && g.P == 0 && flat_tl(T) == 3 &&
                     use_flat(ix, T, Q) && Q < (1 << 20) &&
                     ((ix.ntiles + 7) / 8) * Q < (int64_t)kSplitItemsPerWave * 19 * cus;
  if (split) ix.disp.kernels |= kKRestSplit;
  if (g.P == 0 && Q > 0 && ix.ntiles > 0) {
    // one index: the bound kernel selects theta itself (no key list, no theta
    // kernel); world: the threshold of the whole collection, from every
    // shard's bounds (the keys >= it of this shard go to the W-way merge)
    if (ix.bmax == nullptr || ntg > kBoundMaxTiles || Q > 0x7FFFFFFF || T > kBoundMaxTerms)
      return hipErrorInvalidValue;
    if (seg_entries(ix, Q, T) > 0) launch_seg_table(ix, d_queries, Q, T, ws, stream);
    ix.disp.kernels |= kKBound;
    // the pooled bounds where they hold enough groups (a quarter of the bytes;
    // the threshold only needs k groups' bounds, DevIndex::bpool)
    const bool pool =
        ix.opt.bound_pool &&
        (world ? ix.wbpool != nullptr && ix.wgroups >= kPoolGroupsPerK * (int64_t)k
               : ix.bpool != nullptr && (ix.ntiles + kPool - 1) / kPool >= kPoolGroupsPerK * (int64_t)k);
    if (pool) ix.disp.kernels |= kKBoundPool;
    const uint16_t* tb = world ? (pool ? ix.wbpool : ix.wbmax) : (pool ? ix.bpool : ix.bmax);
    const int64_t tstride = world ? (pool ? ix.wpstride : ix.wstride) : (pool ? ix.pstride : 0);
    const size_t lds = world ? (size_t)(ix.wW * tstride * 2)
                             : (size_t)((pool ? ix.pstride : bmax_stride(ix.ntiles)) * 2);
    hipLaunchKernelGGL(bound_keys_kernel, dim3((unsigned)Q), dim3(kBoundNT), lds, stream,
                       args_of(ix), tb, d_queries, (int32_t)T,
                       ix.tile_shift, (int64_t)k, (uint64_t*)nullptr, ws.theta, ws.list_cnt,
                       ws.counters, world ? ix.wW : 0, tstride, ws.qw,
                       split ? ws.sub : (uint32_t*)nullptr, ws.sub_ipb, ws.sub_done, (int32_t)Q,
                       64 >> flat_tl(T));
#define CALL(s) finish_s<s>(ix, d_queries, Q, T, k, g, 1, ws.cand, ws, stream, true, nullptr, \
                            nullptr, nullptr, split)
    BM25_SHIFT_DISPATCH(CALL)
#undef CALL
    return hipGetLastError();
  }
  hipError_t e = launch_sample(ix, d_queries, Q, T, g, ws.cand, ws, stream);
  if (e != hipSuccess) return e;
  return launch_finish(ix, d_queries, Q, T, k, g, 1, ws.cand, ws, stream);
}

template <int S>
static void select_stage(const DevIndex& ix, const int32_t* q, int64_t T, int k, const Stage& sg,
                         const Workspace& ws, int32_t* docs, float* scores, hipStream_t st) {
  const int64_t maxflag = maxflag_for(k, sg.nt);
  if (sg.theta && !sg.qmap && sg.nt == 0 && k <= kFastMaxK) {
    // sampled main stage: one wavefront per query; the queries it leaves go
    // to the block merge below (their count on the device, usually 0)
    // (merge_tail_kernel takes the queries it leaves)
    hipLaunchKernelGGL(merge_fast_kernel, dim3((unsigned)((sg.nq_host + kQW - 1) / kQW)), dim3(64 * kQW), 0,
                       st, sg, (int32_t)k, ix.doc_offset, ws, docs, scores);
    return;
  }
  // the fallback stage (query count on the device, usually 0): a few blocks
  const unsigned mgrid = (unsigned)(sg.nq_dev ? std::min<int64_t>(sg.nq_host, kFallbackBlocks)
                                              : sg.nq_host);
  hipLaunchKernelGGL(merge_first_kernel, dim3(mgrid), dim3(kMergeNT), 0, st, sg, (int32_t)k,
                     maxflag, ix.doc_offset, ix.n_docs, ws, docs, scores);
  if (k > kTileM && sg.nt > 0) {  // tiles with exact top-4 candidates may need a rescore
    hipLaunchKernelGGL(rescore_kernel<S>, dim3(sg.nq_dev ? kFallbackBlocks : 256),
                       dim3(kRescoreNT), 0, st, args_of(ix), q, (int32_t)T, (int32_t)k, maxflag,
                       sg, ws);
    hipLaunchKernelGGL(merge_final_kernel, dim3(mgrid), dim3(kMergeNT), 0, st, sg, (int32_t)k,
                       maxflag, ix.doc_offset, ws, docs, scores);
  }
}

template <int S_>
static void select_s(const DevIndex& ix, const int32_t* q, int64_t Q, int64_t T, int k, int P,
                     const Workspace& ws, int32_t* docs, float* scores, hipStream_t st,
                     bool unsorted) {
  Stage ms = main_stage(ix, Q, P, ws);
  ms.unsorted = unsorted;
  select_stage<S_>(ix, q, T, k, ms, ws, docs, scores, st);
  if (P == 1) return;
  // queries whose list overflowed: exact pass over every tile (usually none;
  // the kernels read their count on the device and exit at once).  The
  // rescore queue counters [0], [1] are still 0 from theta_wave_kernel (the
  // sampled main stage has no tile candidates to rescore).
  Stage fb = fallback_stage(ix, Q, ws);
  fb.ctr_region = 2;
  launch_phase<S_, kAll>(ix, q, T, Q, fb, ws, st);
  if (k > kFastMaxK) {  // the block merges throughout
    select_stage<S_>(ix, q, T, k, fb, ws, docs, scores, st);
    return;
  }
  Stage sl = ms;  // the queries merge_fast_kernel left
  sl.qmap = ws.slow;
  sl.nq_dev = ws.counters + 4;
  sl.remap = true;
  hipLaunchKernelGGL(merge_tail_kernel<S_>, dim3((unsigned)std::min<int64_t>(Q, kFallbackBlocks)),
                     dim3(kMergeNT), 0, st, args_of(ix), q, (int32_t)T, sl, fb, (int32_t)k,
                     maxflag_for(k, fb.nt), ws, docs, scores);
}

hipError_t launch_select(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                         int k, int P, const Workspace& ws, int32_t* d_docs, float* d_scores,
                         hipStream_t stream, bool unsorted) {
  if (Q == 0 || k == 0) return hipSuccess;
  if (ix.ntiles == 0) {  // an empty doc shard: an all-padding list (doc -1, score bits ~0)
    hipMemsetAsync(d_docs, 0xFF, sizeof(int32_t) * Q * k, stream);
    hipMemsetAsync(d_scores, 0xFF, sizeof(float) * Q * k, stream);
    return hipGetLastError();
  }
#define CALL(s) select_s<s>(ix, d_queries, Q, T, k, P, ws, d_docs, d_scores, stream, unsorted)
  BM25_SHIFT_DISPATCH(CALL)
#undef CALL
  return hipGetLastError();
}

hipError_t launch_scores_dense(const DevIndex& ix, const int32_t* d_query, int64_t T,
                               float* d_out, hipStream_t stream) {
  if (ix.ntiles == 0) return hipSuccess;
  if (ix.tile_shift != BM25_TILE_SHIFT) return hipErrorInvalidValue;
  hipLaunchKernelGGL(scores_dense_kernel<BM25_TILE_SHIFT>, dim3((unsigned)ix.ntiles), dim3(64),
                     0, stream, args_of(ix), d_query, (int32_t)T, d_out);
  return hipGetLastError();
}

hipError_t launch_scores_batch(const DevIndex& ix, const int32_t* d_queries, int64_t G, int64_t T,
                               int64_t stride, float* d_out, hipStream_t stream) {
  if (ix.ntiles == 0 || G == 0) return hipSuccess;
  if (ix.tile_shift != BM25_TILE_SHIFT || G > 65535 || stride < (ix.ntiles << ix.tile_shift))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(scores_batch_kernel<BM25_TILE_SHIFT>, dim3((unsigned)ix.ntiles, (unsigned)G),
                     dim3(64), 0, stream, args_of(ix), d_queries, (int32_t)T, stride, d_out);
  return hipGetLastError();
}

hipError_t launch_merge_lists(const int32_t* d_docs, const float* d_scores, int64_t W,
                              int64_t Q, int k, int64_t rank_stride, bool sorted,
                              int32_t* d_out_docs, float* d_out_scores, hipStream_t stream) {
  if (Q == 0 || k == 0) return hipSuccess;
  if (k > kMaxK)  // the sort-based merge of the large-k path (bm25mi_large.hip)
    return launch_merge_large(d_docs, d_scores, W, Q, k, rank_stride, d_out_docs, d_out_scores,
                              stream);
  if (sorted && W * k <= kMergeSortedCap && W <= 64) {
    hipLaunchKernelGGL(merge_sorted_kernel, dim3((unsigned)((Q + kQW - 1) / kQW)), dim3(64 * kQW), 0, stream,
                       d_docs, d_scores, (int32_t)W, Q, (int32_t)k, rank_stride, d_out_docs,
                       d_out_scores);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(merge_lists_kernel, dim3((unsigned)Q), dim3(kMergeNT), 0, stream, d_docs,
                     d_scores, W, Q, (int32_t)k, rank_stride, d_out_docs, d_out_scores);
  return hipGetLastError();
}

}  // namespace bm25mi

#if BM25_TRACE
// Dev variant builds only: the last REST pass's per-wave trace (4 u64 per
// wave: start clock, end clock, items, rows; 100 MHz clock).
extern "C" int bm25_debug_trace(uint64_t* out, int64_t n_waves) {
  const int64_t n = n_waves < bm25mi::kTraceWaves ? n_waves : bm25mi::kTraceWaves;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(bm25mi::g_bm25_trace), sizeof(uint64_t) * 4 * n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 2;
}
#endif
