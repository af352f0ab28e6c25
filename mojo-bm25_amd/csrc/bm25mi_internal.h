// bm25mi_internal.h — shared declarations between the C-ABI host code
// (bm25mi_capi.cpp) and the gfx950 kernels (bm25mi_kernels.hip).
//
// Device layout of one index:
//   val   f32 [nnz+pad]      the CSC `data` array, unchanged order (term-major,
//                            doc-ascending inside a term)
//   ldoc  u16 [nnz+pad]      LDS slot of the doc inside its tile: the doc's
//                            tile-local id (doc & (D-1)) through the fixed
//                            accumulator permutation acc_slot() below; the
//                            tile of a posting is implied by its position
//                            (pad: kPostingPad elements so 4-posting vector
//                            loads of a segment's last row stay in bounds)
//   indptr i64 [V+1]         CSC column pointers
//   rel   u32 [V][ntiles+1]  rel[t][j] = first posting of term t whose doc is
//                            in tile j or later, relative to indptr[t]
// so the postings of term t inside doc tile j are
//   [indptr[t] + rel[t][j], indptr[t] + rel[t][j+1]).
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>

namespace bm25mi {

// Candidate key: (sortable f32 score bits) << 32 | (0xFFFFFFFF - doc).
// Larger key == better: higher score first, then smaller doc id.
// Key 0 never encodes a real (non-NaN) score and marks an empty slot.
__host__ __device__ inline uint32_t score_key(float s) {
  uint32_t u;
  __builtin_memcpy(&u, &s, 4);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__host__ __device__ inline float key_score(uint32_t k) {
  uint32_t u = (k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k;
  float s;
  __builtin_memcpy(&s, &u, 4);
  return s;
}
__host__ __device__ inline uint64_t make_key(float s, uint32_t doc) {
  return ((uint64_t)score_key(s) << 32) | (uint64_t)(0xFFFFFFFFu - doc);
}

// Per-tile candidates emitted by the score pass.
constexpr int kTileM = 4;
// Largest k served by the tile/merge path.
constexpr int kMaxK = 4096;
// Merge kernel LDS: number of u64 keys sorted at once.
constexpr int kMergeP = 8192;
// One full posting row (4 postings x 1024 lanes) past the end, so row loads
// never need clamping (their out-of-segment lanes are masked, not skipped).
constexpr int64_t kPostingPad = 4 * 1024 + 8;

struct DevIndex {
  int device = 0;
  int64_t n_docs = 0, n_terms = 0, nnz = 0, doc_offset = 0;
  int tile_shift = 14;
  int64_t ntiles = 0;
  int64_t* indptr = nullptr;
  uint32_t* rel = nullptr;
  uint16_t* ldoc = nullptr;
  float* val = nullptr;
};

// Segment descriptor of one (item, query term): the term's postings inside
// the item's tile are [beg, beg + len); pre = postings of the item's earlier
// terms (the term's offset in the item's concatenated posting stream).
struct SegDesc {
  int64_t beg;
  uint32_t len;
  uint32_t pre;
};

struct Workspace {
  int64_t cap_q = 0, cap_k = 0;
  uint64_t* cand = nullptr;      // [Q][ntiles][kTileM]
  uint64_t* theta = nullptr;     // [Q] k-th key of the sample tiles' candidates
  uint64_t* cand2 = nullptr;     // [Q][maxflag][k]  exact top-k of re-scored tiles
  int32_t* flag_tiles = nullptr; // [Q][maxflag]
  int32_t* nflag = nullptr;      // [Q]
  int32_t* counters = nullptr;   // [0]/[1] rescore queue length / pop cursor,
                                 // [2]/[3] overflow queue length / pop cursor
  int32_t* ovq = nullptr;        // [Q*ntiles] REST tiles to fix up (q*ntiles + tile)
  int32_t* queue = nullptr;      // [Q*maxflag] items = q*maxflag + i
  SegDesc* desc = nullptr;       // [ntiles][Q][T] when T <= 16
  int64_t cap_desc = 0;
  int32_t* wctr = nullptr;       // [16] per-XCD-group item counters (2 score phases)
};

// Flag slots per query: a flagged tile holds kTileM keys of the top-(k-1), so
// at most (k-1)/kTileM tiles (and never more than the tiles that exist).
// Accumulator layout of a tile of D = 2^S docs: tile-local doc d belongs to
// selection thread t = d / 32 (entry e = d % 32, so lane order == doc order)
// and lives at float index ((e/4) * NT + t) * 4 + e % 4 with NT = D / 32:
// the selection's float4 reads (j*NT + t) are then conflict-free.
__host__ __device__ inline uint32_t acc_slot(uint32_t d, int S) {
  return ((d & 28u) << (S - 5)) | ((d >> 3) & ~3u) | (d & 3u);
}

inline int64_t maxflag_for(int k, int64_t ntiles) {
  const int64_t m = (k + kTileM - 1) / kTileM;
  return m < ntiles ? m : (ntiles > 0 ? ntiles : 1);
}

// Kernel launchers (bm25mi_kernels.hip).  All enqueue on `stream`.
hipError_t launch_build_tables(const DevIndex& ix, const int32_t* d_indices,
                               int32_t* d_err, hipStream_t stream);
// Score pass: every (tile, query) -> kTileM candidate keys per tile
// (sample tiles: exact top-kTileM; other tiles: the keys above the sample's
// k-th key, or their exact top-kTileM when more than kTileM pass).
hipError_t launch_score_tiles(const DevIndex& ix, const int32_t* d_queries,
                              int64_t Q, int64_t T, int k, const Workspace& ws,
                              hipStream_t stream);
// Queries with at most this many terms use per-batch segment descriptors.
constexpr int kDescMaxT = 16;
// Merge + rescore + final merge.
hipError_t launch_select(const DevIndex& ix, const int32_t* d_queries,
                         int64_t Q, int64_t T, int k, const Workspace& ws,
                         int32_t* d_docs, float* d_scores, hipStream_t stream);
hipError_t launch_scores_dense(const DevIndex& ix, const int32_t* d_query,
                               int64_t T, float* d_out, hipStream_t stream);
hipError_t launch_merge_lists(const int32_t* d_docs, const float* d_scores,
                              int64_t W, int64_t Q, int k, int32_t* d_out_docs,
                              float* d_out_scores, hipStream_t stream);

// Tile shifts with compiled kernels.
bool tile_shift_supported(int s);

}  // namespace bm25mi
