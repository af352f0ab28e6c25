// bm25mi_internal.h — shared declarations between the C-ABI host code
// (bm25mi_capi.cpp) and the gfx950 kernels (bm25mi_kernels.hip).
//
// Device layout of one index, tiles of D = 2^S docs (S = 11):
//   val   f32 [nnz+64]       the CSC `data` array, unchanged order (term-major,
//                            doc-ascending inside a term)
//   ldoc  u16 [nnz+64]       the doc's tile-local id (= its LDS accumulator
//                            slot); the tile of a posting is implied by its
//                            position
//   indptr i64 [V+1]         CSC column pointers
//   rel   u32 [V][ntiles+1]  rel[t][j] = first posting of term t whose doc is
//                            in tile j or later, relative to indptr[t]
// so the postings of term t inside tile j are
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

// Exact candidates kept per sample tile.
constexpr int kTileM = 4;
// Keys per sample tile of the large-k list path (the best of each 256-doc slice).
constexpr int kLargeM = 8;
constexpr int kSplitM = 3;  // the REST build over split items (bm25mi_kernels.hip)
constexpr int kSplitItemsPerWave = 48;  // split REST items below this many items per wave
// Largest k of the sampled-threshold pipeline; larger k (up to n_docs) take
// the large-k path (bm25mi_large.hip).
constexpr int kMaxK = 4096;
// Merge kernel LDS: number of u64 keys sorted at once.
constexpr int kMergeP = 8192;
// Posting arrays carry a small tail (so posting 0 exists for an empty index).
constexpr int64_t kPostingPad = 64;
// Tile: 2^11 = 2048 docs, one wavefront's LDS accumulator (8 KB).
constexpr int kDefaultTileShift = 11;

// Item claims of the flat score kernel (bm25mi_kernels.hip): counters per
// XCD (allocated), int32 stride between counters (256 B).
constexpr int kClaimM = 8;
constexpr int kCtrStride = 64;
// Sample tiles come in groups of kSampleGroup consecutive tiles (sample_geom).
constexpr int kSampleGroup = 8;
constexpr int kWctrInts = 8 * kClaimM * kCtrStride;
// Finished-wave count of a claim counter's waves: 128 B past the counter.
constexpr int kDoneOff = 32;
// Claim-counter regions of a search: SAMPLE, REST (or the exact pass), fallback.
constexpr int kWctrRegions = 3;

// Search dispatch options of one index handle: a snapshot of the BM25_*
// environment at bm25_index_create, changed by bm25_index_set_option
// (include/bm25mi.h lists the names).  Read per search — never cached in
// function statics — so every option takes effect on the next search.
struct SearchOpts {
  int flat = 1;            // 0: score_wave_kernel for every phase
  int flat_bw = 0;         // tiles per flat item: 0 = auto, else 1, 2, 4 or 8
  int items_per_wave = 4;  // auto flat_bw: halve while a phase gives fewer items per wave (c2: 4 > 8)
  int sample_p = 8;        // largest sampling stride (1: the exact pass over every tile)
  int list_cap = 0;        // candidate-list capacity per query (0: auto)
  int claim_ch = 1;        // flat items per claim
  int claim_m = 4;         // claim counters per XCD (1..kClaimM)
  int tile_bound = 1;      // REST skips tiles whose term-maxima sum is below theta (needs bmax)
  int theta_bound = 1;     // threshold keys from the tile bounds instead of a SAMPLE pass
                           // (needs bmax; search_geom)
  int count_skips = 0;     // REST counts the postings its tile bound skips (a build of its own)
  int grid_pct = 100;      // percent of the resident slots the persistent score kernels take
  int large_lists = 1;     // k > kMaxK: the list path (0: dense score rows for every query)
  int rest_split = 0;      // REST over split items where the waves get few items (measured: no gain)
  int bound_pool = 1;      // the tile-bound threshold from the pooled bounds (bpool / wbpool) where
                           // they hold >= kPoolGroupsPerK * k groups
};

// What the last search launched (bm25_search_dispatch).
enum {
  kKFlatSample = 1, kKFlatRest = 2, kKFlatAll = 4,
  kKWaveSample = 8, kKWaveRest = 16, kKWaveAll = 32,
  kKLarge = 64,  // the large-k path (k > kMaxK): dense scores + radix selection
  kKBound = 128, // tile-bound threshold keys (bound_keys_kernel) instead of a SAMPLE pass
  kKBoundOff = 256,  // (not a kernel) the tile-bound threshold was off for this search:
                     // earlier ones overflowed with it (DevIndex::bound_weak)
  kKCountSkips = 512,  // (a flag) REST counted the postings its tile bound skipped
  kKRestSplit = 1024,  // (a flag) REST ran over split items (heavy queries' bands in pieces)
  kKBoundPool = 2048,  // (a flag) the tile-bound threshold came from the pooled bounds
};
struct Dispatch {
  uint32_t kernels = 0;       // kK* bits of the score kernels launched
  int32_t term_lanes = 0;     // flat kernel: term lanes per tile (8, 16, 32, 64)
  int32_t band_tiles[3] = {0, 0, 0};  // flat kernel: tiles per item of ALL, SAMPLE, REST
  int32_t sample_p = 0;       // sampling stride (1: exact pass, 0: tile-bound keys)
};

// Row stride of the tile-bound table: whole groups of four tiles (8 B).
__host__ __device__ inline int64_t bmax_stride(int64_t ntiles) { return (ntiles + 3) & ~(int64_t)3; }

struct DevIndex {
  int device = 0;
  int64_t n_docs = 0, n_terms = 0, nnz = 0, doc_offset = 0;
  int tile_shift = kDefaultTileShift;
  bool nonneg = false;  // every CSC value is 0 or >= FLT_MIN (running sums are monotone)
  int64_t ntiles = 0;
  int64_t* indptr = nullptr;
  // Segment table, dense or sparse: the postings of term t in
  // tile j are [indptr[t] + r(t, j), indptr[t] + r(t, j + 1)) where
  //   dense:  r(t, j) = rel[t * (ntiles + 1) + j]          (V x (ntiles+1) u32)
  //   sparse: the term's non-empty tiles tl_tile[tl_ptr[t] .. tl_ptr[t+1])
  //           (ascending u16) with their first postings tl_start (u32,
  //           relative to indptr[t]) — O(non-empty (term, tile) pairs).
  bool sparse = false;
  uint32_t* rel = nullptr;
  int64_t* tl_ptr = nullptr;
  uint16_t* tl_tile = nullptr;
  uint32_t* tl_start = nullptr;
  int64_t n_pairs = 0;
  uint16_t* ldoc = nullptr;
  float* val = nullptr;
  double* val64 = nullptr;  // float64 values of the same postings (bm25.BM25's path; optional)
  // Tile bounds (dense segment table, non-negative index): each (term,
  // tile)'s largest score as f16 bits rounded DOWN, [V][bmax_stride] — a lower
  // bound of that score (threshold keys) and, one f16 step up, an upper bound
  // (the REST pass's tile skip)
  uint16_t* bmax = nullptr;
  // The same bounds pooled over groups of kPool consecutive tiles (the max of
  // each group's entries, [V][pstride], pstride = bmax_stride(ceil(ntiles /
  // kPool))): the threshold kernel's input where it holds enough groups — a
  // group's bound is still <= one of its documents' scores, and distinct
  // groups hold distinct documents, at a quarter of the bytes
  uint16_t* bpool = nullptr;
  int64_t pstride = 0;
  // The tile-bound threshold is off for this handle's next searches: the
  // last ones that used it overflowed their candidate lists (weak bounds —
  // an index whose terms weigh alike); set by the host per search
  // (bm25mi_capi.cpp: bound_ok), read by search_geom
  bool bound_weak = false;
  // World tile bounds of a doc-sharded collection (bm25_index_set_world_
  // bounds): every shard's bmax rows, [wW][V][wstride] (a caller-owned device
  // buffer, zero past each shard's tiles), so a shard's search
  // (bm25_search_shard_device) takes the whole collection's tile-bound
  // threshold by itself — no key exchange; wtiles = the collection's tiles
  const uint16_t* wbmax = nullptr;
  int32_t wW = 0;
  int64_t wstride = 0;
  int64_t wtiles = 0;
  // ... and pooled as bpool (handle-owned, built by bm25_index_set_world_bounds):
  // [wW][V][wpstride], wpstride = bmax_stride(wstride / kPool); wgroups = the
  // collection's groups (each shard's ceil(tiles / kPool), summed)
  uint16_t* wbpool = nullptr;
  int64_t wpstride = 0;
  int64_t wgroups = 0;
  SearchOpts opt;
  mutable Dispatch disp;  // written by the launchers (callers hold the handle's mutex)
};

constexpr int kCounters = 8;  // Workspace::counters

// A handle's reusable scratch for the large-k paths (bm25mi_large.hip): one
// device allocation, bump-allocated by each search (nested uses stack), sized
// by the host before a search to what the last searches asked for — so a
// search makes no allocation of its own once the handle has seen its shape.
struct LargeArena {
  char* base = nullptr;
  size_t bytes = 0;
  size_t used = 0;     // bump offset of the live scratch users
  size_t need = 0;     // the most the last searches asked for
  int64_t budget = 0;  // bytes one search may take (large_budget(), fixed at first use)
};

struct Workspace {
  int64_t cap_q = 0, cap_k = 0;
  LargeArena* arena = nullptr;   // the handle's large-k scratch (null: per-search allocations)
  uint64_t* cand = nullptr;      // [Q][ntiles][kTileM] exact top-kTileM keys of sample (or all) tiles
  uint64_t* theta = nullptr;     // [Q] k-th best sample key
  uint64_t* list = nullptr;      // [Q][list_cap] keys above theta of the other tiles
  int32_t* list_cnt = nullptr;   // [Q] keys appended (> list_cap: overflow)
  int32_t list_cap = 0;
  int32_t* fb = nullptr;         // [Q] queries whose list overflowed (fallback stage)
  uint64_t* cand2 = nullptr;     // [Q][maxflag][k] exact top-k of re-scored tiles
  int32_t* flag_tiles = nullptr; // [Q][maxflag]
  int32_t* nflag = nullptr;      // [Q]
  int32_t* queue = nullptr;      // [Q*maxflag] items = qi*maxflag + i
  int32_t* counters = nullptr;   // [kCounters]: [0]/[1] rescore queue length / pop cursor,
                                 // [2] fallback queries, [3] tiles re-scored this search,
                                 // [4] queries left to the block merge (slow),
                                 // [5] (query, tile) pairs REST skipped by their tile bound,
                                 // [6..7] (a u64) the postings of those pairs
  int32_t* slow = nullptr;       // [Q] those queries
  // the large-k list path's REST (bm25mi_large.hip sets them on its copy):
  // per-(query, tile) slots of slot_cap keys and their counts; null otherwise
  uint64_t* slots = nullptr;
  int32_t* slot_cnt = nullptr;
  int32_t slot_cap = 0;
  int32_t* wctr = nullptr;       // [kWctrRegions][kWctrInts] item-claim counters: zeroed once
                                 // at allocation; the last wave of each counter's sharers
                                 // re-zeroes it (and its finished count) at the end of every
                                 // flat launch, so each launch finds its region zeroed
  int32_t* report = nullptr;     // host-mapped [2]: merge_tail_kernel writes the search's
                                 // fallback query count, then `seq` (null: no report)
  int32_t seq = 0;               // the search's sequence number on its handle
  // split REST items (bound_keys_kernel builds the table per search): per
  // query its weight, then the band's item table (<= 8 per query), the items
  // per band, and the finished-block count of the build (self-resetting)
  uint32_t* qw = nullptr;
  uint32_t* sub = nullptr;
  int32_t* sub_ipb = nullptr;
  int32_t* sub_done = nullptr;
  uint64_t* seg = nullptr;       // sparse index: [Q][tiles/8][TT][8] segment of each (query,
                                 // term position, tile) (start | len << 32), built per search
  int64_t cap_seg = 0;           // u64 entries of seg
};

// Flag slots per query: a flagged tile holds kTileM keys of the top-(k-1), so
// at most (k-1)/kTileM tiles (and never more than the candidate tiles).
inline int64_t maxflag_for(int k, int64_t ntiles) {
  const int64_t m = (k + kTileM - 1) / kTileM;
  return m < ntiles ? m : (ntiles > 0 ? ntiles : 1);
}

// Threshold geometry of a search over W doc shards of ntiles tiles each:
// stride P (1 = no sampling), m keys per sample tile, S keys per query per
// shard, sample tiles in groups of G consecutive tiles (one group per G*P).
// P = 0: no SAMPLE pass — each shard's S best tile-bound keys
// (bound_keys_kernel).
struct SampleGeom {
  int P, m;
  int64_t S;
  int G;  // sample tiles come in groups of G consecutive tiles (bm25mi_kernels.hip)
};
SampleGeom sample_geom(int64_t ntiles, int k, int W, int pmax);
// The geometry a search of T-term queries takes: tile-bound keys when the
// handle has tile bounds (and the theta_bound option) and the queries are
// short, else sample_geom; the key width S is sample_geom's either way.
// ntiles: the widest shard's tiles (every shard of a search must take the
// same geometry).
SampleGeom search_geom(const DevIndex& ix, int64_t ntiles, int k, int W, int64_t T);
// Most tiles a shard may have for tile-bound keys (one wave's LDS per query).
constexpr int64_t kBoundMaxTiles = 30720;
// ... and at least this many tiles per wanted key over the whole collection.
constexpr int64_t kBoundTilesPerK = 16;
// Pooled bounds: tiles per group, and the groups per wanted key the pooled
// threshold needs (else the per-tile bounds: top-k tiles sharing a group
// lower the threshold by about k^2 (kPool - 1) / (2 ntiles) ranks).
constexpr int64_t kPool = 4;
constexpr int64_t kPoolGroupsPerK = 8;
// ... and queries of at most this many terms (search_geom; the bound kernel's
// per-tile loads in flight).
#ifndef BM25_BOUND_TERMS
#define BM25_BOUND_TERMS 16
#endif
constexpr int64_t kBoundMaxTerms = BM25_BOUND_TERMS;

// Kernel launchers (bm25mi_kernels.hip).  All enqueue on `stream`.
hipError_t launch_build_tables(const DevIndex& ix, const int32_t* d_indices,
                               int32_t* d_err, hipStream_t stream);
// Tile bounds ix.bmax from the dense segment table and the scores.
hipError_t launch_build_bmax(const DevIndex& ix, hipStream_t stream);
// out[r][g] = the max of in[r][kPool g .. kPool g + kPool - 1] (u16 f16 bits,
// all >= 0) for rows r < rows, g < out_stride (zero past in_stride).
hipError_t launch_pool_bounds(const uint16_t* in, int64_t rows, int64_t in_stride, uint16_t* out,
                              int64_t out_stride, hipStream_t stream);
// Sparse segment table: non-empty tiles per term -> d_cnt[V] (also writes
// ldoc and validates, as launch_build_tables), then (after the caller's scan
// into ix.tl_ptr) the tile lists.
hipError_t launch_count_tiles(const DevIndex& ix, const int32_t* d_indices, int64_t* d_cnt,
                              int32_t* d_err, hipStream_t stream);
hipError_t launch_fill_tiles(const DevIndex& ix, const int32_t* d_indices, hipStream_t stream);
// u64 entries of Workspace::seg a search of Q queries of T terms needs (0:
// dense index, or a search the flat kernel does not serve).
int64_t seg_entries(const DevIndex& ix, int64_t Q, int64_t T);
// Score pass of a single-index search: SAMPLE + theta + REST (or the exact
// pass when the index is too small to sample).
// The threshold geometry of a search; world (a shard with world bounds): the
// collection's tile-bound threshold when it serves (P = 0), else the shard's own.
SampleGeom shard_geom_world(const DevIndex& ix, int k, int64_t T, bool world);
// world: the threshold from the world tile bounds (ix.wbmax; a shard's
// search for the W-way merge), else from this index's own.
hipError_t launch_score(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                        int k, const Workspace& ws, hipStream_t stream, bool world = false);
// The same in two halves for W doc shards searched together: each shard's
// sample keys [Q][g.S] -> (all-gather across shards) -> theta over [W][Q][g.S]
// + REST.
hipError_t launch_sample(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                         const SampleGeom& g, uint64_t* keys, const Workspace& ws,
                         hipStream_t stream);
// rest_stream (when not null and not `stream`): the REST pass runs there,
// after theta (join: recorded on `stream`, waited on rest_stream); rest_timing
// (optional) is recorded on rest_stream just before the REST pass.
hipError_t launch_finish(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                         int k, const SampleGeom& g, int W, const uint64_t* all_keys,
                         const Workspace& ws, hipStream_t stream,
                         hipStream_t rest_stream = nullptr, hipEvent_t join = nullptr,
                         hipEvent_t rest_timing = nullptr);
// Merge (+ rescore + final merge), then the exact fallback stage; P = the
// search's sampling stride.  unsorted: a doc shard's list for the W-way merge
// (the keys >= its k-th key in no order, padding last: merge_fast skips the
// sort; the fallback stages still write sorted lists).
hipError_t launch_select(const DevIndex& ix, const int32_t* d_queries,
                         int64_t Q, int64_t T, int k, int P, const Workspace& ws,
                         int32_t* d_docs, float* d_scores, hipStream_t stream, bool unsorted = false);
hipError_t launch_scores_dense(const DevIndex& ix, const int32_t* d_query,
                               int64_t T, float* d_out, hipStream_t stream);
// W lists [Q, k] at element w * rank_stride (docs and scores alike) -> [Q, k];
// sorted: every list is already best-first (W-way merge instead of a sort).
hipError_t launch_merge_lists(const int32_t* d_docs, const float* d_scores,
                              int64_t W, int64_t Q, int k, int64_t rank_stride, bool sorted,
                              int32_t* d_out_docs, float* d_out_scores, hipStream_t stream);

// Dense scores of G queries (rows of T terms) into d_out[g * stride + doc];
// stride >= ntiles << tile_shift (whole tiles are stored; docs past n_docs
// hold 0).  G <= 65535.
hipError_t launch_scores_batch(const DevIndex& ix, const int32_t* d_queries, int64_t G, int64_t T,
                               int64_t stride, float* d_out, hipStream_t stream);

// Exact top-k for any k (the path of k > kMaxK, bm25mi_large.hip): per chunk
// of queries the dense scores, a radix selection of the k-th key, the keys
// >= it compacted and sorted.  k > n_docs (a doc shard smaller than k) pads
// each row with doc -1 / score bits 0xFFFFFFFF.  Scratch comes from the
// handle's arena; what does not fit is taken stream-ordered (hipMallocAsync)
// and released at the end of the launch sequence.  budget: the bytes this
// call may take (<= 0: the arena's budget; a nested call passes what its
// caller leaves).
hipError_t launch_search_large(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                               int k, int32_t* d_docs, float* d_scores, hipStream_t stream,
                               LargeArena* arena = nullptr, int64_t budget = 0);
// The large-k list path's passes (bm25mi_kernels.hip; used by
// bm25mi_large.hip): SAMPLE with kLargeM keys per sample tile into keys[Q][g.S]
// (g.m == kLargeM), and REST into the workspace's theta / list / list_cnt /
// list_cap (the caller's buffers).  large_list_supported: the flat kernel
// serves the batch and the index is non-negative.
hipError_t launch_sample_large(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                               const SampleGeom& g, uint64_t* keys, const Workspace& ws,
                               hipStream_t stream);
hipError_t launch_rest_lists(const DevIndex& ix, const int32_t* d_queries, int64_t Q, int64_t T,
                             const SampleGeom& g, const Workspace& ws, hipStream_t stream);
bool large_list_supported(const DevIndex& ix, int64_t T, int64_t Q);

// The large-k list path (bm25mi_large.hip) for kMaxK < k <= kLargeListMaxK:
// large_geom's SAMPLE (P = 0: not applicable), theta, REST into lists, the
// k-th key of each list, compaction and a row sort; queries the lists cannot
// serve go through launch_search_large on their own (*n_fallback of them;
// the path synchronises the stream once to count them).  ws: the handle's
// workspace (claim counters, counters, segment table).
constexpr int64_t kLargeListMaxK = 131072;
SampleGeom large_geom(const DevIndex& ix, int64_t k);
hipError_t launch_search_large_lists(const DevIndex& ix, const int32_t* d_queries, int64_t Q,
                                     int64_t T, int k, const Workspace& ws, int32_t* d_docs,
                                     float* d_scores, int64_t* n_fallback, hipStream_t stream);

// W lists [Q, k] (docs and scores at element w * rank_stride) -> the best k
// of each query by (score desc, doc asc), for any k (a segmented sort of the
// W k keys of each query).  Padding (doc -1, score bits ~0) sorts last.
hipError_t launch_merge_large(const int32_t* d_docs, const float* d_scores, int64_t W, int64_t Q,
                              int k, int64_t rank_stride, int32_t* d_out_docs,
                              float* d_out_scores, hipStream_t stream);

// Largest token id of [n] device ids (0 if none is positive) into *d_out.
hipError_t launch_max_token(const int32_t* d_queries, int64_t n, int32_t* d_out,
                            hipStream_t stream);

// Tile shifts with compiled kernels, and the one a new index takes.
bool tile_shift_supported(int s);
int build_tile_shift();

// Device sort and scan (bm25mi_sort.hip; hand-written, no hipCUB).
// Stable LSD radix sort of n (u64 key, u32 value) pairs: by the key bits
// [key_bits_lo, key_bits_hi) (descending: of ~key), then by the value bits
// [0, val_bits_hi) (vals may be null when val_bits_hi == 0).  keys_alt /
// vals_alt are same-sized buffers; *result_in_alt tells which pair of buffers
// holds the result.  scratch: radix_sort_scratch_bytes(n) bytes.
size_t radix_sort_scratch_bytes(int64_t n);
hipError_t radix_sort_pairs(uint64_t* keys, uint32_t* vals, uint64_t* keys_alt, uint32_t* vals_alt,
                            int64_t n, int key_bits_lo, int key_bits_hi, bool descending,
                            int val_bits_hi, void* scratch, bool* result_in_alt, hipStream_t st);
// G rows of n keys each ([G][n]), every row sorted descending in place of
// the segmented sort (rows / rows_alt: G * n u32 of scratch values).
hipError_t radix_sort_rows_desc(uint64_t* keys, uint64_t* keys_alt, uint32_t* rows,
                                uint32_t* rows_alt, int64_t G, int64_t n, void* scratch,
                                bool* result_in_alt, hipStream_t st);
// out[i] = in[0] + ... + in[i - 1] (out[0] = 0) for n u64 counts.
size_t exclusive_scan_scratch_bytes(int64_t n);
hipError_t exclusive_scan_u64(const unsigned long long* in, int64_t* out, int64_t n, void* scratch,
                              hipStream_t st);

// bm25.BM25's float64 path (bm25mi_dense.hip): dense sums of one query from
// the index's float64 values (numpy's order), and the n best of a dense
// float64 vector by (score desc, doc asc).
hipError_t launch_dense_f64(const DevIndex& ix, const double* val64, const int32_t* d_query,
                            int64_t T, double* d_out, hipStream_t st);
size_t topn_f64_scratch_bytes(int64_t n_docs);
hipError_t launch_topn_f64(const double* d_scores, int64_t n_docs, int64_t n, void* scratch,
                           int32_t* d_docs, double* d_out_scores, hipStream_t st);

// GPU index build (bm25mi_build.hip): scoring rules of bm25_build_scores.
enum { kLucene = 0, kBm25Py = 1 };
// (doc, term, tf) triples + document lengths -> CSC indptr [n_terms+1] (i64),
// indices/data [n] (+ f64 data when d_data64 != null), all on the device;
// d_err |= 1 (id out of range), 2 (tf not positive finite), 4 (duplicate
// (doc, term)).  Synchronises `stream` before returning.
hipError_t build_scores(int64_t n_docs, int64_t n_terms, int64_t n, const int32_t* d_docs,
                        const int32_t* d_terms, const float* d_tfs, const int32_t* d_doc_len,
                        double avgdl, double k1, double b, int method, const float* d_idf,
                        int64_t* d_indptr, int32_t* d_indices, float* d_data, double* d_data64,
                        int32_t* d_err, hipStream_t stream);

}  // namespace bm25mi
