/*
 * bm25mi.h — C-ABI of libbm25mi.so, the MI355X-native BM25 CSC query engine.
 *
 * This is the drop-in boundary for the reference's batched BM25 scoring path
 * (SURVEY.md §8(b)).  Every entry point is plain C: pointers, sizes and error
 * codes, no torch / HIP types in the signatures.  Each function cites the
 * reference interface it replaces (paths relative to the reference checkout
 * yuhuishi-convect/mojo-bm25 @ 2025-06-20).
 *
 * Conventions
 *   - Return 0 on success, a BM25_E* code otherwise; the message of the last
 *     failure on the calling thread is bm25_last_error().
 *   - Host buffers are C-order numpy-compatible arrays owned by the caller.
 *   - Device buffers (the *_device entry points) are caller-owned HIP device
 *     allocations on the index's device; `stream` is a hipStream_t passed as
 *     void* (NULL = the legacy default stream).  *_device calls are
 *     asynchronous with respect to the host.
 *   - One index handle is not re-entrant: calls on the same handle are
 *     serialised by an internal mutex.
 *   - Doc ids are int32, scores float32, token ids int32; negative token ids
 *     are padding and are skipped (bm25_native.py:151).
 *   - Results are sorted by score descending; equal scores are ordered by doc
 *     id ascending (the deterministic rule of the MAX CPU top-k,
 *     operations/topk.mojo:234-258 / test_topk.mojo:222-238; bm25_native's
 *     own tie order is numpy-implementation-defined).
 */
#ifndef BM25MI_H
#define BM25MI_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BM25MI_ABI_VERSION 1

enum {
  BM25_OK = 0,
  BM25_EINVAL = 1, /* bad argument (bad shape, token id >= n_terms, k > n_docs ...) */
  BM25_EHIP = 2,   /* HIP runtime failure, or no usable GPU */
  /* 3 is unused: the one-process sharded handle moves its keys and lists with
   * peer copies, and the multi-process path's collectives run in the caller
   * (torch.distributed over RCCL, bm25mi.dist), not in this library */
  BM25_ENOMEM = 4  /* device or host allocation failed */
};

typedef struct bm25_index bm25_index;

/* ABI version of the loaded library (== BM25MI_ABI_VERSION it was built with). */
int bm25_abi_version(void);

/* Message of the last failing call on this thread ("" if none).  The pointer
 * stays valid until the next failing call on the same thread. */
const char* bm25_last_error(void);

/* Number of HIP devices visible to the process (0 on a host without a GPU;
 * never fails). */
int bm25_device_count(void);

/*
 * Build a device-resident index from a CSC doc x term score matrix.
 * Replaces: BM25v.index(doc_toks: scipy csc_matrix, doc_lengths)
 *           (bm25_native.py:59-74) and the host->device copy of the MAX path
 *           (gpu_bm25/common.py:38).
 *   indptr  [n_terms+1]  int32 (indptr_is_i64 = 0) or int64 (= 1), indptr[0]=0,
 *                        indptr[n_terms] = nnz, non-decreasing
 *   indices [nnz] int32  doc ids of each column, sorted ascending and unique
 *                        within a column (canonical CSC, as bm25s writes it)
 *   data    [nnz] f32    precomputed per-(doc, term) BM25 scores
 * The arrays are copied; the caller may free them when this returns.
 * doc_offset is added to every doc id the index returns (shards of a larger
 * collection pass the global id of their first document; 0 otherwise).
 */
int bm25_index_create(int device, int64_t n_docs, int64_t n_terms, int64_t nnz,
                      const void* indptr, int indptr_is_i64,
                      const int32_t* indices, const float* data,
                      int64_t doc_offset, bm25_index** out);

/* Release every device allocation and stream of the handle (the index
 * arrays once no fork of the handle is left). */
int bm25_index_destroy(bm25_index* idx);

/*
 * A second search context on the same device-resident index: it shares the
 * CSC arrays, segment table and tile bounds of `base` (no copy) and has its
 * own workspace, staging buffers, options (copied from base) and internal
 * stream, so searches on base and on its forks may run concurrently on
 * different streams (the doc-sharded search pipelines the parts of a batch
 * this way: bm25mi.dist.sharded_search(parts=2)).  Each handle is destroyed
 * on its own; the index arrays are released with the last one.
 * Replaces no reference call: BM25v.search is stateless per call
 * (bm25_native.py:76-158), which a fork per concurrent caller restores.
 */
int bm25_index_fork(bm25_index* base, bm25_index** out);

/* Geometry of a built index (any pointer may be NULL). */
int bm25_index_info(const bm25_index* idx, int64_t* n_docs, int64_t* n_terms,
                    int64_t* nnz, int32_t* tile_docs, int64_t* n_tiles,
                    int64_t* device_bytes);

/*
 * Segment table of a built index: *sparse = 0 for the dense
 * V x (n_tiles+1) table, 1 for per-term tile lists (chosen at create time:
 * env BM25_SEGMENTS=dense|sparse, else dense unless it would exceed twice the
 * posting arrays); *n_pairs = non-empty (term, tile) pairs held (sparse).
 */
int bm25_index_segments(const bm25_index* idx, int32_t* sparse, int64_t* n_pairs);

/*
 * Tile bounds of a built index: *has_bounds = 1 when it keeps
 * each (term, tile)'s largest score (a dense, non-negative index whose table
 * fit in device memory) — the tile-bound threshold and the REST tile skip
 * need it; *bytes = the table's device bytes.  Any pointer may be NULL.
 */
int bm25_index_bounds(const bm25_index* idx, int32_t* has_bounds, int64_t* bytes);

/*
 * Batched top-k search, host buffers, synchronous.
 * Replaces: BM25v.search / get_scores / _compute_relevance_from_scores / _topk
 *           (bm25_native.py:76-158, 204-214).
 *   queries    [Q, T] int32, negative = padding, every id < n_terms
 *   out_docs   [Q, k] int32
 *   out_scores [Q, k] f32
 * Every 0 <= k <= n_docs is served (k > 4096 by the exact large-k path: a
 * sampled threshold, the keys above it listed, selected and sorted — or
 * dense score rows with a radix selection where lists cannot serve).  That
 * path's scratch (up to a quarter of the free device memory, at most 4 GiB)
 * stays with the handle after its first such search, for the next ones,
 * until bm25_index_destroy.
 * Errors: EINVAL when a token id >= n_terms (message matches
 * bm25_native.py:118-121), when k < 0 or k > n_docs.
 */
int bm25_search(bm25_index* idx, const int32_t* queries, int64_t Q, int64_t T,
                int32_t k, int32_t* out_docs, float* out_scores);

/*
 * Same as bm25_search with device-resident queries and results, enqueued on
 * `stream` without host synchronisation (the bench's timed step: inputs
 * already resident in HBM).  Token ids are NOT validated here: ids >=
 * n_terms are treated as padding by the kernels (bm25_max_token_device is
 * the opt-in check).
 */
int bm25_search_device(bm25_index* idx, const int32_t* d_queries, int64_t Q,
                       int64_t T, int32_t k, int32_t* d_docs, float* d_scores,
                       void* stream);

/*
 * Opt-in validation of a device-resident batch: *max_token = the largest
 * token id of d_queries[Q, T] (0 when none is positive), computed on the
 * device on `stream`, which is synchronised.  A caller of bm25_search_device
 * that wants the reference's check raises when *max_token >= n_terms.
 * Replaces: bm25_native.py:91-96 (queries.max(initial=0) >= n_terms ->
 *           ValueError).
 */
int bm25_max_token_device(bm25_index* idx, const int32_t* d_queries, int64_t Q,
                          int64_t T, int32_t* max_token, void* stream);

/*
 * GPU index build: (doc, term, tf) triples + document lengths -> the CSC
 * score matrix (term-major, doc ids ascending per term = what
 * bm25_index_create and the bm25s on-disk format hold).
 * Replaces: the scoring half of the bm25s writer that produced the
 *           reference's index (animal_index_bm25/, params.index.json:1-11,
 *           bm25_test.py:19-38; method 0) and BM25.fit's matrix
 *           (bm25.py:30-121; method 1).
 *   docs/terms [n] int32, tfs [n] f32 (> 0), any order, one triple per
 *   (doc, term); doc_len [n_docs] int32; avgdl = the mean document length
 *   (bm25.py:62 / bm25s); idf [n_terms] f32 or NULL (computed on the device:
 *   ln(1 + (N - df + 0.5) / (df + 0.5)), df = triples per term);
 *   method 0 = lucene: idf * tf / (tf + k1 * (1 - b + b * dl / avgdl)),
 *   method 1 = bm25.py: idf * tf * (k1 + 1) / (tf + k1 * (1 - b + b * dl / avgdl)).
 *   Outputs (host): out_indptr [n_terms+1] int64, out_indices [n] int32,
 *   out_data [n] f32, out_data64 [n] f64 or NULL (method 1: the float64
 *   bm25_matrix entries).  Operation order and precision follow the code each
 *   method stands in for (bm25mi_build.hip), so the values are bit-identical.
 * Errors: EINVAL for ids out of range, tf <= 0, duplicate (doc, term).
 */
int bm25_build_scores(int device, int64_t n_docs, int64_t n_terms, int64_t n_triples,
                      const int32_t* docs, const int32_t* terms, const float* tfs,
                      const int32_t* doc_len, double avgdl, double k1, double b, int method,
                      const float* idf, int64_t* out_indptr, int32_t* out_indices,
                      float* out_data, double* out_data64);

/*
 * Dense per-document scores of one query (all n_docs fp32 sums, query-term
 * order, zero for untouched documents), host buffers.
 * Replaces: the dense gather+sum of the MAX graph (gpu_bm25/common.py:64-74)
 *           and BM25.get_scores (bm25.py:124-145) over a CSC index.
 */
int bm25_scores_dense(bm25_index* idx, const int32_t* query, int64_t T,
                      float* out_scores);

/*
 * bm25.BM25's float64 path (the dense model's API keeps the reference's
 * precision).  bm25_index_set_values_f64 keeps a float64 copy of the index's
 * values beside it (the same CSC order; bm25_build_scores method 1 returns
 * them as out_data64 — the reference's bm25_matrix entries).
 *   bm25_scores_dense_f64: every document's float64 sum over the query's
 *     valid ids in query order from 0 — numpy's np.sum(bm25_matrix[:, ids],
 *     axis=1) bit for bit (column by column; a one-document corpus: numpy's
 *     pairwise order).  Replaces BM25.get_scores (bm25.py:124-145).
 *   bm25_topn_f64: the n best documents of those sums by (score desc, doc
 *     asc), 0 <= n <= n_docs.  Replaces the ranking of BM25.get_top_n
 *     (bm25.py:147-178: argsort(scores)[::-1][:n]; its order among equal
 *     scores is numpy-implementation-defined).
 * Errors: EINVAL when no float64 values were set, a token id >= n_terms
 * (bm25_native's message), n out of range.
 */
int bm25_index_set_values_f64(bm25_index* idx, const double* data64);
int bm25_scores_dense_f64(bm25_index* idx, const int32_t* query, int64_t T, double* out_scores);
int bm25_topn_f64(bm25_index* idx, const int32_t* query, int64_t T, int64_t n, int32_t* out_docs,
                  double* out_scores);

/*
 * Merge W per-shard top-k lists (global doc ids) into one top-k, device
 * buffers: d_docs/d_scores are [W, Q, k], outputs [Q, k].  Used after the
 * RCCL all-gather of the doc-sharded search; the order rule
 * is the same (score desc, doc asc), so the result equals a single-index
 * search over the whole collection.
 */
int bm25_merge_topk_device(int device, const int32_t* d_docs,
                           const float* d_scores, int64_t W, int64_t Q,
                           int32_t k, int32_t* d_out_docs, float* d_out_scores,
                           void* stream);

/*
 * The same merge for the lists bm25_search_finish_device (world > 1) and
 * bm25_search_shard_device write — a shard's keys in any order, padding
 * (doc -1) anywhere — in one buffer per rank: rank w's [Q, k] docs and scores start at element
 * w * rank_stride of d_docs / d_scores (rank_stride = Q * k for plain
 * [W, Q, k] arrays, 2 * Q * k for the packed [W][docs|scores][Q][k] buffer
 * one all-gather moves).  A W-way merge, one wavefront per query.
 * Replaces: the reference is single-device (main.py:205); SURVEY.md §8(e).
 */
int bm25_merge_sorted_device(int device, const int32_t* d_docs,
                             const float* d_scores, int64_t W, int64_t Q,
                             int32_t k, int64_t rank_stride, int32_t* d_out_docs,
                             float* d_out_scores, void* stream);

/*
 * Doc-sharded search with a GLOBAL threshold, one rank per GPU (the
 * multi-process form of bm25_search_device).  Every rank
 * holds one doc shard (bm25_index_create with its doc_offset) and searches
 * the same query batch in two halves around one all-gather:
 *   bm25_sample_width(idx, shard_docs_max, world, k, &S): keys per query each
 *     rank samples (the same on every rank: shard_docs_max = the largest
 *     shard's document count; S = 0: shards too small to sample, or
 *     k > 4096 — then the finish half lists the shard's exact top-k; the
 *     same S serves the tile-bound threshold, whose keys need no sampling);
 *   bm25_search_sample_device(...): this shard's sample keys -> d_keys
 *     (u64 [Q][S], zero-padded: a SAMPLE pass, or — theta_bound — the best S
 *     tile-bound keys, read from the tile bounds without scoring);
 *   (caller) all-gather d_keys of every rank -> d_all_keys [world][Q][S];
 *   bm25_search_finish_device(...): theta = the k-th best key of the world's
 *     sample (k real documents score at least this), then every key >= theta
 *     of this shard -> [Q, k] (global doc ids; padded with doc -1 / score bits
 *     0xFFFFFFFF where the shard holds fewer), or the shard's exact top-k for
 *     queries the threshold cannot serve.
 * Merging the world's [Q, k] lists with bm25_merge_topk_device (padding
 * sorts last) gives exactly the single-index top-k.  world = 1 is a plain
 * search.  Replaces no reference call: the reference is single-device.
 */
int bm25_sample_width(const bm25_index* idx, int64_t shard_docs_max, int32_t world, int32_t k,
                      int64_t* width);
int bm25_search_sample_device(bm25_index* idx, const int32_t* d_queries, int64_t Q, int64_t T,
                              int32_t k, int32_t world, int64_t shard_docs_max,
                              uint64_t* d_keys, void* stream);
int bm25_search_finish_device(bm25_index* idx, const int32_t* d_queries, int64_t Q, int64_t T,
                              int32_t k, int32_t world, int64_t shard_docs_max,
                              const uint64_t* d_all_keys, int32_t* d_docs, float* d_scores,
                              void* stream);
/*
 * The finish half on three streams, for a caller that pipelines batches
 * (bm25mi.dist.ShardPipeline): theta on stream_theta, the REST pass on
 * stream_rest (after theta), the merges into d_docs / d_scores on
 * stream_select (after REST); the library orders the three with events.
 * The workspace is released on stream_select: the handle's next search on
 * another stream waits for it.  Same results as bm25_search_finish_device
 * (which is this with one stream).  The score pass of a profiled handle is
 * timed on stream_rest from the REST pass's start.
 */
int bm25_search_finish_streams_device(bm25_index* idx, const int32_t* d_queries, int64_t Q,
                                      int64_t T, int32_t k, int32_t world,
                                      int64_t shard_docs_max, const uint64_t* d_all_keys,
                                      int32_t* d_docs, float* d_scores, void* stream_theta,
                                      void* stream_rest, void* stream_select);

/*
 * Doc-sharded search with ONE collective (the multi-process form used by
 * bm25mi.dist when the collection's tile bounds fit one selection block:
 * <= 30720 tiles).  Every rank exports its tile bounds, the ranks all-gather
 * them once (at index build), and each rank's search takes the whole
 * collection's tile-bound threshold by itself:
 *   bm25_index_bounds_export(idx, d_out, stride, stream): this index's tile
 *     bounds [n_terms][stride] u16 (stride: a multiple of 4 >= its tiles,
 *     rounded up to 4; the same on every rank; zero past its tiles);
 *   (caller) all-gather -> d_world [world][n_terms][stride], kept alive;
 *   bm25_index_set_world_bounds(idx, d_world, world, stride, world_tiles):
 *     world_tiles = the collection's tiles (NULL d_world clears); the call
 *     waits for the device (d_world written on any stream before it is
 *     complete) and reads the table once into a pooled copy the handle owns (the max of every 4 tiles, a quarter
 *     of the size: the threshold's input where the collection has >= 8k such
 *     groups — option bound_pool) and keeps the pointer for the rest;
 *   bm25_search_shard_device(...): this shard's keys >= the collection's
 *     threshold (k real documents score at least it) as a [Q, k] list in no
 *     particular order (global doc ids, padding doc -1 / score bits
 *     0xFFFFFFFF last), or its exact top-k for k > 4096 / queries the
 *     threshold cannot serve;
 *   (caller) all-gather the lists, bm25_merge_sorted_device (any order in).
 * The result is exactly the single-index top-k.  Replaces no reference call:
 * the reference is single-device (main.py:205).
 */
int bm25_index_bounds_export(bm25_index* idx, uint16_t* d_out, int64_t stride, void* stream);
int bm25_index_set_world_bounds(bm25_index* idx, const uint16_t* d_world, int32_t world,
                                int64_t stride, int64_t world_tiles);
int bm25_search_shard_device(bm25_index* idx, const int32_t* d_queries, int64_t Q, int64_t T,
                             int32_t k, int32_t* d_docs, float* d_scores, void* stream);

/*
 * Doc-sharded index over several devices of ONE process.
 * The reference is single-device (DEVICE_ID = 0, main.py:205, graph.py:95);
 * this is the build's multi-GPU form of BM25v.index / BM25v.search
 * (bm25_native.py:59-103) for callers that own all local GPUs.  The multi-
 * process form (one rank per GPU, RCCL all-gather) is bm25mi.dist + the
 * *_device calls above.
 *   bm25_sharded_create: same CSC arguments as bm25_index_create; documents
 *     are split into n_dev contiguous, 2048-doc-aligned ranges, shard s on
 *     devices[s] (a device may be listed more than once).
 *   bm25_sharded_search: same contract as bm25_search; the global-threshold
 *     protocol of the *_device calls above with peer copies (xGMI) in place of
 *     the all-gathers: every shard samples on its own stream, every shard's
 *     keys are copied to every device, every shard computes the world's theta
 *     and lists its keys >= theta, and the [Q, k] lists are copied to
 *     devices[0] and merged there; the result equals a single-index search.
 *     Errors as bm25_search (k may exceed a shard's documents: its list is
 *     padded).
 *   bm25_sharded_info: shard count and [lo, hi) doc ranges (arrays of n_dev).
 */
typedef struct bm25_sharded bm25_sharded;

int bm25_sharded_create(int n_dev, const int* devices, int64_t n_docs, int64_t n_terms,
                        int64_t nnz, const void* indptr, int indptr_is_i64,
                        const int32_t* indices, const float* data, bm25_sharded** out);
int bm25_sharded_search(bm25_sharded* s, const int32_t* queries, int64_t Q, int64_t T,
                        int32_t k, int32_t* out_docs, float* out_scores);
int bm25_sharded_info(const bm25_sharded* s, int64_t* n_shards, int64_t* shard_lo,
                      int64_t* shard_hi);
int bm25_sharded_destroy(bm25_sharded* s);

/*
 * Timing of the score pass (sample + theta + rest score kernels, the HBM
 * bound part of a search), measured with HIP events recorded on the search
 * stream around it in every search while enabled.
 * bm25_profile_enable(idx, on) resets the accumulators; on = 1: two events
 * per search (score pass start and end: total_ms reports the score pass);
 * on = 2: a third at the search's end (total_ms = the whole search).  Each
 * event record costs the device a marker packet (~4 us).
 */
int bm25_profile_enable(bm25_index* idx, int on);
int bm25_profile_read(bm25_index* idx, double* score_ms_total,
                      int64_t* score_launches, double* total_ms,
                      int64_t* searches, int64_t* rescored_tiles);

/*
 * Selection statistics of the last search on the handle (diagnostics; waits
 * for the device): tiles whose exact top-k had to be recomputed, and queries
 * that took the exact fallback stage (candidate list overflow).
 */
int bm25_search_stats(bm25_index* idx, int64_t* rescored_tiles,
                      int64_t* fallback_queries);
/* The same plus *bound_skipped: (query, tile) pairs the REST pass skipped
 * because the sum of the query terms' largest scores in the tile (the tile
 * bounds of a dense, non-negative index) is below the query's threshold —
 * counted only by a search with the count_skips option on, else -1.
 * Any pointer may be NULL. */
int bm25_search_stats_ex(bm25_index* idx, int64_t* rescored_tiles,
                         int64_t* fallback_queries, int64_t* bound_skipped);
/* Every selection counter of the last search, the first n of (in order):
 *   [0] tiles re-scored exactly, [1] queries sent to the exact fallback
 *   stage, [2] (query, tile) pairs the REST pass skipped by their tile
 *   bound, [3] the postings of those skipped (query, tile) segments (what
 *   the skip saved of the algorithmic bytes, 8 B each) — [2] and [3]
 *   counted only by a search with the count_skips option on, else -1 —
 *   [4] queries left to
 *   the block merge (lists longer than one wavefront's registers), [5] k >
 *   4096: queries the list path handed to dense score rows (-1: the dense
 *   path served the whole search; 0 after a search of k <= 4096).
 * n must be in 1..6. */
int bm25_search_counters(bm25_index* idx, int64_t* out, int32_t n);

/*
 * Search options of one handle.  A new handle takes them from the
 * environment (BM25_FLAT, BM25_FLAT_BW, BM25_ITEMS_PER_WAVE, BM25_SAMPLE_P,
 * BM25_LIST_CAP, BM25_CLAIM_CH, BM25_CLAIM_M, BM25_TILE_BOUND, BM25_THETA_BOUND,
 * BM25_GRID_PCT, BM25_LARGE_LISTS, BM25_COUNT_SKIPS, BM25_REST_SPLIT,
 * BM25_BOUND_POOL) at
 * bm25_index_create; these
 * calls change or read them afterwards, effective from the next search.
 * Results never depend on them (every setting is bit-exact); they choose
 * kernels and geometry:
 *   "flat"           1 (default): the flat score kernel for queries of 1..64
 *                    terms; 0: score_wave_kernel for every phase
 *   "flat_bw"        tiles per flat-kernel item: 0 = automatic, 1, 2, 4, 8
 *   "items_per_wave" automatic flat_bw: halved while a phase gives the
 *                    resident waves fewer items each (default 4; config 2:
 *                    4-tile items 0.089 ms per batch, 2-tile items at 8: 0.105)
 *   "sample_p"       largest sampling stride, a power of two (default 8;
 *                    1 = no threshold: the exact pass over every tile)
 *   "list_cap"       candidate-list capacity per query (0 = automatic; small
 *                    values force queries through the exact fallback stage)
 *   "claim_ch", "claim_m"  flat-kernel item claims: items per claim (1),
 *                    counters per XCD (4)
 *   "tile_bound"     1 (default): the REST pass skips tiles whose query-term
 *                    maxima (f16 bounds kept per (term, tile) by a dense,
 *                    non-negative index) sum below the threshold;
 *                    0: every tile is scored
 *   "theta_bound"    1 (default): the threshold comes from those tile bounds
 *                    (per tile, its largest query-term maximum is a real
 *                    document's score lower bound) with no SAMPLE pass;
 *                    0: the sampled threshold.  Every shard of a multi-rank
 *                    search needs the same setting (bm25_sample_width).  A
 *                    handle whose tile-bound searches overflowed switches
 *                    itself to the sampled threshold for a while, decided per
 *                    handle from a host-mapped report read without waiting —
 *                    so ranks may mix the two kinds of keys in one search:
 *                    that is exact (both are keys of real documents, the
 *                    width S is the same), only the work differs
 *   "large_lists"    1 (default): k > 4096 takes the list path where it
 *                    applies (a sampled threshold, keys above it listed by the
 *                    REST pass, selected and sorted — no dense score rows);
 *                    0: dense score rows for every query
 *   "count_skips"    1: the REST pass also counts the (query, tile) pairs its
 *                    tile bound skips and their postings (bm25_search_counters
 *                    [2], [3]) — a kernel build of its own: the two counts'
 *                    registers cost the pass 13 % on an 8-way doc shard;
 *                    0 (default): not counted
 *   "rest_split"     1: where the REST pass gives each resident wave few
 *                    items (< 48: a doc shard of a few-GPU collection), a
 *                    heavy query's 8-tile band is split into 2..8 items (a
 *                    per-search table built by the threshold kernel);
 *                    0 (default: measured no faster at W = 8)
 *   "bound_pool"     1 (default): the tile-bound threshold reads the bounds
 *                    pooled over groups of 4 tiles (a group's largest query-
 *                    term maximum is still a lower bound of one of its
 *                    documents' scores) where there are >= 8k groups — a
 *                    quarter of the threshold kernel's bytes; 0: the per-tile
 *                    bounds
 *   "grid_pct"       percent of the device's resident workgroup slots the
 *                    persistent score kernels launch (1..100, default 100):
 *                    below 100 leaves slots for kernels of another stream
 *                    (a concurrent search on a fork, the collectives)
 * Replaces no reference call (the reference has no tuning surface; its MAX
 * custom op takes compile-time parameters, graph.py:72).
 */
int bm25_index_set_option(bm25_index* idx, const char* name, int64_t value);
int bm25_index_get_option(const bm25_index* idx, const char* name, int64_t* value);

/*
 * What the last search on the handle launched (diagnostics, no device wait):
 *   *kernels     bit mask of score kernels: 1 flat SAMPLE, 2 flat REST,
 *                4 flat ALL (exact pass / fallback stage), 8 wave SAMPLE,
 *                16 wave REST, 32 wave ALL, 64 large-k path, 128 tile-bound
 *                threshold keys; 256 (a flag, not a kernel): the tile-bound
 *                threshold was off for this search because earlier searches
 *                on the handle that used it overflowed their candidate lists
 *                (more than 1/16 of their queries took the exact fallback) —
 *                it is retried after 64, 128, ... 4096 searches; 512 (a
 *                flag): REST counted its skipped postings (count_skips);
 *                1024 (a flag): REST ran over split items (rest_split);
 *                2048 (a flag): the threshold read the pooled bounds (bound_pool)
 *   *term_lanes  flat kernel: term lanes per tile (8, 16, 32 or 64)
 *   band_tiles   [3]: flat kernel tiles per item of ALL, SAMPLE, REST
 *   *sample_p    sampling stride of the search (1: exact pass, 0: tile-bound
 *                threshold keys, no SAMPLE pass)
 * Any pointer may be NULL.
 */
int bm25_search_dispatch(bm25_index* idx, uint32_t* kernels, int32_t* term_lanes,
                         int32_t* band_tiles, int32_t* sample_p);

#ifdef __cplusplus
}
#endif

#endif /* BM25MI_H */
