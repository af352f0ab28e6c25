/*
 * bm25_oracle.c — CPU restatement of the reference's BM25 CSC scoring path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker
 * (or the timed CPU baseline) — never as a product code path.
 *
 * It restates bm25_native.BM25v._compute_relevance_from_scores
 * (bm25_native.py:129-158) in its canonical form:
 *   - per query, a dense fp32 accumulator over all documents starting at 0
 *     (scipy csc_matvec's y = zeros, bm25_native.py:152);
 *   - query tokens visited in query order, negative ids skipped
 *     (bm25_native.py:150-151), duplicates visited twice;
 *   - for each column, y[indices[p]] += data[p] (fp32 add, data[p] * 1.0 is
 *     exact) — the same sequence of roundings as csc_matvec, so the dense
 *     scores are bit-identical to `doc_toks[:, query].sum(axis=1).A1`;
 *   - top-k by (score descending, doc id ascending).  bm25_native's _topk
 *     (bm25_native.py:204-214) uses numpy argpartition + argsort, whose order
 *     inside groups of equal scores is implementation-defined; the oracle uses
 *     the deterministic rule of the MAX CPU top-k (operations/topk.mojo:234-258,
 *     KATs test_topk.mojo:222-238).  Parity with bm25_native itself is pinned
 *     by tests/golden/ (tie-aware: ids exact where the score is untied).
 *
 * oracle_search_mt splits the query batch over POSIX threads (each with its
 * own accumulator); per query it is the same computation.
 *
 * Build: gcc -O2 -ffp-contract=off -fPIC -shared -pthread (oracle/Makefile); no
 * -ffast-math: the adds must stay IEEE fp32, unreordered.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

/* same key as the engine: larger = better (score desc, then doc asc) */
static uint64_t okey(float s, uint32_t doc) {
  uint32_t u;
  memcpy(&u, &s, 4);
  u = (u & 0x80000000u) ? ~u : (u | 0x80000000u);
  return ((uint64_t)u << 32) | (uint64_t)(0xFFFFFFFFu - doc);
}

static float okey_score(uint64_t k) {
  uint32_t v = (uint32_t)(k >> 32);
  uint32_t u = (v & 0x80000000u) ? (v & 0x7FFFFFFFu) : ~v;
  float s;
  memcpy(&s, &u, 4);
  return s;
}

/* min-heap of keys, size k */
static void sift_down(uint64_t* h, int64_t n, int64_t i) {
  for (;;) {
    int64_t l = 2 * i + 1, r = l + 1, m = i;
    if (l < n && h[l] < h[m]) m = l;
    if (r < n && h[r] < h[m]) m = r;
    if (m == i) return;
    uint64_t t = h[i]; h[i] = h[m]; h[m] = t;
    i = m;
  }
}

static int cmp_desc(const void* a, const void* b) {
  uint64_t x = *(const uint64_t*)a, y = *(const uint64_t*)b;
  return x < y ? 1 : (x > y ? -1 : 0);
}

/* dense fp32 scores of one query (bm25_native.py:151-152) */
int oracle_scores_dense(int64_t n_docs, int64_t n_terms, const int64_t* indptr,
                        const int32_t* indices, const float* data, const int32_t* query,
                        int64_t T, float* out) {
  for (int64_t d = 0; d < n_docs; ++d) out[d] = 0.0f;
  for (int64_t i = 0; i < T; ++i) {
    const int32_t t = query[i];
    if (t < 0) continue;
    if (t >= n_terms) return 1;
    for (int64_t p = indptr[t]; p < indptr[t + 1]; ++p) out[indices[p]] += data[p];
  }
  return 0;
}

/* top-k of a dense score vector by (score desc, doc asc) */
int oracle_topk(const float* scores, int64_t n, int32_t k, int32_t* out_docs,
                float* out_scores) {
  if (k < 0 || k > n) return 1;
  if (k == 0) return 0;
  uint64_t* h = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)k);
  if (!h) return 2;
  int64_t m = 0;
  for (int64_t d = 0; d < n; ++d) {
    const uint64_t key = okey(scores[d], (uint32_t)d);
    if (m < k) {
      h[m++] = key;
      if (m == k)
        for (int64_t i = k / 2 - 1; i >= 0; --i) sift_down(h, k, i);
    } else if (key > h[0]) {
      h[0] = key;
      sift_down(h, k, 0);
    }
  }
  qsort(h, (size_t)k, sizeof(uint64_t), cmp_desc);
  for (int32_t i = 0; i < k; ++i) {
    out_docs[i] = (int32_t)(0xFFFFFFFFu - (uint32_t)h[i]);
    out_scores[i] = okey_score(h[i]);
  }
  free(h);
  return 0;
}

/* batched search: queries[Q][T] -> out[Q][k] (bm25_native.py:129-158) */
int oracle_search(int64_t n_docs, int64_t n_terms, const int64_t* indptr, const int32_t* indices,
                  const float* data, const int32_t* queries, int64_t Q, int64_t T, int32_t k,
                  int32_t* out_docs, float* out_scores) {
  if (k < 0 || k > n_docs) return 1;
  float* acc = (float*)malloc(sizeof(float) * (size_t)(n_docs > 0 ? n_docs : 1));
  if (!acc) return 2;
  int rc = 0;
  for (int64_t q = 0; q < Q && rc == 0; ++q) {
    rc = oracle_scores_dense(n_docs, n_terms, indptr, indices, data, queries + q * T, T, acc);
    if (rc == 0) rc = oracle_topk(acc, n_docs, k, out_docs + q * k, out_scores + q * k);
  }
  free(acc);
  return rc;
}

/* the same batched search with the queries split over n_threads threads */
typedef struct {
  int64_t n_docs, n_terms;
  const int64_t* indptr;
  const int32_t* indices;
  const float* data;
  const int32_t* queries;
  int64_t q0, q1, T;
  int32_t k;
  int32_t* out_docs;
  float* out_scores;
  int rc;
} oracle_job;

static void* oracle_job_run(void* p) {
  oracle_job* j = (oracle_job*)p;
  j->rc = oracle_search(j->n_docs, j->n_terms, j->indptr, j->indices, j->data,
                        j->queries + j->q0 * j->T, j->q1 - j->q0, j->T, j->k,
                        j->out_docs + j->q0 * j->k, j->out_scores + j->q0 * j->k);
  return NULL;
}

int oracle_search_mt(int64_t n_docs, int64_t n_terms, const int64_t* indptr,
                     const int32_t* indices, const float* data, const int32_t* queries, int64_t Q,
                     int64_t T, int32_t k, int32_t* out_docs, float* out_scores, int n_threads) {
  if (k < 0 || k > n_docs) return 1;
  if (n_threads < 1) n_threads = 1;
  if (n_threads > Q) n_threads = Q > 0 ? (int)Q : 1;
  oracle_job* jobs = (oracle_job*)calloc((size_t)n_threads, sizeof(oracle_job));
  pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
  if (!jobs || !th) {
    free(jobs);
    free(th);
    return 2;
  }
  int rc = 0;
  for (int i = 0; i < n_threads; ++i) {
    oracle_job* j = &jobs[i];
    j->n_docs = n_docs; j->n_terms = n_terms; j->indptr = indptr; j->indices = indices;
    j->data = data; j->queries = queries; j->T = T; j->k = k;
    j->out_docs = out_docs; j->out_scores = out_scores;
    j->q0 = Q * i / n_threads;
    j->q1 = Q * (i + 1) / n_threads;
    if (pthread_create(&th[i], NULL, oracle_job_run, j) != 0) {
      j->rc = 2;
      th[i] = 0;
    }
  }
  for (int i = 0; i < n_threads; ++i) {
    if (th[i]) pthread_join(th[i], NULL);
    if (jobs[i].rc && !rc) rc = jobs[i].rc;
  }
  free(jobs);
  free(th);
  return rc;
}
