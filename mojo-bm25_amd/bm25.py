"""Drop-in replacement of the reference's ``bm25`` module (dense BM25 model).

Same class, constructor, attributes and methods as ``bm25.py:6-178`` of
yuhuishi-convect/mojo-bm25.  ``fit`` counts terms on the host (like the
tokenisation) and builds the BM25 matrix on the MI355X with
``bm25_build_scores`` (bm25.py:106-121: Robertson idf + 1, ``(k1 + 1)``
numerator, the reference's float64 arithmetic and operation order), which
returns the CSC index data and the float64 entries of the reference's dense
``bm25_matrix``; the float64 values stay on the device beside the index.

Numerics: the reference's own precision.  ``get_scores`` is the device's
float64 sum of the query's columns in query order (numpy's column-by-column
reduction of ``np.sum(bm25_matrix[:, ids], axis=1)``, bm25.py:143) — the same
bits; ``get_top_n`` ranks those float64 sums on the device (a stable radix
sort, bm25.py:172-176's ``argsort(...)[::-1]``) — documents with equal scores
by index ascending, where the reference's order among ties is
numpy-implementation-defined.  (bm25_native.BM25v's fp32 CSC scorer is the
engine's batched path; this model keeps float64 like the reference's.)
"""
from __future__ import annotations

import math
from collections import Counter

import numpy as np
import scipy.sparse as sp

from bm25mi.index import GpuIndex
from bm25mi.scoring import build_scores

class BM25:
    """BM25 with a precomputed dense score matrix, scored on the GPU."""

    def __init__(self, k1=1.5, b=0.75, device: int = 0):
        self.k1 = k1
        self.b = b
        self.device = device
        self.corpus_size = 0
        self.avgdl = 0
        self.doc_len = []
        self.doc_freqs = {}
        self.idf = {}
        self.tf = []
        self.vocabulary = []
        self.term_to_id = {}
        self.bm25_matrix = None
        self._gpu: GpuIndex | None = None

    # ------------------------------------------------------------------ fit
    def fit(self, corpus):
        """bm25.py:30-121 (host), then the matrix's non-zeros go to HBM."""
        self.corpus_size = len(corpus)
        if self._gpu is not None:
            self._gpu.close()
            self._gpu = None
        if self.corpus_size == 0:
            self.avgdl = 0
            self.doc_len = []
            self.doc_freqs = {}
            self.idf = {}
            self.tf = np.array([])
            self.vocabulary = []
            self.term_to_id = {}
            return
        all_terms = []
        self.doc_len = []
        for doc_tokens in corpus:
            self.doc_len.append(len(doc_tokens))
            all_terms.extend(doc_tokens)
        self.avgdl = np.mean(self.doc_len)
        self.vocabulary = sorted(set(all_terms))
        self.term_to_id = {term: idx for idx, term in enumerate(self.vocabulary)}
        num_terms = len(self.vocabulary)
        if num_terms == 0:
            self.doc_freqs = {}
            self.idf = {}
            self.tf = np.zeros((self.corpus_size, 0))
            return
        # (doc, term, tf) triples; the counting stays on the host like the
        # tokenisation (bm25.py:76-86)
        docs, terms, tfs = [], [], []
        for i, doc_tokens in enumerate(corpus):
            for term, count in Counter(doc_tokens).items():
                docs.append(i)
                terms.append(self.term_to_id[term])
                tfs.append(count)
        docs = np.asarray(docs, np.int32)
        terms = np.asarray(terms, np.int32)
        tfs = np.asarray(tfs, np.float32)
        doc_freq_counts = np.bincount(terms, minlength=num_terms)
        self.doc_freqs = {self.vocabulary[j]: doc_freq_counts[j] for j in range(num_terms)}
        N = self.corpus_size
        self.idf = {}  # bm25.py:95-103 (math.log, host: V values)
        for term in self.vocabulary:
            df = self.doc_freqs[term]
            if N - df + 0.5 > 0 and df + 0.5 > 0:
                self.idf[term] = math.log((N - df + 0.5) / (df + 0.5) + 1)
            else:
                self.idf[term] = 0.0
        idf_vec = np.array([self.idf[term] for term in self.vocabulary], dtype=np.float32)
        # the matrix (bm25.py:106-121) on the GPU: CSC f32 for the index plus
        # the float64 entries of the reference's dense bm25_matrix
        indptr, indices, data, data64 = build_scores(
            docs, terms, tfs, np.asarray(self.doc_len, np.int32), num_terms, k1=self.k1, b=self.b,
            method="bm25py", avgdl=self.avgdl, idf=idf_vec, device=self.device, want_f64=True)
        shape = (self.corpus_size, num_terms)
        self.tf = sp.csc_matrix((tfs, (docs, terms)), shape=shape).toarray()
        self.bm25_matrix = sp.csc_matrix((data64, indices, indptr), shape=shape).toarray()
        self._gpu = GpuIndex(indptr, indices, data, self.corpus_size, device=self.device)
        self._gpu.set_values_f64(data64)  # get_scores / get_top_n rank in float64

    # --------------------------------------------------------------- scoring
    def _query_ids(self, query):
        return [self.term_to_id[term] for term in query if term in self.term_to_id]

    def get_scores(self, query):
        """bm25.py:124-145: per-document scores (float64 [corpus_size]); OOV
        terms are dropped, an all-OOV query scores 0 everywhere."""
        if not hasattr(self, "bm25_matrix") or self.bm25_matrix is None:
            return np.zeros(self.corpus_size if hasattr(self, "corpus_size") else 0)
        ids = self._query_ids(query)
        if not ids:
            return np.zeros(self.corpus_size)
        return self._gpu.scores_dense_f64(np.asarray(ids, np.int32))

    def get_top_n(self, query, corpus, n=5):
        """bm25.py:147-178: [(score, document)] of the n best documents, best
        first; [] for n <= 0 or an empty corpus."""
        if n <= 0:
            return []
        if self.bm25_matrix is None or self.corpus_size == 0:
            return []
        num = min(n, self.corpus_size)
        ids = self._query_ids(query)
        docs, scores = self._gpu.topn_f64(np.asarray(ids, np.int32), num)
        return [(np.float64(s), corpus[int(d)]) for d, s in zip(docs, scores)]
