"""Drop-in replacement of the reference's ``bm25_native`` module (BM25v).

Same class, constructor, methods, argument meaning, dtypes and error
behaviour as ``bm25_native.py:32-158`` of yuhuishi-convect/mojo-bm25, with the
scoring (posting gather, per-document fp32 scatter-add, top-k) running on an
MI355X through libbm25mi.so.  Put ``mojo-bm25_amd/`` on ``sys.path`` and
``import bm25_native`` as before.

Deliberate differences:
  * invalid query arrays raise ValueError directly (the reference first drops
    into ``breakpoint()``, bm25_native.py:113);
  * documents with equal scores are ordered by doc id ascending (the
    reference's order is numpy-implementation-defined, bm25_native.py:205-212).
Every top_k <= num_docs is served, as by the reference's argpartition
(bm25_native.py:204-214): k <= 4096 by the thresholded pipeline (tile-bound or
sampled threshold, REST lists, wave merges), larger k by the large-k list path
of csrc/bm25mi_large.hip (sampled slice-maximum threshold, REST crossing
lists, selection and row sort), and by dense score rows with a radix
selection only where lists cannot serve (signed indices, k > 131 072, a list
past its capacity).
"""
from __future__ import annotations

import logging
from typing import Optional, Tuple

import numpy as np
import scipy.sparse as sp

from bm25mi.index import GpuIndex

QueryId = np.int32
TokId = np.int32
DocId = np.int32
Score = np.float32


class BM25v:
    """BM25v(ector): BM25 over a precomputed doc x term score matrix in CSC
    form (bm25_native.py:32-38), resident on the GPU."""

    logger = logging.getLogger(__name__)

    def __init__(self, k1: float = 1.5, b: float = 0.75, device: int = 0):
        self.k1 = k1
        self.b = b
        self.dtype = np.float32
        self.device = device
        self.doc_toks: sp.csc_matrix = sp.csc_matrix(np.zeros((0,), dtype=self.dtype))
        self.doc_lengths: np.ndarray = np.zeros((0,), dtype=self.dtype)
        self.avg_doc_length: float = 0.0
        self.num_docs: int = 0
        self._gpu: GpuIndex | None = None

    def index(self, doc_toks: sp.csc_matrix, doc_lengths) -> None:
        """bm25_native.py:59-74.  Copies the CSC matrix into HBM (the doc
        lengths are kept but, as in the reference, not used for scoring)."""
        self.doc_toks = doc_toks
        self.doc_lengths = doc_lengths
        self.avg_doc_length = np.mean(doc_lengths)
        self.num_docs = doc_toks.shape[0]
        if self._gpu is not None:
            self._gpu.close()
        self._gpu = GpuIndex.from_csc(doc_toks, device=self.device)

    @classmethod
    def from_bm25s(cls, path: str, device: int = 0, k1: Optional[float] = None,
                   b: Optional[float] = None) -> "BM25v":
        """A BM25v over a bm25s index directory (indptr/indices/data
        .csc.index.npy + params.index.json, bm25_test.py:35-42), with doc
        lengths of ones (bm25s does not store them; unused for scoring)."""
        from bm25mi.bm25s_io import load_bm25s
        ix = load_bm25s(path)
        m = cls(k1=ix.params.get("k1", 1.5) if k1 is None else k1,
                b=ix.params.get("b", 0.75) if b is None else b, device=device)
        m.vocab = ix.vocab
        n = ix.num_docs
        m.index(sp.csc_matrix((ix.data, ix.indices, ix.indptr), shape=(n, ix.n_terms)),
                np.ones(n, np.float32))
        return m

    def search(self, queries, top_k: int = 100) -> Tuple[np.ndarray, np.ndarray]:
        """bm25_native.py:76-103: sorted top-k doc ids (int32) and scores (f32)."""
        if self.num_docs is None:
            raise ValueError("BM25v index not built. Call index() first.")
        if len(queries) == 0:
            self.logger.info(
                msg="The query is empty. This will result in a zero score for all documents.")
            return np.zeros((0, 0), dtype=self.dtype), np.zeros((0, 0), dtype=self.dtype)
        return self.get_scores(queries, top_k)

    def get_scores(self, queries, top_k: int) -> Tuple[np.ndarray, np.ndarray]:
        """bm25_native.py:105-127 (validation), then the GPU path."""
        if (not isinstance(queries, np.ndarray) or queries.ndim != 2
                or not isinstance(queries[0][0], TokId)):
            raise ValueError("The queries must be a list of list of query token IDs.")
        max_token_id = int(queries.max(initial=0))
        n_terms = self._gpu.n_terms if self._gpu is not None else len(self.doc_toks.indptr) - 1
        if max_token_id >= n_terms:
            raise ValueError(
                f"The maximum token ID in the query ({max_token_id}) is higher than the number "
                "of tokens in the index.")
        return self._compute_relevance_from_scores(queries=queries, top_k=top_k,
                                                   dtype=self.dtype)

    def _compute_relevance_from_scores(self, queries, top_k: int, dtype=np.float32):
        """bm25_native.py:129-158 on the GPU: per query, negative ids dropped,
        postings gathered, fp32 sums in query order, top-k."""
        if top_k < 0:
            raise ValueError("negative dimensions are not allowed")
        return self._gpu.search(queries, top_k)
