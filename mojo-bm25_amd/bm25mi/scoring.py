"""GPU index build: (doc, term, tf) triples -> the CSC score matrix.

Host side of ``bm25_build_scores`` (include/bm25mi.h, kernels in
csrc/bm25mi_build.hip): the step upstream of the search path (SURVEY.md §8(f)
row 2).  Two scoring rules:

``"lucene"``  the bm25s writer that produced the reference's on-disk index
              (params.index.json "method": "lucene"; bm25_test.py:19-38):
              idf * tf / (tf + k1 * (1 - b + b * dl / avgdl)),
              idf = ln(1 + (N - df + 0.5) / (df + 0.5)).
``"bm25py"``  BM25.fit's matrix (bm25.py:108-121): the same with a
              (k1 + 1) numerator, float64 as the reference computes it.

Tokenisation stays on the CPU: callers hand over token
ids; ``triples_from_token_ids`` turns per-document token-id lists into
(doc, term, tf) triples.
"""
from __future__ import annotations

import ctypes
from typing import Iterable, Optional, Tuple

import numpy as np

from ._capi import check, lib

METHODS = {"lucene": 0, "bm25py": 1}


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def triples_from_token_ids(docs_token_ids: Iterable) -> Tuple[np.ndarray, np.ndarray,
                                                                np.ndarray, np.ndarray]:
    """Per-document token-id sequences -> (docs, terms, tfs, doc_len): one
    triple per distinct (doc, term) with its count; doc_len = tokens per doc."""
    d_all, t_all, c_all, dl = [], [], [], []
    for i, ids in enumerate(docs_token_ids):
        ids = np.asarray(ids, dtype=np.int64).ravel()
        dl.append(ids.size)
        if ids.size == 0:
            continue
        u, c = np.unique(ids, return_counts=True)
        d_all.append(np.full(u.size, i, np.int32))
        t_all.append(u.astype(np.int32))
        c_all.append(c.astype(np.float32))
    cat = (lambda xs, dt: np.concatenate(xs).astype(dt) if xs else np.zeros(0, dt))
    return (cat(d_all, np.int32), cat(t_all, np.int32), cat(c_all, np.float32),
            np.asarray(dl, np.int32))


def build_scores(docs, terms, tfs, doc_len, n_terms: int, k1: float = 1.5, b: float = 0.75,
                 method: str = "lucene", avgdl: Optional[float] = None,
                 idf: Optional[np.ndarray] = None, device: int = 0, want_f64: bool = False):
    """CSC (indptr int64 [n_terms+1], indices int32, data f32[, data f64]) of
    the BM25 score matrix, built on the GPU.  ``avgdl`` defaults to
    ``np.mean(doc_len)`` (bm25.py:62); ``idf`` (f32 [n_terms]) defaults to the
    device's ln(1 + (N - df + 0.5) / (df + 0.5))."""
    if method not in METHODS:
        raise ValueError(f"method must be one of {sorted(METHODS)}")
    docs = np.ascontiguousarray(docs, dtype=np.int32).ravel()
    terms = np.ascontiguousarray(terms, dtype=np.int32).ravel()
    tfs = np.ascontiguousarray(tfs, dtype=np.float32).ravel()
    dl = np.ascontiguousarray(doc_len, dtype=np.int32).ravel()
    if not (docs.size == terms.size == tfs.size):
        raise ValueError("docs, terms and tfs must have the same length")
    n_docs = dl.size
    if avgdl is None:
        avgdl = float(np.mean(dl.tolist())) if n_docs else 0.0
    if idf is not None:
        idf = np.ascontiguousarray(idf, dtype=np.float32).ravel()
        if idf.size != n_terms:
            raise ValueError("idf must hold one value per term")
    n = docs.size
    indptr = np.zeros(n_terms + 1, np.int64)
    indices = np.zeros(n, np.int32)
    data = np.zeros(n, np.float32)
    data64 = np.zeros(n, np.float64) if want_f64 else None
    check(lib.bm25_build_scores(int(device), n_docs, int(n_terms), n, _ptr(docs), _ptr(terms),
                                _ptr(tfs), _ptr(dl), float(avgdl), float(k1), float(b),
                                METHODS[method], _ptr(idf), _ptr(indptr), _ptr(indices),
                                _ptr(data), _ptr(data64)))
    return (indptr, indices, data, data64) if want_f64 else (indptr, indices, data)
