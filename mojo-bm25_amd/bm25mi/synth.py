"""Seeded synthetic CSC indices / query batches (ctypes over libbm25synth.so).

The BASELINE.md configs, generated deterministically and shard-independently
(model in csrc/synth.cpp's header).  Data source for bench.py and the parity
tests — not part of the scoring path.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import numpy as np

from .build import SYNTH_LIB

_lib = None


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(SYNTH_LIB):
            raise ImportError(f"{SYNTH_LIB} missing: run __graft_entry__.build()")
        lib = ctypes.CDLL(SYNTH_LIB)
        P = ctypes.c_void_p
        i64 = ctypes.c_int64
        d = ctypes.c_double
        u64 = ctypes.c_uint64
        lib.bm25_synth_df.argtypes = [i64, i64, i64, d, P]
        lib.bm25_synth_count.argtypes = [i64, i64, i64, d, u64, i64, i64, ctypes.c_int, P]
        lib.bm25_synth_fill.argtypes = [i64, i64, i64, d, u64, i64, i64, ctypes.c_int, P, P, P]
        lib.bm25_synth_fill_w.argtypes = [i64, i64, i64, d, u64, i64, i64, ctypes.c_int, P, P,
                                          P, ctypes.c_int]
        lib.bm25_synth_queries.argtypes = [i64, P, i64, i64, d, u64, P]
        for f in (lib.bm25_synth_df, lib.bm25_synth_count, lib.bm25_synth_fill,
                  lib.bm25_synth_fill_w, lib.bm25_synth_queries):
            f.restype = ctypes.c_int
        _lib = lib
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


@dataclass
class Config:
    name: str
    n_docs: int
    n_terms: int
    nnz: int
    n_queries: int
    terms_per_query: int
    k: int
    alpha: float = 1.0
    beta: float = 0.75
    index_seed: int = 0
    query_seed: int = 1
    # posting weights: "idf" (idf * U(0.1, 1), the BASELINE configs),
    # "uniform" (U(0.05, 3) for every term: terms weigh alike), "lucene"
    # (1 + Poisson(0.6) term frequencies scored by bm25s's lucene formula with
    # document lengths on the GPU, bm25_build_scores)
    weights: str = "idf"


WEIGHTS = {"idf": 0, "uniform": 1, "tf": 2}


# BASELINE.json configs (config 1 is the animal_index_bm25 fixture; 4 and 5 are
# config 3 / a 100M-doc index sharded over GPUs).
CONFIGS = {
    "c2": Config("1M docs / 50k vocab, batch=256, k=10", 1_000_000, 50_000, 3_200_000, 256, 8, 10),
    "c3": Config("10M docs / 200k vocab, batch=1024, k=100", 10_000_000, 200_000, 640_000_000,
                 1024, 8, 100),
    "c5": Config("100M docs / 1M vocab, batch=1024, k=100", 100_000_000, 1_000_000,
                 6_400_000_000, 1024, 8, 100),
}
# side lines: config 3's postings and queries, other weights
CONFIGS["c3u"] = Config("10M docs / 200k vocab, uniform U(0.05,3) weights, batch=1024, k=100",
                        10_000_000, 200_000, 640_000_000, 1024, 8, 100, weights="uniform")
CONFIGS["c3l"] = Config("10M docs / 200k vocab, lucene-scored (tf, doc lengths), batch=1024, "
                        "k=100", 10_000_000, 200_000, 640_000_000, 1024, 8, 100,
                        weights="lucene")


def df_target(cfg: Config) -> np.ndarray:
    df = np.zeros(cfg.n_terms, np.int64)
    if _load().bm25_synth_df(cfg.n_docs, cfg.n_terms, cfg.nnz, cfg.alpha, _p(df)):
        raise ValueError("bad synth config")
    return df


def make_index(cfg: Config, doc_lo: int = 0, doc_hi: Optional[int] = None, threads: int = 0,
               device: int = 0):
    """CSC (indptr int64, indices int32 local to doc_lo, data f32) of docs
    [doc_lo, doc_hi) of the config's collection.  weights "lucene": the
    scores come from bm25_build_scores on ``device`` (the GPU; see
    make_lucene_index)."""
    if cfg.weights == "lucene":
        return make_lucene_index(cfg, doc_lo, doc_hi, threads, device)
    return _fill(cfg, doc_lo, doc_hi, threads, WEIGHTS[cfg.weights])


def _fill(cfg: Config, doc_lo, doc_hi, threads, weights):
    doc_hi = cfg.n_docs if doc_hi is None else doc_hi
    lib = _load()
    indptr = np.zeros(cfg.n_terms + 1, np.int64)
    if lib.bm25_synth_count(cfg.n_docs, cfg.n_terms, cfg.nnz, cfg.alpha, cfg.index_seed, doc_lo,
                            doc_hi, threads, _p(indptr)):
        raise ValueError("bad synth range")
    nnz = int(indptr[-1])
    indices = np.empty(nnz, np.int32)
    data = np.empty(nnz, np.float32)
    if lib.bm25_synth_fill_w(cfg.n_docs, cfg.n_terms, cfg.nnz, cfg.alpha, cfg.index_seed, doc_lo,
                             doc_hi, threads, _p(indptr), _p(indices), _p(data), int(weights)):
        raise RuntimeError("synth fill mismatch")
    return indptr, indices, data


def make_lucene_index(cfg: Config, doc_lo: int = 0, doc_hi: Optional[int] = None,
                      threads: int = 0, device: int = 0, k1: float = 1.5, b: float = 0.75):
    """The config's postings with term frequencies 1 + Poisson(0.6), each
    document's length = the sum of its term frequencies, scored on the GPU by
    bm25_build_scores with bm25s's lucene formula (idf * tf / (tf + k1 (1 - b
    + b dl / avgdl)), idf = ln(1 + (N - df + 0.5) / (df + 0.5)) of the shard's
    document frequencies) — the kind of index the reference's bm25s writer
    produces (bm25_test.py:19-38).  avgdl is the shard's own mean."""
    from .scoring import build_scores
    doc_hi = cfg.n_docs if doc_hi is None else doc_hi
    indptr, indices, tf = _fill(cfg, doc_lo, doc_hi, threads, WEIGHTS["tf"])
    n = doc_hi - doc_lo
    terms = np.repeat(np.arange(cfg.n_terms, dtype=np.int32), np.diff(indptr))
    dl = np.bincount(indices, weights=tf, minlength=n).astype(np.int32)
    ip, ix, dt = build_scores(indices, terms, tf, dl, cfg.n_terms, k1=k1, b=b, method="lucene",
                              device=device)
    del terms, tf
    if not np.array_equal(ip, indptr):
        raise RuntimeError("build_scores changed the CSC structure")
    return ip, ix, dt


def make_queries(cfg: Config, df: Optional[np.ndarray] = None, n_queries: Optional[int] = None,
                 seed: Optional[int] = None) -> np.ndarray:
    df = df_target(cfg) if df is None else df
    Q = cfg.n_queries if n_queries is None else n_queries
    out = np.zeros((Q, cfg.terms_per_query), np.int32)
    if _load().bm25_synth_queries(cfg.n_terms, _p(df), Q, cfg.terms_per_query, cfg.beta,
                                  cfg.query_seed if seed is None else seed, _p(out)):
        raise ValueError("bad query config")
    return out


def shard_bounds(n_docs: int, world: int, rank: int, align: int = 16384):
    """Contiguous doc range of a shard (bm25mi.shard.shard_bounds' rule),
    aligned to the generator's 16384-doc chunks (a multiple of the 2048-doc
    tile) so that a shard is generated independently of the others."""
    from .shard import shard_bounds as bounds
    return bounds(n_docs, world, rank, align=align)
