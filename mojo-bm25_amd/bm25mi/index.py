"""GpuIndex — a device-resident BM25 CSC index on one MI355X.

Host mirror of the reference's index object (bm25_native.BM25v.doc_toks,
bm25_native.py:59-74) backed by libbm25mi.so.  All compute goes through the
C-ABI; this module only validates, converts dtypes and owns the handle.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Tuple

import numpy as np

from . import _capi
from ._capi import check, lib


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


class GpuIndex:
    """A doc x term CSC score matrix resident in HBM.

    Arguments mirror ``scipy.sparse.csc_matrix((data, indices, indptr),
    shape=(n_docs, n_terms))`` — the in-memory form of the bm25s on-disk
    index (indptr/indices/data ``.csc.index.npy``)."""

    def __init__(self, indptr, indices, data, n_docs: int, device: int = 0,
                 doc_offset: int = 0, options: Optional[dict] = None):
        indptr = np.asarray(indptr)
        if indptr.ndim != 1 or indptr.size < 1:
            raise ValueError("indptr must be a 1-D array of n_terms + 1 offsets")
        ip_i64 = indptr.dtype == np.int64 or indptr[-1] > np.iinfo(np.int32).max
        self._indptr = np.ascontiguousarray(indptr, dtype=np.int64 if ip_i64 else np.int32)
        self._indices = np.ascontiguousarray(indices, dtype=np.int32)
        self._data = np.ascontiguousarray(data, dtype=np.float32)
        nnz = int(self._indptr[-1])
        if self._indices.size < nnz or self._data.size < nnz:
            raise ValueError("indices/data shorter than indptr[-1]")
        self.n_docs = int(n_docs)
        self.n_terms = int(self._indptr.size - 1)
        self.nnz = nnz
        self.device = int(device)
        self.doc_offset = int(doc_offset)
        h = ctypes.c_void_p()
        self._h = None
        check(lib.bm25_index_create(self.device, self.n_docs, self.n_terms, nnz,
                                    _ptr(self._indptr), int(ip_i64), _ptr(self._indices),
                                    _ptr(self._data), self.doc_offset, ctypes.byref(h)))
        self._h = h
        # the device holds its own copy
        self._indptr = self._indices = self._data = None
        for name, value in (options or {}).items():
            self.set_option(name, value)

    # ------------------------------------------------------------------
    @classmethod
    def from_csc(cls, m, device: int = 0, doc_offset: int = 0) -> "GpuIndex":
        """From a scipy.sparse CSC matrix (doc x term).  Non-canonical input
        (unsorted indices) is sorted on a copy first; duplicate entries are
        summed (scipy semantics for a CSC with duplicates)."""
        import scipy.sparse as sp
        if not sp.issparse(m):
            raise ValueError("doc_toks must be a scipy.sparse matrix")
        m = m.tocsc()
        if not m.has_canonical_format:
            m = m.copy()
            m.sum_duplicates()
        return cls(m.indptr, m.indices, m.data, m.shape[0], device=device, doc_offset=doc_offset)

    def fork(self) -> "GpuIndex":
        """Another search context on the same device arrays (bm25_index_fork):
        its own workspace, options (copied) and stream, so searches on this
        handle and on the fork may run concurrently on different streams."""
        h = ctypes.c_void_p()
        check(lib.bm25_index_fork(self._h, ctypes.byref(h)))
        g = GpuIndex.__new__(GpuIndex)
        g.__dict__.update({k: v for k, v in self.__dict__.items() if not k.startswith("_")})
        g._indptr = g._indices = g._data = None
        g._h = h
        return g

    # ------------------------------------------------------------------
    def close(self) -> None:
        """Destroy the handle and every fork bm25mi.dist cached on it.  The
        device arrays are shared (bm25_index_fork), so they are released only
        when the last of those handles is gone."""
        for f in self.__dict__.pop("_bm25_forks", []):
            f.close()
        self.__dict__.pop("_bm25_part_streams", None)
        if self._h is not None:
            lib.bm25_index_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> dict:
        vals = [ctypes.c_int64() for _ in range(3)]
        td = ctypes.c_int32()
        nt = ctypes.c_int64()
        db = ctypes.c_int64()
        check(lib.bm25_index_info(self._h, *[ctypes.byref(v) for v in vals], ctypes.byref(td),
                                  ctypes.byref(nt), ctypes.byref(db)))
        sp_ = ctypes.c_int32()
        npairs = ctypes.c_int64()
        check(lib.bm25_index_segments(self._h, ctypes.byref(sp_), ctypes.byref(npairs)))
        hb = ctypes.c_int32()
        bb = ctypes.c_int64()
        check(lib.bm25_index_bounds(self._h, ctypes.byref(hb), ctypes.byref(bb)))
        return {"n_docs": vals[0].value, "n_terms": vals[1].value, "nnz": vals[2].value,
                "tile_docs": td.value, "n_tiles": nt.value, "device_bytes": db.value,
                "sparse": bool(sp_.value), "n_pairs": npairs.value,
                "tile_bounds": bool(hb.value), "tile_bound_bytes": bb.value}

    # ------------------------------------------------------------------
    def search(self, queries: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        """Top-k of every query row (host arrays).  queries: int32 [Q, T]."""
        q = np.ascontiguousarray(queries, dtype=np.int32)
        if q.ndim != 2:
            raise ValueError("queries must be a 2-D [Q, T] int32 array")
        Q, T = q.shape
        k = int(k)
        docs = np.zeros((Q, max(k, 0)), np.int32)
        scores = np.zeros((Q, max(k, 0)), np.float32)
        check(lib.bm25_search(self._h, _ptr(q), Q, T, k, _ptr(docs), _ptr(scores)))
        return docs, scores

    def max_token_device(self, d_queries, stream=None) -> int:
        """Largest token id of a device batch (bm25_max_token_device; syncs)."""
        Q, T = d_queries.shape
        s = getattr(stream, "cuda_stream", stream) or 0
        m = ctypes.c_int32()
        check(lib.bm25_max_token_device(self._h, ctypes.c_void_p(d_queries.data_ptr()), Q, T,
                                        ctypes.byref(m), ctypes.c_void_p(s)))
        return m.value

    def search_device(self, d_queries, k: int, d_docs, d_scores, stream=None,
                      validate: bool = False) -> None:
        """Device-resident search: torch int32 [Q, T] in, int32/f32 [Q, k] out,
        enqueued on ``stream`` (a torch.cuda.Stream or raw handle).  Token ids
        >= n_terms count as padding unless ``validate`` (a synchronising
        device check) raises the reference's ValueError (bm25_native.py:91-96)."""
        Q, T = d_queries.shape
        s = getattr(stream, "cuda_stream", stream) or 0
        if validate:
            m = self.max_token_device(d_queries, stream)
            if m >= self.n_terms:
                raise ValueError(
                    f"The maximum token ID in the query ({m}) is higher than the number "
                    "of tokens in the index.")
        check(lib.bm25_search_device(self._h, ctypes.c_void_p(d_queries.data_ptr()), Q, T,
                                     int(k), ctypes.c_void_p(d_docs.data_ptr()),
                                     ctypes.c_void_p(d_scores.data_ptr()), ctypes.c_void_p(s)))

    # -------------------------------------------- doc-sharded, global theta
    def sample_width(self, k: int, world: int, shard_docs_max: int) -> int:
        w = ctypes.c_int64()
        check(lib.bm25_sample_width(self._h, int(shard_docs_max), int(world), int(k),
                                    ctypes.byref(w)))
        return w.value

    def search_sample_device(self, d_queries, k: int, world: int, shard_docs_max: int, d_keys,
                             stream=None) -> None:
        """This shard's sample keys (torch int64/uint64 [Q, S] on the device)."""
        Q, T = d_queries.shape
        s = getattr(stream, "cuda_stream", stream) or 0
        check(lib.bm25_search_sample_device(self._h, ctypes.c_void_p(d_queries.data_ptr()), Q, T,
                                            int(k), int(world), int(shard_docs_max),
                                            ctypes.c_void_p(d_keys.data_ptr()),
                                            ctypes.c_void_p(s)))

    def search_finish_device(self, d_queries, k: int, world: int, shard_docs_max: int,
                             d_all_keys, d_docs, d_scores, stream=None) -> None:
        """Global theta from every shard's sample keys ([W, Q, S]), then this
        shard's keys >= theta as a padded [Q, k] list (global doc ids)."""
        Q, T = d_queries.shape
        s = getattr(stream, "cuda_stream", stream) or 0
        check(lib.bm25_search_finish_device(self._h, ctypes.c_void_p(d_queries.data_ptr()), Q, T,
                                            int(k), int(world), int(shard_docs_max),
                                            ctypes.c_void_p(d_all_keys.data_ptr()),
                                            ctypes.c_void_p(d_docs.data_ptr()),
                                            ctypes.c_void_p(d_scores.data_ptr()),
                                            ctypes.c_void_p(s)))

    def search_finish_streams_device(self, d_queries, k: int, world: int, shard_docs_max: int,
                                     d_all_keys, d_docs, d_scores, stream_theta, stream_rest,
                                     stream_select) -> None:
        """search_finish_device on three streams (bm25_search_finish_streams_
        device): theta, the REST pass and the merges, ordered by events."""
        Q, T = d_queries.shape
        ss = [getattr(x, "cuda_stream", x) or 0 for x in (stream_theta, stream_rest, stream_select)]
        check(lib.bm25_search_finish_streams_device(
            self._h, ctypes.c_void_p(d_queries.data_ptr()), Q, T, int(k), int(world),
            int(shard_docs_max), ctypes.c_void_p(d_all_keys.data_ptr()),
            ctypes.c_void_p(d_docs.data_ptr()), ctypes.c_void_p(d_scores.data_ptr()),
            *[ctypes.c_void_p(x) for x in ss]))

    # ------------------------------- doc-sharded, one collective (world bounds)
    def bounds_stride(self) -> int:
        """u16 per row of this index's tile bounds (its tiles rounded up to 4)."""
        return (int(self.info()["n_tiles"]) + 3) // 4 * 4

    def bounds_export(self, d_out, stride: int, stream=None) -> None:
        """This index's tile bounds into d_out (a torch int16 [n_terms, stride]
        device tensor; bm25_index_bounds_export)."""
        s = getattr(stream, "cuda_stream", stream) or 0
        check(lib.bm25_index_bounds_export(self._h, ctypes.c_void_p(d_out.data_ptr()), int(stride),
                                           ctypes.c_void_p(s)))

    def set_world_bounds(self, d_world, world: int, stride: int, world_tiles: int) -> None:
        """Every shard's tile bounds ([world, n_terms, stride] int16 on this
        device, kept referenced here) for bm25_search_shard_device; None clears."""
        if d_world is None:
            check(lib.bm25_index_set_world_bounds(self._h, None, 0, 0, 0))
            self.__dict__.pop("_bm25_world_bounds", None)
            return
        check(lib.bm25_index_set_world_bounds(self._h, ctypes.c_void_p(d_world.data_ptr()),
                                              int(world), int(stride), int(world_tiles)))
        self._bm25_world_bounds = d_world
        for f in self.__dict__.get("_bm25_forks", []):
            f.set_world_bounds(d_world, world, stride, world_tiles)

    def search_shard_device(self, d_queries, k: int, d_docs, d_scores, stream=None) -> None:
        """This shard's keys >= the collection's threshold (world bounds) as an
        unsorted padded [Q, k] list for the W-way merge (bm25_search_shard_device)."""
        Q, T = d_queries.shape
        s = getattr(stream, "cuda_stream", stream) or 0
        check(lib.bm25_search_shard_device(self._h, ctypes.c_void_p(d_queries.data_ptr()), Q, T,
                                           int(k), ctypes.c_void_p(d_docs.data_ptr()),
                                           ctypes.c_void_p(d_scores.data_ptr()),
                                           ctypes.c_void_p(s)))

    def scores_dense(self, query) -> np.ndarray:
        """All n_docs fp32 scores of one query (zero for untouched docs)."""
        q = np.ascontiguousarray(np.asarray(query).ravel(), dtype=np.int32)
        out = np.zeros(self.n_docs, np.float32)
        check(lib.bm25_scores_dense(self._h, _ptr(q), q.size, _ptr(out)))
        return out

    # ------------------------------------------- bm25.BM25's float64 path
    def set_values_f64(self, data64) -> None:
        """Keep a float64 copy of the values (same CSC order) on the device
        (bm25_index_set_values_f64)."""
        d = np.ascontiguousarray(data64, dtype=np.float64)
        if d.size < self.nnz:
            raise ValueError("data64 shorter than nnz")
        check(lib.bm25_index_set_values_f64(self._h, _ptr(d)))

    def scores_dense_f64(self, query) -> np.ndarray:
        """float64 sums of every document in query order (numpy's
        np.sum(matrix[:, ids], axis=1), bm25.py:143)."""
        q = np.ascontiguousarray(np.asarray(query).ravel(), dtype=np.int32)
        out = np.zeros(self.n_docs, np.float64)
        check(lib.bm25_scores_dense_f64(self._h, _ptr(q), q.size, _ptr(out)))
        return out

    def topn_f64(self, query, n: int) -> Tuple[np.ndarray, np.ndarray]:
        """The n best documents of those float64 sums, (score desc, doc asc)."""
        q = np.ascontiguousarray(np.asarray(query).ravel(), dtype=np.int32)
        docs = np.zeros(max(int(n), 0), np.int32)
        scores = np.zeros(max(int(n), 0), np.float64)
        check(lib.bm25_topn_f64(self._h, _ptr(q), q.size, int(n), _ptr(docs), _ptr(scores)))
        return docs, scores

    # ------------------------------------------------------------------
    def profile_enable(self, on: bool = True) -> None:
        check(lib.bm25_profile_enable(self._h, int(on)))  # (True = 1: score pass events only)

    def profile_read(self) -> dict:
        sm = ctypes.c_double()
        sl = ctypes.c_int64()
        tm = ctypes.c_double()
        ns = ctypes.c_int64()
        rs = ctypes.c_int64()
        check(lib.bm25_profile_read(self._h, ctypes.byref(sm), ctypes.byref(sl), ctypes.byref(tm),
                                    ctypes.byref(ns), ctypes.byref(rs)))
        return {"score_ms": sm.value, "score_launches": sl.value, "total_ms": tm.value,
                "searches": ns.value, "rescored_tiles_last": rs.value}

    # ------------------------------------------------------------------
    def set_option(self, name: str, value: int) -> None:
        """A search option of this handle (bm25_index_set_option: flat,
        flat_bw, items_per_wave, sample_p, list_cap, claim_ch, claim_m,
        tile_bound, theta_bound).  In a multi-rank search every rank must
        change an option together (like a collective): the next
        ``bm25mi.dist.sharded_search`` re-checks the sample width they agree on."""
        check(lib.bm25_index_set_option(self._h, name.encode(), int(value)))
        self.__dict__.pop("_bm25_width_ok", None)  # (bm25mi.dist._agree_width's cache)
        for f in self.__dict__.get("_bm25_forks", []):  # (bm25mi.dist's part contexts)
            f.set_option(name, value)

    def get_option(self, name: str) -> int:
        v = ctypes.c_int64()
        check(lib.bm25_index_get_option(self._h, name.encode(), ctypes.byref(v)))
        return v.value

    KERNELS = {1: "flat_sample", 2: "flat_rest", 4: "flat_all", 8: "wave_sample",
               16: "wave_rest", 32: "wave_all", 64: "large_k", 128: "bound_keys",
               256: "bound_off", 512: "count_skips", 1024: "rest_split",
               2048: "bound_pool"}  # (flags, not
    # kernels: 256 the tile-bound threshold was off, 512 REST counted the postings it
    # skipped, 1024 REST ran over split items, 2048 the threshold read the pooled bounds)

    def last_dispatch(self) -> dict:
        """What the last search launched (bm25_search_dispatch): the score
        kernels by phase, the flat kernel's term lanes and tiles per item
        (ALL, SAMPLE, REST) and the sampling stride."""
        km = ctypes.c_uint32()
        tl = ctypes.c_int32()
        bt = (ctypes.c_int32 * 3)()
        sp_ = ctypes.c_int32()
        check(lib.bm25_search_dispatch(self._h, ctypes.byref(km), ctypes.byref(tl), bt,
                                       ctypes.byref(sp_)))
        return {"kernels": {n for b, n in self.KERNELS.items() if km.value & b},
                "term_lanes": tl.value,
                "band_tiles": {"all": bt[0], "sample": bt[1], "rest": bt[2]},
                "sample_p": sp_.value}

    def search_stats(self) -> dict:
        """Selection statistics of the last search (bm25_search_counters):
        tiles re-scored exactly, queries sent to the exact fallback stage,
        (query, tile) pairs the REST pass skipped by their tile bound and the
        postings of those pairs, queries left to the block merge."""
        v = (ctypes.c_int64 * 6)()
        check(lib.bm25_search_counters(self._h, v, 6))
        return {"rescored_tiles": v[0], "fallback_queries": v[1],
                "bound_skipped_tiles": v[2], "bound_skipped_postings": v[3],
                "block_merge_queries": v[4], "large_dense_queries": v[5]}


def merge_topk_device(device: int, d_docs, d_scores, W: int, Q: int, k: int, d_out_docs,
                      d_out_scores, stream=None) -> None:
    """Merge W per-shard [Q, k] lists (global doc ids) -> [Q, k] on the GPU."""
    s = getattr(stream, "cuda_stream", stream) or 0
    check(lib.bm25_merge_topk_device(int(device), ctypes.c_void_p(d_docs.data_ptr()),
                                     ctypes.c_void_p(d_scores.data_ptr()), int(W), int(Q), int(k),
                                     ctypes.c_void_p(d_out_docs.data_ptr()),
                                     ctypes.c_void_p(d_out_scores.data_ptr()),
                                     ctypes.c_void_p(s)))


def merge_sorted_device(device: int, d_docs, d_scores, W: int, Q: int, k: int, rank_stride: int,
                        d_out_docs, d_out_scores, stream=None) -> None:
    """W-way merge of best-first [Q, k] lists (bm25_merge_sorted_device):
    rank w's lists start at element w * rank_stride of d_docs / d_scores."""
    s = getattr(stream, "cuda_stream", stream) or 0
    check(lib.bm25_merge_sorted_device(int(device), ctypes.c_void_p(d_docs.data_ptr()),
                                       ctypes.c_void_p(d_scores.data_ptr()), int(W), int(Q),
                                       int(k), int(rank_stride),
                                       ctypes.c_void_p(d_out_docs.data_ptr()),
                                       ctypes.c_void_p(d_out_scores.data_ptr()),
                                       ctypes.c_void_p(s)))


class ShardedIndex:
    """A CSC index doc-sharded over several GPUs of this process
    (bm25_sharded_* in include/bm25mi.h): ``search`` has GpuIndex.search's
    contract and returns the single-index result."""

    def __init__(self, indptr, indices, data, n_docs: int, devices):
        devices = [int(d) for d in devices]
        if not devices:
            raise ValueError("need at least one device")
        indptr = np.asarray(indptr)
        ip_i64 = indptr.dtype == np.int64 or indptr[-1] > np.iinfo(np.int32).max
        ip = np.ascontiguousarray(indptr, dtype=np.int64 if ip_i64 else np.int32)
        ix = np.ascontiguousarray(indices, dtype=np.int32)
        dt = np.ascontiguousarray(data, dtype=np.float32)
        devs = np.asarray(devices, np.int32)
        self.n_docs = int(n_docs)
        self.n_terms = int(ip.size - 1)
        self._h = None
        h = ctypes.c_void_p()
        check(lib.bm25_sharded_create(len(devices), _ptr(devs), self.n_docs, self.n_terms,
                                      int(ip[-1]), _ptr(ip), int(ip_i64), _ptr(ix), _ptr(dt),
                                      ctypes.byref(h)))
        self._h = h

    def shards(self):
        n = ctypes.c_int64()
        check(lib.bm25_sharded_info(self._h, ctypes.byref(n), None, None))
        lo = np.zeros(n.value, np.int64)
        hi = np.zeros(n.value, np.int64)
        check(lib.bm25_sharded_info(self._h, ctypes.byref(n), _ptr(lo), _ptr(hi)))
        return list(zip(lo.tolist(), hi.tolist()))

    def search(self, queries: np.ndarray, k: int) -> Tuple[np.ndarray, np.ndarray]:
        q = np.ascontiguousarray(queries, dtype=np.int32)
        if q.ndim != 2:
            raise ValueError("queries must be a 2-D [Q, T] int32 array")
        Q, T = q.shape
        k = int(k)
        docs = np.zeros((Q, max(k, 0)), np.int32)
        scores = np.zeros((Q, max(k, 0)), np.float32)
        check(lib.bm25_sharded_search(self._h, _ptr(q), Q, T, k, _ptr(docs), _ptr(scores)))
        return docs, scores

    def close(self) -> None:
        if self._h is not None:
            lib.bm25_sharded_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def device_count() -> int:
    return _capi.device_count()
