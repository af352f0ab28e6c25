"""Per-rank doc sharding of a CSC index.

A collection larger than one GPU (config 5: 100M docs, 6.4B postings — past
int32 ``indptr``, params.index.json:8) is held as one doc shard per rank.
``shard_csc`` cuts rank r's contiguous doc range out of a global CSC whose
``indptr`` may be int64, streaming over the (possibly memory-mapped) arrays in
bounded column blocks, so the global arrays are never copied whole; the shard
is an ordinary CSC with local doc ids (int32) and its own int64 ``indptr``.
``load_bm25s_shard`` does this straight from a bm25s directory.

``shard_bounds`` is the one definition of the per-rank doc ranges (2048-doc
aligned, the same on every rank); bm25mi.dist and bm25mi.synth use it.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

# postings examined per block (bounded host memory when the arrays are mmaps)
BLOCK_POSTINGS = 1 << 26


def shard_bounds(n_docs: int, world: int, rank: int, align: int = 2048) -> Tuple[int, int]:
    """Contiguous doc range [lo, hi) of ``rank``: an even split with inner
    boundaries rounded to multiples of ``align`` (the 2048-doc LDS tile, so no
    shard carries a partial tile except the last)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad shard {rank} of {world}")

    def b(r: int) -> int:
        if r >= world:
            return int(n_docs)
        x = (int(n_docs) * r) // world
        return min(int(n_docs), (x + align // 2) // align * align)

    return b(rank), b(rank + 1)


def _column_blocks(indptr: np.ndarray, limit: int):
    """[t0, t1) column ranges holding about ``limit`` postings each."""
    V = indptr.size - 1
    t0 = 0
    while t0 < V:
        target = int(indptr[t0]) + limit
        t1 = int(np.searchsorted(indptr, target, side="right")) - 1
        t1 = min(V, max(t1, t0 + 1))
        yield t0, t1
        t0 = t1


def shard_csc(indptr, indices, data, lo: int, hi: int, block: int = BLOCK_POSTINGS):
    """Docs [lo, hi) of a canonical CSC (indices sorted per column) ->
    (indptr int64 [V+1], indices int32 local to lo, data f32)."""
    indptr = np.asarray(indptr)
    if indptr.ndim != 1 or indptr.size < 1 or int(indptr[0]) != 0:
        raise ValueError("indptr must be a 1-D array of n_terms + 1 offsets from 0")
    if not 0 <= lo <= hi:
        raise ValueError(f"bad doc range [{lo}, {hi})")
    V = indptr.size - 1
    p0 = np.empty(V, np.int64)
    p1 = np.empty(V, np.int64)
    ip64 = indptr.astype(np.int64, copy=False)
    for t0, t1 in _column_blocks(ip64, block):
        a, b = int(ip64[t0]), int(ip64[t1])
        seg = np.asarray(indices[a:b])
        off = ip64[t0:t1 + 1] - a
        for bound, out in ((lo, p0), (hi, p1)):
            c = np.zeros(b - a + 1, np.int64)
            np.cumsum(seg < bound, out=c[1:])
            out[t0:t1] = ip64[t0:t1] + (c[off[1:]] - c[off[:-1]])
    n = p1 - p0
    sip = np.zeros(V + 1, np.int64)
    np.cumsum(n, out=sip[1:])
    six = np.empty(int(sip[-1]), np.int32)
    sdt = np.empty(int(sip[-1]), np.float32)
    for t0, t1 in _column_blocks(ip64, block):
        a, b = int(ip64[t0]), int(ip64[t1])
        seg_i = np.asarray(indices[a:b])
        seg_d = np.asarray(data[a:b])
        sel = np.zeros(b - a + 1, np.int64)
        # mark each column's [p0, p1) inside the block, then compress
        np.add.at(sel, p0[t0:t1] - a, 1)
        np.add.at(sel, p1[t0:t1] - a, -1)
        keep = np.cumsum(sel[:-1]) > 0
        d0, d1 = int(sip[t0]), int(sip[t1])
        six[d0:d1] = seg_i[keep] - lo
        sdt[d0:d1] = seg_d[keep]
    return sip, six, sdt


def load_bm25s_shard(path: str, rank: int, world: int):
    """Rank ``rank`` of ``world``'s doc shard of a bm25s directory (arrays
    memory-mapped; int32 or int64 indptr) -> (indptr, indices, data, n_docs,
    doc_offset, Bm25sIndex)."""
    from .bm25s_io import load_bm25s
    ix = load_bm25s(path, mmap=True)
    lo, hi = shard_bounds(ix.num_docs, world, rank)
    ip, ii, dd = shard_csc(ix.indptr, ix.indices, ix.data, lo, hi)
    return ip, ii, dd, hi - lo, lo, ix
