"""Posting-segment statistics of the config-3 batch (CPU, dev tool): per
(query, tile) segments, double rows, rows using <= 64 positions, segment
length histogram, for tile sizes 2^10..2^13.
  python scripts/segment_stats.py > profiles/r03/segment_stats.txt"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
from bm25mi import synth  # noqa: E402

cfg = synth.CONFIGS["c3"]
ip, ix, dt = synth.make_index(cfg, threads=8)
q = synth.make_queries(cfg)
terms, cnt = np.unique(q[q >= 0], return_counts=True)
for S in (10, 11, 12, 13):
    rows = half = post = segs = 0
    hist = np.zeros(9, np.int64)
    for t, c in zip(terms, cnt):
        a, b = int(ip[t]), int(ip[t + 1])
        if b == a:
            continue
        tiles = ix[a:b] >> S
        starts = np.r_[0, np.nonzero(np.diff(tiles))[0] + 1]
        L = np.diff(np.r_[starts, b - a])
        par = (a + starts) & 1
        nr = (par + L + 127) // 128
        last = (par + L) - 128 * (nr - 1)
        rows += c * nr.sum()
        half += c * (last <= 64).sum()
        post += c * L.sum()
        segs += c * len(L)
        hist += c * np.bincount(np.minimum(np.log2(np.maximum(L, 1)).astype(int), 8), minlength=9)[:9]
    print(f"tile 2^{S}: postings {post / 1e9:.3f} G, segments {segs / 1e6:.1f} M, double rows "
          f"{rows / 1e6:.1f} M, rows using <= 64 positions {half / rows:.3f}, lane use "
          f"{post / (rows * 128):.3f}, segment length log2 histogram "
          f"{np.round(hist / segs, 3).tolist()}")
