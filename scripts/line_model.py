"""Cache-line model of the flat kernel's posting reads on the config-3 batch
(CPU, dev tool).  For the rows the REST pass issues (double rows of 128
postings per (query, tile, term) segment, aligned to an even posting; every
lane loads 4 B of ldoc and 8 B of val), count 128-B lines:
  req   : lines per row summed over every query (no reuse at all)
  band  : distinct lines per 8-tile band, summed over bands (perfect reuse
          of a band's lines among the batch's queries, none across bands)
  batch : distinct lines of the whole batch (perfect cache)
each for full-row loads and for loads masked to the row's valid lanes.
  python scripts/line_model.py [--config c3] [--band 8]"""
import argparse
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
from bm25mi import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--band", type=int, default=8)
ap.add_argument("--S", type=int, default=11)
args = ap.parse_args()
cfg = synth.CONFIGS[args.config]
ip, ix, dt = synth.make_index(cfg, threads=8)
q = synth.make_queries(cfg)
terms, cnt = np.unique(q[q >= 0], return_counts=True)
S, BW = args.S, args.band
tot = {k: 0 for k in ("req", "req_m", "band", "band_m", "batch", "batch_m")}
post = 0
for t, c in zip(terms, cnt):
    a, b = int(ip[t]), int(ip[t + 1])
    if b == a:
        continue
    tiles = ix[a:b] >> S
    starts = np.r_[0, np.nonzero(np.diff(tiles))[0] + 1]
    L = np.diff(np.r_[starts, b - a])
    seg0 = a + starts                         # first posting of each segment
    par = seg0 & 1
    nr = (par + L + 127) // 128               # double rows per segment
    segi = np.repeat(np.arange(len(L)), nr)
    k = np.arange(nr.sum()) - np.repeat(np.cumsum(nr) - nr, nr)
    base = (seg0[segi] & ~1) + 128 * k        # even first posting of the row
    hi = np.minimum(128, par[segi] + L[segi] - 128 * k)  # valid positions [.., hi)
    vh = (hi + 1) // 2                        # valid lanes
    band = (tiles[starts][segi] // BW).astype(np.int64)
    post += c * (b - a)
    for m, nl in (("", np.full_like(vh, 64)), ("_m", vh)):
        # ldoc: 4 B per lane at 2 * base; val: 8 B per lane at 4 * base (separate arrays)
        l0 = (2 * base) // 128
        l1 = (2 * base + 4 * nl - 1) // 128
        v0 = (4 * base) // 128
        v1 = (4 * base + 8 * nl - 1) // 128
        tot["req" + m] += c * int((l1 - l0 + 1).sum() + (v1 - v0 + 1).sum())
        # distinct lines per band / per batch: expand the line ranges
        def expand(x0, x1):
            n = x1 - x0 + 1
            return np.repeat(x0, n) + (np.arange(n.sum()) - np.repeat(np.cumsum(n) - n, n))
        lb = np.repeat(band, l1 - l0 + 1)
        vb = np.repeat(band, v1 - v0 + 1)
        L_ = expand(l0, l1)
        V_ = expand(v0, v1)
        tot["band" + m] += len(np.unique(lb * (1 << 40) + L_)) + len(np.unique(vb * (1 << 40) + V_))
        tot["batch" + m] += len(np.unique(L_)) + len(np.unique(V_))
print(f"{args.config} tile 2^{S} band {BW}: postings {post / 1e9:.3f} G "
      f"(6 B each: {post * 6 / 1e9:.2f} GB)")
for key, v in tot.items():
    print(f"  {key:8s} {v / 1e6:9.1f} M lines = {v * 128 / 1e9:7.2f} GB")
