"""Model of the REST pass's tile bound (dev analysis, CPU only).

For a sample of a config's bench queries: the exact k-th best score (C
oracle), the sampled threshold the engine takes (k-th best of the sample
tiles' best sums: groups of 8 tiles every P * 8), a threshold from the
per-(term, tile) maxima alone (k-th best over tiles of the tile's largest
single-term maximum: a real doc's score lower bound, no SAMPLE pass), and the
share of (query, tile) pairs and of postings the tile bound skips at each.

  python scripts/bound_model.py [--config c3] [--queries 16] [--terms 8]
"""
import argparse
import dataclasses
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--queries", type=int, default=16)
    ap.add_argument("--terms", type=int, default=0)
    ap.add_argument("--shard", type=int, default=0, help="c5: rank of the 8-way shard")
    ap.add_argument("--P", type=int, default=8)
    args = ap.parse_args()
    from bm25mi import synth
    from oracle import oracle
    cfg = synth.CONFIGS[args.config]
    if args.terms:
        cfg = dataclasses.replace(cfg, terms_per_query=args.terms)
    lo, hi = (synth.shard_bounds(cfg.n_docs, 8, args.shard) if args.config == "c5"
              else (0, cfg.n_docs))
    t0 = time.time()
    ip, ix, dt = synth.make_index(cfg, lo, hi, threads=8)
    N = hi - lo
    print(f"index {time.time() - t0:.1f}s", file=sys.stderr)
    q = synth.make_queries(cfg)[:args.queries]
    k = cfg.k
    TD = 2048
    nt = (N + TD - 1) // TD
    used = np.unique(q[q >= 0])
    # per-(term, tile) maxima and posting counts of the batch's terms
    tmax = {}
    tcnt = {}
    for t in used:
        a, b = ip[t], ip[t + 1]
        tiles = ix[a:b] // TD
        m = np.zeros(nt, np.float32)
        np.maximum.at(m, tiles, dt[a:b])
        tmax[t] = m
        tcnt[t] = np.bincount(tiles, minlength=nt)
    G, P = 8, args.P
    samp = np.zeros(nt, bool)
    for g0 in range(0, nt, G * P):
        samp[g0:g0 + G] = True
    rows = []
    for row in q:
        terms = row[row >= 0]
        dense = oracle.scores_dense_c(N, ip, ix, dt, terms)
        best = np.zeros(nt, np.float32)
        np.maximum.at(best, np.arange(N) // TD, dense)
        theta_exact = np.partition(dense, -k)[-k]
        sb = np.sort(best[samp])[::-1]
        theta_samp = sb[k - 1] if len(sb) >= k else 0.0
        lb = np.zeros(nt, np.float32)
        ub = np.zeros(nt, np.float32)
        cnt = np.zeros(nt, np.int64)
        for t in terms:
            lb = np.maximum(lb, tmax[t])
            ub = ub + tmax[t]
            cnt += tcnt[t]
        theta_lb = np.sort(lb)[::-1][k - 1]
        r = {"theta_exact": float(theta_exact), "theta_sample": float(theta_samp),
             "theta_lb": float(theta_lb)}
        rest = ~samp
        for name, th in (("sample", theta_samp), ("lb", theta_lb), ("exact", theta_exact)):
            cut = ub * 1.0001 < th
            r[f"skip_tiles_{name}"] = float(cut[rest].mean())
            r[f"skip_post_{name}"] = float(cnt[rest & cut].sum() / max(cnt[rest].sum(), 1))
            r[f"flag_tiles_{name}"] = float((best[rest] >= th).mean())
            r[f"docs_ge_{name}"] = int((dense >= th).sum())
        rows.append(r)
        print(json.dumps(r), flush=True)
    keys = rows[0].keys()
    print(json.dumps({"config": args.config, "terms": int(cfg.terms_per_query),
                      "queries": len(rows),
                      **{f"mean_{kk}": float(np.mean([r[kk] for r in rows])) for kk in keys}}))


if __name__ == "__main__":
    main()
