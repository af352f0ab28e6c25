"""Model of MaxScore-style term pruning on the config-3 workload (dev analysis,
CPU only).  For a sample of the bench's queries: the exact dense scores (C
oracle), theta = the query's R-th best score (the sampled threshold is ~the
900th best), each term's largest score, the non-essential terms
(lowest maxima whose fp32 sum stays below theta), the share of the query's
postings that belong to essential terms, and how many documents an essential-
only pass would flag (partial essential sum + the non-essential bound >= theta).

  python scripts/maxscore_model.py [--config c3] [--queries 32] [--rank 900]
"""
import argparse
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
    ap.add_argument("--queries", type=int, default=32)
    ap.add_argument("--rank", type=int, default=900)
    ap.add_argument("--terms", type=int, default=0)
    args = ap.parse_args()
    from bm25mi import synth
    from oracle import oracle
    import dataclasses
    cfg = synth.CONFIGS[args.config]
    if args.terms:
        cfg = dataclasses.replace(cfg, terms_per_query=args.terms)
    t0 = time.time()
    ip, ix, dt = synth.make_index(cfg, threads=8)
    print(f"index {time.time() - t0:.1f}s", file=sys.stderr)
    q = synth.make_queries(cfg)[:args.queries]
    df = np.diff(ip)
    tmax = np.zeros(len(df), np.float32)
    nz = np.nonzero(df)[0]
    tmax[nz] = np.maximum.reduceat(dt, ip[nz])
    tot_post = ess_post = 0
    flagged = []
    for row in q:
        terms = row[row >= 0]
        dense = oracle.scores_dense_c(cfg.n_docs, ip, ix, dt, terms)
        theta = np.partition(dense, -args.rank)[-args.rank]
        order = np.argsort(tmax[terms], kind="stable")
        bound = np.float32(0)
        ne = []
        for j in order:
            b2 = np.float32(bound + tmax[terms[j]])
            if b2 >= theta:
                break
            bound = b2
            ne.append(j)
        ess = [j for j in range(len(terms)) if j not in ne]
        post = df[terms].sum()
        epost = df[terms[ess]].sum() if ess else 0
        tot_post += post
        ess_post += epost
        part = oracle.scores_dense_c(cfg.n_docs, ip, ix, dt, terms[ess]) if ess else np.zeros(1)
        flagged.append(int(np.sum(part + bound >= theta)))
        print(json.dumps({"theta": float(theta), "ne_terms": len(ne), "terms": len(terms),
                          "postings": int(post), "essential_postings": int(epost),
                          "bound": float(bound), "flagged": flagged[-1]}), flush=True)
    print(json.dumps({"config": args.config, "queries": len(q), "rank": args.rank,
                      "essential_share": ess_post / tot_post,
                      "flagged_median": float(np.median(flagged))}))


if __name__ == "__main__":
    main()
