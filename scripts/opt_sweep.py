"""Time search-option variants of ONE built index in one process (GPU box).

  python scripts/opt_sweep.py --config c3 --terms 8,16 --sets '[{}, {"flat_bw": 4}]'

Per (terms, option set): 3 warm-up searches, then --steps device searches
with the handle's HIP-event profile (score pass = SAMPLE + theta + REST);
prints one JSON line each and checks that every variant returns the same
bits as the first (options never change results).
"""
import argparse
import dataclasses
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(REPO, "mojo-bm25_amd"), REPO):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3")
    ap.add_argument("--terms", default="8")
    ap.add_argument("--sets", default="[{}]")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--segments", default="")
    args = ap.parse_args()
    import torch
    from bm25mi import synth
    from bm25mi.index import GpuIndex
    from bench import algorithmic_bytes
    if args.segments:
        os.environ["BM25_SEGMENTS"] = args.segments
    cfg = synth.CONFIGS[args.config]
    lo, hi = (0, cfg.n_docs) if args.config != "c5" else synth.shard_bounds(cfg.n_docs, 8, 0)
    t0 = time.time()
    ip, ix, dt = synth.make_index(cfg, lo, hi, threads=16)
    print(f"# index generated in {time.time() - t0:.1f}s nnz={int(ip[-1])}", file=sys.stderr,
          flush=True)
    index = GpuIndex(ip, ix, dt, hi - lo, doc_offset=lo)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for T in [int(x) for x in args.terms.split(",")]:
        q = synth.make_queries(dataclasses.replace(cfg, terms_per_query=T))
        Q, k = q.shape[0], cfg.k
        alg = algorithmic_bytes(ip, q, k)
        dq = torch.from_numpy(q).to(dev)
        dd = torch.empty((Q, k), dtype=torch.int32, device=dev)
        ds = torch.empty((Q, k), dtype=torch.float32, device=dev)
        ref = None
        for opts in json.loads(args.sets):
            for name in ("flat", "flat_bw", "items_per_wave", "sample_p", "list_cap",
                         "claim_ch", "claim_m"):
                index.set_option(name, {"flat": 1, "flat_bw": 0, "items_per_wave": 8,
                                        "sample_p": 8, "list_cap": 0, "claim_ch": 1,
                                        "claim_m": 4}[name])
            for name, val in opts.items():
                index.set_option(name, val)
            for _ in range(3):
                index.search_device(dq, k, dd, ds, st)
            torch.cuda.synchronize()
            index.profile_enable(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.steps):
                index.search_device(dq, k, dd, ds, st)
            e1.record(st)
            torch.cuda.synchronize()
            pr = index.profile_read()
            ms = e0.elapsed_time(e1) / args.steps
            score_ms = pr["score_ms"] / max(pr["score_launches"], 1)
            got = (dd.cpu().numpy(), ds.cpu().numpy().view(np.uint32))
            same = None
            if ref is None:
                ref = got
            else:
                same = bool(np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]))
            print(json.dumps({"config": args.config, "terms": T, "opts": opts,
                              "ms_per_search": round(ms, 4), "score_ms": round(score_ms, 4),
                              "qps": round(Q / ms * 1e3, 1),
                              "frac": round(alg / (score_ms * 1e-3) / 8e12, 4),
                              "dispatch": {**index.last_dispatch(),
                                           "kernels": sorted(index.last_dispatch()["kernels"])},
                              "fallback": index.search_stats()["fallback_queries"],
                              "same_bits_as_first": same}), flush=True)
            index.profile_enable(False)


if __name__ == "__main__":
    main()
