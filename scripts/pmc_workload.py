"""A short search workload for profilers (dev tool, not part of the product):
the config's index and query batch, 2 warm-up + 5 profiled searches.

  python scripts/pmc_workload.py [--config c3] [--terms 8] [--c5-rank 0]
"""
import argparse
import dataclasses
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--terms", type=int, default=0)
ap.add_argument("--c5-rank", type=int, default=0)
ap.add_argument("--searches", type=int, default=5)
args = ap.parse_args()

import torch  # noqa: E402
if os.environ.get("VLIB"):  # a variant build (scripts/build_variant.sh)
    import importlib  # (bm25mi.build as an attribute is the build() function)
    importlib.import_module("bm25mi.build").LIB = os.path.abspath(os.environ["VLIB"])
from bm25mi import synth  # noqa: E402
from bm25mi.index import GpuIndex  # noqa: E402

cfg = synth.CONFIGS[args.config]
if args.terms:
    cfg = dataclasses.replace(cfg, terms_per_query=args.terms)
lo, hi = (synth.shard_bounds(cfg.n_docs, 8, args.c5_rank) if args.config == "c5"
          else (0, cfg.n_docs))
ip, ix, dt = synth.make_index(cfg, lo, hi, threads=16)
index = GpuIndex(ip, ix, dt, hi - lo, doc_offset=lo)
q = torch.from_numpy(synth.make_queries(cfg)).cuda()
Q, k = q.shape[0], cfg.k
d = torch.empty((Q, k), dtype=torch.int32, device="cuda")
s = torch.empty((Q, k), device="cuda")
st = torch.cuda.current_stream()
for _ in range(2):
    index.search_device(q, k, d, s, st)
torch.cuda.synchronize()
index.profile_enable(2)  # (score pass and whole search)
for _ in range(args.searches):
    index.search_device(q, k, d, s, st)
p = index.profile_read()
print(json.dumps({"config": args.config, "terms": cfg.terms_per_query,
                  "score_ms": p["score_ms"] / p["score_launches"],
                  "total_ms": p["total_ms"] / p["searches"],
                  "dispatch": sorted(index.last_dispatch()["kernels"])}), flush=True)
