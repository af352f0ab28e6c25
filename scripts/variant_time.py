"""Time the config-3 search with the libbm25mi of a variant package copy
(a directory holding bm25mi/ with its own libbm25mi.so, e.g. built with
-DBM25_KJ=4).  Dev tool (not part of the product):
python scripts/variant_time.py <variant-dir>   -> one JSON line (score/total ms, result hash)"""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
var = sys.argv[1]
sys.path[:0] = [os.path.join(REPO, var), os.path.join(REPO, "mojo-bm25_amd"), REPO]
import torch
from bm25mi import synth, _capi
from bm25mi.index import GpuIndex
cfg = synth.CONFIGS["c3"]
ip, ix, dt = synth.make_index(cfg, threads=16)
index = GpuIndex(ip, ix, dt, cfg.n_docs)
del ip, ix, dt
q = torch.from_numpy(synth.make_queries(cfg)).cuda()
Q, k = q.shape[0], cfg.k
d = torch.empty((Q, k), dtype=torch.int32, device="cuda"); s = torch.empty((Q, k), device="cuda")
st = torch.cuda.current_stream()
for _ in range(2):
    index.search_device(q, k, d, s, st)
torch.cuda.synchronize()
index.profile_enable(True)
for _ in range(10):
    index.search_device(q, k, d, s, st)
p = index.profile_read()
torch.cuda.synchronize()
h = int((d.to(torch.int64) * 1000003 + s.view(torch.int32).to(torch.int64)).sum().item())
print(json.dumps({"variant": var, "lib": _capi.LIB, "score_ms": round(p["score_ms"] / p["score_launches"], 4),
                  "total_ms": round(p["total_ms"] / p["searches"], 4), "hash": h}), flush=True)
