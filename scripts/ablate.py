"""Time score_tiles on config 3 under the BM25_ABLATE mode of this process.
Dev tool (not part of the product): python scripts/ablate.py [config]"""
import json, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
import torch
from bm25mi import synth
from bm25mi.index import GpuIndex
cfg = synth.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
ip, ix, dt = synth.make_index(cfg, threads=16)
index = GpuIndex(ip, ix, dt, cfg.n_docs)
q = torch.from_numpy(synth.make_queries(cfg)).cuda()
Q, k = q.shape[0], cfg.k
d = torch.empty((Q, k), dtype=torch.int32, device="cuda"); s = torch.empty((Q, k), device="cuda")
st = torch.cuda.current_stream()
for _ in range(2):
    index.search_device(q, k, d, s, st)
torch.cuda.synchronize()
index.profile_enable(True)
for _ in range(5):
    index.search_device(q, k, d, s, st)
p = index.profile_read()
print(json.dumps({"mode": os.environ.get("BM25_ABLATE", "0"), "tile_shift": os.environ.get("BM25_TILE_SHIFT", "14"),
                  "score_ms": p["score_ms"] / p["score_launches"], "total_ms": p["total_ms"] / p["searches"]}), flush=True)
