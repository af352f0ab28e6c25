"""Sweep the launch-geometry knobs of the score pass (BM25_SAMPLE_P,
BM25_CLAIM_CH, BM25_CLAIM_M) on one resident index, one process.
Dev tool (not part of the product): python scripts/sweep.py [config]
Every setting's result is checked against the default setting's (bit-exact)."""
import itertools, json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
import torch
from bm25mi import synth
from bm25mi.index import GpuIndex
cfg = synth.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "c3"]
ip, ix, dt = synth.make_index(cfg, threads=16)
index = GpuIndex(ip, ix, dt, cfg.n_docs)
del ip, ix, dt
q = torch.from_numpy(synth.make_queries(cfg)).cuda()
Q, k = q.shape[0], cfg.k
d = torch.empty((Q, k), dtype=torch.int32, device="cuda"); s = torch.empty((Q, k), device="cuda")
st = torch.cuda.current_stream()
ref = None
for P, ch, m in itertools.product((4, 8, 16), (4, 8, 16), (2, 4, 8)):
    os.environ.update(BM25_SAMPLE_P=str(P), BM25_CLAIM_CH=str(ch), BM25_CLAIM_M=str(m))
    for _ in range(2):
        index.search_device(q, k, d, s, st)
    torch.cuda.synchronize()
    if ref is None:
        ref = (d.clone(), s.clone())
    same = bool(torch.equal(d, ref[0]) and torch.equal(s.view(torch.int32), ref[1].view(torch.int32)))
    index.profile_enable(True)
    for _ in range(5):
        index.search_device(q, k, d, s, st)
    p = index.profile_read()
    index.profile_enable(False)
    print(json.dumps({"P": P, "claim_ch": ch, "claim_m": m, "same": same,
                      "score_ms": round(p["score_ms"] / p["score_launches"], 4),
                      "total_ms": round(p["total_ms"] / p["searches"], 4)}), flush=True)
