"""Dev probe: time rank 0's shard of the config-3 index for W = 1, 2, 4, 8 on
one GPU (the per-rank work of the N-GPU bench without the collective)."""
import json, os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
import torch
from bm25mi import synth
from bm25mi.index import GpuIndex
cfg = synth.CONFIGS["c3"]
q = torch.from_numpy(synth.make_queries(cfg)).cuda()
Q, k = q.shape[0], cfg.k
for W in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8"])]:
    lo, hi = synth.shard_bounds(cfg.n_docs, W, 0)
    ip, ix, dt = synth.make_index(cfg, lo, hi, threads=16)
    index = GpuIndex(ip, ix, dt, hi - lo, doc_offset=lo)
    d = torch.empty((Q, k), dtype=torch.int32, device="cuda"); s = torch.empty((Q, k), device="cuda")
    st = torch.cuda.current_stream()
    from bm25mi.dist import sharded_search

    class Ex:  # all-gather stand-in: every rank's sample = this shard's
        world = W

        def __call__(self, keys):
            return keys.unsqueeze(0).expand(W, -1, -1).contiguous()

    def one():
        if W == 1:
            index.search_device(q, k, d, s, st)
        else:
            sharded_search(index, q, k, hi - lo, d, s, None, st, exchange=Ex())

    for _ in range(3):
        one()
    torch.cuda.synchronize()
    index.profile_enable(True)
    t0 = time.perf_counter()
    n = 10
    for _ in range(n):
        one()
    torch.cuda.synchronize()
    dt_ms = (time.perf_counter() - t0) * 1e3 / n
    p = index.profile_read()
    fb = index.search_stats()["fallback_queries"]
    print(json.dumps({"W": W, "shard_docs": hi - lo, "ms_per_batch": round(dt_ms, 3),
                      "score_ms": round(p["score_ms"] / p["score_launches"], 3),
                      "qps_if_all_ranks_equal": round(Q / dt_ms * 1e3, 1),
                      "fallback_queries": fb}), flush=True)
    index.close()
    del ip, ix, dt
