"""Dev probe: the per-rank work of the N-GPU config-3 bench on ONE GPU, for
W = 1, 2, 4, 8, with every rank's real data in place of the collectives.

For each W, all W shards of the config-3 collection are built on the one GPU.
Each shard runs its SAMPLE half once; the W sample blocks are stacked as the
key all-gather would deliver them, every shard runs its finish half against
that stack, and the W lists are packed [W, 2, Q, k] as the list all-gather
would deliver them.  The timed loop is then exactly one rank's batch: SAMPLE
(its own slot of the stack rewritten, as the gather would), finish (theta over
the WHOLE real sample, REST, list into its own slot of the packed buffer) and
the W-way merge of the packed lists -- everything but the two collectives.  It
is timed for every rank; the bench's step is the max over ranks.

The two all-gathers are modelled, not measured (no multi-GPU box here):
  t(bytes per rank) = ALPHA + bytes * (W - 1) / (LINKS_USED * LINK_GBS)
with RCCL's direct all-gather over the point-to-point xGMI mesh: each rank's
block goes to its W - 1 peers over W - 1 distinct links in parallel.  The
constants are stated in the output line.

  python scripts/shard_probe.py [W ...]     (env VLIB: a variant library;
                                             PROBE_Q: batch size; PROBE_RANKS, PROBE_ITERS)
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
import torch  # noqa: E402

if os.environ.get("VLIB"):  # a variant build of libbm25mi (dev: scripts/build_variant.sh)
    import importlib
    importlib.import_module("bm25mi.build").LIB = os.path.abspath(os.environ["VLIB"])
from bm25mi import synth  # noqa: E402
from bm25mi.index import GpuIndex, merge_sorted_device  # noqa: E402

ALPHA_US = 10.0       # per-collective latency (RCCL launch + xGMI handshake)
LINK_GBS = 64.0       # one xGMI link, one direction, achieved by a copy engine/kernel


def model_gather_us(bytes_per_rank: int, W: int) -> float:
    if W == 1:
        return 0.0
    # W - 1 peers over W - 1 links in parallel: one block per link
    return ALPHA_US + bytes_per_rank / (LINK_GBS * 1e3)


def main():
    cfg = synth.CONFIGS["c3"]
    nq = int(os.environ.get("PROBE_Q", "0")) or None  # batch size (default: the config's 1024)
    q = torch.from_numpy(synth.make_queries(cfg, n_queries=nq)).cuda()
    Q, k = q.shape[0], cfg.k
    dev = q.device.index
    st = torch.cuda.current_stream()
    n = int(os.environ.get("PROBE_ITERS", "10"))
    ranks_env = os.environ.get("PROBE_RANKS")
    w1_ms = None
    for W in [int(x) for x in (sys.argv[1:] or ["1", "2", "4", "8"])]:
        bounds = [synth.shard_bounds(cfg.n_docs, W, r) for r in range(W)]
        smax = max(hi - lo for lo, hi in bounds)
        shards = []
        for lo, hi in bounds:
            ip, ix, dt = synth.make_index(cfg, lo, hi, threads=16)
            shards.append(GpuIndex(ip, ix, dt, hi - lo, doc_offset=lo))
            del ip, ix, dt
        S = shards[0].sample_width(k, W, smax)
        out_d = torch.empty((Q, k), dtype=torch.int32, device="cuda")
        out_s = torch.empty((Q, k), dtype=torch.float32, device="cuda")
        if W == 1:
            def one(r):
                shards[0].search_device(q, k, out_d, out_s, st)
        else:
            keys = torch.empty((W, Q, S), dtype=torch.int64, device="cuda")
            for r, ix_ in enumerate(shards):
                ix_.search_sample_device(q, k, W, smax, keys[r], st)
            g = torch.empty((W, 2, Q, k), dtype=torch.int32, device="cuda")
            for r, ix_ in enumerate(shards):
                ix_.search_finish_device(q, k, W, smax, keys, g[r, 0], g[r, 1].view(torch.float32), st)
            torch.cuda.synchronize()

            def one(r):
                ix_ = shards[r]
                ix_.search_sample_device(q, k, W, smax, keys[r], st)
                ix_.search_finish_device(q, k, W, smax, keys, g[r, 0], g[r, 1].view(torch.float32), st)
                merge_sorted_device(dev, g, g[:, 1].view(torch.float32), W, Q, k, 2 * Q * k,
                                    out_d, out_s, st)
        ranks = range(W) if not ranks_env else [int(x) for x in ranks_env.split(",") if int(x) < W]
        per_rank = []
        for r in ranks:
            for _ in range(3):
                one(r)
            torch.cuda.synchronize()
            shards[r].profile_enable(True)
            t0 = time.perf_counter()
            for _ in range(n):
                one(r)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) * 1e3 / n
            p = shards[r].profile_read()
            shards[r].profile_enable(False)
            per_rank.append({"rank": r, "ms": round(ms, 4),
                             "score_ms": round(p["score_ms"] / max(p["score_launches"], 1), 4),
                             "fallback_queries": shards[r].search_stats()["fallback_queries"]})
        worst = max(x["ms"] for x in per_rank)
        keys_b = Q * S * 8
        list_b = Q * k * 8
        coll_us = model_gather_us(keys_b, W) + model_gather_us(list_b, W)
        proj = worst + coll_us * 1e-3
        if W == 1:
            w1_ms = worst
        line = {"W": W, "shard_docs_max": smax, "sample_width": S, "per_rank": per_rank,
                "max_rank_ms": round(worst, 4),
                "model": {"alpha_us": ALPHA_US, "link_GBps": LINK_GBS,
                          "keys_bytes_per_rank": keys_b, "list_bytes_per_rank": list_b,
                          "collectives_us": round(coll_us, 1)},
                "projected_ms": round(proj, 4),
                "projected_qps": round(Q / proj * 1e3, 1)}
        if w1_ms is not None:
            line["speedup_vs_W1"] = round(w1_ms / proj, 3)
        print(json.dumps(line), flush=True)
        for s_ in shards:
            s_.close()
        del shards
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
