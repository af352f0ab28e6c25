"""The N>1 path on the CPU: world_size-2 ``gloo`` process groups run the
doc-sharded protocol of bench.py / bm25mi.dist (each rank searches its shard,
all-gather of the [Q, k] lists, merge by (score desc, doc asc)) and must
reproduce the single-index top-k bit for bit.  The per-shard search and the
merge are the oracle's here (no GPU); the GPU merge kernel is covered by
tests/test_gpu_parity.py::test_sharded_merge_equals_single_index."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _merge_cpu(g_docs: torch.Tensor, g_scores: torch.Tensor):
    """Reference merge: top-k of the W*k candidates by (score desc, doc asc)."""
    W, Q, k = g_docs.shape
    d = g_docs.permute(1, 0, 2).reshape(Q, W * k).numpy()
    s = g_scores.permute(1, 0, 2).reshape(Q, W * k).numpy()
    out_d = np.zeros((Q, k), np.int32)
    out_s = np.zeros((Q, k), np.float32)
    for q in range(Q):
        order = np.lexsort((d[q], -s[q].astype(np.float64)))[:k]
        out_d[q], out_s[q] = d[q][order], s[q][order]
    return torch.from_numpy(out_d), torch.from_numpy(out_s)


def _worker(rank, world, port, cfg_args, k, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bm25mi import synth
        from bm25mi.dist import sharded_topk
        from oracle import oracle
        cfg = synth.Config(*cfg_args)
        lo, hi = synth.shard_bounds(cfg.n_docs, world, rank)
        ip, ix, dt = synth.make_index(cfg, lo, hi)
        q = synth.make_queries(cfg)
        d, s = oracle.search_c(hi - lo, ip, ix, dt, q, k)   # this shard's top-k
        d = d + lo                                          # global doc ids
        gd, gs = sharded_topk(torch.from_numpy(d), torch.from_numpy(s), _merge_cpu)
        if rank == 0:
            np.savez(result_path, docs=gd.numpy(), scores=gs.numpy())
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_sharded_search_equals_single_index(tmp_path, world):
    from bm25mi import synth
    from oracle import oracle
    args = ("t", 120_000, 900, 500_000, 24, 6, 20)
    cfg = synth.Config(*args)
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(world, _free_port(), args, cfg.k, out), nprocs=world, join=True)
    got = np.load(out)
    ref = oracle.search_c(cfg.n_docs, *synth.make_index(cfg), synth.make_queries(cfg), cfg.k)
    assert np.array_equal(got["docs"], ref[0])
    assert np.array_equal(got["scores"].view(np.uint32), ref[1].view(np.uint32))


def test_shard_bounds_tile_aligned_cover():
    from bm25mi.dist import shard_bounds
    for n in (1, 2047, 10_000_000, 12_345_679):
        for w in (1, 2, 3, 8):
            b = [shard_bounds(n, w, r) for r in range(w)]
            assert b[0][0] == 0 and b[-1][1] == n
            assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))
            assert all(x[0] % 2048 == 0 for x in b if x[1] > x[0])
    with pytest.raises(ValueError):
        shard_bounds(10, 2, 2)


def test_single_rank_is_identity():
    from bm25mi.dist import sharded_topk
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        d = torch.arange(6, dtype=torch.int32).reshape(2, 3)
        s = torch.ones((2, 3))
        gd, gs = sharded_topk(d, s, _merge_cpu)
        assert gd is d and gs is s
    finally:
        dist.destroy_process_group()
