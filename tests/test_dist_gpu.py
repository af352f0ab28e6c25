"""The N>1 bench path through REAL process groups on one GPU: 2 and 3 ranks
(``gloo``, since RCCL wants one GPU per rank) each own a doc shard on
cuda:0 and run exactly what bench.py runs for N > 1 — bm25mi.dist.
sharded_search: the HIP sample pass, a real all-gather of the sample keys,
the global threshold + REST pass, a real all-gather of the [Q, k] lists and
the HIP merge.  Rank 0's result must equal the single-index oracle bit for
bit.  The process group is initialised before any GPU call in each rank."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


CASES = {
    # (n_docs, n_terms, nnz, n_queries, terms_per_query, k)
    "synth": ("t", 1_000_000, 8000, 8_000_000, 64, 8, 100),
    # shards smaller than k: lists padded, then merged
    "small": ("s", 5_000, 300, 40_000, 16, 6, 3000),
}


def _worker(rank, world, port, case, out, parts=1, world_bounds=False):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bm25mi import synth
        from bm25mi.dist import gpu_merge, sharded_search, shard_bounds
        from bm25mi.index import GpuIndex
        cfg = synth.Config(*CASES[case])
        bounds = synth.shard_bounds if case == "synth" else shard_bounds
        lo, hi = bounds(cfg.n_docs, world, rank)
        sdm = max(b - a for a, b in (bounds(cfg.n_docs, world, r) for r in range(world)))
        ip, ix, dt = synth.make_index(cfg, lo, hi)
        index = GpuIndex(ip, ix, dt, hi - lo, device=0, doc_offset=lo)
        q = synth.make_queries(cfg)
        q[2, 3:] = -1
        dq = torch.from_numpy(q).cuda()
        d_docs = torch.empty((len(q), cfg.k), dtype=torch.int32, device="cuda")
        d_scores = torch.empty((len(q), cfg.k), dtype=torch.float32, device="cuda")
        stream = torch.cuda.Stream()   # a non-current stream: the body must order on it
        merge = gpu_merge(0, stream) if os.environ.get("BM25_TEST_MERGE") == "sort" else None
        if world_bounds:  # the one-collective protocol: the world's tile bounds on every rank
            from bm25mi.dist import setup_world_bounds
            assert setup_world_bounds(index)
        docs, scores = sharded_search(index, dq, cfg.k, sdm, d_docs, d_scores, merge, stream,
                                      parts=parts)
        if parts > 1:  # the parts ran on forks of the index, each on its own stream
            assert len(index.__dict__["_bm25_forks"]) == parts - 1
        torch.cuda.synchronize()
        if rank == 0:
            np.savez(out, docs=docs.cpu().numpy(), scores=scores.cpu().numpy())
        index.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", ["synth", "small"])
def test_sharded_search_real_process_group(gpu, tmp_path, world, case):
    _run_case(tmp_path, world, case, 1)


@pytest.mark.parametrize("world,case,parts", [(2, "synth", 2), (3, "small", 3), (2, "synth", 4)])
def test_sharded_search_parts_real_process_group(gpu, tmp_path, world, case, parts):
    """sharded_search(parts=P): the batch pipelined as P row ranges over forks
    of each rank's shard (bm25_index_fork), each part on its own stream with
    its own all-gathers — bit-exact like the unsplit search."""
    _run_case(tmp_path, world, case, parts)


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("case", ["synth", "small"])
def test_world_bounds_one_collective_real_process_group(gpu, tmp_path, world, case):
    """The one-collective protocol (setup_world_bounds once, then per batch
    bm25_search_shard_device + one all-gather of the lists + the W-way
    merge) through real gloo groups: bit-exact vs the single-index oracle,
    including shards smaller than k (padding)."""
    _run_case(tmp_path, world, case, 1, True)


def _run_case(tmp_path, world, case, parts, world_bounds=False):
    from bm25mi import synth
    from oracle import oracle
    cfg = synth.Config(*CASES[case])
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(world, _free_port(), case, out, parts, world_bounds), nprocs=world,
             join=True)
    got = np.load(out)
    q = synth.make_queries(cfg)
    q[2, 3:] = -1
    ref = oracle.search_c(cfg.n_docs, *synth.make_index(cfg), q, cfg.k)
    assert np.array_equal(got["docs"], ref[0])
    assert np.array_equal(got["scores"].view(np.uint32), ref[1].view(np.uint32))
