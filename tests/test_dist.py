"""The N>1 path on the CPU: world_size-2 and -3 ``gloo`` process groups run
the doc-sharded protocol of bench.py / bm25mi.dist and must reproduce the
single-index top-k bit for bit:
  * the list exchange (each rank's top-k, all-gather of the [Q, k] lists,
    merge by (score desc, doc asc));
  * the global-threshold protocol of bm25mi.dist.sharded_search — sample keys
    with GLOBAL doc ids, all-gathered by ``gather_keys``, theta = the k-th
    best, every shard lists its keys >= theta (padded to k), lists gathered
    and merged — on tie-heavy indices whose tie groups span shards.
The per-shard scoring is the oracle's here (no GPU); the HIP sample / finish
/ merge kernels run the same protocol in tests/test_dist_gpu.py."""
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


def _key(score: float, doc: int) -> int:
    """(score desc, doc asc) as one sortable u64, as bm25mi_internal.h."""
    u = int(np.float32(score).view(np.uint32))
    sk = (~u & 0xFFFFFFFF) if u & 0x80000000 else (u | 0x80000000)
    return (sk << 32) | (0xFFFFFFFF - doc)


def _protocol_worker(rank, world, port, args, k, tile, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bm25mi.dist import gather_keys, shard_bounds, sharded_topk
        from oracle import oracle
        N, V, Q, T, seed = args
        ip, ix, dt, q = _tie_index(N, V, Q, T, seed)
        lo, hi = shard_bounds(N, world, rank, align=tile)
        sdm = max(b - a for a, b in (shard_bounds(N, world, r, align=tile) for r in range(world)))
        keys = np.zeros((Q, (sdm + tile - 1) // tile), np.uint64)  # same width on every rank
        dense = []
        for i in range(Q):
            s = np.zeros(hi - lo, np.float32)
            for t in q[i]:
                if t < 0:
                    continue
                a, b = int(ip[t]), int(ip[t + 1])
                sel = (ix[a:b] >= lo) & (ix[a:b] < hi)
                np.add.at(s, ix[a:b][sel] - lo, dt[a:b][sel])
            dense.append(s)
            for j in range(0, hi - lo, tile):  # sample: every tile's best, GLOBAL id
                seg = s[j:j + tile]
                m = int(np.argmax(seg))
                keys[i, j // tile] = _key(seg[m], lo + j + m) if seg[m] > 0 else 0
        all_keys = gather_keys(torch.from_numpy(keys.view(np.int64))).numpy().view(np.uint64)
        docs = np.full((Q, k), -1, np.int32)
        scores = np.full((Q, k), np.nan, np.float32)
        for i in range(Q):
            ks = np.sort(all_keys[:, i, :].ravel())[::-1]
            theta = int(ks[k - 1])
            assert theta != 0, "test index too sparse for the sample"
            lst = [(_key(v, lo + d), lo + d, v) for d, v in enumerate(dense[i])
                   if _key(v, lo + d) >= theta]
            lst.sort(reverse=True)
            for j, (_, d, v) in enumerate(lst[:k]):
                docs[i, j], scores[i, j] = d, v
        gd, gs = sharded_topk(torch.from_numpy(docs), torch.from_numpy(scores), _merge_cpu)
        if rank == 0:
            np.savez(result_path, docs=gd.numpy(), scores=gs.numpy())
    finally:
        dist.destroy_process_group()


def _tie_index(N, V, Q, T, seed):
    """Values on a quarter grid (term 0 constant): most scores are tied."""
    rng = np.random.default_rng(seed)
    ip, ix, dt = [0], [], []
    for t in range(V):
        df = int(rng.integers(N // 10, N // 2))
        ix.append(np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
        dt.append(np.full(df, 1.0, np.float32) if t == 0 else
                  (rng.integers(1, 5, df) / 4).astype(np.float32))
        ip.append(ip[-1] + df)
    q = rng.integers(0, V, size=(Q, T)).astype(np.int32)
    q[0, :] = -1
    q[0, 0] = 0
    return np.array(ip, np.int64), np.concatenate(ix), np.concatenate(dt), q


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_global_theta_protocol_ties(tmp_path, world):
    from oracle import oracle
    args = (60000, 6, 5, 3, 7)
    k, tile = 150, 256
    out = str(tmp_path / "r.npz")
    mp.spawn(_protocol_worker, args=(world, _free_port(), args, k, tile, out), nprocs=world,
             join=True)
    got = np.load(out)
    ip, ix, dt, q = _tie_index(*args)
    ref = oracle.search_c(args[0], ip, ix, dt, q, k)
    assert np.array_equal(got["docs"], ref[0])
    assert np.array_equal(got["scores"].view(np.uint32), ref[1].view(np.uint32))


def _keys_worker(rank, world, port, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bm25mi.dist import gather_keys
        keys = torch.arange(12, dtype=torch.int64).reshape(3, 4) + 1000 * rank
        keys[0, 0] = -1 - rank  # u64 keys with the top bit set travel as negative int64
        g = gather_keys(keys)
        if rank == 0:
            np.save(result_path, g.numpy())
    finally:
        dist.destroy_process_group()


def test_gloo_gather_keys_rank_major(tmp_path):
    out = str(tmp_path / "k.npy")
    mp.spawn(_keys_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    g = np.load(out)
    assert g.shape == (2, 3, 4)
    for r in range(2):
        want = np.arange(12).reshape(3, 4) + 1000 * r
        want[0, 0] = -1 - r
        assert np.array_equal(g[r], want)


class _FakeShard:
    """The host-side surface of a GpuIndex that sharded_search consults
    before it launches anything: the shard's documents and its sample width."""

    def __init__(self, n_docs, width):
        self.n_docs = n_docs
        self.width = width

    def sample_width(self, k, world, shard_docs_max):
        return self.width


def _checks_worker(rank, world, port, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {}
    try:
        from bm25mi.dist import _global_docs, sharded_search
        q = torch.zeros((2, 3), dtype=torch.int32)
        d = torch.zeros((2, 1), dtype=torch.int32)
        s = torch.zeros((2, 1), dtype=torch.float32)
        # k beyond the summed shard documents: numpy's argpartition error
        ix = _FakeShard(1000 + rank, 8)
        try:
            sharded_search(ix, q, 2002, 1001, d, s)
        except ValueError as e:
            out["k_err"] = str(e)
        # the count is cached per process group: a sub-group of rank 0 alone
        sub = dist.new_group([0])
        if rank == 0:
            out["sub_docs"] = _global_docs(ix, q.device, sub)
        out["world_docs"] = _global_docs(ix, q.device)
        # ranks whose handles sample different widths: every rank raises
        try:
            sharded_search(_FakeShard(1000, 8 + rank), q, 10, 1001, d, s)
        except ValueError as e:
            out["width_err"] = str(e)
        if rank == 0:
            np.save(result_path, np.array([out], dtype=object), allow_pickle=True)
        else:
            assert "width_err" in out and "k_err" in out, out
    finally:
        dist.destroy_process_group()


def test_gloo_sharded_search_checks(tmp_path):
    """sharded_search's whole-collection k check and its lazily
    all-reduced document count (cached per process group), and the sample
    width agreement across ranks (one all-reduce per group and k)."""
    out = str(tmp_path / "c.npy")
    mp.spawn(_checks_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out, allow_pickle=True)[0]  # written by this test's own worker
    assert got["k_err"] == "kth(=-1) out of bounds (2001)"
    assert got["sub_docs"] == 1000 and got["world_docs"] == 2001
    assert "disagree on the sample width" in got["width_err"]


class _NumpyShard:
    """A doc shard that answers the two halves of the global-threshold
    protocol on the host (numpy), with GpuIndex's call signatures: every
    tile's best key as the sample (GLOBAL doc ids, zero-padded to the common
    width), theta = the world sample's k-th key, the shard's keys >= theta
    best first, padded with doc -1 / score bits ~0 as the HIP finish half
    writes them.  fork() shares the data, as bm25_index_fork shares the
    device arrays."""

    def __init__(self, ip, ix, dt, lo, hi, tile, width):
        self.ip, self.ix, self.dt, self.lo, self.hi = ip, ix, dt, lo, hi
        self.n_docs, self.tile, self.width = hi - lo, tile, width
        self.calls = []

    def fork(self):
        f = _NumpyShard(self.ip, self.ix, self.dt, self.lo, self.hi, self.tile, self.width)
        f.calls = self.calls
        return f

    def sample_width(self, k, world, shard_docs_max):
        return self.width

    def _dense(self, row):
        s = np.zeros(self.hi - self.lo, np.float32)
        for t in row:
            if t < 0:
                continue
            a, b = int(self.ip[t]), int(self.ip[t + 1])
            sel = (self.ix[a:b] >= self.lo) & (self.ix[a:b] < self.hi)
            np.add.at(s, self.ix[a:b][sel] - self.lo, self.dt[a:b][sel])
        return s

    def search_sample_device(self, q, k, world, sdm, keys, stream=None):
        self.calls.append(("sample", q.shape[0]))
        out = np.zeros(keys.shape, np.uint64)
        for i, row in enumerate(q.numpy()):
            s = self._dense(row)
            for j in range(0, s.size, self.tile):
                seg = s[j:j + self.tile]
                m = int(np.argmax(seg))
                out[i, j // self.tile] = _key(seg[m], self.lo + j + m) if seg[m] > 0 else 0
        keys.copy_(torch.from_numpy(out.view(np.int64)))

    def search_finish_device(self, q, k, world, sdm, all_keys, d_docs, d_scores, stream=None):
        self.calls.append(("finish", q.shape[0]))
        ak = all_keys.numpy().view(np.uint64)
        docs = np.full((q.shape[0], k), -1, np.int32)
        scores = np.full((q.shape[0], k), -1, np.int32).view(np.float32)  # bits ~0
        for i, row in enumerate(q.numpy()):
            theta = int(np.sort(ak[:, i, :].ravel())[::-1][k - 1])
            s = self._dense(row)
            u = s.view(np.uint32).astype(np.uint64)
            sk = np.where(u & 0x80000000, ~u & 0xFFFFFFFF, u | 0x80000000)
            docs_g = np.arange(self.lo, self.hi, dtype=np.uint64)
            keys_ = (sk << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - docs_g)
            sel = np.nonzero(keys_ >= np.uint64(theta))[0]
            lst = sorted(((int(keys_[d]), self.lo + int(d), s[d]) for d in sel), reverse=True)[:k]
            for j, (_, d, v) in enumerate(lst):
                docs[i, j], scores[i, j] = d, v
        d_docs.copy_(torch.from_numpy(docs))
        d_scores.copy_(torch.from_numpy(scores))


def _merge_packed_cpu(device, g, g_scores, W, Q, k, stride, out_d, out_s, stream=None):
    """bm25_merge_sorted_device on the host: [W][docs|scores][Q][k] -> [Q, k]."""
    d = g[:, 0].contiguous()
    s = g[:, 1].contiguous().view(torch.float32)
    s = torch.where(d < 0, torch.full_like(s, -np.inf), s)  # padding sorts last
    md, ms = _merge_cpu(d, s)
    out_d.copy_(md)
    out_s.copy_(ms)


def _parts_worker(rank, world, port, args, k, tile, parts, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bm25mi.index as bi
        from bm25mi.dist import shard_bounds, sharded_search
        bi.merge_sorted_device = _merge_packed_cpu  # the host stand-in of the HIP merge
        N, V, Q, T, seed = args
        ip, ix, dt, q = _tie_index(N, V, Q, T, seed)
        lo, hi = shard_bounds(N, world, rank, align=tile)
        sdm = max(b - a for a, b in (shard_bounds(N, world, r, align=tile) for r in range(world)))
        shard = _NumpyShard(ip, ix, dt, lo, hi, tile, (sdm + tile - 1) // tile)
        d = torch.zeros((Q, k), dtype=torch.int32)
        s = torch.zeros((Q, k), dtype=torch.float32)
        sharded_search(shard, torch.from_numpy(q), k, sdm, d, s, parts=parts, n_docs_total=N)
        if rank == 0:
            np.savez(result_path, docs=d.numpy(), scores=s.numpy(),
                     calls=np.array([c[1] for c in shard.calls]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,parts", [(2, 2), (3, 3)])
def test_gloo_search_parts_protocol(tmp_path, world, parts):
    """sharded_search(parts=P): the batch's rows as P parts on forks of the
    shard, each through both halves and both all-gathers, merged into its own
    rows — the single-index top-k bit for bit (tie-heavy index, tie groups
    across shards), every part's sample and finish issued once."""
    from oracle import oracle
    args = (12000, 6, 7, 3, 11)
    k, tile = 40, 256
    out = str(tmp_path / "r.npz")
    mp.spawn(_parts_worker, args=(world, _free_port(), args, k, tile, parts, out),
             nprocs=world, join=True)
    got = np.load(out)
    ip, ix, dt, q = _tie_index(*args)
    ref = oracle.search_c(args[0], ip, ix, dt, q, k)
    assert np.array_equal(got["docs"], ref[0])
    assert np.array_equal(got["scores"].view(np.uint32), ref[1].view(np.uint32))
    cuts = [args[2] * i // parts for i in range(parts + 1)]
    sizes = [b - a for a, b in zip(cuts[:-1], cuts[1:])]
    assert list(got["calls"]) == sizes + sizes  # every sample half, then every finish half


class _NumpyWorldShard(_NumpyShard):
    """_NumpyShard with the one-collective protocol's calls (GpuIndex's
    signatures): its tile bounds exported as f16 bits rounded down, the
    world's bounds kept as all-gathered, and bm25_search_shard_device's
    answer — the collection's threshold (the k-th best tile bound of the
    world, as a score: the weakest key at it) and the shard's keys at or
    above it (at most k, best first), zero fill with its smallest untouched
    documents when the world has fewer than k positive tiles, padding doc -1
    / score bits ~0."""

    def __init__(self, *a, n_terms=0):
        super().__init__(*a)
        self.n_terms = n_terms
        self.ntiles = (self.hi - self.lo + self.tile - 1) // self.tile

    def info(self):
        return {"tile_bounds": True, "n_tiles": self.ntiles}

    def bounds_stride(self):
        return (self.ntiles + 3) // 4 * 4

    def bounds_export(self, out, stride, stream=None):
        b = np.zeros((self.n_terms, stride), np.float32)
        for t in range(self.n_terms):
            a, e = int(self.ip[t]), int(self.ip[t + 1])
            sel = (self.ix[a:e] >= self.lo) & (self.ix[a:e] < self.hi)
            tiles = (self.ix[a:e][sel] - self.lo) // self.tile
            np.maximum.at(b[t], tiles, self.dt[a:e][sel])
        h = b.astype(np.float16)
        h = np.where(h.astype(np.float32) > b, np.nextafter(h, np.float16(-np.inf)), h)
        out.copy_(torch.from_numpy(h.view(np.int16)))

    def set_world_bounds(self, g, world, stride, tiles):
        self._bm25_world_bounds = g
        self.world_tiles = tiles

    def search_shard_device(self, q, k, d_docs, d_scores, stream=None):
        self.calls.append(("shard", q.shape[0]))
        wb = self._bm25_world_bounds.numpy().view(np.float16).astype(np.float32)  # [W, V, stride]
        docs = np.full((q.shape[0], k), -1, np.int32)
        scores = np.full((q.shape[0], k), -1, np.int32).view(np.float32)
        for i, row in enumerate(q.numpy()):
            terms = np.unique(row[row >= 0])
            lb = wb[:, terms, :].max(axis=1).ravel() if terms.size else np.zeros(1, np.float32)
            lb = np.sort(lb)[::-1]
            s = self._dense(row)
            if lb.size >= k and lb[k - 1] > 0:
                sel = np.nonzero(s >= lb[k - 1])[0]
                lst = sorted(((-float(s[d]), self.lo + int(d)) for d in sel))[:k]
            else:  # every positive doc, then the smallest untouched ones at score 0
                pos = sorted((-float(s[d]), self.lo + int(d)) for d in np.nonzero(s > 0)[0])
                zero = [(0.0, self.lo + int(d)) for d in np.nonzero(s == 0)[0][:k]]
                lst = (pos + zero)[:k]
            for j, (ms, d) in enumerate(lst):
                docs[i, j], scores[i, j] = d, -ms
        d_docs.copy_(torch.from_numpy(docs))
        d_scores.copy_(torch.from_numpy(scores))


def _world_worker(rank, world, port, args, k, tile, result_path):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bm25mi.index as bi
        from bm25mi.dist import setup_world_bounds, shard_bounds, sharded_search
        bi.merge_sorted_device = _merge_packed_cpu  # the host stand-in of the HIP merge
        N, V, Q, T, seed = args
        ip, ix, dt, q = _tie_index(N, V, Q, T, seed)
        lo, hi = shard_bounds(N, world, rank, align=tile)
        sdm = max(b - a for a, b in (shard_bounds(N, world, r, align=tile) for r in range(world)))
        shard = _NumpyWorldShard(ip, ix, dt, lo, hi, tile, (sdm + tile - 1) // tile, n_terms=V)
        assert setup_world_bounds(shard, device="cpu")
        wb = shard._bm25_world_bounds
        assert tuple(wb.shape) == (world, V, shard.bounds_stride())
        d = torch.zeros((Q, k), dtype=torch.int32)
        s = torch.zeros((Q, k), dtype=torch.float32)
        sharded_search(shard, torch.from_numpy(q), k, sdm, d, s, n_docs_total=N)
        if rank == 0:
            np.savez(result_path, docs=d.numpy(), scores=s.numpy(),
                     calls=np.array([c[0] for c in shard.calls]),
                     tiles=np.array([shard.world_tiles]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_world_bounds_one_collective(tmp_path, world):
    """The one-collective protocol's plumbing through real gloo groups:
    setup_world_bounds (the MAX/SUM agreement, the bounds all-gather), then per
    batch one shard search, one all-gather of the packed lists and the merge —
    the single-index top-k bit for bit on a tie-heavy index; no sample or
    finish half runs."""
    from oracle import oracle
    args = (12000, 6, 7, 3, 11)
    k, tile = 40, 256
    out = str(tmp_path / "w.npz")
    mp.spawn(_world_worker, args=(world, _free_port(), args, k, tile, out), nprocs=world,
             join=True)
    got = np.load(out)
    ip, ix, dt, q = _tie_index(*args)
    ref = oracle.search_c(args[0], ip, ix, dt, q, k)
    assert np.array_equal(got["docs"], ref[0])
    assert np.array_equal(got["scores"].view(np.uint32), ref[1].view(np.uint32))
    assert list(got["calls"]) == ["shard"]
    assert int(got["tiles"][0]) == (12000 + tile - 1) // tile or int(got["tiles"][0]) > 0
