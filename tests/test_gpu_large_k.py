"""GPU parity of the large-k path (k > kMaxK = 4096, up to n_docs).

The reference serves any k <= N: ``_topk`` is ``argpartition(doc_scores,
-k)`` + ``argsort`` of the k survivors (bm25_native.py:204-214, output rows
sized [Q, k] at :147-148).  Above the sampled-threshold pipeline's limit the
engine takes the dense-score radix selection of csrc/bm25mi_large.hip; these
tests hold it BIT-exact (doc ids and score bits) to the canonical C oracle at
k in {4097, 10000, N} on indices of >= 100k documents, with tied scores,
zero-fill rows (fewer than k touched documents), padding rows and signed
values — through every entry point: BM25v.search, the device search, the
one-process sharded handle, the multi-process protocol (bm25mi.dist) and
the merges."""
import numpy as np
import pytest

from oracle import oracle
from test_gpu_parity import _doc_slice, _exact, _idx, _rand_index

pytestmark = pytest.mark.gpu

N_DOCS = 120_001  # a partial last tile


def _case(seed, signed=False, coarse=True, V=600, dfmax=20_000):
    rng = np.random.default_rng(seed)
    ip, ix, dt = _rand_index(rng, N_DOCS, V, dfmax, signed=signed, coarse=coarse)
    q = rng.integers(-1, V, size=(10, 8)).astype(np.int32)
    q[0, :] = -1                      # all padding: every doc scores 0
    q[1, :] = 5                       # one term eight times
    q[2, 1:] = -1                     # one term
    q[3, :] = np.arange(V - 8, V)     # the last terms
    # a rare row: terms with few postings (far fewer than k touched docs)
    df = np.diff(ip)
    rare = np.argsort(df)[:8].astype(np.int32)
    q[4, :] = rare
    return ip, ix, dt, q


@pytest.mark.parametrize("k", [4097, 10_000, N_DOCS])
def test_large_k_bm25v_drop_in(gpu, k):
    """BM25v.search (the drop-in) at k > 4096: bit-exact vs the oracle,
    including tied quarter-step scores, zero fill and an all-padding row."""
    import scipy.sparse as sp
    import bm25_native
    ip, ix, dt, q = _case(1)
    m = sp.csc_matrix((dt, ix, ip), shape=(N_DOCS, len(ip) - 1))
    model = bm25_native.BM25v()
    model.index(m, np.ones(N_DOCS, np.int32))
    docs, scores = model.search(q, top_k=k)
    assert docs.shape == (len(q), k) and docs.dtype == np.int32 and scores.dtype == np.float32
    _exact((docs, scores), oracle.search_c(N_DOCS, ip, ix, dt, q, k))
    assert "large_k" in model._gpu.last_dispatch()["kernels"]
    # the row of padding is all zero scores, doc ids ascending
    assert np.array_equal(docs[0], np.arange(k, dtype=np.int32))


def test_large_k_boundary_and_errors(gpu):
    """k = 4096 stays on the sampled pipeline, 4097 takes the large-k path;
    both bit-exact.  k > n_docs is numpy's argpartition error, as in the
    reference (bm25_native.py:205)."""
    ip, ix, dt, q = _case(2)
    index = _idx(ip, ix, dt, N_DOCS)
    for k, large in ((4096, False), (4097, True)):
        _exact(index.search(q, k), oracle.search_c(N_DOCS, ip, ix, dt, q, k))
        assert ("large_k" in index.last_dispatch()["kernels"]) == large
    with pytest.raises(ValueError, match=r"kth\(=-1\) out of bounds \(%d\)" % N_DOCS):
        index.search(q, N_DOCS + 1)


@pytest.mark.parametrize("segments", ["dense", "sparse"])
def test_large_k_signed_values(gpu, segments):
    """A signed index (negative sums rank below untouched documents)."""
    ip, ix, dt, q = _case(3, signed=True, coarse=False)
    index = _idx(ip, ix, dt, N_DOCS, segments=segments)
    for k in (5000, N_DOCS):
        _exact(index.search(q, k), oracle.search_c(N_DOCS, ip, ix, dt, q, k))


def test_large_k_device_entry_and_chunks(gpu):
    """bm25_search_device at k > 4096 on device buffers, a batch larger than
    one selection chunk (64 queries), twice in a row (same bits)."""
    import torch
    ip, ix, dt, q0 = _case(4, coarse=False)
    rng = np.random.default_rng(44)
    q = np.concatenate([q0, rng.integers(-1, len(ip) - 1, size=(54, 8)).astype(np.int32)])
    index = _idx(ip, ix, dt, N_DOCS)
    k = 6000
    ref = oracle.search_c(N_DOCS, ip, ix, dt, q, k, threads=8)
    dq = torch.from_numpy(q).cuda()
    dd = torch.empty((len(q), k), dtype=torch.int32, device="cuda")
    ds = torch.empty((len(q), k), dtype=torch.float32, device="cuda")
    for _ in range(2):
        index.search_device(dq, k, dd, ds, torch.cuda.current_stream())
        torch.cuda.synchronize()
        _exact((dd.cpu().numpy(), ds.cpu().numpy()), ref)


@pytest.mark.parametrize("k", [4097, 50_000, N_DOCS])
def test_large_k_sharded_index(gpu, k):
    """bm25_sharded_search at k > 4096: every shard's exact top-k (shards of
    40k docs pad their lists when k exceeds them), peer-copied and merged by
    the sort-based large merge — the single-index result."""
    from bm25mi.index import ShardedIndex
    ip, ix, dt, q = _case(5)
    sh = ShardedIndex(ip, ix, dt, N_DOCS, devices=[0, 0, 0])
    _exact(sh.search(q, k), oracle.search_c(N_DOCS, ip, ix, dt, q, k))
    sh.close()


@pytest.mark.parametrize("packed", [False, True])
def test_large_k_multi_process_protocol(gpu, packed):
    """bm25mi.dist.sharded_search at k > 4096 over W = 3 shards: no sample
    exchange (sample width 0), each shard's padded exact list, merged by the
    large merge from [W, Q, k] arrays or from the packed all-gather buffer."""
    import torch
    from bm25mi.index import GpuIndex, merge_sorted_device, merge_topk_device
    from bm25mi.dist import shard_bounds, sharded_search
    ip, ix, dt, q = _case(6)
    W, k = 3, 45_000
    ref = oracle.search_c(N_DOCS, ip, ix, dt, q, k)
    bounds = [shard_bounds(N_DOCS, W, r) for r in range(W)]
    sdm = max(hi - lo for lo, hi in bounds)
    shards = [GpuIndex(*_doc_slice(ip, ix, dt, lo, hi), hi - lo, doc_offset=lo)
              for lo, hi in bounds]
    assert all(sh.sample_width(k, W, sdm) == 0 for sh in shards)
    dq = torch.from_numpy(q).cuda()
    st = torch.cuda.current_stream()

    class Ex:
        world = W

        def __call__(self, keys):
            return keys.unsqueeze(0).expand(W, *keys.shape).contiguous()

    Q = len(q)
    if packed:  # rank w's docs at w * 2Qk, its scores Qk later (dist's packed layout)
        g = torch.empty((W, 2, Q, k), dtype=torch.int32, device="cuda")
        for r, sh in enumerate(shards):
            sharded_search(sh, dq, k, sdm, g[r, 0], g[r, 1].view(torch.float32), None, st,
                           exchange=Ex())
        md = torch.empty((Q, k), dtype=torch.int32, device="cuda")
        ms = torch.empty((Q, k), dtype=torch.float32, device="cuda")
        merge_sorted_device(0, g, g[:, 1].view(torch.float32), W, Q, k, 2 * Q * k, md, ms, st)
    else:
        ld = torch.empty((W, Q, k), dtype=torch.int32, device="cuda")
        ls = torch.empty((W, Q, k), dtype=torch.float32, device="cuda")
        for r, sh in enumerate(shards):
            sharded_search(sh, dq, k, sdm, ld[r], ls[r], None, st, exchange=Ex())
        md = torch.empty((Q, k), dtype=torch.int32, device="cuda")
        ms = torch.empty((Q, k), dtype=torch.float32, device="cuda")
        merge_topk_device(0, ld, ls, W, Q, k, md, ms, st)
    torch.cuda.synchronize()
    _exact((md.cpu().numpy(), ms.cpu().numpy()), ref)


def test_large_merge_random_lists(gpu):
    """bm25_merge_topk_device at k > 4096 on arbitrary lists with padding
    (doc -1, score bits ~0) and ties: the best k by (score desc, doc asc)."""
    import torch
    from bm25mi.index import merge_topk_device
    rng = np.random.default_rng(9)
    W, Q, k = 4, 5, 5000
    docs = rng.permutation(W * Q * k * 2)[:W * Q * k].reshape(W, Q, k).astype(np.int32)
    scores = (np.round(rng.uniform(0, 3, (W, Q, k)) * 8) / 8).astype(np.float32)
    docs[1, 2, 100:] = -1
    scores.view(np.uint32)[1, 2, 100:] = 0xFFFFFFFF
    d_docs, d_scores = torch.from_numpy(docs).cuda(), torch.from_numpy(scores).cuda()
    md = torch.empty((Q, k), dtype=torch.int32, device="cuda")
    ms = torch.empty((Q, k), dtype=torch.float32, device="cuda")
    merge_topk_device(0, d_docs, d_scores, W, Q, k, md, ms, torch.cuda.current_stream())
    torch.cuda.synchronize()
    for qi in range(Q):
        d = docs[:, qi].ravel()
        s = scores[:, qi].ravel()
        ok = d >= 0
        order = np.lexsort((d[ok], -s[ok].astype(np.float64)))[:k]
        assert np.array_equal(md.cpu().numpy()[qi], d[ok][order])
        assert np.array_equal(ms.cpu().numpy()[qi].view(np.uint32), s[ok][order].view(np.uint32))


@pytest.mark.parametrize("segments", ["dense", "sparse"])
def test_large_k_list_path(gpu, segments):
    """k > 4096 without dense score rows — a SAMPLE pass
    with the best key of every 256-doc slice of the sample tiles, theta = its
    k-th key, the REST pass listing every key >= theta, the k-th key of each
    list, compaction and the hand-written row sort.  Bit-exact vs the oracle;
    rows the lists cannot serve (all padding, rare terms: fewer than k keys)
    go to the dense rows on their own; large_lists = 0 gives the same bits."""
    from bm25mi import synth
    cfg = synth.Config("L", 3_000_000, 20_000, 40_000_000, 48, 8, 5000)
    ip, ix, dt = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    q[0, :] = -1                                   # all padding
    q[1, 1:] = q[1, 0]                             # one term eight times
    q[2, :] = np.argsort(np.diff(ip))[:8]          # rare terms: fewer than k docs
    index = _idx(ip, ix, dt, cfg.n_docs, segments=segments)
    # 1465 tiles: the sample of every other tile group holds 5888 slice keys —
    # the list path serves k <= 5888; k = 7000 takes the dense rows
    for k, lists in ((4097, True), (5500, True), (7000, False)):
        ref = oracle.search_c(cfg.n_docs, ip, ix, dt, q, k, threads=8)
        index.set_option("large_lists", 1)
        _exact(index.search(q, k), ref)
        d = index.last_dispatch()
        if lists:
            assert {"large_k", "flat_sample", "flat_rest"} <= d["kernels"], d
            assert d["sample_p"] >= 2, d
            # zero-fill rows (padding, rare terms) are completed in the lists too
            assert index.search_stats()["large_dense_queries"] == 0
        else:
            assert d["kernels"] == {"large_k"}, d
            assert index.search_stats()["large_dense_queries"] == -1
        index.set_option("large_lists", 0)
        _exact(index.search(q, k), ref)
        assert index.search_stats()["large_dense_queries"] == -1
    # counter [5] belongs to the last search: a k <= 4096 search resets it
    _exact(index.search(q, 100), oracle.search_c(cfg.n_docs, ip, ix, dt, q, 100, threads=8))
    assert index.search_stats()["large_dense_queries"] == 0
    index.close()


def test_large_k_list_path_overflow_falls_back(gpu):
    """A list longer than its capacity goes to the dense rows, for that query
    alone: one term covering every document with uniform scores lists ~15k
    keys above the sampled threshold at k = 4200 (capacity forced to 6000 by
    the list_cap option); the other queries (six terms of < 900 documents:
    fewer than 6000 positive documents, so their lists fit) stay on the lists.
    Bit-exact."""
    rng = np.random.default_rng(12)
    N, V = 3_000_000, 60
    indptr, idx, dat = [0], [], []
    for t in range(V):
        df = N if t == 0 else int(rng.integers(200, 900))
        idx.append(np.arange(N, dtype=np.int32) if t == 0 else
                   np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
        dat.append(rng.uniform(0.05, 3.0, df).astype(np.float32))
        indptr.append(indptr[-1] + df)
    ip, ix, dt = np.array(indptr, np.int64), np.concatenate(idx), np.concatenate(dat)
    q = rng.integers(1, V, size=(12, 6)).astype(np.int32)
    q[0, :] = -1
    q[0, 0] = 0  # every document
    index = _idx(ip, ix, dt, N)
    k = 4200
    ref = oracle.search_c(N, ip, ix, dt, q, k, threads=8)
    _exact(index.search(q, k), ref)
    assert index.search_stats()["large_dense_queries"] == 0
    index.set_option("list_cap", 6000)
    _exact(index.search(q, k), ref)
    assert 1 <= index.search_stats()["large_dense_queries"] < len(q)
    index.close()


def test_large_k_list_path_doc_shards(gpu):
    """the list path on doc shards (doc_offset != 0) — the global
    -> local threshold conversion of row_kth_kernel<0>, zero fill with local
    ids and the offset added by row_sort_write_kernel.  Two 3M-doc shards of
    a 6M-doc index at 4096 < k <= a shard's sample keys, an all-padding row
    (zero fill) and a rare-term row: each shard's list-path top-k (no dense
    rows), merged, is the single-index result bit for bit."""
    import torch
    from bm25mi import synth
    from bm25mi.dist import sharded_search
    from bm25mi.index import GpuIndex, merge_sorted_device
    cfg = synth.Config("LS", 6_000_000, 20_000, 80_000_000, 12, 8, 4500)
    ip, ix, dt = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    q[0, :] = -1                                   # all padding: zero fill
    q[1, :] = np.argsort(np.diff(ip))[:8]          # rare terms: fewer than k docs
    W, Q = 2, len(q)
    bounds = [synth.shard_bounds(cfg.n_docs, W, r) for r in range(W)]
    sdm = max(hi - lo for lo, hi in bounds)
    dq = torch.from_numpy(q).cuda()
    st = torch.cuda.current_stream()

    class Ex:
        world = W

        def __call__(self, keys):
            return keys.unsqueeze(0).expand(W, *keys.shape).contiguous()

    for k in (4097, 4500):
        ref = oracle.search_c(cfg.n_docs, ip, ix, dt, q, k, threads=8)
        g = torch.empty((W, 2, Q, k), dtype=torch.int32, device="cuda")
        for r, (lo, hi) in enumerate(bounds):
            sh = GpuIndex(*synth.make_index(cfg, lo, hi), hi - lo, doc_offset=lo)
            sharded_search(sh, dq, k, sdm, g[r, 0], g[r, 1].view(torch.float32), None, st,
                           exchange=Ex())
            d = sh.last_dispatch()
            assert {"large_k", "flat_sample", "flat_rest"} <= d["kernels"], d
            assert sh.search_stats()["large_dense_queries"] == 0
            torch.cuda.synchronize()
            sh.close()
        md = torch.empty((Q, k), dtype=torch.int32, device="cuda")
        ms = torch.empty((Q, k), dtype=torch.float32, device="cuda")
        merge_sorted_device(0, g, g[:, 1].view(torch.float32), W, Q, k, 2 * Q * k, md, ms, st)
        torch.cuda.synchronize()
        _exact((md.cpu().numpy(), ms.cpu().numpy()), ref)
