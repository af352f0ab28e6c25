"""GPU parity: the HIP path (through the C-ABI) against the oracle and the
reference's golden vectors.  Bar: top-k doc ids and scores BIT-exact against
the canonical oracle (same fp32 adds in the same order, same (score desc,
doc asc) rule); against bm25_native's golden outputs, scores bit-exact and
ids exact wherever the reference score is untied (tie-aware, tolerance 0)."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle

pytestmark = pytest.mark.gpu


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def _idx(indptr, indices, data, n_docs, doc_offset=0, segments=None, options=None):
    """A GpuIndex; ``segments`` = "dense" / "sparse" forces the segment table
    (BM25_SEGMENTS, read at create), ``options`` are bm25_index_set_option's."""
    from bm25mi.index import GpuIndex
    old = os.environ.get("BM25_SEGMENTS")
    if segments is not None:
        os.environ["BM25_SEGMENTS"] = segments
    try:
        return GpuIndex(indptr, indices, data, n_docs, doc_offset=doc_offset, options=options)
    finally:
        if segments is not None:
            if old is None:
                os.environ.pop("BM25_SEGMENTS")
            else:
                os.environ["BM25_SEGMENTS"] = old


# what a search launches: SAMPLE + REST (+ the fallback stage's ALL launch,
# which reads its query count on the device), or one exact ALL pass
FLAT_SAMPLED = {"flat_sample", "flat_rest", "flat_all"}
WAVE_SAMPLED = {"wave_sample", "wave_rest", "wave_all"}
FLAT_BOUND = {"bound_keys", "flat_rest", "flat_all"}
WAVE_BOUND = {"bound_keys", "wave_rest", "wave_all"}


def _want_kernels(P, flat=True):
    """The score kernels a search of threshold geometry P launches."""
    if P == 1:
        return {"flat_all" if flat else "wave_all"}
    if P == 0:
        return FLAT_BOUND if flat else WAVE_BOUND
    return FLAT_SAMPLED if flat else WAVE_SAMPLED


def _progress(msg):
    """A line per stage of the long full-workload tests (run with -s, so a
    GPU run shows progress)."""
    import time
    print(f"  [{time.strftime('%H:%M:%S')}] {msg}", flush=True)


def _exact(a, b):
    assert a[0].shape == b[0].shape
    diff = np.nonzero((a[0] != b[0]) | (a[1].view(np.uint32) != b[1].view(np.uint32)))
    assert diff[0].size == 0, (f"{diff[0].size} mismatches, first at {diff[0][0]},{diff[1][0]}: "
                               f"gpu {a[0][diff[0][0]][:6]} {a[1][diff[0][0]][:6]} "
                               f"oracle {b[0][diff[0][0]][:6]} {b[1][diff[0][0]][:6]}")


def _rand_index(rng, N, V, dfmax, signed=False, coarse=False):
    indptr, idx, dat = [0], [], []
    for t in range(V):
        df = int(rng.integers(0, min(dfmax, N) + 1))
        idx.append(np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
        v = rng.uniform(-2.0 if signed else 0.05, 3.0, df)
        if coarse:
            v = np.round(v * 4) / 4
        dat.append(v.astype(np.float32))
        indptr.append(indptr[-1] + df)
    return (np.array(indptr, np.int64), np.concatenate(idx) if idx else np.zeros(0, np.int32),
            np.concatenate(dat) if dat else np.zeros(0, np.float32))


# ---------------------------------------------------------------- golden
@pytest.mark.parametrize("case", ["q1", "dup", "pad", "batch", "allk"])
def test_animal_golden_bm25v(gpu, case):
    import scipy.sparse as sp
    import bm25_native
    g = _load("animal.npz")
    n = int(g["n_docs"])
    m = sp.csc_matrix((g["data"], g["indices"], g["indptr"]), shape=(n, len(g["indptr"]) - 1))
    model = bm25_native.BM25v()
    model.index(m, np.ones(n, np.int32))
    q, k = g[f"{case}_queries"], int(g[f"{case}_k"])
    docs, scores = model.search(q, top_k=k)
    assert docs.dtype == np.int32 and scores.dtype == np.float32 and docs.shape == (len(q), k)
    bad = oracle.compare_topk(docs, scores, g[f"{case}_docs"], g[f"{case}_scores"],
                              tied=g[f"{case}_tied"], atol=0.0)
    assert not bad, bad
    _exact((docs, scores), oracle.search_c(n, g["indptr"], g["indices"], g["data"], q, k))


def test_animal_errors_match_reference(gpu):
    import scipy.sparse as sp
    import bm25_native
    g = _load("animal.npz")
    m = sp.csc_matrix((g["data"], g["indices"], g["indptr"]), shape=(4, 20))
    model = bm25_native.BM25v()
    model.index(m, np.ones(4, np.int32))
    with pytest.raises(ValueError) as e:
        model.search(np.array([[20]], np.int32), 1)
    assert f"ValueError: {e.value}" == str(g["err_token"])
    with pytest.raises(ValueError) as e:
        model.search(np.array([[0]], np.int32), 5)
    assert f"ValueError: {e.value}" == str(g["err_k"])
    d, s = model.search(np.zeros((0, 4), np.int32), 3)
    assert d.shape == (0, 0) and str(d.dtype) == str(g["empty_docs_dtype"])
    d, s = model.search(np.array([[1, 2]], np.int32), 0)
    assert d.shape == (1, 0) and s.shape == (1, 0)


def test_main_demo(gpu):
    import scipy.sparse as sp
    import bm25_native
    from gpu_bm25.common import gpu_execute_query
    g = _load("main_demo.npz")
    m = sp.csc_matrix(g["dense"])
    model = bm25_native.BM25v()
    model.index(m, np.array([2], np.int32))
    d, s = model.search(g["queries"], top_k=1)
    assert d.tolist() == [[1]] and s.tolist() == [[6.0]]
    idx, w = gpu_execute_query(g["dense"], np.array([0, 1], np.int32), None, None)
    assert idx.item() == 1 and w.item() == 6.0


@pytest.mark.parametrize("k", [1, 10, 100])
def test_synth_small_golden(gpu, k):
    g = _load("synth_small.npz")
    n = int(g["n_docs"])
    ix = _idx(g["indptr"], g["indices"], g["data"], n)
    docs, scores = ix.search(g["queries"], k)
    bad = oracle.compare_topk(docs, scores, g[f"docs_k{k}"], g[f"scores_k{k}"],
                              tied=g[f"tied_k{k}"], atol=0.0)
    assert not bad, bad[:4]
    _exact((docs, scores), oracle.search_c(n, g["indptr"], g["indices"], g["data"],
                                           g["queries"], k))


def test_dense_scores_bit_exact(gpu):
    g = _load("synth_small.npz")
    n = int(g["n_docs"])
    ix = _idx(g["indptr"], g["indices"], g["data"], n)
    for i, key in ((0, "dense0"), (8, "dense8")):
        d = ix.scores_dense(g["queries"][i])
        assert np.array_equal(d.view(np.uint32), g[key].view(np.uint32))


# ------------------------------------------------------- synthetic parity
@pytest.mark.parametrize("seed", [10, 11])
def test_random_ragged_index(gpu, seed):
    rng = np.random.default_rng(seed)
    N, V = 70_001, 700  # a partial last tile
    ip, ix, dt = _rand_index(rng, N, V, 6000)
    q = rng.integers(-1, V, size=(37, 9)).astype(np.int32)
    index = _idx(ip, ix, dt, N)
    for k in (1, 4, 5, 64, 300):
        _exact(index.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))
    assert index.last_dispatch()["term_lanes"] == 16  # T = 9: 16 term lanes, 4 tiles per item


def test_signed_and_tied_values(gpu):
    rng = np.random.default_rng(11)
    N, V = 40_000, 300
    ip, ix, dt = _rand_index(rng, N, V, 8000, signed=True, coarse=True)
    q = rng.integers(-2, V, size=(50, 6)).astype(np.int32)
    index = _idx(ip, ix, dt, N)
    for k in (3, 50, 1000):
        _exact(index.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))


def test_zero_fill_and_k_equals_n(gpu):
    rng = np.random.default_rng(3)
    N, V = 1000, 50
    ip, ix, dt = _rand_index(rng, N, V, 5)
    q = np.array([[1, 2, -1], [-1, -1, -1], [3, 3, 3], [49, 0, 7]], np.int32)
    index = _idx(ip, ix, dt, N)
    for k in (10, 200, N):
        _exact(index.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))


@pytest.mark.parametrize("T,lanes", [(1, 8), (12, 16), (16, 16), (17, 32), (32, 32), (45, 64),
                                     (64, 64)])
@pytest.mark.parametrize("segments", ["dense", "sparse"])
def test_flat_kernel_query_widths(gpu, T, lanes, segments):
    """Queries of 1..64 terms take the flat kernel with 8/16/32/64 term lanes
    per tile (64 / lanes tiles per item), on both segment tables: padding,
    a term repeated across the whole row, duplicates — bit-exact."""
    rng = np.random.default_rng(T)
    N, V = 120_000, 500
    ip, ix, dt = _rand_index(rng, N, V, 12_000)
    q = rng.integers(-1, V, size=(33, T)).astype(np.int32)
    q[0, :] = 7          # one term T times
    q[1, :] = -1         # all padding
    q[2, T // 2:] = -1
    index = _idx(ip, ix, dt, N, segments=segments)
    assert index.info()["sparse"] == (segments == "sparse")
    for k in (1, 25, 300):
        _exact(index.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))
        d = _check_dispatch(index, k, T=T)
        assert d["term_lanes"] == lanes, d
        assert 1 <= d["band_tiles"]["rest" if d["sample_p"] != 1 else "all"] <= 64 // lanes


@pytest.mark.parametrize("T", [0, 65, 80])
def test_wave_kernel_long_and_empty_queries(gpu, T):
    """Queries of 0 or more than 64 terms take score_wave_kernel (LDS float
    adds in query-term order) for SAMPLE, REST and ALL — bit-exact."""
    rng = np.random.default_rng(80 + T)
    N, V = 60_000, 400
    ip, ix, dt = _rand_index(rng, N, V, 6000)
    q = rng.integers(-1, V, size=(11, T)).astype(np.int32)
    if T:
        q[0, :] = 3
        q[1, :40] = -1
    index = _idx(ip, ix, dt, N)
    for k in (1, 30, 200):
        _exact(index.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))
        _check_dispatch(index, k, T=T, flat=False)
    index.set_option("sample_p", 1)  # the exact pass over every tile
    _exact(index.search(q, 30), oracle.search_c(N, ip, ix, dt, q, 30))
    assert index.last_dispatch()["kernels"] - {"bound_off", "rest_split", "bound_pool"} == {"wave_all"}
    index.set_option("list_cap", 4)  # every query through the fallback stage
    index.set_option("sample_p", 8)
    _exact(index.search(q, 30), oracle.search_c(N, ip, ix, dt, q, 30))
    if T:
        assert index.search_stats()["fallback_queries"] > 0


def test_tiny_and_empty_shapes(gpu):
    ip = np.array([0, 1, 1, 3], np.int32)
    ix = np.array([0, 0, 2], np.int32)
    dt = np.array([1.0, 0.5, 2.0], np.float32)
    index = _idx(ip, ix, dt, 3)
    q = np.array([[0, 1, 2]], np.int32)
    _exact(index.search(q, 3), oracle.search_c(3, ip, ix, dt, q, 3))
    d, s = index.search(np.zeros((2, 0), np.int32), 2)  # T = 0: all zero, smallest ids
    assert d.tolist() == [[0, 1], [0, 1]] and not s.any()
    one = _idx(np.array([0, 1], np.int32), np.array([0], np.int32), np.array([3.0], np.float32), 1)
    assert one.search(np.array([[0]], np.int32), 1)[0].tolist() == [[0]]


def test_rescore_path_clustered_tile(gpu):
    # every high score sits in tiles 0-2, so the exact path (no sampling) must
    # rescore them
    N, V = 200_000, 3
    ip = np.array([0, 5000, 5000 + N // 2, 5000 + N // 2 + 10], np.int64)
    ix = np.concatenate([np.arange(5000, dtype=np.int32),
                         np.arange(0, N, 2, dtype=np.int32),
                         np.arange(10, dtype=np.int32) * 1000]).astype(np.int32)
    rng = np.random.default_rng(8)
    dt = np.concatenate([rng.uniform(10, 20, 5000), rng.uniform(0, 1, N // 2),
                         rng.uniform(0, 30, 10)]).astype(np.float32)
    q = np.array([[0, 1, 2], [1, 0, -1], [2, 2, 1]], np.int32)
    for flat in (1, 0):
        index = _idx(ip, ix, dt, N, options={"sample_p": 1, "flat": flat})
        index.profile_enable(True)
        for k in (100, 2048):
            got = index.search(q, k)
            _exact(got, oracle.search_c(N, ip, ix, dt, q, k))
            assert index.profile_read()["rescored_tiles_last"] > 0
            assert (index.last_dispatch()["kernels"] - {"bound_off", "rest_split", "bound_pool"}
                    == {"flat_all" if flat else "wave_all"})


def test_search_device_torch(gpu):
    import torch
    g = _load("synth_small.npz")
    n = int(g["n_docs"])
    ix = _idx(g["indptr"], g["indices"], g["data"], n)
    dq = torch.from_numpy(g["queries"]).to("cuda:0")
    dd = torch.empty((dq.shape[0], 10), dtype=torch.int32, device="cuda:0")
    ds = torch.empty((dq.shape[0], 10), dtype=torch.float32, device="cuda:0")
    stream = torch.cuda.current_stream()
    ix.search_device(dq, 10, dd, ds, stream)
    torch.cuda.synchronize()
    _exact((dd.cpu().numpy(), ds.cpu().numpy()),
           oracle.search_c(n, g["indptr"], g["indices"], g["data"], g["queries"], 10))


def test_search_device_opt_in_validation(gpu):
    """bm25_max_token_device: the reference's max-token check
    (bm25_native.py:91-96) on a device batch; search_device(validate=True)
    raises its ValueError, the default treats the id as padding."""
    import torch
    g = _load("synth_small.npz")
    n = int(g["n_docs"])
    ix = _idx(g["indptr"], g["indices"], g["data"], n)
    q = g["queries"].copy()
    assert ix.max_token_device(torch.from_numpy(q).to("cuda:0")) == int(q.max(initial=0))
    assert ix.max_token_device(torch.full((3, 4), -1, dtype=torch.int32, device="cuda:0")) == 0
    q[1, 0] = ix.n_terms + 5
    dq = torch.from_numpy(q).to("cuda:0")
    dd = torch.empty((q.shape[0], 10), dtype=torch.int32, device="cuda:0")
    ds = torch.empty((q.shape[0], 10), dtype=torch.float32, device="cuda:0")
    with pytest.raises(ValueError, match=r"maximum token ID in the query \(%d\)" % (ix.n_terms + 5)):
        ix.search_device(dq, 10, dd, ds, validate=True)
    ix.search_device(dq, 10, dd, ds)  # unchecked: the id is padding
    torch.cuda.synchronize()
    q[1, 0] = -1
    _exact((dd.cpu().numpy(), ds.cpu().numpy()),
           oracle.search_c(n, g["indptr"], g["indices"], g["data"], q, 10))


def test_sharded_merge_equals_single_index(gpu):
    import torch
    from bm25mi import synth
    from bm25mi.index import GpuIndex, merge_topk_device
    cfg = synth.Config("t", 300_000, 5000, 2_000_000, 64, 8, 100)
    full = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    ref = oracle.search_c(cfg.n_docs, *full, q, cfg.k)
    W = 3
    dq = torch.from_numpy(q).cuda()
    outs_d = torch.empty((W, len(q), cfg.k), dtype=torch.int32, device="cuda")
    outs_s = torch.empty((W, len(q), cfg.k), dtype=torch.float32, device="cuda")
    shards = []
    for r in range(W):
        lo, hi = synth.shard_bounds(cfg.n_docs, W, r)
        ip, ix, dt = synth.make_index(cfg, lo, hi)
        sh = GpuIndex(ip, ix, dt, hi - lo, doc_offset=lo)
        shards.append(sh)
        sh.search_device(dq, cfg.k, outs_d[r], outs_s[r], torch.cuda.current_stream())
    md = torch.empty((len(q), cfg.k), dtype=torch.int32, device="cuda")
    ms = torch.empty((len(q), cfg.k), dtype=torch.float32, device="cuda")
    merge_topk_device(0, outs_d, outs_s, W, len(q), cfg.k, md, ms, torch.cuda.current_stream())
    torch.cuda.synchronize()
    _exact((md.cpu().numpy(), ms.cpu().numpy()), ref)


@pytest.mark.parametrize("W,k", [(2, 1), (3, 100), (8, 100), (8, 128), (5, 300)])
def test_merge_sorted_packed_lists(gpu, W, k):
    """bm25_merge_sorted_device on the packed [W][docs|scores][Q][k] buffer of
    the doc-sharded path: best-first lists (global doc ids, some padded with
    doc -1 / key 0, tied scores across ranks) merge to the (score desc, doc
    asc) top-k — the same bits as the sort-based bm25_merge_topk_device, and
    as a numpy merge.  W * k > 1024 takes the sort kernel with the stride."""
    import torch
    from bm25mi.index import merge_sorted_device, merge_topk_device
    rng = np.random.default_rng(W * 1000 + k)
    Q = 37
    docs = np.full((W, Q, k), -1, np.int32)
    scores = np.full((W, Q, k), np.uint32(0xFFFFFFFF).view(np.float32), np.float32)
    for w in range(W):
        for q in range(Q):
            n = int(rng.integers(0, k + 1)) if q % 5 else k
            d = rng.choice(np.arange(w, 200_000, W), size=n, replace=False).astype(np.int32)
            s = np.round(rng.uniform(0, 4, size=n) * 8).astype(np.float32) / 8  # ties
            o = np.lexsort((d, -s))
            docs[w, q, :n], scores[w, q, :n] = d[o], s[o]
    pk = np.stack([docs, scores.view(np.int32)], axis=1)  # [W, 2, Q, k]
    g = torch.from_numpy(np.ascontiguousarray(pk)).cuda()
    md = torch.empty((Q, k), dtype=torch.int32, device="cuda")
    ms = torch.empty((Q, k), dtype=torch.float32, device="cuda")
    merge_sorted_device(0, g, g[:, 1].view(torch.float32), W, Q, k, 2 * Q * k, md, ms)
    rd = torch.empty_like(md)
    rs = torch.empty_like(ms)
    merge_topk_device(0, torch.from_numpy(docs).cuda(), torch.from_numpy(scores).cuda(), W, Q, k,
                      rd, rs)
    torch.cuda.synchronize()
    _exact((md.cpu().numpy(), ms.cpu().numpy()), (rd.cpu().numpy(), rs.cpu().numpy()))
    for q in range(Q):
        d, s = docs[:, q].ravel(), scores[:, q].ravel()
        real = d >= 0
        o = np.lexsort((d[real], -s[real]))[:k]
        n = len(o)
        assert np.array_equal(md[q, :n].cpu().numpy(), d[real][o])
        assert (md[q, n:].cpu().numpy() == -1).all()


def test_config2_full_parity(gpu):
    from bm25mi import synth
    cfg = synth.CONFIGS["c2"]
    ip, ix, dt = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    index = _idx(ip, ix, dt, cfg.n_docs)
    _exact(index.search(q, cfg.k), oracle.search_c(cfg.n_docs, ip, ix, dt, q, cfg.k))


def test_config3_full_batch_parity(gpu):
    """The headline 10M-doc / 200k-vocab / 640M-posting index, k=100: all
    1024 queries of the bench batch checked bit-exactly against the C oracle
    (threaded over the host's cores), plus size-independent properties."""
    from bm25mi import synth
    cfg = synth.CONFIGS["c3"]
    ip, ix, dt = synth.make_index(cfg, threads=16)
    q = synth.make_queries(cfg)
    index = _idx(ip, ix, dt, cfg.n_docs)
    docs, scores = index.search(q, cfg.k)
    ref = oracle.search_c(cfg.n_docs, ip, ix, dt, q, cfg.k, threads=16)
    _exact((docs, scores), ref)
    # the threshold read the pooled bounds (1221 groups >= 8k); the per-tile
    # bounds give the same bits
    assert "bound_pool" in index.last_dispatch()["kernels"]
    index.set_option("bound_pool", 0)
    _exact(index.search(q, cfg.k), ref)
    assert "bound_pool" not in index.last_dispatch()["kernels"]
    index.set_option("bound_pool", 1)
    # whole batch: sorted, unique ids in range, ties ordered by id
    assert np.all(np.diff(scores, axis=1) <= 0)
    assert all(len(set(r)) == cfg.k for r in docs.tolist())
    assert docs.min() >= 0 and docs.max() < cfg.n_docs
    eq = np.diff(scores, axis=1) == 0
    assert np.all(np.diff(docs, axis=1)[eq] > 0)
    # the sampled threshold path handles every query: no fallback, few rescored tiles
    st = index.search_stats()
    assert st["fallback_queries"] == 0 and st["rescored_tiles"] < len(q)
    # idempotent: a second search returns the same bits
    d2, s2 = index.search(q, cfg.k)
    assert np.array_equal(d2, docs) and np.array_equal(s2.view(np.uint32), scores.view(np.uint32))


def _sample_p(ntiles, k, W=1, pmax=8):
    """The sampling stride sample_geom picks (bm25mi_kernels.hip): the first
    P = pmax, pmax / 2, ... 2 whose sample of m = 1, 2 or 4 keys per sample
    tile holds >= 2k keys; 1 (the exact pass) otherwise."""
    P = 64
    while P >= 2:
        if P <= pmax and ntiles >= 2 * P:
            G = 8 if ntiles >= 4 * 8 * P else 1
            nS = (ntiles // (G * P)) * G + min(ntiles % (G * P), G)
            if any(nS * m * W >= 2 * k for m in (1, 2, 4)):
                return P
        P //= 2
    return 1


def _geom_p(index, k, W=1, ntiles=None, opts=None, T=8, weak=False):
    """The threshold geometry search_geom picks (bm25mi_kernels.hip): 0 =
    tile-bound keys (a sampled geometry, the index keeps tile bounds,
    theta_bound on, queries of 1..16 terms, at most 30720 tiles, a collection
    of >= 16k tiles, and not turned off for the handle after overflowing
    searches — ``weak``, the dispatch's "bound_off" flag), else _sample_p's
    stride."""
    opts = opts or {}
    info = index.info()
    nt = info["n_tiles"] if ntiles is None else ntiles
    pmax = opts.get("sample_p", 8)
    P = _sample_p(nt, k, W, pmax)
    if (P > 1 and opts.get("theta_bound", 1) and info["tile_bounds"] and 1 <= T <= 16
            and nt <= 30720 and nt * W >= 16 * k and not weak):
        return 0
    return P


def _check_dispatch(index, k, W=1, ntiles=None, opts=None, T=8, flat=True):
    """The last search launched the kernels of the geometry it should have
    taken (with the tile-bound threshold off when the dispatch says the
    handle turned it off after overflowing searches); returns the report."""
    d = index.last_dispatch()
    weak = "bound_off" in d["kernels"]
    P = _geom_p(index, k, W, ntiles, opts, T=T, weak=weak)
    want = _want_kernels(P, flat)
    assert d["kernels"] - {"bound_off", "rest_split", "bound_pool"} == want and d["sample_p"] == P, (k, d, want, P)
    return d


# (options, segment table)
VARIANTS = [
    ({}, "dense"), ({"sample_p": 1}, "dense"), ({"sample_p": 2}, "dense"),
    ({"sample_p": 16}, "dense"), ({"list_cap": 8}, "dense"), ({"flat": 0}, "dense"),
    ({"flat": 0, "list_cap": 8}, "dense"), ({"flat": 0, "sample_p": 1}, "dense"),
    ({}, "sparse"), ({"sample_p": 1}, "sparse"), ({"list_cap": 8}, "sparse"),
    ({"flat": 0}, "sparse"), ({"flat_bw": 1}, "dense"), ({"flat_bw": 2}, "sparse"),
    ({"flat_bw": 4, "sample_p": 2}, "dense"), ({"flat_bw": 8, "list_cap": 40}, "sparse"),
    ({"claim_ch": 4, "claim_m": 1}, "dense"), ({"items_per_wave": 1000}, "dense"),
]


@pytest.mark.parametrize("T", [8, 16])
@pytest.mark.parametrize("opts,segments", VARIANTS)
def test_kernel_variants_bit_exact(gpu, opts, segments, T):
    """Every search configuration gives the oracle's bits, and the search
    reports that it ran the kernels the configuration selects
    (bm25_search_dispatch): sampling strides (1 = one exact pass over every
    tile), both score kernels, forced item widths, tiny candidate lists that
    send queries through the exact fallback stage, both segment tables.
    Options are set on the handle after it is built: they apply per search."""
    rng = np.random.default_rng(21)
    N, V = 400_000, 900
    ip, ix, dt = _rand_index(rng, N, V, 20_000)
    q = rng.integers(-1, V, size=(70, T)).astype(np.int32)
    q[3, :] = -1
    q[4, 2:] = q[4, 1]
    index = _idx(ip, ix, dt, N, segments=segments)
    _exact(index.search(q, 7), oracle.search_c(N, ip, ix, dt, q, 7))  # defaults first
    _check_dispatch(index, 7, T=T)
    assert index.info()["tile_bounds"] == (segments == "dense")
    for name, val in opts.items():
        index.set_option(name, val)
        assert index.get_option(name) == val
    flat = opts.get("flat", 1)
    ntiles = index.info()["n_tiles"]
    fallback = 0
    for k in (1, 7, 100):
        _exact(index.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))
        d = _check_dispatch(index, k, 1, ntiles, opts, T=T, flat=flat)
        P = d["sample_p"]
        if flat:
            assert d["term_lanes"] == (8 if T == 8 else 16)
            phase = "rest" if P != 1 else "all"
            if "flat_bw" in opts:
                assert d["band_tiles"][phase] == min(opts["flat_bw"], 64 // d["term_lanes"])
        fallback += index.search_stats()["fallback_queries"]
    if "list_cap" in opts:
        assert fallback > 0


def test_options_rejected(gpu):
    ip = np.array([0, 1], np.int32)
    index = _idx(ip, np.array([0], np.int32), np.array([1.0], np.float32), 1)
    for name, val in (("flat", 2), ("flat_bw", 3), ("sample_p", 3), ("claim_m", 9),
                      ("count_skips", 2), ("nope", 1)):
        with pytest.raises(ValueError):
            index.set_option(name, val)


def test_sharded_index_multi_shard_one_process(gpu):
    """bm25_sharded_*: the same GPU listed three times = three shards on their
    own streams, peer-copied lists, HIP merge; bit-exact vs the oracle."""
    from bm25mi import synth
    from bm25mi.index import ShardedIndex
    cfg = synth.Config("t", 400_000, 6000, 3_000_000, 96, 8, 100)
    ip, ix, dt = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    q[5, 3:] = -1
    sh = ShardedIndex(ip, ix, dt, cfg.n_docs, devices=[0, 0, 0])
    b = sh.shards()
    assert len(b) == 3 and b[0][0] == 0 and b[-1][1] == cfg.n_docs
    for k in (1, 17, 100):
        _exact(sh.search(q, k), oracle.search_c(cfg.n_docs, ip, ix, dt, q, k))
    with pytest.raises(ValueError, match="maximum token ID"):
        sh.search(np.array([[cfg.n_terms]], np.int32), 3)
    sh.close()


def _bm25_golden_check(name, n_top):
    import bm25
    g = _load(name)
    corpus = [d.lower().split() for d in g["docs"].tolist()]
    m = bm25.BM25()
    m.fit(corpus)
    # the GPU-built float64 matrix is the reference's, bit for bit
    assert m.vocabulary == g["vocabulary"].tolist() if "vocabulary" in g else True
    assert m.bm25_matrix.dtype == np.float64
    if "bm25_matrix" in g:
        assert np.array_equal(m.bm25_matrix, g["bm25_matrix"])
    for i, q in enumerate(g["queries"].tolist()):
        toks = q.lower().split()
        s = m.get_scores(toks)
        ref = g[f"scores_{i}"]
        assert s.dtype == np.float64 and s.shape == (len(corpus),)
        assert np.array_equal(s.view(np.uint64), ref.view(np.uint64)), q  # bit-exact
        top = m.get_top_n(toks, corpus, n=n_top)
        rs, rd = g[f"top_scores_{i}"], g[f"top_docs_{i}"]
        got_s = np.array([t[0] for t in top])
        assert np.array_equal(got_s, rs), q
        # documents: exact wherever the reference's score is untied in the
        # whole score vector (its order among ties is numpy's choice)
        vals, cnt = np.unique(ref, return_counts=True)
        rep = dict(zip(vals.tolist(), cnt.tolist()))
        for j, (sc, doc) in enumerate(top):
            if rep[float(rs[j])] == 1:
                assert doc == corpus[rd[j]], (q, j)
            else:
                assert float(ref[corpus.index(doc)]) == float(sc)
    return m, g


def test_bm25_dense_model_golden(gpu):
    """bm25.BM25 (drop-in of bm25.py:6-178) against the reference's own
    outputs: the GPU-built float64 matrix, get_scores bit for bit (the
    device's float64 sums in numpy's order), get_top_n's scores bit for bit
    and its documents exact wherever the reference's score is untied."""
    _bm25_golden_check("bm25_dense.npz", 5)


def test_bm25_near_ties_rank_in_float64(gpu):
    """a corpus + queries whose float64 ranking differs from
    the same sums' fp32 ranking (golden bm25_near_ties.npz, from the
    reference): get_scores bit-exact, get_top_n(n=20) documents exact where
    untied — so ranking is float64 end to end."""
    m, g = _bm25_golden_check("bm25_near_ties.npz", 20)
    assert len(g["fp32_differs"]) > 0


def test_bm25_top_n_whole_corpus_and_one_doc(gpu):
    """get_top_n for n up to the whole corpus (the reference ranks every
    document, bm25.py:172-178): the device's float64 ranking equals the
    oracle's (score desc, doc asc) order of the oracle's float64 sums; and a
    one-document corpus (numpy's pairwise row sum) bit for bit."""
    import bm25
    rng = np.random.default_rng(7)
    words = [f"w{i}" for i in range(60)]
    corpus = [list(rng.choice(words, size=int(rng.integers(3, 12)))) for _ in range(5000)]
    m = bm25.BM25()
    m.fit(corpus)
    q = ["w1", "w7", "w30", "w59", "w7"]
    ids = [m.term_to_id[t] for t in q]
    import scipy.sparse as sp
    csc = sp.csc_matrix(m.bm25_matrix)
    want = oracle.scores_f64(len(corpus), csc.indptr, csc.indices, csc.data, ids)
    s = m.get_scores(q)
    assert np.array_equal(s.view(np.uint64), want.view(np.uint64))
    full = m.get_top_n(q, corpus, n=len(corpus))
    assert len(full) == len(corpus)
    od, osc = oracle.topn_f64(want, len(corpus))
    assert [t[0] for t in full] == list(osc)
    assert [t[1] for t in full] == [corpus[i] for i in od]
    one = [["a", "b", "c", "d", "e", "f", "g", "h", "i", "j", "k"]]
    m1 = bm25.BM25()
    m1.fit(one)
    q1 = ["a", "c", "e", "g", "i", "k", "b", "d", "f", "h"]
    ref1 = np.sum(m1.bm25_matrix[:, [m1.term_to_id[t] for t in q1]], axis=1)
    assert np.array_equal(m1.get_scores(q1), ref1)


def test_bm25s_directory_drop_in(gpu, tmp_path):
    """BM25v.from_bm25s over a bm25s index directory (the animal fixture written
    back to disk): the bm25_test.py:23 query returns the reference's golden."""
    import bm25_native
    from test_bm25s_io import write_animal
    from bm25mi.bm25s_io import query_ids
    g, _ = write_animal(str(tmp_path))
    m = bm25_native.BM25v.from_bm25s(str(tmp_path))
    q = query_ids([["fish", "purr", "like", "cat"]], m.vocab, 20)
    docs, scores = m.search(q, top_k=2)
    assert np.array_equal(docs, g["q1_docs"])
    assert np.array_equal(scores.view(np.uint32), g["q1_scores"].view(np.uint32))


def test_sample_keys_per_tile_geometries(gpu):
    """The sampled search with m = 1, 2 and 4 keys per sample tile (the
    geometry a doc shard of the 8-GPU config uses: few tiles, k = 100)."""
    from bm25mi import synth
    cfg = synth.Config("t", 600_000, 4000, 4_000_000, 48, 8, 10)
    ip, ix, dt = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    index = _idx(ip, ix, dt, cfg.n_docs)
    for k in (10, 30, 70):  # 293 tiles, P = 8: m = 1, 2, 4
        _exact(index.search(q, k), oracle.search_c(cfg.n_docs, ip, ix, dt, q, k))
        assert index.search_stats()["fallback_queries"] == 0


def test_merge_paths_long_lists(gpu):
    """The sampled main stage's merges: one wavefront per query for lists of
    up to 2048 keys and k <= 1024 (merge_fast_kernel), the block merge for
    longer lists (k = 600: ~8k keys above the sampled threshold) and larger
    k (1500) — bit-exact either way."""
    rng = np.random.default_rng(33)
    N, V = 6_000_000, 300
    ip, ix, dt = _rand_index(rng, N, V, 400_000)
    q = rng.integers(-1, V, size=(24, 8)).astype(np.int32)
    index = _idx(ip, ix, dt, N, options={"theta_bound": 0})
    for k in (10, 250, 600, 1500):
        _exact(index.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))
        assert index.last_dispatch()["sample_p"] == _geom_p(index, k, opts={"theta_bound": 0})
        assert index.search_stats()["fallback_queries"] == 0
    # the tile-bound threshold on this index (every term equally weighted, so
    # a tile's largest single-term score is far below the best sums): lists
    # overflow and the queries take the exact fallback stage — still exact
    index.set_option("theta_bound", 1)
    _exact(index.search(q, 10), oracle.search_c(N, ip, ix, dt, q, 10))
    assert index.last_dispatch()["sample_p"] == 0


def test_weak_bounds_switch_to_sampled_threshold(gpu):
    """on an index whose terms all weigh alike, the
    tile-bound threshold sits far below the best sums and the lists
    overflow.  The first search with it sends its queries to the exact
    fallback (still exact); the handle reads that overflow from the search's
    report and its next 64 searches take the sampled threshold — exact, no
    fallback — before the tile-bound one is retried (and, failing again, off
    for 128)."""
    rng = np.random.default_rng(33)
    N, V = 6_000_000, 300
    ip, ix, dt = _rand_index(rng, N, V, 400_000)
    q = rng.integers(-1, V, size=(24, 8)).astype(np.int32)
    ref = oracle.search_c(N, ip, ix, dt, q, 10)
    index = _idx(ip, ix, dt, N)
    _exact(index.search(q, 10), ref)
    d = index.last_dispatch()
    assert d["sample_p"] == 0 and "bound_off" not in d["kernels"], d
    assert index.search_stats()["fallback_queries"] * 16 > len(q)
    for i in range(64):
        _exact(index.search(q, 10), ref)
        d = _check_dispatch(index, 10)
        assert "bound_off" in d["kernels"] and d["sample_p"] > 1, (i, d)
        assert index.search_stats()["fallback_queries"] == 0
    _exact(index.search(q, 10), ref)  # the retry
    assert index.last_dispatch()["sample_p"] == 0
    for i in range(128):
        _exact(index.search(q, 10), ref) if i % 32 == 0 else index.search(q, 10)
        assert "bound_off" in index.last_dispatch()["kernels"], i
    # a skewed index keeps the tile-bound threshold
    from bm25mi import synth
    cfg = synth.Config("s", 2_000_000, 20_000, 12_000_000, 40, 8, 10)
    ip2, ix2, dt2 = synth.make_index(cfg)
    q2 = synth.make_queries(cfg)
    index2 = _idx(ip2, ix2, dt2, cfg.n_docs)
    ref2 = oracle.search_c(cfg.n_docs, ip2, ix2, dt2, q2, cfg.k)
    for _ in range(4):
        _exact(index2.search(q2, cfg.k), ref2)
        d = index2.last_dispatch()
        assert d["sample_p"] == 0 and "bound_off" not in d["kernels"], d


def test_lucene_synth_index_built_on_gpu(gpu):
    """bench --config c3l's generator at a small scale: term frequencies and
    document lengths scored on the GPU by bm25_build_scores (lucene rule) are
    the oracle restatement's bits (oracle.build_scores_numpy, pinned by the
    animal fixture), and a search of the result is the oracle's."""
    from bm25mi import synth
    cfg = synth.Config("l", 300_000, 3000, 2_000_000, 48, 8, 20, weights="lucene")
    ip, ix, dt = synth.make_index(cfg)
    _, _, tf = synth._fill(cfg, 0, None, 0, synth.WEIGHTS["tf"])
    terms = np.repeat(np.arange(cfg.n_terms), np.diff(ip))
    dl = np.bincount(ix, weights=tf, minlength=cfg.n_docs).astype(np.int32)
    rip, rix, rdt, _ = oracle.build_scores_numpy(ix, terms, tf, dl, cfg.n_terms, 1.5, 0.75,
                                                 "lucene", float(np.mean(dl.tolist())))
    assert np.array_equal(rip, ip) and np.array_equal(rix, ix)
    assert np.array_equal(rdt.view(np.uint32), dt.view(np.uint32))
    q = synth.make_queries(cfg)
    index = _idx(ip, ix, dt, cfg.n_docs)
    _exact(index.search(q, cfg.k), oracle.search_c(cfg.n_docs, ip, ix, dt, q, cfg.k))


def test_rare_queries_zero_fill_path(gpu):
    """Queries with fewer than k positive docs in the sample (rare terms) on a
    non-negative index: every positive doc + the smallest untouched ids —
    no fallback pass — bit-exact vs the oracle; a signed index takes the exact
    fallback for the same queries."""
    rng = np.random.default_rng(17)
    N, V = 2_000_000, 600
    ip, ix, dt = _rand_index(rng, N, V, 40)  # every term has <= 40 postings
    q = rng.integers(-1, V, size=(40, 5)).astype(np.int32)
    q[0, :] = -1
    index = _idx(ip, ix, dt, N)
    for k in (50, 300):
        _exact(index.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))
        assert index.search_stats()["fallback_queries"] == 0
    dt2 = dt.copy()
    dt2[::7] *= -1
    index2 = _idx(ip, ix, dt2, N)
    _exact(index2.search(q, 50), oracle.search_c(N, ip, ix, dt2, q, 50))
    assert index2.search_stats()["fallback_queries"] > 0


@pytest.mark.parametrize("W", [1, 3, 8])
def test_global_theta_sharded_search(gpu, W):
    """bm25_search_sample/finish_device: W doc shards on one GPU, their sample
    keys concatenated (the all-gather of bm25mi.dist.sharded_search), theta
    from the whole sample, per-shard padded lists merged by the HIP merge —
    bit-exact vs the single-index oracle."""
    import torch
    from bm25mi import synth
    from bm25mi.index import GpuIndex, merge_topk_device
    from bm25mi.dist import sharded_search
    cfg = synth.Config("t", 1_200_000, 8000, 9_000_000, 64, 8, 100)
    full = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    q[3, 2:] = -1
    q[7, :] = [7990, 7991, 7992, 7993, -1, -1, -1, -1]  # rare terms: fewer than k hits
    ref = oracle.search_c(cfg.n_docs, *full, q, cfg.k)
    dq = torch.from_numpy(q).cuda()
    st = torch.cuda.current_stream()
    bounds = [synth.shard_bounds(cfg.n_docs, W, r) for r in range(W)]
    sdm = max(hi - lo for lo, hi in bounds)
    shards = [GpuIndex(*synth.make_index(cfg, lo, hi), hi - lo, doc_offset=lo) for lo, hi in bounds]
    # phase 1 on every shard, then the "all-gather"
    keys = []
    for sh in shards:
        S = sh.sample_width(cfg.k, W, sdm)
        kk = torch.zeros((len(q), max(S, 1)), dtype=torch.int64, device="cuda")
        if S > 0:
            sh.search_sample_device(dq, cfg.k, W, sdm, kk, st)
        keys.append(kk)
    all_keys = torch.stack(keys)

    class Ex:
        world = W

        def __call__(self, _):
            return all_keys

    lists_d = torch.empty((W, len(q), cfg.k), dtype=torch.int32, device="cuda")
    lists_s = torch.empty((W, len(q), cfg.k), dtype=torch.float32, device="cuda")
    for r, sh in enumerate(shards):
        sharded_search(sh, dq, cfg.k, sdm, lists_d[r], lists_s[r], None, st, exchange=Ex())
    md = torch.empty((len(q), cfg.k), dtype=torch.int32, device="cuda")
    ms = torch.empty((len(q), cfg.k), dtype=torch.float32, device="cuda")
    merge_topk_device(0, lists_d, lists_s, W, len(q), cfg.k, md, ms, st)
    torch.cuda.synchronize()
    _exact((md.cpu().numpy(), ms.cpu().numpy()), ref)


def test_split_halves_all_padding_row_k1(gpu):
    """The two halves of the sharded protocol on a 2-tile index with an
    all-padding row at k = 1 (the case round 4's debug probes chased): the
    row's top-1 is doc 0 at score 0 whether the world's sample holds this
    shard's own keys or only zeros (a world whose other shards hold nothing),
    and the other row is the oracle's."""
    import torch
    rng = np.random.default_rng(1)
    N, V = 3000, 20
    ip, ix, dt = _rand_index(rng, N, V, N // 3)
    index = _idx(ip, ix, dt, N)
    q = np.array([[-1, -1, -1], [1, 2, -1]], np.int32)
    dq = torch.from_numpy(q).cuda()
    for k in (1, 3):
        ref = oracle.search_c(N, ip, ix, dt, q, k)
        S = index.sample_width(k, 1, N)
        for world_keys in ("own", "zeros"):
            keys = torch.full((2, max(S, 1)), 7, dtype=torch.int64, device="cuda")
            if S > 0:
                index.search_sample_device(dq, k, 1, N, keys)
            ak = keys if world_keys == "own" else torch.zeros_like(keys)
            d = torch.empty((2, k), dtype=torch.int32, device="cuda")
            s = torch.empty((2, k), dtype=torch.float32, device="cuda")
            index.search_finish_device(dq, k, 1, N, ak.unsqueeze(0), d, s)
            torch.cuda.synchronize()
            _exact((d.cpu().numpy(), s.cpu().numpy()), ref)
    index.close()


def _doc_slice(indptr, indices, data, lo, hi):
    """The CSC of documents [lo, hi) (local ids), columns kept."""
    ip = np.zeros(len(indptr), np.int64)
    ix, dt = [], []
    for t in range(len(indptr) - 1):
        a, b = int(indptr[t]), int(indptr[t + 1])
        col = indices[a:b]
        p0, p1 = np.searchsorted(col, lo), np.searchsorted(col, hi)
        ix.append(col[p0:p1] - lo)
        dt.append(data[a + p0:a + p1])
        ip[t + 1] = ip[t] + (p1 - p0)
    return ip, np.concatenate(ix).astype(np.int32), np.concatenate(dt).astype(np.float32)


@pytest.mark.parametrize("W", [2, 3])
def test_global_theta_ties_across_shards(gpu, W):
    """the global threshold is a (score, doc) key; sample
    keys carry global doc ids and each shard moves theta into its own frame,
    so a tie group cut by k that spans shards keeps the smallest GLOBAL ids.
    Columns of constant or quarter-step values make nearly every score tied."""
    import torch
    from bm25mi.index import GpuIndex, merge_topk_device
    from bm25mi.dist import shard_bounds, sharded_search
    rng = np.random.default_rng(40 + W)
    N, V = 700_000, 12
    ip, ix, dt = _rand_index(rng, N, V, 300_000, coarse=True)
    dt[ip[0]:ip[1]] = 1.0          # term 0: one score everywhere
    q = np.array([[0, -1, -1], [0, 0, -1], [1, 2, 3], [4, 4, 5], [0, 6, 7], [8, 9, 10]],
                 np.int32)
    dq = torch.from_numpy(q).cuda()
    st = torch.cuda.current_stream()
    bounds = [shard_bounds(N, W, r) for r in range(W)]
    sdm = max(hi - lo for lo, hi in bounds)
    shards = [GpuIndex(*_doc_slice(ip, ix, dt, lo, hi), hi - lo, doc_offset=lo) for lo, hi in bounds]
    for k in (100, 777):
        ref = oracle.search_c(N, ip, ix, dt, q, k)
        keys = []
        for sh in shards:
            S = sh.sample_width(k, W, sdm)
            kk = torch.zeros((len(q), max(S, 1)), dtype=torch.int64, device="cuda")
            if S > 0:
                sh.search_sample_device(dq, k, W, sdm, kk, st)
            keys.append(kk)
        all_keys = torch.stack(keys)

        class Ex:
            world = W

            def __call__(self, _):
                return all_keys

        lists_d = torch.empty((W, len(q), k), dtype=torch.int32, device="cuda")
        lists_s = torch.empty((W, len(q), k), dtype=torch.float32, device="cuda")
        for r, sh in enumerate(shards):
            sharded_search(sh, dq, k, sdm, lists_d[r], lists_s[r], None, st, exchange=Ex())
        md = torch.empty((len(q), k), dtype=torch.int32, device="cuda")
        ms = torch.empty((len(q), k), dtype=torch.float32, device="cuda")
        merge_topk_device(0, lists_d, lists_s, W, len(q), k, md, ms, st)
        torch.cuda.synchronize()
        _exact((md.cpu().numpy(), ms.cpu().numpy()), ref)


def test_sharded_index_global_theta_ties_and_small_shards(gpu):
    """bm25_sharded_search runs the global-threshold protocol (every shard's
    sample keys peer-copied to every device): tie groups cut by k that span
    shards keep the smallest global ids; shards smaller than k pad their
    lists; a one-tile collection split over more devices than tiles works."""
    from bm25mi.index import ShardedIndex
    rng = np.random.default_rng(77)
    N, V = 700_000, 12
    ip, ix, dt = _rand_index(rng, N, V, 300_000, coarse=True)
    dt[ip[0]:ip[1]] = 1.0
    q = np.array([[0, -1, -1], [0, 0, -1], [1, 2, 3], [4, 4, 5], [0, 6, 7], [8, 9, 10]],
                 np.int32)
    sh = ShardedIndex(ip, ix, dt, N, devices=[0, 0, 0])
    for k in (100, 777):
        _exact(sh.search(q, k), oracle.search_c(N, ip, ix, dt, q, k))
    sh.close()
    for N, devs, k in ((3000, [0, 0], 2500), (1500, [0, 0, 0], 1500)):
        ip, ix, dt = _rand_index(rng, N, 40, 4000)
        qq = rng.integers(-1, 40, size=(9, 4)).astype(np.int32)
        sh = ShardedIndex(ip, ix, dt, N, devices=devs)
        _exact(sh.search(qq, k), oracle.search_c(N, ip, ix, dt, qq, k))
        sh.close()


# ------------------------------------------------- GPU index build (§8(f) 2)
def test_build_scores_lucene_animal_fixture(gpu):
    """bm25_build_scores (lucene, device idf) rebuilds animal_index_bm25's CSC
    from (doc, term, tf) triples: indptr, indices and every data bit."""
    from bm25mi.scoring import build_scores
    g = _load("animal.npz")
    ip0, ix0 = g["indptr"].astype(np.int64), g["indices"]
    terms = np.repeat(np.arange(len(ip0) - 1), np.diff(ip0)).astype(np.int32)
    dl = np.bincount(ix0, minlength=int(g["n_docs"]))
    perm = np.random.default_rng(3).permutation(len(ix0))  # any triple order
    ip, ix, dt = build_scores(ix0[perm], terms[perm], np.ones(len(ix0), np.float32), dl,
                              len(ip0) - 1, k1=1.5, b=0.75, method="lucene")
    assert np.array_equal(ip, ip0) and np.array_equal(ix, ix0)
    assert np.array_equal(dt.view(np.uint32), g["data"].view(np.uint32))


@pytest.mark.parametrize("method", ["lucene", "bm25py"])
def test_build_scores_random_corpus(gpu, method):
    """A 20k-doc random corpus (Zipf token ids, repeated tokens): the GPU
    build equals the numpy restatement bit for bit with the host idf, and
    within 1 f32 ulp with the device idf; the built index then searches
    bit-exactly against the oracle."""
    from bm25mi.scoring import build_scores, triples_from_token_ids
    rng = np.random.default_rng(11)
    V = 3000
    docs_tok = [np.minimum(rng.zipf(1.3, size=int(rng.integers(0, 300))) - 1, V - 1)
                for _ in range(20_000)]
    docs, terms, tfs, dl = triples_from_token_ids(docs_tok)
    avgdl = float(np.mean(dl.tolist()))
    df = np.bincount(terms, minlength=V)
    idf = oracle.idf_numpy(df, len(dl))
    ref = oracle.build_scores_numpy(docs, terms, tfs, dl, V, 1.2, 0.7, method, avgdl, idf=idf)
    got = build_scores(docs, terms, tfs, dl, V, k1=1.2, b=0.7, method=method, idf=idf,
                       want_f64=True)
    assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1])
    assert np.array_equal(got[2].view(np.uint32), ref[2].view(np.uint32))
    assert np.array_equal(got[3].view(np.uint64), ref[3].view(np.uint64))
    dev = build_scores(docs, terms, tfs, dl, V, k1=1.2, b=0.7, method=method)
    ulp = np.abs(dev[2].view(np.int32).astype(np.int64) - ref[2].view(np.int32))
    assert ulp.max() <= 1 and np.mean(ulp == 0) > 0.999
    q = rng.integers(-1, V, size=(40, 6)).astype(np.int32)
    index = _idx(got[0], got[1], got[2], len(dl))
    _exact(index.search(q, 50), oracle.search_c(len(dl), got[0], got[1], got[2], q, 50))


def test_build_scores_rejects_bad_triples(gpu):
    from bm25mi.scoring import build_scores
    with pytest.raises(ValueError, match="duplicate"):
        build_scores([0, 0], [1, 1], [1.0, 2.0], [3], 2)
    with pytest.raises(ValueError, match="out of range"):
        build_scores([0, 5], [1, 1], [1.0, 2.0], [3, 3], 2)
    with pytest.raises(ValueError, match="positive"):
        build_scores([0], [1], [0.0], [3], 2)
    # ids that would index doc_len / idf out of bounds stop the
    # build before scoring — negative ids and ids near 2^30, docs and terms
    rng = np.random.default_rng(5)
    n = 50_000
    docs = rng.integers(0, 1000, n).astype(np.int32)
    terms = rng.integers(0, 30, n).astype(np.int32)
    tfs = np.ones(n, np.float32)
    dl = np.full(1000, 7, np.int32)
    for bad_d, bad_t in ((-1, None), (-(1 << 30), None), ((1 << 30) - 1, None), (1 << 30, None),
                         (None, -1), (None, (1 << 30) + 7), (None, 2**31 - 1)):
        d2, t2 = docs.copy(), terms.copy()
        if bad_d is not None:
            d2[n // 2] = bad_d
        if bad_t is not None:
            t2[n - 1] = bad_t
        with pytest.raises(ValueError, match="out of range"):
            build_scores(d2, t2, tfs, dl, 30)
    ip, ix, dt = build_scores([], [], [], [0, 0], 4)
    assert np.array_equal(ip, np.zeros(5, np.int64)) and ix.size == 0


# ------------------------------------------------- sparse segments / config 5
def test_config3_sparse_segments_full_batch(gpu, monkeypatch):
    """The headline batch on the O(pairs) segment table (tile lists + the
    per-search seg table of the band kernel): all 1024 queries bit-exact."""
    from bm25mi import synth
    monkeypatch.setenv("BM25_SEGMENTS", "sparse")
    cfg = synth.CONFIGS["c3"]
    ip, ix, dt = synth.make_index(cfg, threads=16)
    q = synth.make_queries(cfg)
    index = _idx(ip, ix, dt, cfg.n_docs)
    info = index.info()
    assert info["sparse"] and 0 < info["n_pairs"] <= len(ix)
    assert info["device_bytes"] < 6 * len(ix) + 2_000_000_000  # no dense V x ntiles table
    _exact(index.search(q, cfg.k), oracle.search_c(cfg.n_docs, ip, ix, dt, q, cfg.k, threads=16))


def test_config5_shape_int64_shards_sparse(gpu, tmp_path, monkeypatch):
    """Config 5 in miniature: a collection written as a bm25s directory with
    an int64 indptr, cut per rank by bm25mi.shard (streamed column blocks),
    each rank's shard on the sparse segment table, searched with the global
    threshold protocol and merged — bit-exact vs the oracle on the whole
    collection."""
    import torch
    monkeypatch.setenv("BM25_SEGMENTS", "sparse")
    from bm25mi import synth
    from bm25mi.bm25s_io import save_bm25s
    from bm25mi.shard import load_bm25s_shard
    from bm25mi.index import GpuIndex, merge_topk_device
    from bm25mi.dist import sharded_search
    cfg = synth.Config("c5-mini", 2_000_000, 400_000, 16_000_000, 128, 8, 100)
    ip, ix, dt = synth.make_index(cfg, threads=16)
    q = synth.make_queries(cfg)
    save_bm25s(str(tmp_path), ip.astype(np.int64), ix, dt, cfg.n_docs)
    W = 4
    dq = torch.from_numpy(q).cuda()
    st = torch.cuda.current_stream()
    shards, sdm = [], 0
    for r in range(W):
        sip, six, sdt, n, lo, _ = load_bm25s_shard(str(tmp_path), r, W)
        sh = GpuIndex(sip, six, sdt, n, doc_offset=lo)
        assert sh.info()["sparse"]
        shards.append(sh)
        sdm = max(sdm, n)
    ref = oracle.search_c(cfg.n_docs, ip, ix, dt, q, cfg.k, threads=16)
    keys = []
    for sh in shards:
        S = sh.sample_width(cfg.k, W, sdm)
        kk = torch.zeros((len(q), max(S, 1)), dtype=torch.int64, device="cuda")
        if S > 0:
            sh.search_sample_device(dq, cfg.k, W, sdm, kk, st)
        keys.append(kk)
    all_keys = torch.stack(keys)

    class Ex:
        world = W

        def __call__(self, _):
            return all_keys

    lists_d = torch.empty((W, len(q), cfg.k), dtype=torch.int32, device="cuda")
    lists_s = torch.empty((W, len(q), cfg.k), dtype=torch.float32, device="cuda")
    for r, sh in enumerate(shards):
        sharded_search(sh, dq, cfg.k, sdm, lists_d[r], lists_s[r], None, st, exchange=Ex())
    md = torch.empty((len(q), cfg.k), dtype=torch.int32, device="cuda")
    ms = torch.empty((len(q), cfg.k), dtype=torch.float32, device="cuda")
    merge_topk_device(0, lists_d, lists_s, W, len(q), cfg.k, md, ms, st)
    torch.cuda.synchronize()
    _exact((md.cpu().numpy(), ms.cpu().numpy()), ref)


# ------------------------------------------------ configs 4 and 5 in full
def _protocol_search(shards, dq, k, sdm):
    """bm25mi.dist.sharded_search (the bench's N > 1 step) over doc shards
    held by this process, the two all-gathers replaced by concatenation;
    returns the merged [Q, k] (docs, scores) on the host."""
    import torch
    from bm25mi.dist import sharded_search
    from bm25mi.index import merge_topk_device
    W, Q = len(shards), dq.shape[0]
    st = torch.cuda.current_stream()
    keys = []
    for sh in shards:
        S = sh.sample_width(k, W, sdm)
        kk = torch.zeros((Q, max(S, 1)), dtype=torch.int64, device="cuda")
        if S > 0:
            sh.search_sample_device(dq, k, W, sdm, kk, st)
        keys.append(kk)
    all_keys = torch.stack(keys)

    class Ex:
        world = W

        def __call__(self, _):
            return all_keys

    lists_d = torch.empty((W, Q, k), dtype=torch.int32, device="cuda")
    lists_s = torch.empty((W, Q, k), dtype=torch.float32, device="cuda")
    for r, sh in enumerate(shards):
        sharded_search(sh, dq, k, sdm, lists_d[r], lists_s[r], None, st, exchange=Ex())
    md = torch.empty((Q, k), dtype=torch.int32, device="cuda")
    ms = torch.empty((Q, k), dtype=torch.float32, device="cuda")
    merge_topk_device(0, lists_d, lists_s, W, Q, k, md, ms, st)
    torch.cuda.synchronize()
    return md.cpu().numpy(), ms.cpu().numpy()


def test_config4_c3_index_eight_shards_full_batch(gpu):
    """Config 4 at its own workload: the headline 10M-doc / 640M-posting
    index doc-sharded 8 ways, all 1024 queries bit-exact vs the oracle on the
    whole collection — (i) bm25_sharded_* (eight shards on cuda:0, global
    threshold, peer-copied keys and lists, HIP merge); (ii) the
    multi-process protocol of bench.py's N > 1 step (bm25mi.dist.
    sharded_search over the per-rank shards the bench generates)."""
    import torch
    from bm25mi import synth
    from bm25mi.index import GpuIndex, ShardedIndex
    cfg = synth.CONFIGS["c3"]
    ip, ix, dt = synth.make_index(cfg, threads=16)
    q = synth.make_queries(cfg)
    _progress("c4: index generated")
    ref = oracle.search_c(cfg.n_docs, ip, ix, dt, q, cfg.k, threads=16)
    _progress("c4: oracle done")
    sh = ShardedIndex(ip, ix, dt, cfg.n_docs, devices=[0] * 8)
    assert len(sh.shards()) == 8
    _progress("c4: 8 shards built")
    _exact(sh.search(q, cfg.k), ref)
    sh.close()
    del ip, ix, dt
    _progress("c4: bm25_sharded_search bit-exact")
    W = 8
    bounds = [synth.shard_bounds(cfg.n_docs, W, r) for r in range(W)]
    sdm = max(hi - lo for lo, hi in bounds)
    shards = []
    for lo, hi in bounds:
        shards.append(GpuIndex(*synth.make_index(cfg, lo, hi, threads=16), hi - lo, doc_offset=lo))
        _progress(f"c4: rank shard [{lo}, {hi}) built")
    dq = torch.from_numpy(q).cuda()
    _exact(_protocol_search(shards, dq, cfg.k, sdm), ref)
    d = shards[0].last_dispatch()
    assert d["kernels"] - {"bound_off", "rest_split", "bound_pool"} == _want_kernels(
        _geom_p(shards[0], cfg.k, W, (sdm + 2047) // 2048, weak="bound_off" in d["kernels"])), d
    _progress("c4: two-collective protocol bit-exact")
    _exact(_world_bounds_search(shards, dq, cfg.k), ref)
    assert {"bound_keys", "bound_pool"} <= shards[0].last_dispatch()["kernels"]
    _progress("c4: one-collective protocol (world tile bounds) bit-exact")
    for s in shards:
        s.close()


def _world_bounds_search(shards, dq, k):
    """The one-collective protocol over doc shards held by this process: the
    world's tile bounds stacked as their all-gather delivers them, each
    shard's bm25_search_shard_device list in the packed [W, 2, Q, k] buffer
    as the list all-gather delivers it, the W-way merge."""
    import torch
    from bm25mi.index import merge_sorted_device
    W, Q = len(shards), dq.shape[0]
    stride = max(s.bounds_stride() for s in shards)
    wb = torch.empty((W, shards[0].n_terms, stride), dtype=torch.int16, device="cuda")
    for r, s in enumerate(shards):
        s.bounds_export(wb[r], stride)
    tiles = sum(int(s.info()["n_tiles"]) for s in shards)
    g = torch.empty((W, 2, Q, k), dtype=torch.int32, device="cuda")
    for r, s in enumerate(shards):
        s.set_world_bounds(wb, W, stride, tiles)
        s.search_shard_device(dq, k, g[r, 0], g[r, 1].view(torch.float32))
    md = torch.empty((Q, k), dtype=torch.int32, device="cuda")
    ms = torch.empty((Q, k), dtype=torch.float32, device="cuda")
    merge_sorted_device(0, g, g[:, 1].view(torch.float32), W, Q, k, 2 * Q * k, md, ms)
    torch.cuda.synchronize()
    for s in shards:
        s.set_world_bounds(None, 0, 0, 0)
    return md.cpu().numpy(), ms.cpu().numpy()


def test_world_bounds_shards_ties_small_shards(gpu):
    """bm25_search_shard_device with world tile bounds on uneven shards (40
    tiles, 160 tiles, the rest): the collection's threshold taken by each
    shard, quarter-step ties at it, zero-fill rows, k above a shard's tiles
    and k > 4096 (each shard's exact top-k) — merged, bit-exact vs the
    single-index oracle; without world bounds the entry point refuses."""
    import scipy.sparse as sp
    import torch
    N, V = 600_000, 200
    ip, ix, dt = _bound_case(91, N, V, 20)
    rng = np.random.default_rng(6)
    q = np.concatenate([rng.integers(0, 20, size=(24, 3)),
                        rng.integers(20, V, size=(24, 3))], axis=1).astype(np.int32)
    q[0, :] = -1
    q[1, :] = -1
    q[1, 0] = 20 + int(np.argmin(np.diff(ip)[20:]))  # a rare term: fewer than k positive docs
    cuts = [0, 2048 * 40, 2048 * 200, N]
    m = sp.csc_matrix((dt, ix, ip), shape=(N, V))
    shards = []
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        s = m[lo:hi].tocsc()
        s.sort_indices()
        shards.append(_idx(s.indptr.astype(np.int64), s.indices.astype(np.int32),
                           s.data.astype(np.float32), hi - lo, doc_offset=lo, segments="dense"))
    dq = torch.from_numpy(q).cuda()
    d = torch.empty((len(q), 10), dtype=torch.int32, device="cuda")
    with pytest.raises(ValueError, match="world bounds"):
        shards[0].search_shard_device(dq, 10, d, d.view(torch.float32))
    for k in (1, 10, 16, 5000):
        ref = oracle.search_c(N, ip, ix, dt, q, k, threads=8)
        _exact(_world_bounds_search(shards, dq, k), ref)
        # the pooled world bounds: 293 tiles, 74 groups of 4 serve k <= 9
        assert ("bound_pool" in shards[1].last_dispatch()["kernels"]) == (k == 1), k
        if k == 1:
            for s in shards:
                s.set_option("bound_pool", 0)
            _exact(_world_bounds_search(shards, dq, k), ref)
            assert "bound_pool" not in shards[1].last_dispatch()["kernels"]
            for s in shards:
                s.set_option("bound_pool", 1)
        if k <= 16:  # REST over split items (rest_split: heavy queries' bands in pieces)
            for s in shards:
                s.set_option("rest_split", 1)
            _exact(_world_bounds_search(shards, dq, k), ref)
            assert "rest_split" in shards[1].last_dispatch()["kernels"]
            for s in shards:
                s.set_option("rest_split", 0)
    for s in shards:
        s.close()


def test_world_bounds_set_while_export_in_flight(gpu):
    """bm25_index_set_world_bounds reads the caller's table into its pooled
    copy only once the device is idle: the table is first filled with the
    largest f16 bound (65504: a threshold no document reaches), then each
    shard's export is queued on a side stream behind a spin kernel and the
    world bounds are set at once, with no wait by the caller — a copy taken
    before the exports land would hold 65504 and zero-fill every row."""
    import scipy.sparse as sp
    import torch
    N, V = 600_000, 200
    ip, ix, dt = _bound_case(93, N, V, 20)
    rng = np.random.default_rng(9)
    q = np.concatenate([rng.integers(0, 20, size=(32, 3)),
                        rng.integers(20, V, size=(32, 3))], axis=1).astype(np.int32)
    cuts = [0, 2048 * 100, N]
    m = sp.csc_matrix((dt, ix, ip), shape=(N, V))
    shards = []
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        s_ = m[lo:hi].tocsc()
        s_.sort_indices()
        shards.append(_idx(s_.indptr.astype(np.int64), s_.indices.astype(np.int32),
                           s_.data.astype(np.float32), hi - lo, doc_offset=lo, segments="dense"))
    W, k = len(shards), 1
    stride = max(s_.bounds_stride() for s_ in shards)
    tiles = sum(int(s_.info()["n_tiles"]) for s_ in shards)
    wb = torch.full((W, V, stride), 0x7BFF, dtype=torch.int16, device="cuda")
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        torch.cuda._sleep(200_000_000)  # (~0.1 s of spinning ahead of the exports)
    for r, s_ in enumerate(shards):
        s_.bounds_export(wb[r], stride, side)
    for s_ in shards:
        s_.set_world_bounds(wb, W, stride, tiles)
    dq = torch.from_numpy(q).cuda()
    g = torch.empty((W, 2, len(q), k), dtype=torch.int32, device="cuda")
    for r, s_ in enumerate(shards):
        s_.search_shard_device(dq, k, g[r, 0], g[r, 1].view(torch.float32))
        assert "bound_pool" in s_.last_dispatch()["kernels"]
    from bm25mi.index import merge_sorted_device
    md = torch.empty((len(q), k), dtype=torch.int32, device="cuda")
    ms = torch.empty((len(q), k), dtype=torch.float32, device="cuda")
    merge_sorted_device(0, g, g[:, 1].view(torch.float32), W, len(q), k, 2 * len(q) * k, md, ms)
    torch.cuda.synchronize()
    _exact((md.cpu().numpy(), ms.cpu().numpy()), oracle.search_c(N, ip, ix, dt, q, k, threads=8))
    for s_ in shards:
        s_.close()


@pytest.mark.parametrize("segments", ["dense", "sparse"])
def test_config5_rank_shard_full_batch(gpu, segments):
    """Config 5 at its own per-rank workload: one rank's doc shard of the
    100M-doc / 1M-term / 6.4B-posting collection (12.5M docs, ~800M
    postings, the global ids of rank 3: doc_offset 37.5M), all 1024 queries
    bit-exact vs the oracle on that shard, on both segment tables (dense: 24
    GB, the bench's; sparse: tile lists + the per-search table)."""
    from bm25mi import synth
    cfg = synth.CONFIGS["c5"]
    lo, hi = synth.shard_bounds(cfg.n_docs, 8, 3)
    ip, ix, dt = synth.make_index(cfg, lo, hi, threads=16)
    assert ip.dtype == np.int64 and int(ip[-1]) > 700_000_000
    q = synth.make_queries(cfg)
    _progress(f"c5: rank shard [{lo}, {hi}) generated, nnz {int(ip[-1])}")
    rd, rs = oracle.search_c(hi - lo, ip, ix, dt, q, cfg.k, threads=16)
    _progress("c5: oracle done")
    index = _idx(ip, ix, dt, hi - lo, doc_offset=lo, segments=segments)
    _progress(f"c5: {segments} index built")
    assert index.info()["sparse"] == (segments == "sparse")
    _exact(index.search(q, cfg.k), (rd + lo, rs))
    _check_dispatch(index, cfg.k)
    assert index.info()["tile_bounds"] == (segments == "dense")
    assert index.search_stats()["fallback_queries"] == 0
    index.close()


def test_rccl_all_gather_branch(gpu):
    """bm25mi.dist's device all-gather (the RCCL branch: nccl backend,
    all_gather_into_tensor on the search stream) on a real one-rank RCCL
    communicator: shape [W, ...], rank-major, the packed [W, 2, Q, k] list
    layout the merge reads."""
    import torch
    import torch.distributed as dist
    from bm25mi.dist import _all_gather, gather_keys
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        pk = torch.arange(2 * 5 * 7, dtype=torch.int32, device="cuda").view(2, 5, 7)
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            g = _all_gather(pk)
            kk = gather_keys(torch.arange(5 * 3, dtype=torch.int64, device="cuda").view(5, 3))
        s.synchronize()
        assert tuple(g.shape) == (1, 2, 5, 7) and g.is_contiguous() and torch.equal(g[0], pk)
        assert tuple(kk.shape) == (1, 5, 3) and int(kk[0, 4, 2]) == 14
    finally:
        dist.destroy_process_group()


def test_rccl_one_collective_protocol_one_rank(gpu):
    """The one-collective protocol end to end over a real one-rank RCCL
    communicator (the driver's N > 1 bench path, minus the peers):
    setup_world_bounds' MAX / SUM all-reduces and the int32-view all-gather
    of the bounds on RCCL, the pooled world table, bm25_search_shard_device
    and the W-way merge of sharded_search (its list all-gather is the
    identity at one rank: test_rccl_all_gather_branch covers it) —
    bit-exact against the oracle; a second search reuses the setup."""
    import torch
    import torch.distributed as dist
    from bm25mi.dist import setup_world_bounds, sharded_search
    N, V = 1_200_000, 300
    ip, ix, dt = _bound_case(95, N, V, 30)
    rng = np.random.default_rng(12)
    q = np.concatenate([rng.integers(0, 30, size=(64, 4)),
                        rng.integers(30, V, size=(64, 4))], axis=1).astype(np.int32)
    k = 10
    ref = oracle.search_c(N, ip, ix, dt, q, k, threads=8)
    dist.init_process_group("nccl", store=dist.HashStore(), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    try:
        index = _idx(ip, ix, dt, N, segments="dense")
        assert setup_world_bounds(index)
        dq = torch.from_numpy(q).cuda()
        d = torch.empty((len(q), k), dtype=torch.int32, device="cuda")
        sc = torch.empty((len(q), k), dtype=torch.float32, device="cuda")
        for _ in range(2):
            docs, scores = sharded_search(index, dq, k, N, d, sc)
            torch.cuda.synchronize()
            _exact((docs.cpu().numpy(), scores.cpu().numpy()), ref)
            assert {"bound_keys", "bound_pool"} <= index.last_dispatch()["kernels"]
        index.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("T", [4, 8])
def test_tile_bound_skips_exact(gpu, T):
    """The REST pass skips the (query, tile) pairs whose query-term maxima
    (f16 upper bounds per (term, tile)) sum below the threshold: same bits
    with and without (tile_bound option), and tiles are actually skipped —
    rare high-scoring terms (present in few tiles) beside common low-scoring
    ones, ties at the threshold from quarter-step values."""
    rng = np.random.default_rng(50 + T)
    N, V = 3_000_000, 400
    indptr, idx, dat = [0], [], []
    for t in range(V):
        df = int(rng.integers(200_000, 900_000)) if t < 40 else int(rng.integers(5, 400))
        idx.append(np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
        hi = 1.0 if t < 40 else 9.0
        dat.append((np.round(rng.uniform(0.1, hi, df) * 4) / 4 + 0.25).astype(np.float32))
        indptr.append(indptr[-1] + df)
    ip, ix, dt = np.array(indptr, np.int64), np.concatenate(idx), np.concatenate(dat)
    q = np.concatenate([rng.integers(0, 40, size=(48, T // 2)),
                        rng.integers(40, V, size=(48, T - T // 2))], axis=1).astype(np.int32)
    q[0, :] = -1
    q[1, 1:] = q[1, 0]
    index = _idx(ip, ix, dt, N, segments="dense")
    assert index.get_option("tile_bound") == 1
    _exact(index.search(q, 10), oracle.search_c(N, ip, ix, dt, q, 10, threads=8))
    # the skipped postings are counted by the count_skips build only
    assert index.search_stats()["bound_skipped_postings"] == -1
    assert "count_skips" not in index.last_dispatch()["kernels"]
    index.set_option("count_skips", 1)
    for k in (10, 100):
        ref = oracle.search_c(N, ip, ix, dt, q, k, threads=8)
        _exact(index.search(q, k), ref)
        st = index.search_stats()
        assert "count_skips" in index.last_dispatch()["kernels"]
        skipped = st["bound_skipped_tiles"]
        assert skipped > 0, skipped
        # the postings of the skipped pairs (bench.py's roofline.bound_skip): the
        # all-padding row skips every tile with no posting in it; at k = 10
        # (tile-bound theta) the other rows skip tiles of their common terms too
        df = np.diff(ip)
        per_query = sum(int(df[np.unique(r[r >= 0])].sum()) for r in q)
        ntiles = index.info()["n_tiles"]
        assert 0 <= st["bound_skipped_postings"] < per_query, (st, per_query)
        assert (st["bound_skipped_postings"] > 0) == (skipped > ntiles), (st, ntiles)
        if k == 10:
            assert skipped > ntiles, st
        index.set_option("tile_bound", 0)
        _exact(index.search(q, k), ref)
        st = index.search_stats()
        assert st["bound_skipped_tiles"] == 0 and st["bound_skipped_postings"] == 0
        index.set_option("tile_bound", 1)


def _bound_case(seed, N, V, heavy, big=False):
    """CSC with `heavy` common low-scoring terms and rare high-scoring ones
    (quarter-step values: ties); big: also scores past f16's range and below
    its smallest subnormal (the rounding edges of the tile bounds)."""
    rng = np.random.default_rng(seed)
    indptr, idx, dat = [0], [], []
    for t in range(V):
        df = int(rng.integers(N // 15, N // 4)) if t < heavy else int(rng.integers(1, 300))
        idx.append(np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
        hi = 1.0 if t < heavy else 9.0
        v = (np.round(rng.uniform(0.1, hi, df) * 4) / 4 + 0.25).astype(np.float32)
        if big and t % 7 == 3:
            v[::3] = np.float32(70000.0) + np.float32(t)
        if big and t % 7 == 5:
            v[::2] = np.float32(1e-30)
        dat.append(v)
        indptr.append(indptr[-1] + df)
    return np.array(indptr, np.int64), np.concatenate(idx), np.concatenate(dat)


@pytest.mark.parametrize("T,big", [(4, False), (8, True), (3, True), (12, False), (70, False)])
def test_theta_bound_exact(gpu, T, big):
    """Threshold keys from the tile bounds (theta_bound, no SAMPLE pass): the
    same bits as the sampled threshold and as the oracle, with and without
    the REST tile skip — ties at the threshold (quarter-step values), rows
    with fewer positive tiles than k (zero-fill), padding, duplicates, scores
    past f16's range and below its subnormals, and T > 64 (the wave kernel's
    REST); the threshold from the pooled bounds (bound_pool: 428 groups of 4
    tiles serve k <= 53) and from the per-tile bounds."""
    N, V = 3_500_000, 300  # 1709 tiles: >= 16k at k = 100 (search_geom)
    ip, ix, dt = _bound_case(70 + T, N, V, 30, big)
    rng = np.random.default_rng(T)
    q = np.concatenate([rng.integers(0, 30, size=(40, T // 2)),
                        rng.integers(30, V, size=(40, T - T // 2))], axis=1).astype(np.int32)
    q[0, :] = -1
    q[1, 1:] = q[1, 0]
    q[2, :] = -1
    q[2, 0] = 30 + int(np.argmin(np.diff(ip)[30:]))  # one rare term: < k positive tiles
    index = _idx(ip, ix, dt, N, segments="dense")
    assert index.get_option("theta_bound") == 1
    for k in (1, 10, 100):
        ref = oracle.search_c(N, ip, ix, dt, q, k, threads=8)
        for tb in (1, 0):
            for tl in (1, 0):
                for pool in (1, 0):
                    index.set_option("theta_bound", tb)
                    index.set_option("tile_bound", tl)
                    index.set_option("bound_pool", pool)
                    _exact(index.search(q, k), ref)
                    d = _check_dispatch(index, k, opts={"theta_bound": tb}, T=T, flat=T <= 64)
                    P = d["sample_p"]
                    assert (P == 0) == (bool(tb) and T <= 16 and "bound_off" not in d["kernels"]), \
                        (P, tb, T, d)
                    assert ("bound_pool" in d["kernels"]) == (P == 0 and bool(pool) and
                                                              428 >= 8 * k), (pool, k, d)
    index.set_option("theta_bound", 1)
    index.set_option("tile_bound", 1)
    index.set_option("bound_pool", 1)
    index.close()


def test_theta_bound_sharded_protocol(gpu):
    """The two-half sharded protocol with tile-bound keys: S = k per shard,
    every shard's best k keys all-gathered (here: stacked on one GPU), the
    world's k-th key as theta, lists merged — bit-exact vs the single-index
    oracle, also with one empty-ish shard and k above a shard's tiles."""
    import torch
    from bm25mi.index import merge_topk_device
    N, V = 600_000, 200
    ip, ix, dt = _bound_case(91, N, V, 20)
    rng = np.random.default_rng(5)
    q = np.concatenate([rng.integers(0, 20, size=(24, 3)),
                        rng.integers(20, V, size=(24, 3))], axis=1).astype(np.int32)
    cuts = [0, 2048 * 40, 2048 * 200, N]
    import scipy.sparse as sp
    m = sp.csc_matrix((dt, ix, ip), shape=(N, V))
    shards = []
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        s = m[lo:hi].tocsc()
        s.sort_indices()
        shards.append(_idx(s.indptr.astype(np.int64), s.indices.astype(np.int32),
                           s.data.astype(np.float32), hi - lo, doc_offset=lo, segments="dense"))
    W = len(shards)
    smax = max(hi - lo for lo, hi in zip(cuts[:-1], cuts[1:]))
    dq = torch.from_numpy(q).cuda()
    for k in (10, 16):  # (3 x 93 tiles >= 16k)
        S = shards[0].sample_width(k, W, smax)
        assert S > 0 and S * W >= 2 * k, S
        keys = torch.zeros((W, q.shape[0], S), dtype=torch.int64, device="cuda")
        for r, s in enumerate(shards):
            s.search_sample_device(dq, k, W, smax, keys[r])
        d = torch.empty((W, q.shape[0], k), dtype=torch.int32, device="cuda")
        sc = torch.empty((W, q.shape[0], k), dtype=torch.float32, device="cuda")
        for r, s in enumerate(shards):
            s.search_finish_device(dq, k, W, smax, keys, d[r], sc[r])
            assert "bound_keys" in s.last_dispatch()["kernels"]
        od = torch.empty((q.shape[0], k), dtype=torch.int32, device="cuda")
        os_ = torch.empty((q.shape[0], k), dtype=torch.float32, device="cuda")
        merge_topk_device(0, d, sc, W, q.shape[0], k, od, os_)
        torch.cuda.synchronize()
        ref = oracle.search_c(N, ip, ix, dt, q, k, threads=8)
        _exact((od.cpu().numpy(), os_.cpu().numpy()), ref)
    for s in shards:
        s.close()


def test_fork_shares_arrays_concurrent_streams(gpu):
    """bm25_index_fork: a second context on the same device arrays with its
    own workspace — two halves of a batch searched at once on two streams
    (one per handle) give the oracle's bits; options are copied at fork time
    and follow set_option; the fork outlives its base (shared arrays)."""
    import torch
    from bm25mi import synth
    cfg = synth.Config("f", 700_000, 3000, 5_000_000, 96, 8, 50)
    ip, ix, dt = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    ref = oracle.search_c(cfg.n_docs, ip, ix, dt, q, cfg.k)
    base = _idx(ip, ix, dt, cfg.n_docs, options={"grid_pct": 60})
    fork = base.fork()
    assert fork.get_option("grid_pct") == 60 and fork.info() == base.info()
    dq = torch.from_numpy(q).cuda()
    d = torch.empty((len(q), cfg.k), dtype=torch.int32, device="cuda")
    s = torch.empty((len(q), cfg.k), dtype=torch.float32, device="cuda")
    h = len(q) // 2
    s0, s1 = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        base.search_device(dq[:h], cfg.k, d[:h], s[:h], s0)
        fork.search_device(dq[h:], cfg.k, d[h:], s[h:], s1)
    torch.cuda.synchronize()
    _exact((d.cpu().numpy(), s.cpu().numpy()), ref)
    with pytest.raises(ValueError, match="grid_pct"):
        base.set_option("grid_pct", 0)
    base.close()  # the fork keeps the arrays
    _exact(fork.search(q, cfg.k), ref)
    fork.close()


# ------------------------------------------------- round 6: stream order, close
def test_fork_first_search_fresh_stream_reallocates(gpu):
    """a (re)allocated workspace's claim counters are zeroed
    on the search's own stream, not on the null stream a non-blocking stream
    does not wait for.  A fresh fork's first search on a new non-blocking
    torch stream — and later searches on new streams with batches that force
    the workspace to grow — give the oracle's bits."""
    import torch
    from bm25mi import synth
    cfg = synth.Config("fs", 900_000, 4000, 7_000_000, 200, 8, 40)
    ip, ix, dt = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    ref = oracle.search_c(cfg.n_docs, ip, ix, dt, q, cfg.k)
    base = _idx(ip, ix, dt, cfg.n_docs)
    dq = torch.from_numpy(q).cuda()
    d = torch.empty((len(q), cfg.k), dtype=torch.int32, device="cuda")
    s = torch.empty((len(q), cfg.k), dtype=torch.float32, device="cuda")
    base.search_device(dq[:8], cfg.k, d[:8], s[:8], torch.cuda.Stream())
    torch.cuda.synchronize()
    for rows in (16, 64, len(q)):  # each a larger batch: the fork's workspace grows
        fork = base.fork()
        st = torch.cuda.Stream()
        assert st.query()  # a new non-blocking stream with nothing on it
        fork.search_device(dq[:rows], cfg.k, d[:rows], s[:rows], st)
        grow = base.fork()
        st2 = torch.cuda.Stream()
        grow.search_device(dq[:4], cfg.k, d[:4], s[:4], st2)
        grow.search_device(dq[:rows], cfg.k, d[:rows], s[:rows], st2)  # reallocates on st2
        torch.cuda.synchronize()
        _exact((d[:rows].cpu().numpy(), s[:rows].cpu().numpy()), (ref[0][:rows], ref[1][:rows]))
        fork.close()
        grow.close()
    base.close()


def test_close_releases_cached_forks(gpu):
    """GpuIndex.close() also closes the forks bm25mi.dist caches on
    the index (parts > 1), so the shared device arrays and every fork's
    workspace are released at close, not at garbage collection."""
    import gc
    import torch
    from bm25mi import synth
    from bm25mi.dist import _forks
    cfg = synth.Config("cl", 2_000_000, 5000, 30_000_000, 64, 8, 10)
    ip, ix, dt = synth.make_index(cfg)
    q = synth.make_queries(cfg)
    torch.cuda.synchronize()
    gc.collect()
    free0 = torch.cuda.mem_get_info()[0]
    index = _idx(ip, ix, dt, cfg.n_docs)
    ctxs = _forks(index, 3)
    assert len(ctxs) == 3 and index._bm25_forks
    for c in ctxs:
        c.search(q, cfg.k)
    held = free0 - torch.cuda.mem_get_info()[0]
    assert held > 200 << 20, held  # the index arrays (~300 MB) and three workspaces
    index.close()
    assert "_bm25_forks" not in index.__dict__ and all(c._h is None for c in ctxs)
    torch.cuda.synchronize()
    left = free0 - torch.cuda.mem_get_info()[0]
    assert left < 16 << 20, (held, left)


def test_gpu_execute_query_realistic_matrix(gpu):
    """gpu_execute_query (gpu_bm25/common.py:28-85) fed as
    the reference's driver feeds it (main.py:238-252) — bm25.py's fitted dense
    matrix cast to f32 (bm25_dense.npz, generated by the reference itself),
    query vectors from term_to_id with OOV terms mapped to id 0 — plus
    duplicate ids, negative ids (normalised as MAX gather does) and a
    corpus-sized sparse-ish dense matrix.  The top-1 index / weight match the
    oracle's top-1 on the same fp32 columns in query order.  Parity with MAX
    itself is unpinned (MAX is not importable here)."""
    import scipy.sparse as sp
    from gpu_bm25.common import gpu_execute_query
    g = _load("bm25_dense.npz")
    m = g["bm25_matrix"].astype(np.float32)
    term_to_id = {t: i for i, t in enumerate(g["vocabulary"].tolist())}
    cases = [[term_to_id.get(t, 0) for t in str(qs).lower().split()] for qs in g["queries"]]
    cases += [[term_to_id["fox"]] * 3 + [term_to_id["dog"]], [-1, 0, -2], [0, 0, 0, 0]]

    def check(mat, qv):
        qv = np.asarray(qv, np.int32)
        idx, w = gpu_execute_query(mat, qv, None, None)
        assert idx.shape == (1, 1) and idx.dtype == np.int64 and w.dtype == np.float32
        norm = np.where(qv < 0, qv + mat.shape[1], qv).astype(np.int32)
        c = sp.csc_matrix(mat)
        rd, rs = oracle.search_c(mat.shape[0], c.indptr, c.indices, c.data, norm[None, :], 1)
        assert idx.item() == int(rd[0, 0]) and w.view(np.uint32).item() == rs.view(np.uint32)[0, 0], \
            (qv, idx, w, rd, rs)

    for qv in cases:
        check(m, qv)
    rng = np.random.default_rng(66)
    big = rng.uniform(0.0, 4.0, (50_000, 300)).astype(np.float32)
    big[rng.random(big.shape) < 0.9] = 0.0
    for _ in range(4):
        qv = rng.integers(0, 300, size=6)
        qv[rng.random(6) < 0.3] = 0  # OOV -> 0
        check(big, qv)
    check(big, [17, 17, -300, -1])
