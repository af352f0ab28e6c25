"""CPU tests of the host side: the C-ABI library loads and exports every
symbol of include/bm25mi.h, error paths that need no GPU, the synthetic
generator, and the drop-in modules' validation (which runs before any GPU
call)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import gpu_available


def test_lib_exports_every_header_symbol():
    from bm25mi import _capi
    syms = _capi.header_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(_capi.lib, s), s
    assert _capi.abi_version() == 1


def test_header_abi_define_matches():
    from bm25mi import _capi
    text = open(_capi.HEADER).read()
    assert "#define BM25MI_ABI_VERSION 1" in text


def test_device_count_never_fails():
    from bm25mi import _capi
    assert _capi.device_count() >= 0


@pytest.mark.skipif(gpu_available(), reason="exercises the no-GPU error path")
def test_create_without_gpu_fails_loudly():
    from bm25mi.index import GpuIndex
    from bm25mi._capi import HipError
    with pytest.raises(HipError, match="no HIP device"):
        GpuIndex(np.array([0, 1], np.int32), np.array([0], np.int32),
                 np.array([1.0], np.float32), 1)


def test_create_argument_validation():
    from bm25mi._capi import lib, BM25_EINVAL
    h = ctypes.c_void_p()
    ip = np.array([0, 2, 1], np.int64)  # decreasing
    ix = np.array([0, 1], np.int32)
    dt = np.ones(2, np.float32)
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    rc = lib.bm25_index_create(0, 4, 2, 1, p(ip), 1, p(ix), p(dt), 0, ctypes.byref(h))
    assert rc == BM25_EINVAL
    assert b"indptr" in lib.bm25_last_error()
    rc = lib.bm25_index_create(0, -1, 2, 1, p(ip), 1, p(ix), p(dt), 0, ctypes.byref(h))
    assert rc == BM25_EINVAL


def test_merge_rejects_bad_shape():
    from bm25mi._capi import lib, BM25_EINVAL
    assert lib.bm25_merge_topk_device(0, None, None, 0, 1, 1, None, None, None) == BM25_EINVAL


# ----------------------------------------------------------------- synth
def test_synth_deterministic_and_canonical():
    from bm25mi import synth
    cfg = synth.Config("t", 50_000, 3000, 150_000, 8, 8, 10)
    a = synth.make_index(cfg)
    b = synth.make_index(cfg, threads=3)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    indptr, indices, data = a
    assert abs(int(indptr[-1]) - cfg.nnz) < 0.05 * cfg.nnz
    for t in range(0, 3000, 97):
        col = indices[indptr[t]:indptr[t + 1]]
        assert np.all(np.diff(col) > 0) and (col.size == 0 or (col[0] >= 0 and col[-1] < 50_000))
    assert np.all(data > 0)


def test_synth_shards_concatenate_to_full():
    from bm25mi import synth
    cfg = synth.Config("t", 70_000, 500, 100_000, 4, 4, 5)
    full = synth.make_index(cfg)
    parts = [synth.make_index(cfg, *synth.shard_bounds(cfg.n_docs, 3, r)) for r in range(3)]
    for t in range(500):
        col = full[1][full[0][t]:full[0][t + 1]]
        vals = full[2][full[0][t]:full[0][t + 1]]
        got, gv = [], []
        for r, (ip, ix, dt) in enumerate(parts):
            lo, _ = synth.shard_bounds(cfg.n_docs, 3, r)
            got.append(ix[ip[t]:ip[t + 1]] + lo)
            gv.append(dt[ip[t]:ip[t + 1]])
        assert np.array_equal(np.concatenate(got), col)
        assert np.array_equal(np.concatenate(gv), vals)


def test_synth_queries_distinct_terms():
    from bm25mi import synth
    cfg = synth.CONFIGS["c2"]
    q = synth.make_queries(cfg)
    assert q.shape == (256, 8) and q.dtype == np.int32
    assert all(len(set(r)) == 8 for r in q.tolist())
    assert q.min() >= 0 and q.max() < cfg.n_terms


def test_shard_bounds_cover():
    from bm25mi import synth
    for w in (1, 2, 4, 8):
        b = [synth.shard_bounds(10_000_000, w, r) for r in range(w)]
        assert b[0][0] == 0 and b[-1][1] == 10_000_000
        assert all(b[i][1] == b[i + 1][0] for i in range(w - 1))


# ----------------------------------------------------------- drop-in shims
def test_bm25v_empty_batch_no_gpu():
    import bm25_native
    m = bm25_native.BM25v()
    d, s = m.search([], top_k=10)
    assert d.shape == (0, 0) and s.shape == (0, 0)
    assert d.dtype == np.float32 and s.dtype == np.float32  # as bm25_native.py:96-98


def test_bm25v_validation_before_gpu():
    import bm25_native
    m = bm25_native.BM25v()
    with pytest.raises(ValueError, match="list of list"):
        m.search(np.array([[1, 2]], np.int64), 3)
    with pytest.raises(ValueError, match="list of list"):
        m.search([[1, 2]], 3)
    with pytest.raises(ValueError, match=r"maximum token ID in the query \(5\)"):
        m.search(np.array([[5, -1]], np.int32), 3)
    with pytest.raises(IndexError):
        m.search(np.zeros((2, 0), np.int32), 3)


def test_gpu_execute_query_validates_indices():
    from gpu_bm25.common import gpu_execute_query
    with pytest.raises(ValueError, match="out of range"):
        gpu_execute_query(np.ones((3, 2), np.float32), np.array([2], np.int32), None, None)


@pytest.mark.skipif(gpu_available(), reason="exercises the no-GPU error path")
def test_sharded_create_without_gpu_fails_loudly():
    from bm25mi.index import ShardedIndex
    from bm25mi._capi import HipError
    with pytest.raises(HipError, match="no HIP device"):
        ShardedIndex(np.array([0, 1], np.int32), np.array([0], np.int32),
                     np.array([1.0], np.float32), 1, devices=[0, 0])


def test_bm25_fit_builds_on_the_gpu_only():
    """bm25.BM25.fit builds its matrix with bm25_build_scores: without a GPU
    it fails loudly (no host fallback); the matrix itself is checked against
    the reference in tests/test_gpu_parity.py."""
    import os
    import bm25
    from bm25mi._capi import HipError
    from conftest import GOLDEN
    g = np.load(os.path.join(GOLDEN, "bm25_dense.npz"), allow_pickle=False)
    corpus = [d.lower().split() for d in g["docs"].tolist()]
    m = bm25.BM25()
    if not gpu_available():
        with pytest.raises(HipError, match="no HIP device"):
            m.fit(corpus)
    assert m.vocabulary == g["vocabulary"].tolist()
    assert bm25.BM25().get_top_n(["x"], corpus, n=0) == []
    e = bm25.BM25()
    e.fit([])
    assert e.get_scores(["a"]).shape == (0,)


def test_build_scores_validation_without_gpu():
    from bm25mi.scoring import build_scores
    with pytest.raises(ValueError, match="method"):
        build_scores([0], [0], [1.0], [1], 1, method="okapi")
    with pytest.raises(ValueError, match="same length"):
        build_scores([0, 1], [0], [1.0], [1, 1], 1)


def test_synth_weight_modes_share_postings():
    """The side-line weightings (bench --config c3u / c3l) keep config 3's
    postings: same indptr/indices, uniform values in [0.05, 3], term
    frequencies 1 + Poisson(0.6) (mean 1.6), all deterministic."""
    from bm25mi import synth
    cfg = synth.Config("t", 60_000, 900, 300_000, 8, 6, 10)
    a = synth.make_index(cfg)
    u = synth.make_index(synth.Config(*list(cfg.__dict__.values())[:-1], weights="uniform"))
    assert np.array_equal(a[0], u[0]) and np.array_equal(a[1], u[1])
    assert u[2].min() >= 0.05 and u[2].max() <= 3.0 and not np.array_equal(a[2], u[2])
    ip, ix, tf = synth._fill(cfg, 0, None, 0, synth.WEIGHTS["tf"])
    assert np.array_equal(ip, a[0]) and np.all(tf >= 1) and np.all(tf == np.round(tf))
    assert abs(float(tf.mean()) - 1.6) < 0.02
    assert np.array_equal(tf, synth._fill(cfg, 0, None, 0, synth.WEIGHTS["tf"])[2])


def test_capi_host_asan():
    """SURVEY.md:235 / VERDICT r4 item 8: the C-ABI's host code under
    AddressSanitizer.  tests/asan/host_check.cpp drives every argument check,
    error path and NULL-handle rejection of include/bm25mi.h (here, with no GPU
    visible, the device calls end in EHIP); ASan aborts the run on any
    out-of-bounds access or use-after-free of the host side."""
    import subprocess
    from bm25mi.build import build_asan_check
    exe = build_asan_check()
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0 and "AddressSanitizer" not in r.stderr, (r.stdout, r.stderr[-2000:])
    assert "asan host check ok" in r.stdout
