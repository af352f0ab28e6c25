"""CPU tests: pin the oracle to the reference (golden vectors made by importing
bm25_native.py, tests/golden/make_golden.py) and to the top-k KATs of
test_topk.mojo.  No GPU needed."""
import os

import numpy as np
import pytest

from conftest import GOLDEN
from oracle import oracle


def _load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


ANIMAL_CASES = ["q1", "dup", "pad", "batch", "allk"]


@pytest.mark.parametrize("case", ANIMAL_CASES)
@pytest.mark.parametrize("impl", ["c", "numpy", "faithful"])
def test_animal_golden(case, impl):
    g = _load("animal.npz")
    n = int(g["n_docs"])
    q, k = g[f"{case}_queries"], int(g[f"{case}_k"])
    fn = {"c": oracle.search_c, "numpy": oracle.search_numpy,
          "faithful": oracle.search_faithful}[impl]
    docs, scores = fn(n, g["indptr"], g["indices"], g["data"], q, k)
    assert docs.dtype == np.int32 and scores.dtype == np.float32
    bad = oracle.compare_topk(docs, scores, g[f"{case}_docs"], g[f"{case}_scores"],
                              tied=g[f"{case}_tied"], atol=0.0)
    assert not bad, bad


def test_animal_dense_bit_exact():
    g = _load("animal.npz")
    n = int(g["n_docs"])
    for case in ANIMAL_CASES:
        for i, row in enumerate(g[f"{case}_queries"]):
            ref = g[f"{case}_dense"][i]
            c = oracle.scores_dense_c(n, g["indptr"], g["indices"], g["data"], row)
            npy = oracle.scores_dense_numpy(n, g["indptr"], g["indices"], g["data"], row)
            assert np.array_equal(c.view(np.uint32), ref.view(np.uint32))
            assert np.array_equal(npy.view(np.uint32), ref.view(np.uint32))


def test_animal_known_values():
    # query "does the fish purr like a cat?" -> [[0, 3]]
    g = _load("animal.npz")
    d, s = oracle.search_c(int(g["n_docs"]), g["indptr"], g["indices"], g["data"],
                           np.array([[17, 16, 0, 2]], np.int32), 2)
    assert d.tolist() == [[0, 3]]
    assert s.tolist() == [[np.float32(1.5876564), np.float32(0.48158914)]]
    d, s = oracle.search_c(int(g["n_docs"]), g["indptr"], g["indices"], g["data"],
                           np.array([[2, 2]], np.int32), 1)
    assert d.tolist() == [[0]] and s[0, 0] == np.float32(1.0584376)


def test_animal_error_messages_recorded():
    g = _load("animal.npz")
    assert str(g["err_token"]).startswith("ValueError: The maximum token ID in the query (20)")
    assert str(g["err_k"]) == "ValueError: kth(=-1) out of bounds (4)"
    assert str(g["empty_docs_dtype"]) == "float32" and g["empty_shape"].tolist() == [0, 0]


def test_main_demo():
    import scipy.sparse as sp
    g = _load("main_demo.npz")
    m = sp.csc_matrix(g["dense"])
    for fn in (oracle.search_c, oracle.search_numpy, oracle.search_faithful):
        d, s = fn(m.shape[0], m.indptr, m.indices, m.data, g["queries"], 1)
        assert d.tolist() == g["docs"].tolist() == [[1]]
        assert s.tolist() == g["scores"].tolist() == [[6.0]]


@pytest.mark.parametrize("k", [1, 10, 100])
@pytest.mark.parametrize("impl", ["c", "numpy", "faithful"])
def test_synth_small_golden(k, impl):
    g = _load("synth_small.npz")
    fn = {"c": oracle.search_c, "numpy": oracle.search_numpy,
          "faithful": oracle.search_faithful}[impl]
    docs, scores = fn(int(g["n_docs"]), g["indptr"], g["indices"], g["data"], g["queries"], k)
    bad = oracle.compare_topk(docs, scores, g[f"docs_k{k}"], g[f"scores_k{k}"],
                              tied=g[f"tied_k{k}"], atol=0.0)
    assert not bad, bad[:5]
    # scores bit-identical (same fp32 additions, same order)
    assert np.array_equal(scores.view(np.uint32), g[f"scores_k{k}"].view(np.uint32))


def test_synth_small_dense_bit_exact():
    g = _load("synth_small.npz")
    for i, key in ((0, "dense0"), (8, "dense8")):
        c = oracle.scores_dense_c(int(g["n_docs"]), g["indptr"], g["indices"], g["data"],
                                  g["queries"][i])
        assert np.array_equal(c.view(np.uint32), g[key].view(np.uint32))


def test_c_matches_numpy_canonical_exactly():
    g = _load("synth_small.npz")
    a = oracle.search_c(int(g["n_docs"]), g["indptr"], g["indices"], g["data"], g["queries"], 100)
    b = oracle.search_numpy(int(g["n_docs"]), g["indptr"], g["indices"], g["data"],
                            g["queries"], 100)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


# test_topk.mojo KATs for the tie / order rule adopted (MAX CPU top-k)
def test_topk_kat_1d_sorted():  # test_topk.mojo:152-161
    d, s = oracle.topk_c(np.arange(10, dtype=np.float32), 5)
    assert s.tolist() == [9, 8, 7, 6, 5] and d.tolist() == [9, 8, 7, 6, 5]


def test_topk_kat_identical():  # test_topk.mojo:222-238: ties -> ascending index
    d, s = oracle.topk_c(np.ones(4, np.float32), 3)
    assert d.tolist() == [0, 1, 2]
    d, s = oracle.topk_c(np.ones(33, np.float32), 3)
    assert d.tolist() == [0, 1, 2] and s.tolist() == [1, 1, 1]
    d, s = oracle.topk_numpy(np.ones(33, np.float32), 3)
    assert d.tolist() == [0, 1, 2]


def test_topk_kat_max_k():  # test_topk.mojo:240-248 (one column of the 3x4 iota)
    d, s = oracle.topk_c(np.array([0, 4, 8], np.float32), 3)
    assert d.tolist() == [2, 1, 0] and s.tolist() == [8, 4, 0]


def test_c_vs_faithful_random_untied():
    rng = np.random.default_rng(5)
    N, V = 5000, 300
    indptr = [0]
    idx, dat = [], []
    for t in range(V):
        df = int(rng.integers(1, 400))
        idx.append(np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
        dat.append(rng.uniform(0.1, 5.0, df).astype(np.float32))
        indptr.append(indptr[-1] + df)
    indptr = np.array(indptr, np.int64)
    indices, data = np.concatenate(idx), np.concatenate(dat)
    q = rng.integers(-1, V, size=(40, 6)).astype(np.int32)
    a = oracle.search_c(N, indptr, indices, data, q, 20)
    b = oracle.search_faithful(N, indptr, indices, data, q, 20)
    assert not oracle.compare_topk(*a, *b, atol=0.0)
    assert np.array_equal(a[1].view(np.uint32), b[1].view(np.uint32))


def test_faithful_k_too_large_raises():
    g = _load("animal.npz")
    with pytest.raises(ValueError, match="out of bounds"):
        oracle.search_faithful(4, g["indptr"], g["indices"], g["data"],
                               np.array([[0]], np.int32), 5)


def _animal_triples():
    """(doc, term, tf=1) triples and document lengths of animal_index_bm25
    (every term occurs once per document there: dl = postings per doc)."""
    g = np.load(os.path.join(GOLDEN, "animal.npz"), allow_pickle=False)
    ip, ix = g["indptr"].astype(np.int64), g["indices"]
    terms = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
    dl = np.bincount(ix, minlength=int(g["n_docs"]))
    return g, ix, terms, np.ones(len(ix), np.float32), dl


def test_build_scores_lucene_restatement_matches_fixture():
    """The lucene build rule (bm25s writer) reproduces every value of
    animal_index_bm25/data.csc.index.npy bit for bit."""
    g, docs, terms, tfs, dl = _animal_triples()
    ip, ix, d32, _ = oracle.build_scores_numpy(docs, terms, tfs, dl, len(g["indptr"]) - 1,
                                               1.5, 0.75, "lucene", float(np.mean(dl)))
    assert np.array_equal(ip, g["indptr"]) and np.array_equal(ix, g["indices"])
    assert np.array_equal(d32.view(np.uint32), g["data"].view(np.uint32))


def test_build_scores_bm25py_restatement_matches_reference_matrix():
    """The bm25.py build rule reproduces the reference's float64 bm25_matrix
    (golden bm25_dense.npz, generated by importing bm25.py) bit for bit."""
    from collections import Counter
    import scipy.sparse as sp
    g = np.load(os.path.join(GOLDEN, "bm25_dense.npz"), allow_pickle=False)
    corpus = [d.lower().split() for d in g["docs"].tolist()]
    tid = {t: i for i, t in enumerate(g["vocabulary"].tolist())}
    docs, terms, tfs = [], [], []
    for i, d in enumerate(corpus):
        for t, c in Counter(d).items():
            docs.append(i), terms.append(tid[t]), tfs.append(c)
    dl = [len(d) for d in corpus]
    ip, ix, _, d64 = oracle.build_scores_numpy(docs, terms, tfs, dl, len(tid), 1.5, 0.75,
                                               "bm25py", np.mean(dl))
    m = sp.csc_matrix((d64, ix, ip), shape=(len(corpus), len(tid))).toarray()
    assert np.array_equal(m, g["bm25_matrix"])


def _bm25_corpus_csc(docs_text, vocab=None):
    """The bm25.py matrix (build_scores_numpy "bm25py") of a text corpus as
    CSC with its float64 values; vocab = sorted words (bm25.py:73)."""
    from collections import Counter
    corpus = [d.lower().split() for d in docs_text]
    vocab = sorted({t for d in corpus for t in d}) if vocab is None else vocab
    tid = {t: i for i, t in enumerate(vocab)}
    docs, terms, tfs = [], [], []
    for i, d in enumerate(corpus):
        for t, c in Counter(d).items():
            docs.append(i), terms.append(tid[t]), tfs.append(c)
    dl = [len(d) for d in corpus]
    ip, ix, _, d64 = oracle.build_scores_numpy(docs, terms, tfs, dl, len(vocab), 1.5, 0.75,
                                               "bm25py", float(np.mean(dl)))
    return corpus, tid, ip, ix, d64


@pytest.mark.parametrize("name", ["bm25_dense.npz", "bm25_near_ties.npz"])
def test_bm25_f64_scores_restatement_matches_reference(name):
    """oracle.scores_f64 (bm25.py:143's column-by-column float64 sum, restated
    on the CSC) reproduces the reference's get_scores bit for bit, and
    oracle.topn_f64 its get_top_n scores — on the reference's own corpus and on
    the near-tie corpus whose fp32 ranking differs from float64's."""
    g = np.load(os.path.join(GOLDEN, name), allow_pickle=False)
    corpus, tid, ip, ix, d64 = _bm25_corpus_csc(g["docs"].tolist())
    for i, q in enumerate(g["queries"].tolist()):
        ids = [tid[t] for t in q.lower().split() if t in tid]
        s = oracle.scores_f64(len(corpus), ip, ix, d64, ids)
        assert np.array_equal(s.view(np.uint64), g[f"scores_{i}"].view(np.uint64)), (name, q)
        n = len(g[f"top_scores_{i}"])
        d, sc = oracle.topn_f64(s, n)
        assert np.array_equal(sc, g[f"top_scores_{i}"])
    if name == "bm25_near_ties.npz":
        assert len(g["fp32_differs"]) > 0


def test_bm25_f64_one_document_corpus_is_pairwise():
    """A one-document corpus: numpy sums the one gathered row pairwise (T >=
    8 differs from the in-order sum), and the restatement follows it."""
    rng = np.random.default_rng(3)
    v = rng.random(40) * 7
    ip = np.arange(41, dtype=np.int64)
    ix = np.zeros(40, np.int32)
    for T in (3, 8, 9, 17, 40):
        ids = list(rng.integers(0, 40, T))
        want = np.sum(v[None, :][:, ids], axis=1)
        got = oracle.scores_f64(1, ip, ix, v, ids)
        assert np.array_equal(got, want), T
