"""Generate the golden vectors of tests/golden/ from the REFERENCE itself.

Runs only in the build container, where the reference checkout is mounted
read-only at /root/reference: it imports the reference's bm25_native.py
(BM25v, bm25_native.py:32-214) and records inputs + outputs as .npz files.
Nothing of the reference's source is copied; the GPU box never runs this.

  python tests/golden/make_golden.py [/root/reference]

Fixtures
  animal.npz     the checked-in bm25s index animal_index_bm25/ (its
                 indptr/indices/data arrays and params), queries derived from
                 bm25_test.py:23 through vocab.index.json, outputs of
                 BM25v.search, plus the two error messages
  main_demo.npz  bm25_native.py:219-248 (2x3 dense -> CSC, query [[0,1]], k=1)
  bm25_near_ties.npz  a seeded corpus + queries where the reference's float64
                 ranking differs from fp32 sums' (bm25.BM25 must rank in f64)
  bm25_dense.npz the reference's dense BM25 model (bm25.py:6-178) fitted on
                 its own __main__ corpus (bm25.py:182-196): bm25_matrix, and
                 get_scores / get_top_n(n=5) of a few queries (OOV, duplicate
                 terms, duplicate documents -> tied scores)
  synth_small.npz  numpy-seeded 3000-doc / 400-term index; 48 queries with -1
                 padding, duplicate tokens, all-padding rows and rare-term rows
                 (zero-fill); k in {1, 10, 100}; outputs + `tied` masks computed
                 from the reference's full dense score vectors
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

REF = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
import scipy.sparse as sp  # noqa: E402

import bm25_native as bn  # noqa: E402  (the reference)


def run(m, queries, k):
    model = bn.BM25v()
    model.index(m, np.ones(m.shape[0], np.int32))
    return model.search(np.asarray(queries, np.int32), top_k=k)


def dense_rows(m, queries):
    rows = []
    for q in np.asarray(queries):
        q = q[q >= 0]
        rows.append(np.asarray(m[:, q].sum(axis=1)).ravel().astype(np.float32))
    return rows


def tied(rows, scores):
    t = np.zeros(scores.shape, bool)
    for i, d in enumerate(rows):
        vals, counts = np.unique(d, return_counts=True)
        c = dict(zip(vals.tolist(), counts.tolist()))
        for j, s in enumerate(scores[i]):
            t[i, j] = c.get(float(s), 0) > 1
    return t


def err_msg(m, queries, k):
    try:
        run(m, queries, k)
    except Exception as e:  # noqa: BLE001
        return f"{type(e).__name__}: {e}"
    return ""


def animal():
    d = os.path.join(REF, "animal_index_bm25")
    indptr = np.load(os.path.join(d, "indptr.csc.index.npy"))
    indices = np.load(os.path.join(d, "indices.csc.index.npy"))
    data = np.load(os.path.join(d, "data.csc.index.npy"))
    params = json.load(open(os.path.join(d, "params.index.json")))
    vocab = json.load(open(os.path.join(d, "vocab.index.json")))
    n = params["num_docs"]
    V = len(indptr) - 1
    m = sp.csc_matrix((data, indices, indptr), shape=(n, V))
    # bm25_test.py:23 "does the fish purr like a cat?" after stemming/stopwords
    q1 = [vocab["fish"], vocab["purr"], vocab["like"], vocab["cat"]]
    out = {"indptr": indptr, "indices": indices, "data": data, "n_docs": np.int64(n),
           "vocab_keys": np.array(list(vocab.keys())), "vocab_ids": np.array(list(vocab.values()))}
    cases = [
        ("q1", [q1], 2),
        ("dup", [[vocab["cat"], vocab["cat"]]], 1),
        ("pad", [[-1, -1]], 3),
        ("batch", [q1, [vocab["cat"], vocab["cat"], -1, -1], [vocab["dog"], 3, 5, 7],
                   [-1, -1, -1, -1], [vocab["bird"], -5, vocab["swim"], vocab["fish"]]], 4),
        ("allk", [[vocab["dog"], vocab["bird"]]], 4),
    ]
    for name, q, k in cases:
        q = np.asarray(q, np.int32)
        docs, scores = run(m, q, k)
        rows = dense_rows(m, q)
        out[f"{name}_queries"] = q
        out[f"{name}_k"] = np.int64(k)
        out[f"{name}_docs"] = docs
        out[f"{name}_scores"] = scores
        out[f"{name}_tied"] = tied(rows, scores)
        out[f"{name}_dense"] = np.stack(rows)
    out["err_token"] = np.array(err_msg(m, np.array([[V]], np.int32), 1))
    out["err_k"] = np.array(err_msg(m, np.array([[0]], np.int32), n + 1))
    e_docs, e_scores = run(m, np.zeros((0, 4), np.int32), 3)
    out["empty_docs_dtype"] = np.array(str(e_docs.dtype))
    out["empty_shape"] = np.array(e_docs.shape)
    np.savez(os.path.join(OUT, "animal.npz"), **out)


def main_demo():
    dense = np.array([[1.0, 2.0, 3.0], [2.0, 4.0, 1.0]], np.float32)
    m = sp.csc_matrix(dense, dense.shape, dtype=np.float32)
    docs, scores = run(m, np.array([[0, 1]], np.int32), 1)
    np.savez(os.path.join(OUT, "main_demo.npz"), dense=dense, queries=np.array([[0, 1]], np.int32),
             docs=docs, scores=scores)


def synth_small():
    rng = np.random.default_rng(20250620)
    N, V = 3000, 400
    cols_i, cols_d, indptr = [], [], [0]
    for t in range(V):
        df = int(min(N // 2, max(1, round(600 / (t + 1) ** 0.9))))
        docs = np.sort(rng.choice(N, size=df, replace=False)).astype(np.int32)
        idf = np.float32(np.log(1 + (N - df + 0.5) / (df + 0.5)))
        # coarse values (multiples of 1/64) create exact score ties on purpose
        vals = (idf * (np.floor(rng.uniform(0.1, 1.0, df) * 64) / 64)).astype(np.float32)
        cols_i.append(docs)
        cols_d.append(vals)
        indptr.append(indptr[-1] + df)
    indptr = np.array(indptr, np.int32)
    indices = np.concatenate(cols_i)
    data = np.concatenate(cols_d)
    m = sp.csc_matrix((data, indices, indptr), shape=(N, V))
    Q, T = 48, 8
    p = np.diff(indptr).astype(np.float64) ** 0.75
    p /= p.sum()
    q = rng.choice(V, size=(Q, T), p=p).astype(np.int32)
    q[0:8, 6:] = -1                      # padding
    q[8:12, 1] = q[8:12, 0]              # duplicate tokens (counted twice)
    q[12, :] = -1                        # all padding
    q[13, :] = [V - 1, V - 2, -1, -1, -1, -1, -1, -1]  # rare terms -> zero-fill
    q[14, :] = [V - 3] * 8               # same rare term 8 times
    q[15, :] = -7                        # any negative id is padding
    out = {"indptr": indptr, "indices": indices, "data": data, "n_docs": np.int64(N),
           "queries": q}
    rows = dense_rows(m, q)
    for k in (1, 10, 100):
        docs, scores = run(m, q, k)
        out[f"docs_k{k}"] = docs
        out[f"scores_k{k}"] = scores
        out[f"tied_k{k}"] = tied(rows, scores)
    out["dense0"] = rows[0]
    out["dense8"] = rows[8]
    np.savez_compressed(os.path.join(OUT, "synth_small.npz"), **out)


def bm25_dense():
    import bm25 as ref_bm25  # the reference's dense model (pure numpy)
    docs = [
        "The quick brown fox jumps over the lazy dog",
        "Some other text",
        "The quick rabbit runs past the brown fox",
        "The quick rabbit jumps over the brown dog",
        "The quick dog chases past the lazy fox",
        "The quick dog runs through the tall trees",
        "The quick brown fox jumps over the lazy dog",
        "The brown dog sleeps under the shady tree",
        "The brown rabbit hops under the tall tree",
        "The brown fox runs through the forest trees",
        "The brown fox watches the sleeping rabbit",
        "The lazy fox watches over the sleeping dog",
        "The lazy dog watches the quick rabbit",
    ]  # bm25.py:182-196
    corpus = [d.lower().split() for d in docs]
    queries = ["quick brown fox", "lazy dog", "sleeping rabbit tree", "fox fox fox",
               "unknown words only", "the", "tall trees shady forest watches"]
    model = ref_bm25.BM25()
    model.fit(corpus)
    out = {"docs": np.array(docs), "queries": np.array(queries),
           "bm25_matrix": model.bm25_matrix, "vocabulary": np.array(model.vocabulary)}
    for i, q in enumerate(queries):
        toks = q.lower().split()
        out[f"scores_{i}"] = np.asarray(model.get_scores(toks))
        top = model.get_top_n(toks, corpus, n=5)
        out[f"top_scores_{i}"] = np.array([t[0] for t in top], np.float64)
        # the returned documents, as corpus indices (duplicate documents: first match)
        out[f"top_docs_{i}"] = np.array([corpus.index(t[1]) for t in top], np.int64)
    np.savez(os.path.join(OUT, "bm25_dense.npz"), **out)


def bm25_near_ties():
    """bm25_near_ties.npz: a seeded random corpus (2000 docs over 30 words) and
    queries whose float64 ranking (the reference's get_top_n) differs from the
    ranking of the same sums in fp32: two documents whose float64 scores are
    distinct but round to one fp32 value (found by search, seed 2024)."""
    import bm25 as ref_bm25
    rng = np.random.default_rng(2024)
    words = [f"w{i}" for i in range(30)]
    for attempt in range(200):
        corpus = [list(rng.choice(words, size=int(rng.integers(3, 12)))) for _ in range(2000)]
        model = ref_bm25.BM25()
        model.fit(corpus)
        m32 = model.bm25_matrix.astype(np.float32)
        ar = np.arange(len(corpus))
        hits, queries = [], []
        for _ in range(40):
            q = [str(w) for w in rng.choice(words, size=int(rng.integers(2, 6)))]
            s64 = model.get_scores(q)
            s32 = np.zeros(len(corpus), np.float32)
            for t in q:
                s32 = s32 + m32[:, model.term_to_id[t]]
            o64 = np.lexsort((ar, -s64))[:20]
            o32 = np.lexsort((ar, -s32.astype(np.float64)))[:20]
            vals, c = np.unique(s64, return_counts=True)
            rep = dict(zip(vals.tolist(), c.tolist()))
            if any(o64[j] != o32[j] and rep[s64[o64[j]]] == 1 for j in range(20)):
                hits.append(len(queries))
            queries.append(" ".join(q))
        if hits:
            break
    out = {"docs": np.array([" ".join(d) for d in corpus]), "queries": np.array(queries),
           "fp32_differs": np.array(hits, np.int64)}
    for i, q in enumerate(queries):
        toks = q.split()
        out[f"scores_{i}"] = np.asarray(model.get_scores(toks))
        top = model.get_top_n(toks, corpus, n=20)
        out[f"top_scores_{i}"] = np.array([t[0] for t in top], np.float64)
        out[f"top_docs_{i}"] = np.array([corpus.index(t[1]) for t in top], np.int64)
    np.savez_compressed(os.path.join(OUT, "bm25_near_ties.npz"), **out)


if __name__ == "__main__":
    bm25_near_ties()
    bm25_dense()
    animal()
    main_demo()
    synth_small()
    print("wrote", sorted(f for f in os.listdir(OUT) if f.endswith(".npz")))
