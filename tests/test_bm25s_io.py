"""The bm25s on-disk index format (bm25mi.bm25s_io): a directory written from
the reference's checked-in fixture (animal_index_bm25/, recorded in
tests/golden/animal.npz) loads back memory-mapped, validated, with the
token -> id mapping of its vocab.index.json."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

PARAMS = {"k1": 1.5, "b": 0.75, "delta": 0.5, "method": "lucene", "idf_method": "lucene",
          "dtype": "float32", "int_dtype": "int32", "num_docs": 4, "version": "0.2.12",
          "backend": "numpy"}  # params.index.json:1-11 of the fixture


def write_animal(d):
    g = np.load(os.path.join(GOLDEN, "animal.npz"), allow_pickle=False)
    for name in ("indptr", "indices", "data"):
        np.save(os.path.join(d, f"{name}.csc.index.npy"), g[name])
    with open(os.path.join(d, "params.index.json"), "w") as f:
        json.dump(PARAMS, f)
    vocab = dict(zip(g["vocab_keys"].tolist(), g["vocab_ids"].tolist()))
    with open(os.path.join(d, "vocab.index.json"), "w") as f:
        json.dump(vocab, f)
    texts = ["a cat is a feline and likes to purr", "a dog is the human's best friend and "
             "loves to play", "a bird is a beautiful animal that can fly",
             "a fish is a creature that lives in water and swims"]
    offs, pos = [], 0
    with open(os.path.join(d, "corpus.jsonl"), "wb") as f:
        for i, t in enumerate(texts):
            line = (json.dumps({"id": i, "text": t}) + "\n").encode()
            offs.append(pos)
            pos += len(line)
            f.write(line)
    with open(os.path.join(d, "corpus.mmindex.json"), "w") as f:
        json.dump(offs, f)
    return g, vocab


def test_load_animal_directory(tmp_path):
    from bm25mi.bm25s_io import load_bm25s, query_ids
    g, vocab = write_animal(str(tmp_path))
    ix = load_bm25s(str(tmp_path))
    assert isinstance(ix.indptr, np.memmap)
    assert ix.num_docs == 4 and ix.n_terms == 20
    assert np.array_equal(ix.data, g["data"]) and np.array_equal(ix.indices, g["indices"])
    assert ix.vocab == vocab
    # bm25_test.py:23 query, stemmed: fish purr like cat; "" (id 20) has no column
    q = query_ids([["fish", "purr", "like", "cat"], ["", "zzz"], ["dog"]], ix.vocab, ix.n_terms)
    assert q.tolist() == [[17, 16, 0, 2], [-1, -1, -1, -1], [19, -1, -1, -1]]
    assert np.array_equal(q[:1], g["q1_queries"])
    assert ix.document(3)["text"].startswith("a fish")
    assert len(ix.corpus()) == 4


def test_load_rejects_inconsistent_arrays(tmp_path):
    from bm25mi.bm25s_io import load_bm25s
    write_animal(str(tmp_path))
    np.save(os.path.join(str(tmp_path), "data.csc.index.npy"), np.zeros(3, np.float32))
    with pytest.raises(ValueError, match="indptr"):
        load_bm25s(str(tmp_path))


@pytest.mark.skipif(not os.path.isdir("/root/reference/animal_index_bm25"),
                    reason="the reference checkout is only in the build container")
def test_load_reference_fixture_directory():
    from bm25mi.bm25s_io import load_bm25s
    g = np.load(os.path.join(GOLDEN, "animal.npz"), allow_pickle=False)
    ix = load_bm25s("/root/reference/animal_index_bm25")
    assert ix.params["num_docs"] == 4 and ix.params["method"] == "lucene"
    for name in ("indptr", "indices", "data"):
        assert np.array_equal(getattr(ix, name), g[name])
    assert ix.document(0)["text"] == "a cat is a feline and likes to purr"


def test_shard_csc_int64_indptr_concatenates_to_full(tmp_path):
    """bm25mi.shard: a bm25s directory with an int64 indptr (the config-5
    form) cut into rank shards — every shard is canonical CSC with local ids,
    and the shards together are the whole index (small column blocks force
    the streaming path across block edges)."""
    from bm25mi import shard
    from bm25mi.bm25s_io import load_bm25s, save_bm25s
    rng = np.random.default_rng(5)
    N, V = 50_000, 300
    cols = [np.sort(rng.choice(N, int(rng.integers(0, 3000)), replace=False)) for _ in range(V)]
    ip = np.zeros(V + 1, np.int64)
    ip[1:] = np.cumsum([len(c) for c in cols])
    ix = np.concatenate(cols).astype(np.int32)
    dt = rng.random(ix.size).astype(np.float32)
    save_bm25s(str(tmp_path), ip, ix, dt, N, vocab={"a": 0})
    assert load_bm25s(str(tmp_path)).indptr.dtype == np.int64
    for W in (1, 3, 8):
        parts = []
        for r in range(W):
            sip, six, sdt, n, lo, _ = shard.load_bm25s_shard(str(tmp_path), r, W)
            assert sip.dtype == np.int64 and six.dtype == np.int32
            a, b = shard.shard_bounds(N, W, r)
            assert (lo, n) == (a, b - a)
            if six.size:
                assert six.min() >= 0 and six.max() < n
            parts.append((sip, six, sdt, lo))
            blk = shard.shard_csc(ip, ix, dt, a, b, block=777)
            assert all(np.array_equal(x, y) for x, y in zip(blk, (sip, six, sdt)))
        for t in range(V):
            d = np.concatenate([p[1][p[0][t]:p[0][t + 1]] + p[3] for p in parts])
            v = np.concatenate([p[2][p[0][t]:p[0][t + 1]] for p in parts])
            assert np.array_equal(d, ix[ip[t]:ip[t + 1]]) and np.array_equal(v, dt[ip[t]:ip[t + 1]])
