"""bm25s on-disk index format (§3D).

A bm25s index directory — what ``retriever.save(dir)`` writes
(bm25_test.py:35-38; the reference's fixture ``animal_index_bm25/``) — holds

  indptr.csc.index.npy   int32 (``int_dtype``) or int64, [V + 1]
  indices.csc.index.npy  int32, [nnz] doc ids, sorted per column
  data.csc.index.npy     float32 (``dtype``), [nnz] precomputed BM25 scores
  params.index.json      k1, b, delta, method, idf_method, dtype, int_dtype,
                         num_docs, version, backend (params.index.json:1-11)
  vocab.index.json       {token: id}; ids may exceed the CSC's column count
                         (the fixture's "" -> 20 has no column)
  corpus.jsonl + corpus.mmindex.json   optional documents + byte offsets

``load_bm25s`` memory-maps the three arrays (``numpy.load(mmap_mode="r")``,
never unpickling) and validates their shapes; ``open_index`` uploads them to a
GPU (the device build rejects unsorted / out-of-range doc ids);
``query_ids`` maps tokens to ids the way a caller of ``BM25v.search`` would;
``save_bm25s`` writes the same layout (e.g. from bm25mi.scoring's GPU build);
bm25mi.shard.load_bm25s_shard reads one rank's doc shard of it.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass
from typing import Dict, Iterable, List, Optional

import numpy as np

ARRAYS = ("indptr", "indices", "data")


@dataclass
class Bm25sIndex:
    indptr: np.ndarray
    indices: np.ndarray
    data: np.ndarray
    params: dict
    vocab: Dict[str, int]
    path: str

    @property
    def num_docs(self) -> int:
        return int(self.params["num_docs"])

    @property
    def n_terms(self) -> int:
        return int(self.indptr.size - 1)

    def corpus(self) -> Optional[List[dict]]:
        """The saved documents (corpus.jsonl), or None when not saved."""
        p = os.path.join(self.path, "corpus.jsonl")
        if not os.path.exists(p):
            return None
        with open(p, encoding="utf-8") as f:
            return [json.loads(line) for line in f if line.strip()]

    def document(self, i: int) -> Optional[dict]:
        """Document i through the byte-offset index (corpus.mmindex.json)."""
        pi = os.path.join(self.path, "corpus.mmindex.json")
        pc = os.path.join(self.path, "corpus.jsonl")
        if not (os.path.exists(pi) and os.path.exists(pc)):
            return None
        with open(pi) as f:
            offs = json.load(f)
        with open(pc, "rb") as f:
            f.seek(int(offs[i]))
            return json.loads(f.readline().decode("utf-8"))


def load_bm25s(path: str, mmap: bool = True) -> Bm25sIndex:
    """Read a bm25s index directory (arrays memory-mapped, not copied)."""
    with open(os.path.join(path, "params.index.json")) as f:
        params = json.load(f)
    vocab: Dict[str, int] = {}
    vp = os.path.join(path, "vocab.index.json")
    if os.path.exists(vp):
        with open(vp, encoding="utf-8") as f:
            vocab = {str(k): int(v) for k, v in json.load(f).items()}
    arrs = {}
    for name in ARRAYS:
        arrs[name] = np.load(os.path.join(path, f"{name}.csc.index.npy"),
                             mmap_mode="r" if mmap else None, allow_pickle=False)
    ip, ix, dt = arrs["indptr"], arrs["indices"], arrs["data"]
    if ip.ndim != 1 or ix.ndim != 1 or dt.ndim != 1 or ip.size < 1:
        raise ValueError(f"{path}: CSC arrays must be 1-D")
    if ip.dtype not in (np.int32, np.int64) or ix.dtype not in (np.int32, np.int64):
        raise ValueError(f"{path}: integer arrays must be int32/int64 (got {ip.dtype}, {ix.dtype})")
    if not np.issubdtype(dt.dtype, np.floating):
        raise ValueError(f"{path}: data must be floating point (got {dt.dtype})")
    nnz = int(ip[-1])
    if int(ip[0]) != 0 or ix.size != nnz or dt.size != nnz:
        raise ValueError(f"{path}: indptr[0]={int(ip[0])}, indptr[-1]={nnz}, "
                         f"indices {ix.size}, data {dt.size}")
    if "num_docs" not in params:
        raise ValueError(f"{path}: params.index.json has no num_docs")
    return Bm25sIndex(ip, ix, dt, params, vocab, path)


def save_bm25s(path: str, indptr, indices, data, num_docs: int,
               vocab: Optional[Dict[str, int]] = None, params: Optional[dict] = None,
               corpus: Optional[List[dict]] = None) -> None:
    """Write a bm25s index directory (the layout ``load_bm25s`` reads:
    ``.npy`` arrays without pickles, params/vocab JSON, optional corpus.jsonl
    + corpus.mmindex.json byte offsets).  ``indptr`` keeps its integer width
    (int64 once nnz passes 2^31)."""
    os.makedirs(path, exist_ok=True)
    ip = np.asarray(indptr)
    if ip.dtype not in (np.int32, np.int64):
        ip = ip.astype(np.int64)
    for name, arr in (("indptr", ip), ("indices", np.asarray(indices, np.int32)),
                      ("data", np.asarray(data, np.float32))):
        np.save(os.path.join(path, f"{name}.csc.index.npy"), arr, allow_pickle=False)
    prm = {"k1": 1.5, "b": 0.75, "delta": 0.5, "method": "lucene", "idf_method": "lucene",
           "dtype": "float32", "int_dtype": "int64" if ip.dtype == np.int64 else "int32",
           "num_docs": int(num_docs), "version": "0.2.12", "backend": "numpy"}
    prm.update(params or {})
    prm["num_docs"] = int(num_docs)
    with open(os.path.join(path, "params.index.json"), "w") as f:
        json.dump(prm, f, indent=4)
    with open(os.path.join(path, "vocab.index.json"), "w", encoding="utf-8") as f:
        json.dump(vocab or {}, f)
    if corpus is not None:
        offs = []
        with open(os.path.join(path, "corpus.jsonl"), "wb") as f:
            for doc in corpus:
                offs.append(f.tell())
                f.write((json.dumps(doc) + "\n").encode("utf-8"))
        with open(os.path.join(path, "corpus.mmindex.json"), "w") as f:
            json.dump(offs, f)


def open_index(path: str, device: int = 0):
    """Load a bm25s directory straight into HBM as a GpuIndex."""
    from .index import GpuIndex
    ix = load_bm25s(path)
    return GpuIndex(ix.indptr, ix.indices, ix.data, ix.num_docs, device=device)


def query_ids(queries: Iterable[Iterable[str]], vocab: Dict[str, int], n_terms: int,
              width: Optional[int] = None) -> np.ndarray:
    """Token lists -> int32 [Q, width] ids, -1 padded (BM25v padding,
    bm25_native.py:151); tokens absent from the vocabulary or without a CSC
    column (id >= n_terms) are dropped, as bm25s drops unknown query tokens."""
    rows = [[vocab[t] for t in q if t in vocab and vocab[t] < n_terms] for q in queries]
    w = width if width is not None else max([len(r) for r in rows] + [1])
    out = np.full((len(rows), w), -1, np.int32)
    for i, r in enumerate(rows):
        r = r[:w]
        out[i, :len(r)] = r
    return out
