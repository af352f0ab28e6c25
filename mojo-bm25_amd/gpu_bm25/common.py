"""Drop-in replacement of the reference's ``gpu_bm25.common`` module.

``gpu_execute_query`` keeps the signature and results of
gpu_bm25/common.py:28-85 (called by main.py:250, results read with
``.item()`` at main.py:251-252): a dense [num_docs, vocab] f32 score matrix
and an int32 query vector in, the top-1 ``(index[1, 1], weight[1, 1])`` out.

The reference builds and compiles a MAX graph per call
(ops.gather -> ops.sum -> ops.top_k over the dense matrix, :40-84).  Here the
dense matrix becomes a CSC index (zeros dropped — they add nothing to a sum)
and the query runs through the same HIP kernels as BM25v.search with k = 1.
``session`` / ``device`` are accepted for signature compatibility; ``device``
may be an int GPU ordinal.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np
import scipy.sparse as sp

from bm25mi.index import GpuIndex


def gpu_execute_query(score_matrix, query_vector, session=None, device=None,
                      ) -> Tuple[np.ndarray, np.ndarray]:
    m = np.asarray(score_matrix, dtype=np.float32)
    if m.ndim != 2:
        raise ValueError("score_matrix must be [num_docs, num_terms]")
    n_docs, n_terms = m.shape
    q = np.asarray(query_vector).astype(np.int64).ravel()
    # MAX gather normalises negative indices (gather_scatter.mojo normalize_neg_index)
    q = np.where(q < 0, q + n_terms, q)
    if q.size and (q.min() < 0 or q.max() >= n_terms):
        raise ValueError(f"gather index out of range for axis of size {n_terms}")
    dev = device if isinstance(device, int) else 0
    index = GpuIndex.from_csc(sp.csc_matrix(m), device=dev)
    try:
        docs, scores = index.search(q.astype(np.int32)[None, :], 1)
    finally:
        index.close()
    # ops.top_k returns int64 indices and f32 values of shape [1, 1]
    return docs.astype(np.int64), scores
