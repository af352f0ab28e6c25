"""Dev probe: the REST tile skip on test_tile_bound_skips_exact's index —
pairs and postings skipped per setting (band width, padding row, k)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
from bm25mi.index import GpuIndex
T = 4
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
os.environ["BM25_SEGMENTS"] = "dense"
index = GpuIndex(ip, ix, dt, N)
print("info", index.info(), flush=True)
for name, qq, opts in (("all", q, {}), ("no-pad", q[1:], {}), ("bw8", q, {"flat_bw": 8}),
                       ("bw1", q, {"flat_bw": 1}), ("one", q[1:2], {})):
    for kk, v in opts.items():
        index.set_option(kk, v)
    for k in (10, 100):
        index.search(qq, k)
        print(name, k, index.last_dispatch(), index.search_stats(), flush=True)
    for kk in opts:
        index.set_option(kk, 0)
