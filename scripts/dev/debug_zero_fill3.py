"""Dev probe: all-padding row, k = 1, tile-bound threshold, small indices."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
from bm25mi.index import GpuIndex
rng = np.random.default_rng(1)
for N in (3000, 4096, 6000, 8192, 20000):
    V = 20
    indptr, idx, dat = [0], [], []
    for t in range(V):
        df = int(rng.integers(1, N // 3))
        idx.append(np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
        dat.append(rng.uniform(0.5, 3, df).astype(np.float32))
        indptr.append(indptr[-1] + df)
    ip, ix_, dt = np.array(indptr, np.int64), np.concatenate(idx), np.concatenate(dat)
    ix = GpuIndex(ip, ix_, dt, N)
    for qrow in ([-1, -1, -1], [1, 2, -1]):
        q = np.array([qrow], np.int32)
        for k in (1, 2, 3):
            d, s = ix.search(q, k)
            print(N, qrow, k, ix.last_dispatch()["sample_p"], ix.last_dispatch()["band_tiles"], d[0], s[0], ix.search_stats(), flush=True)
    ix.close()
