"""Dev probe: all-padding / rare rows through the sampled and tile-bound thresholds."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
from bm25mi.index import GpuIndex
from oracle import oracle
rng = np.random.default_rng(1)
N, V = 100_000, 50
indptr, idx, dat = [0], [], []
for t in range(V):
    df = int(rng.integers(1, 20000)) if t else 3
    idx.append(np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
    dat.append(rng.uniform(0.5, 3, df).astype(np.float32))
    indptr.append(indptr[-1] + df)
ip, ix_, dt = np.array(indptr, np.int64), np.concatenate(idx), np.concatenate(dat)
q = np.array([[-1, -1, -1], [1, 2, 3], [0, -1, -1], [4, 4, 4]], np.int32)
ix = GpuIndex(ip, ix_, dt, N)
for tb in (0, 1):
    ix.set_option("theta_bound", tb)
    for k in (1, 2, 5, 10):
        d, s = ix.search(q, k)
        ref = oracle.search_c(N, ip, ix_, dt, q, k, threads=4)
        ok = [bool((d[i] == ref[0][i]).all() and (s[i].view(np.uint32) == ref[1][i].view(np.uint32)).all()) for i in range(len(q))]
        print(tb, k, ix.last_dispatch()["sample_p"], sorted(ix.last_dispatch()["kernels"]), ok, d[0][:3], s[0][:3], d[2][:3], s[2][:3], flush=True)
