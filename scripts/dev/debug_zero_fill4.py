"""Dev probe: the two halves on a 2-tile index, all-padding row, k = 1."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
import torch
from bm25mi.index import GpuIndex
rng = np.random.default_rng(1)
N, V = 3000, 20
indptr, idx, dat = [0], [], []
for t in range(V):
    df = int(rng.integers(1, N // 3))
    idx.append(np.sort(rng.choice(N, df, replace=False)).astype(np.int32))
    dat.append(rng.uniform(0.5, 3, df).astype(np.float32))
    indptr.append(indptr[-1] + df)
ip, ix_, dt = np.array(indptr, np.int64), np.concatenate(idx), np.concatenate(dat)
ix = GpuIndex(ip, ix_, dt, N)
q = torch.tensor([[-1, -1, -1], [1, 2, -1]], dtype=torch.int32, device="cuda")
for k in (1,):
    S = ix.sample_width(k, 1, N)
    keys = torch.full((2, S), 7, dtype=torch.int64, device="cuda")
    ix.search_sample_device(q, k, 1, N, keys)
    torch.cuda.synchronize()
    print("S", S, "keys", [hex(x & 0xFFFFFFFFFFFFFFFF) for x in keys.flatten().tolist()], flush=True)
    for name, ak in (("own", keys), ("zeros", torch.zeros_like(keys))):
        d = torch.empty((2, k), dtype=torch.int32, device="cuda")
        s = torch.empty((2, k), dtype=torch.float32, device="cuda")
        if name == "zeros":
            ix.search_sample_device(q, k, 1, N, keys)
        ix.search_finish_device(q, k, 1, N, ak.unsqueeze(0), d, s)
        torch.cuda.synchronize()
        print(name, d.tolist(), s.tolist(), ix.search_stats(), ix.last_dispatch(), flush=True)
