"""Dev probe: all-padding rows through the tile-bound threshold (synth_small)."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
from bm25mi.index import GpuIndex
g = np.load(os.path.join(REPO, "tests/golden/synth_small.npz"))
n = int(g["n_docs"])
ix = GpuIndex(g["indptr"], g["indices"], g["data"], n)
print("info", ix.info())
for tb in (1, 0):
    for tl in (1, 0):
        ix.set_option("theta_bound", tb)
        ix.set_option("tile_bound", tl)
        for k in (1, 2, 10):
            for rows in ([12], [11, 12], list(range(48))):
                q = g["queries"][rows]
                d, s = ix.search(q, k)
                bad = [r for i, r in enumerate(rows) if np.isnan(s[i]).any()]
                print(tb, tl, k, len(rows), "dispatch", ix.last_dispatch(), "nan rows", bad,
                      "row12", d[rows.index(12)][:3], s[rows.index(12)][:3], ix.search_stats(), flush=True)
