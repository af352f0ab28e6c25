"""Model of the sampled threshold on config 3 (CPU, dev tool): for 16 of the
1,024 queries, the exact dense scores (scipy, as bm25_native), the SAMPLE
keys (best sum of each sample tile: bands of 8 tiles, every 8th band), theta
= the k-th best key, and what REST then emits: keys >= theta outside the
skipped sample tiles, and the tiles holding any.
  python scripts/theta_model.py"""
import sys, os, numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
from bm25mi import synth
import scipy.sparse as sp
cfg = synth.CONFIGS["c3"]
ip, ix, dt = synth.make_index(cfg, threads=8)
q = synth.make_queries(cfg)
N = cfg.n_docs; k = 100; D = 2048; nt = (N + D - 1) // D
A = sp.csc_matrix((dt, ix, ip), shape=(N, cfg.n_terms))
tiles = np.arange(nt)
sample = ((tiles >> 3) & 7) == 0
res = []
for qi in range(0, 1024, 64):
    t = q[qi][q[qi] >= 0]
    s = np.asarray(A[:, t].sum(axis=1)).ravel().astype(np.float32)
    pad = np.zeros(nt * D, np.float32); pad[:N] = s
    tm = pad.reshape(nt, D).max(axis=1)
    skeys = np.sort(tm[sample])[::-1]
    th = skeys[k - 1]
    true_k = np.sort(s)[-k]
    above = pad.reshape(nt, D) >= th
    rest_tiles = ~sample | (tm >= th)
    n_keys = int(above[rest_tiles].sum())
    n_tiles = int((above.any(axis=1) & rest_tiles).sum())
    res.append((th, true_k, n_keys, n_tiles))
    print(qi, f"theta {th:.4f} true_kth {true_k:.4f} keys>=theta {n_keys} emitting tiles {n_tiles} of {nt}")
r = np.array(res)
print("mean keys", r[:, 2].mean(), "mean emitting tiles", r[:, 3].mean(), "of", nt)
