"""Dev probe (variant build -DBM25_TRACE=1): per-wave start/end of the REST
pass on config 3's index (W=1) and on one 8-way doc shard (W=8), to see how
much of the pass is the tail (waves finishing while others still run).
  VLIB=exp/libbm25mi_trace.so python scripts/dev/rest_trace.py"""
import ctypes, json, os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "mojo-bm25_amd"), REPO]
import torch
import importlib
importlib.import_module("bm25mi.build").LIB = os.path.abspath(os.environ["VLIB"])
from bm25mi import synth, _capi
from bm25mi.index import GpuIndex
lib = _capi.lib
lib.bm25_debug_trace.argtypes = [ctypes.c_void_p, ctypes.c_int64]
cfg = synth.CONFIGS["c3"]
q = torch.from_numpy(synth.make_queries(cfg)).cuda()
for W in (1, 8):
    lo, hi = synth.shard_bounds(cfg.n_docs, W, 0)
    ip, ix, dt = synth.make_index(cfg, lo, hi, threads=16)
    index = GpuIndex(ip, ix, dt, hi - lo, doc_offset=lo)
    d = torch.empty((q.shape[0], cfg.k), dtype=torch.int32, device="cuda")
    s = torch.empty((q.shape[0], cfg.k), dtype=torch.float32, device="cuda")
    for _ in range(3):
        index.search_device(q, cfg.k, d, s)
    torch.cuda.synchronize()
    for rep in range(2):
        index.search_device(q, cfg.k, d, s)
        torch.cuda.synchronize()
        n = 16384
        buf = np.zeros((n, 4), np.uint64)
        assert lib.bm25_debug_trace(buf.ctypes.data_as(ctypes.c_void_p), n) == 0
        used = buf[:, 1] > 0
        b = buf[used].astype(np.int64)
        t0 = b[:, 0].min()
        st = (b[:, 0] - t0) / 100.0  # us (100 MHz)
        en = (b[:, 1] - t0) / 100.0
        span = en.max()
        pct = lambda a, p: float(np.percentile(a, p))
        late = en > pct(en, 99)
        print(json.dumps({"W": W, "waves": int(used.sum()), "span_us": round(span, 1),
                          "start_us_p50_max": [round(pct(st, 50), 1), round(st.max(), 1)],
                          "end_us_p1_p10_p50_p90_p99": [round(pct(en, p), 1) for p in (1, 10, 50, 90, 99)],
                          "items_mean_max": [float(b[:, 2].mean()), int(b[:, 2].max())],
                          "rows_mean_max": [float(b[:, 3].mean()), int(b[:, 3].max())],
                          "late_waves_rows_mean": float(b[late, 3].mean()),
                          "late_waves_items_mean": float(b[late, 2].mean()),
                          "busy_fraction": round(float((en - st).sum() / (span * used.sum())), 3),
                          # per XCD (workgroup i runs on XCD i % 8): end p50 / max, rows
                          "xcd_end_p50_max_rows": [[round(pct(en[xs], 50), 1), round(float(en[xs].max()), 1),
                                                    int(b[xs, 3].sum())]
                                                   for xs in (np.nonzero(used)[0] % 8 == x for x in range(8))]}),
              flush=True)
    index.close()
