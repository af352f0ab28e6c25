"""Selection counters of one config-3 search (dev): block-merge queries, the
lists' lengths are not exposed, so the counters only (bm25_search_counters)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "mojo-bm25_amd"))
from bm25mi import synth  # noqa: E402
from bm25mi.index import GpuIndex  # noqa: E402

cfg = synth.CONFIGS[os.environ.get("CFG", "c3")]
ip, ix, dt = synth.make_index(cfg, threads=16)
q = synth.make_queries(cfg)
g = GpuIndex(ip, ix, dt, cfg.n_docs)
for _ in range(2):
    g.search(q, cfg.k)
print(cfg, g.search_stats(), g.last_dispatch(), flush=True)
g.close()
