"""Time the config-3 search with variant builds of libbm25mi (dev tool, not
part of the product).  python scripts/variant_lib_time.py exp/libbm25mi_A.so ...
Each library runs in its own child process (one HIP runtime per library);
the index arrays are cached under /tmp between children.  One JSON line per
library: score-pass / search ms and a hash of the results."""
import json, os, subprocess, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import json, os, sys, numpy as np
sys.path[:0] = [os.path.join(sys.argv[1], "mojo-bm25_amd"), sys.argv[1]]
import torch
import importlib  # (bm25mi.build as an attribute is the build() function)
importlib.import_module("bm25mi.build").LIB = os.environ["VLIB"]  # this child's variant library
from bm25mi import synth, _capi
from bm25mi.index import GpuIndex
cfg = synth.CONFIGS[os.environ.get("VCFG", "c3")]
if os.environ.get("VTERMS"):
    import dataclasses
    cfg = dataclasses.replace(cfg, terms_per_query=int(os.environ["VTERMS"]))
c = "/tmp/vt_" + cfg.name.split()[0]
# config 5: one rank's doc shard (rank 0 of 8), as bench.py --config c5
lo, hi = synth.shard_bounds(cfg.n_docs, 8, 0) if os.environ.get("VCFG") == "c5" else (0, cfg.n_docs)
if not os.path.exists(c + "_dt.npy"):
    ip, ix, dt = synth.make_index(cfg, lo, hi, threads=16)
    for n, a in (("ip", ip), ("ix", ix), ("dt", dt)): np.save(c + "_" + n + ".npy", a)
ip, ix, dt = (np.load(c + "_" + n + ".npy", mmap_mode="r") for n in ("ip", "ix", "dt"))
index = GpuIndex(np.ascontiguousarray(ip), ix, dt, hi - lo, doc_offset=lo)
q = torch.from_numpy(synth.make_queries(cfg)).cuda()
Q, k = q.shape[0], int(os.environ.get("VK", cfg.k))
d = torch.empty((Q, k), dtype=torch.int32, device="cuda"); s = torch.empty((Q, k), device="cuda")
st = torch.cuda.current_stream()
for _ in range(3):
    index.search_device(q, k, d, s, st)
torch.cuda.synchronize()
index.profile_enable(2)  # (score pass and whole search)
for _ in range(20):
    index.search_device(q, k, d, s, st)
p = index.profile_read()
torch.cuda.synchronize()
h = int((d.to(torch.int64) * 1000003 + s.view(torch.int32).to(torch.int64)).sum().item())
ss = index.search_stats()
print(json.dumps({"lib": os.path.basename(_capi.LIB), "env": os.environ.get("VENV", ""),
                  "cfg": os.environ.get("VCFG", "c3"), "k": k, "terms": cfg.terms_per_query, "score_ms": round(p["score_ms"] / p["score_launches"], 4),
                  "total_ms": round(p["total_ms"] / p["searches"], 4), "hash": h,
                  "kernels": sorted(index.last_dispatch()["kernels"]),
                  "fallback_queries": ss["fallback_queries"],
                  "bound_skipped_tiles": ss["bound_skipped_tiles"]}), flush=True)
'''
for arg in sys.argv[1:]:  # LIB[:NAME=VAL,NAME=VAL]: per-library environment
    lib, _, kv = arg.partition(":")
    env = dict(os.environ, VLIB=os.path.abspath(lib))
    env.update(dict(x.split("=", 1) for x in kv.split(",") if x))
    env["VENV"] = kv
    r = subprocess.run(["timeout", "-k", "10", "240", sys.executable, "-c", CHILD, REPO], env=env,
                       capture_output=True, text=True)
    out = r.stdout.strip().splitlines()
    print(out[-1] if r.returncode == 0 and out else json.dumps({"lib": lib, "rc": r.returncode,
                                                               "err": r.stderr[-800:]}), flush=True)
    if r.returncode != 0:
        sys.exit(r.returncode)
