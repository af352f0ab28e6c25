"""Bytes per memory-side read request, from the traffic_calib PMC passes
(profiles/r02/traffic_calib): for each pattern, requested bytes (printed by
traffic_calib) / TCC_EA0_RDREQ and / FETCH_SIZE.  Dev tool:
python scripts/calib/summarize.py profiles/r02/traffic_calib"""
import csv, json, sys, os

d = sys.argv[1] if len(sys.argv) > 1 else "profiles/r02/traffic_calib"
pats = [json.loads(l) for l in open(os.path.join(d, "patterns.jsonl"))]
ctr = {}
for f in ("calib_p1.csv", "calib_p2.csv"):
    for r in csv.DictReader(open(os.path.join(d, f))):
        if "fillBuffer" in r["Kernel_Name"]:
            continue
        ctr.setdefault(int(r["Dispatch_Id"]), {})[r["Counter_Name"]] = float(r["Counter_Value"])
rows = [ctr[k] for k in sorted(ctr)]
out = []
for p, c in zip(pats, rows):
    b = p["requested_bytes"]
    out.append({"pattern": p["pattern"], "requested_bytes": b,
                "tcc_ea0_rdreq": c["TCC_EA0_RDREQ_sum"],
                "bytes_per_rdreq": round(b / c["TCC_EA0_RDREQ_sum"], 2),
                "fetch_size_bytes": c["FETCH_SIZE"] * 1024,
                "requested_over_fetch_size": round(b / (c["FETCH_SIZE"] * 1024), 3)})
print(json.dumps(out, indent=1))
