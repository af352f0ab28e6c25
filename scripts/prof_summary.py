"""Summarise rocprofv3 outputs of scripts/gpu_evidence.sh (PART=prof): the
kernel stats of the bench run, then the PMC counters per workload tag and
score phase (mean per dispatch) with derived per-row / traffic figures.
With --traffic OUT.json, also write the per-workload HBM traffic of one
search (EA read requests x 128 B + WRITE_SIZE, summed over the score
phases) that bench.py reports as roofline.traffic.
Dev tool: python scripts/prof_summary.py gpurun_out/<NAME> [--traffic profiles/traffic.json]"""
import collections
import csv
import glob
import os
import re
import sys

import json

args = [a for a in sys.argv[1:] if not a.startswith("--")]
d = args[0] if args else "gpurun_out"
traffic_out = sys.argv[sys.argv.index("--traffic") + 1] if "--traffic" in sys.argv else None
if traffic_out in args:
    args.remove(traffic_out)
for f in sorted(glob.glob(os.path.join(d, "trace*", "*kernel_stats.csv"))):
    print("== kernel stats", os.path.relpath(f, d))
    for r in csv.DictReader(open(f)):
        name = r["Name"].split("(")[0].replace("void ", "").replace("bm25mi::", "")
        print(f"  {name:44s} calls={int(r['Calls']):5d} avg={float(r['AverageNs'])/1e3:10.1f} us"
              f"  pct={float(r['Percentage']):6.2f}")
PH = {"0": "ALL", "1": "SAMPLE", "2": "REST"}
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    tag = os.path.relpath(f, d).split(os.sep)[0].split("_")[1]
    for r in csv.DictReader(open(f)):
        m = re.search(r"score_flat_kernel<(\d+), (\d), (\d), (\w+), (\d)>", r["Kernel_Name"])
        key = (tag, PH[m.group(2)] + f" SM={m.group(3)} sparse={m.group(4)} TL={m.group(5)}") if m else (tag, r["Kernel_Name"][:40])
        agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
        agg[key]["_dur_us"].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for (tag, ph), cs in sorted(agg.items()):
    mean = {c: sum(v) / len(v) for c, v in cs.items()}
    print(f"== PMC {tag} {ph}")
    for c, v in sorted(mean.items()):
        print(f"  {c:24s} {v:16.5g}")
    if mean.get("SQ_INSTS_VMEM_RD", 0) > 0:
        rows = mean["SQ_INSTS_VMEM_RD"] / 2
        print(f"  -> rows {rows:.4g}; per row: VALU {mean.get('SQ_INSTS_VALU', 0) / rows:.1f} "
              f"SALU {mean.get('SQ_INSTS_SALU', 0) / rows:.1f} LDS {mean.get('SQ_INSTS_LDS', 0) / rows:.2f}")
    if mean.get("SQ_LDS_IDX_ACTIVE", 0) > 0 and "SQ_LDS_BANK_CONFLICT" in mean:
        print(f"  -> LDS bank-conflict share {mean['SQ_LDS_BANK_CONFLICT'] / mean['SQ_LDS_IDX_ACTIVE']:.3f}")
    if "TCC_EA0_RDREQ_sum" in mean:
        h, m = mean.get("TCC_HIT_sum", 0), mean.get("TCC_MISS_sum", 0)
        print(f"  -> EA read bytes {mean['TCC_EA0_RDREQ_sum'] * 128 / 1e9:.3f} GB (x128 B/req), "
              f"DRAM-side {mean.get('TCC_EA0_RDREQ_DRAM_sum', 0) * 128 / 1e9:.3f} GB, L2 hit {h / max(h + m, 1):.3f}")
    if mean.get("SQ_WAVE_CYCLES", 0) > 0:
        w = mean["SQ_WAVE_CYCLES"]
        print(f"  -> wave cycles: wait {mean.get('SQ_WAIT_ANY', 0) / w:.2f}, "
              f"issue-stall {mean.get('SQ_WAIT_INST_ANY', 0) / w:.2f}, active {mean.get('SQ_ACTIVE_INST_ANY', 0) / w:.2f}")

# per-workload traffic of one search (each phase is one dispatch per search)
WL = {"c3": ("c3", 8), "t16": ("c3", 16), "c5": ("c5", 8)}
if traffic_out:
    entries = []
    for tag, (config, terms) in WL.items():
        ph = {p: {c: sum(v) / len(v) for c, v in cs.items()} for (t, p), cs in agg.items() if t == tag}
        if not ph:
            continue
        rd = sum(m.get("TCC_EA0_RDREQ_sum", 0) for m in ph.values())
        wr = sum(m.get("WRITE_SIZE", 0) for m in ph.values()) * 1024
        hit = sum(m.get("TCC_HIT_sum", 0) for m in ph.values())
        miss = sum(m.get("TCC_MISS_sum", 0) for m in ph.values())
        entries.append({"config": config, "terms_per_query": terms, "tile_shift": 11,
                        "hbm_bytes_per_launch": int(rd * 128 + wr), "read_bytes": int(rd * 128),
                        "write_size_bytes": int(wr), "tcc_ea0_rdreq": int(rd),
                        "l2_hit_rate": round(hit / max(hit + miss, 1), 3),
                        "phases": sorted(ph)})
    json.dump({"source": os.path.relpath(d), "kernels": "the score pass of one search: bound_keys_kernel or score_flat_kernel SAMPLE, score_flat_kernel REST (+ the fallback ALL launch)",
               "method": ("rocprofv3 --pmc, one counter group per pass (scripts/gpu_r5.sh STEPS=prof); "
                          "read bytes = TCC_EA0_RDREQ x 128 B, the bytes per request measured for this "
                          "kernel's 4-B and 8-B-per-lane buffer loads by the calibration kernel "
                          "(profiles/r02/traffic_calib/summary.json: 128.0 B/RDREQ, FETCH_SIZE reports "
                          "half); + WRITE_SIZE (KB); Infinity-Cache hits are included (not separable)"),
               "entries": entries}, open(traffic_out, "w"), indent=1)
    print("wrote", traffic_out, [(e["config"], e["terms_per_query"], e["hbm_bytes_per_launch"]) for e in entries])
