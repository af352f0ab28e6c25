"""Summarise rocprofv3 outputs under a gpurun_out dir: kernel stats + PMC
counters per kernel (averaged per dispatch).  Dev tool."""
import csv, glob, os, sys, collections
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out"
for f in glob.glob(os.path.join(d, "trace", "*kernel_stats.csv")):
    print("== kernel stats", f)
    for r in csv.DictReader(open(f)):
        name = r["Name"].split("(")[0].replace("void ", "").replace("bm25mi::", "")
        print(f"  {name:38s} calls={int(r['Calls']):5d} avg={float(r['AverageNs'])/1e3:10.1f} us  pct={float(r['Percentage']):6.2f}")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
meta = {}
for f in sorted(glob.glob(os.path.join(d, "pmc*", "**", "*counter_collection.csv"), recursive=True)):
    tag = os.path.relpath(f, d).split(os.sep)[0]
    for r in csv.DictReader(open(f)):
        name = tag + ":" + r["Kernel_Name"].split("(")[0].replace("void ", "").replace("bm25mi::", "")
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        meta[name] = (r["VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"], r["Workgroup_Size"])
        dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        agg[name]["_dur_ns"].append(dur)
for name, cs in agg.items():
    print("== PMC", name, "vgpr/sgpr/lds/wg =", meta[name])
    for c, v in sorted(cs.items()):
        print(f"  {c:24s} {sum(v)/len(v):16.4g}  (n={len(v)})")
