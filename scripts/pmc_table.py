"""Mean counter values per score kernel phase from rocprofv3 --pmc csv dirs.
Dev tool: python scripts/pmc_table.py gpurun_out/pmcq_*"""
import collections, csv, glob, sys

for d in sys.argv[1:]:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        per = collections.defaultdict(dict)
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            kind = "band" if "score_band" in name else "pipe"
            ph = kind + ("_SAMPLE" if "<11, 1," in name else "_REST" if "<11, 2," in name else "_ALL" if "<11, 0," in name else name[:30])
            per[(r["Dispatch_Id"], ph)][r["Counter_Name"]] = float(r["Counter_Value"])
        for (_, ph), cs in per.items():
            for c, v in cs.items():
                acc[ph][c].append(v)
    for ph, cs in acc.items():
        print(d, ph, {c: round(sum(v) / len(v)) for c, v in cs.items()})
