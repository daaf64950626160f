"""Summarise rocprofv3 PMC csv dirs: python scripts/pmc_summary.py DIR [DIR ...] [--kernel substr]"""
import csv, glob, sys, collections
args = [a for a in sys.argv[1:] if not a.startswith("--")]
ksub = "decode"
for a in sys.argv[1:]:
    if a.startswith("--kernel="):
        ksub = a.split("=", 1)[1]
tot = collections.defaultdict(float)
disp = collections.defaultdict(set)
for d in args:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if ksub in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
for k, v in sorted(tot.items()):
    n = max(1, len(disp[k]))
    print(f"{k:24s} total {v:16.0f}  per-dispatch {v / n:16.0f}  dispatches {n}")
