"""Sum rocprofv3 --pmc counter_collection.csv values per (kernel, counter), averaged per dispatch.
usage: pmc_sum.py DIR [DIR...] [--kernel SUBSTR]"""
import csv, glob, sys, collections, os
args = [a for a in sys.argv[1:] if not a.startswith("--")]
ksub = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else "irls"
tot = collections.defaultdict(float); disp = collections.defaultdict(set); dur = {}
for d in args:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if ksub not in k or k == ksub:
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add((f, r["Dispatch_Id"]))
for c in sorted(tot):
    print(f"{c:32s} {tot[c] / max(len(disp[c]), 1):.6g}")
