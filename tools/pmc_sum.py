"""Per-kernel averages (per dispatch) of rocprofv3 --pmc counter_collection.csv files, with the
kernel durations from the matching kernel_trace.csv.
usage: pmc_sum.py DIR [DIR...] [--kernel SUBSTR] [--json]"""
import csv, glob, json, os, sys, collections
args = [a for a in sys.argv[1:] if not a.startswith("--") and a != (sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else None)]
ksub = sys.argv[sys.argv.index("--kernel") + 1] if "--kernel" in sys.argv else ""
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(lambda: collections.defaultdict(int))
dur = collections.defaultdict(list)
for d in args:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if ksub not in k or "rocclr" in k:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            cnt[k][r["Counter_Name"]] += 1
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if ksub in k and "rocclr" not in k:
                dur[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6)
out = {}
for k in tot:
    e = {c: tot[k][c] / cnt[k][c] for c in tot[k]}
    ds = dur.get(k, [])
    e["avg_ms"] = sum(ds) / len(ds) if ds else None
    e["dispatches"] = len(ds)
    out[k] = e
if "--json" in sys.argv:
    print(json.dumps(out, indent=1))
else:
    for k, e in out.items():
        print(k[:90])
        for c in sorted(e):
            print(f"   {c:28s} {e[c]:.6g}" if e[c] is not None else f"   {c:28s} -")
