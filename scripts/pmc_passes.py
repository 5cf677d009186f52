"""Per-dispatch PMC counters of k_corr in launch order (rocprofv3 --pmc csv), for the bench's first timed
(cold) registration: dispatches [first, first + n).   python scripts/pmc_passes.py DIR [first] [n]"""
import csv, glob, sys, collections
root = sys.argv[1]
first = int(sys.argv[2]) if len(sys.argv) > 2 else 5
n = int(sys.argv[3]) if len(sys.argv) > 3 else 30
rows = collections.defaultdict(dict)
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_corr" not in r["Kernel_Name"]:
            continue
        rows[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
ids = sorted(rows)
names = sorted({c for d in rows.values() for c in d})
print("pass " + " ".join(f"{c[:14]:>14s}" for c in names))
for k, i in enumerate(ids[first:first + n]):
    print(f"{k:4d} " + " ".join(f"{rows[i].get(c, float('nan')):14.0f}" for c in names))
