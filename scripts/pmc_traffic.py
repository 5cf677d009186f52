"""Per-launch HBM-side traffic of a kernel from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes,
corrected as MI355X_MICROARCH.md §HBM prescribes (gfx950 FETCH_SIZE counts half the bytes of a
16-B/lane read stream: doubled; WRITE_SIZE as is; both in KiB).

    python scripts/pmc_traffic.py <pmc dir> <out.json> [kernel substring] [workload] [first] [passes]

first = the command's --warmup, passes = its --steps: the summary is keyed by (workload, steps, warmup) and
bench.py reports it only for that exact command.

Besides the mean over every launch of the command, per pass of the timed registration (dispatches
[first, first + passes) of the kernel: bench.py's 5 warmup launches come first): pass 0, the mean of
passes 1-10 (moving) and of the last 10 (converged)."""
import csv, glob, json, sys
root, out = sys.argv[1], sys.argv[2]
kern = sys.argv[3] if len(sys.argv) > 3 else "k_corr"
workload = sys.argv[4] if len(sys.argv) > 4 else ""
first = int(sys.argv[5]) if len(sys.argv) > 5 else 5
passes = int(sys.argv[6]) if len(sys.argv) > 6 else 30
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
by_id = {"FETCH_SIZE": {}, "WRITE_SIZE": {}}
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"] and r["Counter_Name"] in vals:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
            by_id[r["Counter_Name"]][(f, int(r["Dispatch_Id"]))] = float(r["Counter_Value"])


def timed(counter):
    ids = sorted(by_id[counter], key=lambda k: k[1])
    return [by_id[counter][k] for k in ids[first:first + passes]]


fp, wp = timed("FETCH_SIZE"), timed("WRITE_SIZE")
per = [(2.0 * a + b) * 1024.0 for a, b in zip(fp, wp)] if len(fp) == len(wp) else []
fetch = sum(vals["FETCH_SIZE"]) / max(1, len(vals["FETCH_SIZE"]))
write = sum(vals["WRITE_SIZE"]) / max(1, len(vals["WRITE_SIZE"]))
res = {"kernel": kern, "workload": workload, "steps": passes, "warmup": first,
       "command": f"bench.py --gpus 1 --steps {passes} --warmup {first}",
       "launches": len(vals["FETCH_SIZE"]),
       "fetch_size_kib": fetch, "write_size_kib": write,
       "traffic_bytes_per_launch": (2.0 * fetch + write) * 1024.0,
       "per_pass": None if not per else {
           "first_pass": per[0], "moving_mean": sum(per[1:11]) / len(per[1:11]) if len(per) > 1 else None,
           "converged_mean": sum(per[-10:]) / len(per[-10:]), "timed_mean": sum(per) / len(per),
           "bytes_by_pass": [round(x) for x in per],
           "note": "timed cold registration of bench.py (dispatches first..first+passes), FETCH and WRITE "
                   "from separate runs of the same command"},
       "correction": "2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes), MI355X_MICROARCH.md HBM section; "
                     "Infinity-Cache hits are counted as memory-side traffic"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
