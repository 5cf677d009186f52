"""Per-iteration timeline from a rocprofv3 kernel trace: durations and gaps between kernels."""
import csv, glob, sys, statistics as st
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = [(r["Kernel_Name"].split("(")[0].replace("void ", "")[:40], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
# last 20 k_corr launches and what follows each
idx = [i for i, s in enumerate(seq) if "k_corr" in s[0]][-21:]
per = []
for a, b in zip(idx, idx[1:]):
    chunk = seq[a:b]
    period = seq[b][1] - seq[a][1]
    per.append(period)
    if len(per) <= 2:
        prev_end = None
        for name, s, e in chunk:
            gap = (s - prev_end) / 1e3 if prev_end else 0.0
            print(f"  {name:40s} dur {(e - s) / 1e3:8.2f} us  gap-before {gap:7.2f} us")
            prev_end = e
        print(f"  -> period {period / 1e3:.2f} us")
print("median iteration period (us):", st.median(per) / 1e3)
