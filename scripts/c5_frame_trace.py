"""C5 per-frame timeline from a rocprofv3 kernel trace of bench_odometry.py: for the registration of each frame,
the k_corr launches on the registration stream, their summed duration, the gaps between them and the gap
from the last launch of one frame to the first of the next (host work between registrations)."""
import csv
import glob
import statistics as st
import sys

f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
corr = [r for r in rows if "k_corr" in r["Kernel_Name"]]
# frames: a k_corr whose start follows the previous one's end by more than 30 us starts a new registration
frames, cur = [], []
for r in corr:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    if cur and s - cur[-1][1] > 30_000:
        frames.append(cur)
        cur = []
    cur.append((s, e))
frames.append(cur)
frames = frames[len(frames) // 4:]   # past the warmup
busy = [sum(e - s for s, e in fr) / 1e3 for fr in frames]
span = [(fr[-1][1] - fr[0][0]) / 1e3 for fr in frames]
inner = [sum(b[0] - a[1] for a, b in zip(fr, fr[1:])) / 1e3 for fr in frames]
between = [(b[0][0] - a[-1][1]) / 1e3 for a, b in zip(frames, frames[1:])]
n = [len(fr) for fr in frames]
print(f"frames {len(frames)}: launches/frame {st.mean(n):.2f}; k_corr busy {st.mean(busy):.1f} us/frame, span "
      f"{st.mean(span):.1f} us (gaps inside {st.mean(inner):.1f}), between frames {st.median(between):.1f} us median "
      f"({st.mean(between):.1f} mean)")
per = {}
for fr in frames:
    for k, (s, e) in enumerate(fr):
        per.setdefault(k, []).append((e - s) / 1e3)
print("k_corr us by iteration of the frame:", " ".join(f"{st.mean(v):.0f}" for k, v in sorted(per.items()) if len(v) > len(frames) // 2))
others = {}
t0, t1 = frames[0][0][0], frames[-1][-1][1]
for r in rows:
    s = int(r["Start_Timestamp"])
    if t0 <= s <= t1 and "k_corr" not in r["Kernel_Name"]:
        nm = r["Kernel_Name"].split("(")[0].replace("void ", "")[:50]
        others.setdefault(nm, []).append((int(r["End_Timestamp"]) - s) / 1e3)
for nm, v in sorted(others.items(), key=lambda kv: -sum(kv[1])):
    print(f"  {nm:50s} {len(v) / len(frames):5.2f}/frame  {st.mean(v):8.1f} us")
