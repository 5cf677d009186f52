"""Occupancy timeline of one k_corr launch from a stamps dump (GICP_STAMPS_DUMP, stamps build).

    python scripts/timeline.py gpurun_out/st.2 [kCorrWaves=4] [heavy_waves=512]"""
import sys
import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 20).astype(np.int64)
cw = int(sys.argv[2]) if len(sys.argv) > 2 else 4
hw = int(sys.argv[3]) if len(sys.argv) > 3 else 512
live = a[:, 16] > 0
idx = np.flatnonzero(live)
t0, t1 = a[live, 16], a[live, 17]
base = t0.min()
t0 = (t0 - base) / 100.0   # us (100 MHz)
t1 = (t1 - base) / 100.0
span = t1.max()
print(f"waves {live.sum()}  span {span:.1f} us  mean wave {np.mean(t1 - t0):.1f} us  p50 {np.median(t1 - t0):.1f}"
      f"  p99 {np.percentile(t1 - t0, 99):.1f}  max {np.max(t1 - t0):.1f}")
edges = np.arange(0, span + 5, 5.0)
act = [(np.sum((t0 < e + 5) & (t1 > e))) for e in edges]
print("active waves per 5 us:", " ".join(str(int(x)) for x in act))
print("start times: first 1% / 50% / last 1% of waves:", np.percentile(t0, [1, 50, 99]).round(1))
print("waves finishing in the last 10% of the span:", int(np.sum(t1 > 0.9 * span)))
o = np.argsort(-t1)[:8]
for k in o:
    w = idx[k]
    print(f"  wave {w:6d} ({'heavy' if w < hw else 'tile'}) start {t0[k]:6.1f} end {t1[k]:6.1f} dur {t1[k]-t0[k]:6.1f}"
          f" visits {a[w, 8]} scanned {a[w, 9]} rows {a[w, 7]} list {a[w, 11]} xcc {a[w, 19]}")
xcc = a[live, 19] & 7
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"  xcc {x}: waves {m.sum()} last end {t1[m].max():.1f} us")
