"""Pass-0 launch order, from a timeline dump (scripts/tl_run.sh keeps gpurun_out/tl/st.30 = the first pass of
a cold 1M/1M registration): list-schedules the measured wave durations onto the 6144 wave slots in launch
order, longest-first by the true duration (the bound any cost-ordered launch could reach) and longest-first
by a setup-time predictor (the source tile's radius, its point count).

    python scripts/launch_order.py gpurun_out/tl/st.30"""
import heapq
import sys

import numpy as np

a = np.fromfile(sys.argv[1], dtype=np.uint64).reshape(-1, 20).astype(np.int64)
live = a[:, 17] > 0
t0, t1 = a[live, 16], a[live, 17]
base = t0.min()
dur = (t1 - t0) / 100.0                      # us (100 MHz realtime)
rad = a[live, 1].astype(np.uint32).view(np.float32)
cnt = a[live, 2]


def sched(order, slots=6144):
    h = [0.0] * slots
    end = 0.0
    for i in order:
        t = heapq.heappop(h)
        e = t + dur[i]
        end = max(end, e)
        heapq.heappush(h, e)
    return end


print(f"waves {live.sum()}  measured span {(t1.max() - base) / 100:.1f} us  mean wave {dur.mean():.1f} us"
      f"  (all waves packed on 6144 slots: {dur.sum() / 6144:.1f} us)")
print(f"corr(duration, tile radius) {np.corrcoef(dur, rad)[0, 1]:.2f}  corr(duration, tile size) {np.corrcoef(dur, cnt)[0, 1]:.2f}")
print(f"list schedule, launch order          {sched(range(len(dur))):6.1f} us")
print(f"list schedule, longest first (oracle) {sched(np.argsort(-dur)):6.1f} us")
print(f"list schedule, largest radius first   {sched(np.argsort(-rad)):6.1f} us")
print(f"list schedule, largest tile first     {sched(np.argsort(-cnt, kind='stable')):6.1f} us")
# per XCD (workgroup b runs on XCD b % 8, 768 wave slots each), in launch order and longest-first within the XCD
idx = np.flatnonzero(live)
xcd = (idx // 4) % 8
ends = [sched(np.flatnonzero(xcd == x)[np.argsort(np.zeros(np.sum(xcd == x)), kind='stable')], 768) for x in range(8)]
# (sched orders by position in dur: pass indices)
def sched_sub(sel, order_key=None, slots=768):
    o = sel if order_key is None else sel[np.argsort(-order_key[sel], kind="stable")]
    return sched(o, slots)
e0 = [sched_sub(np.flatnonzero(xcd == x)) for x in range(8)]
e1 = [sched_sub(np.flatnonzero(xcd == x), dur) for x in range(8)]
print("per XCD, launch order:  " + " ".join(f"{e:5.1f}" for e in e0) + f"   max {max(e0):.1f} us")
print("per XCD, longest first: " + " ".join(f"{e:5.1f}" for e in e1) + f"   max {max(e1):.1f} us")
xe = [(t1[xcd == x].max() - base) / 100 for x in range(8)]
print("per XCD, measured:      " + " ".join(f"{e:5.1f}" for e in xe))
