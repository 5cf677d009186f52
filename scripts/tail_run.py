"""Per-launch tail breakdown of k_corr (the fixed floor of a pass), from the GICP_TAIL diagnostic build.

    make -C generalized-icp_amd/csrc VARIANT=tail VDEFS=-DGICP_TAIL
    GICP_LIB_VARIANT=tail python scripts/tail_run.py [--n 1000000] [--shard-sim 1] [--steps 30]

One cold registration of --steps fixed iterations with every launch timed by a HIP event pair and its tail
record dumped (gicp_internal.h kTailWords, 100 MHz realtime stamps).  Prints, per iteration: the event time,
the waves' phase (first workgroup start -> last partial stored) and each step of the tail: the group ticket,
the group sum, the final ticket, the final sum, the exchange, the statistics store, the solve."""
import argparse
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "generalized-icp_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--shard-sim", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import gicp
    from gicp import synthetic as S
    src, tgt, _ = S.scene_pair_3d(a.n)
    p = gicp.default_params(3, fixed_iterations=1, max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)
    e = gicp.Engine(0)
    e.set_target(tgt, p)
    e.set_source(src, p, shard=0, nshards=a.shard_sim)
    p.max_iterations = a.warmup
    e.align(None, p)
    p.max_iterations = a.steps
    p.timing_stride = 1
    d = tempfile.mkdtemp()
    os.environ["GICP_TAIL_DUMP"] = os.path.join(d, "tail")
    recs, evs = [], []
    for r in range(a.reps):
        e.reset_cache()
        e.align(None, p)
        evs.append(np.array(e.iteration_times()) * 1e3)
    del os.environ["GICP_TAIL_DUMP"]
    for r in range(a.reps):
        recs.append(np.fromfile(os.path.join(d, f"tail.{r}"), dtype=np.uint64).reshape(-1, 16).astype(np.int64))
    e.close()
    R = np.stack(recs)            # [rep][iter][16]
    for k in range(2, 9):         # a stage the launch skipped (one-level reduction: no group sum) takes no time
        R[:, :, k] = np.where(R[:, :, k] == 0, R[:, :, k - 1], R[:, :, k])
    ev = np.stack(evs)            # [rep][iter] us
    us = lambda x: x / 100.0      # 100 MHz
    waves = us(R[:, :, 1] - R[:, :, 0])
    names = ["grp_ticket", "grp_sum", "fin_ticket", "fin_sum", "exchange", "stats_st", "solve"]
    steps = [us(R[:, :, k + 1] - R[:, :, k]) for k in range(1, 8)]
    span = us(R[:, :, 8] - R[:, :, 0])
    print(f"n={a.n} shard 0 of {a.shard_sim}, {a.steps} iterations, {a.reps} cold reps; us, median over reps")
    print("iter  event   span  waves | " + " ".join(f"{n:>10s}" for n in names) + " | tail")
    for i in range(R.shape[1]):
        row = [np.median(ev[:, i]), np.median(span[:, i]), np.median(waves[:, i])] + [np.median(s[:, i]) for s in steps]
        tail = np.median(us(R[:, i, 8] - R[:, i, 1]))
        print(f"{i:4d} {row[0]:6.1f} {row[1]:6.1f} {row[2]:6.1f} | " + " ".join(f"{x:10.2f}" for x in row[3:]) +
              f" | {tail:6.2f}")
    conv = slice(max(0, R.shape[1] - 10), R.shape[1])
    print("last 10 (converged) mean: event %.1f span %.1f waves %.1f tail %.2f | " % (
        ev[:, conv].mean(), span[:, conv].mean(), waves[:, conv].mean(), us(R[:, conv, 8] - R[:, conv, 1]).mean()) +
        " ".join(f"{n} {s[:, conv].mean():.2f}" for n, s in zip(names, steps)))
    print("launch overhead (event - span), converged mean: %.1f us" % (ev[:, conv] - span[:, conv]).mean())
    print("descent outcomes (rep 0): iter | descending | proved: start-node-min  start-row  after-hop  tie | walking lanes  waves")
    for i in range(R.shape[1]):
        w = R[0, i, 9:16]
        print(f"{i:4d} | {w[0]:8d} {w[1]:8d} {w[2]:8d} {w[3]:8d} | {w[4]:8d} {w[5]:7d} {w[6]:7d}")


if __name__ == "__main__":
    main()
