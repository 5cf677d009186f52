"""GICP iterations/sec on MI355X (BASELINE.json metric), one process per GPU.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n POINTS] [--dim 3]

A step is one outer GICP iteration (gicp.py:116-167): correspondences + weights +
statistics on the GPU (k_corr, reduced inside the launch), the RCCL all-reduce of the
statistics when N > 1 (80 fp64 in 3-D = 74 statistics + 6 pass diagnostics; 32 = 26 + 6 in 2-D),
and the pose solve + convergence test on the device (k_solve).  Default workload = BASELINE.json
configs[2]: two synthetic 3-D clouds of 1M points, k = 20 covariances, d_c = 0.5 m,
d_n = 1.0 m; with --gpus N the source is sharded over N ranks (configs[3]).
Convergence is disabled so every run does exactly K iterations.

Ranks: under a launcher (torch.distributed.run sets WORLD_SIZE) every process is one rank and
--gpus must equal WORLD_SIZE.  Without one, --gpus N > 1 starts N rank processes itself -- as
children (python -m torch.distributed.run --nproc-per-node N ... bench.py ...), before anything
touches the GPU -- forwards rank 0's line and exits with the launcher's status; with fewer than N
GPUs visible it exits non-zero naming the count (never a silent 1-GPU run).  --dry-run starts the
ranks on the CPU (gloo) and only reports the rank plumbing.

The timed registration starts COLD: the engine's pose-dependent caches (candidate lists,
nearest-neighbour certificates, last matches) are dropped after the warmup (gicp_reset_cache), so
the K iterations pay the first full walks from the identity exactly as a fresh registration does.
roofline.achieved follows SURVEY.md §8(d): algorithmic bytes per k_corr launch
B = 8 dim (N/G + M) (fp32 xyz + fp32 normal of every source point of the shard and every target
point, read once: 24 B in 3-D, 16 B in 2-D) over the HIP-event mean k_corr duration.
"""
import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "generalized-icp_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md, HBM3E peak
FP32_PEAK_TFLOPS = 157.3     # MI355X vector FP32 peak
IMPL_BYTES_PER_POINT = 80    # DESIGN.md §3 layout actually read: fp32 screen (16) + fp64 xyz (32) + covariance (32)
FLOP_PER_PAIR = 8            # 3 sub + 1 mul + 2 fma (counted as 2) in the fp32 screen
# gicp.py itself (2-D only), timed in the build container on 1 core: context for
# cpu_baseline, never the comparator (the reference cannot travel to the GPU box)
GICP_PY_IT_S = {100_000: 0.062, 1_000_000: 0.0063}


def bytes_per_point(dim):
    """SURVEY.md §8(d) contract: fp32 coordinates + fp32 unit normal, read once (24 B 3-D, 16 B 2-D)."""
    return 8 * dim


def stats_exchanged(dim):
    """fp64 values the per-iteration all-reduce carries: the statistics + GICP_PASS_INFO diagnostics."""
    ns = dim * (dim + 1) // 2
    return ns * ns + ns * dim + ns + dim * dim + dim + 2 + 6


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--n", "--points", dest="n", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-workers", type=int, default=16,
                    help="cKDTree workers of the CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--warm", action="store_true",
                    help="diagnostic: time the registration warm (caches left by the warmup), not the metric")
    ap.add_argument("--shard-sim", type=int, default=1,
                    help="diagnostic: one process runs only shard 0 of S (no collective) to time a rank of an "
                         "S-GPU job; the line is marked and is not the metric")
    ap.add_argument("--shard-index", type=int, default=0, help="diagnostic: which shard --shard-sim runs")
    ap.add_argument("--dry-run", action="store_true",
                    help="start the ranks (gloo, CPU only) and report RANK / WORLD_SIZE; no GPU work")
    ap.add_argument("--exchange", choices=("peer", "rccl"), default="peer",
                    help="N > 1: the statistics exchange -- 'peer' (in-kernel, IPC-mapped areas; falls back to "
                         "RCCL when its probe fails on any rank) or 'rccl' (ncclAllReduce + k_solve)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="diagnostic: the N ranks share GPU 0 (peer exchange only; RCCL refuses); times the "
                         "protocol, not a multi-GPU job")
    return ap.parse_args()


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(a):
    """--gpus N > 1 without a launcher: N rank processes under torch.distributed.run, as CHILD
    processes (never exec: nothing here has touched the GPU, and nothing may before the ranks do).
    Returns the exit status to leave with."""
    if not a.dry_run and not a.share_gpu:
        import torch
        ngpu = torch.cuda.device_count()   # counts devices without initialising HIP on this image
        if ngpu < a.gpus:
            print(f"bench.py: --gpus {a.gpus} needs {a.gpus} GPUs, but {ngpu} GPU(s) are visible; "
                  "refusing to run (no fallback to fewer GPUs)", file=sys.stderr)
            return 2
    import subprocess
    # (the launcher's own parser reads every "--x" token, the script's too: "--n" would be an ambiguous
    # prefix of its options, so it travels as --points)
    args = ["--points" + x[3:] if x == "--n" or x.startswith("--n=") else x for x in sys.argv[1:]]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()), os.path.abspath(__file__), *args]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC: RCCL's only mode on this driver
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def dry_run(world, rank, local, points):
    """Rank plumbing only (CPU, gloo): every rank reports itself, rank 0 prints the gathered list."""
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")
        got = [None] * world
        dist.all_gather_object(got, {"rank": rank, "local_rank": local, "world_size": world})
        dist.destroy_process_group()
    else:
        got = [{"rank": rank, "local_rank": local, "world_size": world}]
    if rank == 0:
        print(json.dumps({"dry_run": True, "world_size": world, "ranks": got, "points": points}))


def workload(n, dim):
    from gicp import synthetic as S
    if dim == 3:
        src, tgt, Tgt = S.scene_pair_3d(n)
        return src, tgt, Tgt, dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0), \
            f"3d_room_{n // 1000}k_{n // 1000}k_k20"
    src, tgt, Tgt = S.segment_scene_2d(n)
    return src, tgt, Tgt, dict(max_distance_correspondence=20.0, max_distance_nearest_neighbors=25.0), \
        f"2d_segments_{n // 1000}k_k6"


def measured_traffic(workload, steps, warmup):
    """HBM-side bytes per k_corr launch from the newest committed PMC summary of THIS command -- the same
    workload, --steps and --warmup (scripts/profile_round.sh -> profiles/rNN/pmc_traffic.json); the counters
    cannot be read in-process.  Returns (bytes, file, per_pass, note); bytes is None, with the reason in
    note, when no profile of this exact command exists (another command's bytes are never reported)."""
    import glob
    seen = []
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*", "pmc_traffic.json")), reverse=True):
        try:
            d = json.load(open(f))
        except (OSError, ValueError):
            continue
        if d.get("workload") != workload:
            continue
        key = (d.get("steps"), d.get("warmup"))
        if key == (steps, warmup):
            return d["traffic_bytes_per_launch"], os.path.relpath(f, ROOT), d.get("per_pass"), \
                f"profiled: rocprofv3 --pmc of bench.py --gpus 1 --steps {steps} --warmup {warmup} ({d.get('launches')} launches)"
        seen.append(f"{os.path.relpath(f, ROOT)} (steps {key[0]}, warmup {key[1]})")
    return None, None, None, ("no PMC profile of this command (steps %d, warmup %d)%s" %
                              (steps, warmup, ("; other commands' profiles not used: " + ", ".join(seen)) if seen else ""))


def cpu_baseline(src, tgt, kw, workers, iters=1):
    """The oracle (NumPy/SciPy restatement) on the host: setup + `iters` outer iterations."""
    from scipy.spatial import cKDTree

    from oracle import gicp_oracle as O
    d = src.shape[1]
    t0 = time.perf_counter()
    Ct, _ = O.covariances(tgt, kw["max_distance_nearest_neighbors"], workers=workers)
    Cs, _ = O.covariances(src, kw["max_distance_nearest_neighbors"], workers=workers)
    tree = cKDTree(tgt)
    setup = time.perf_counter() - t0
    T = np.eye(d + 1)
    t1 = time.perf_counter()
    for _ in range(iters):
        moved = O.apply_transformation(src, T)
        idx, _ = O.correspondences(moved, tgt, kw["max_distance_correspondence"], tree=tree, workers=workers)
        R = T[:d, :d]
        W = O.weights(np.einsum("ab,nbc,dc->nad", R, Cs, R), Ct, idx)
        q = np.zeros_like(src)
        q[idx >= 0] = tgt[idx[idx >= 0]]
        T, _ = O.inner_gn(src, q, W, idx, T)
    dt = time.perf_counter() - t1
    return iters / dt, setup, dt


def setup_exchange(eng, gd, rank, world, exchange, share_gpu):
    """The statistics exchange of a multi-rank run, agreed by every rank: 'peer' tries the in-kernel peer
    exchange (gd.init_peer returns the same note on every rank when any rank's export, IPC open or probe
    failed, with the peer path closed everywhere) and then every rank takes RCCL together; 'rccl' goes
    straight to RCCL.  Two ranks on one GPU (share_gpu) have no RCCL: a failed peer set-up ends the run.
    Returns (peer_note, comm_ranks, comm_kind) as the context reports them, after checking that they are
    what was agreed."""
    peer_note = None
    if world > 1:
        if exchange == "peer":
            peer_note = gd.init_peer(eng, rank, world)
        if exchange == "rccl" or peer_note is not None:   # asked for, or the peer probe failed on some rank
            if share_gpu:
                raise SystemExit(f"rank {rank}: the peer exchange failed on one GPU: {peer_note}")
            gd.init_comm(eng, rank, world)
    comm_ranks, _, comm_kind = eng.comm_ranks()
    want = "peer" if (exchange == "peer" and peer_note is None) else "rccl"
    if world > 1 and (comm_ranks != world or comm_kind != want):
        raise SystemExit(f"rank {rank}: the exchange reports {comm_ranks} ranks ({comm_kind}), expected {world} ({want})")
    return peer_note, comm_ranks, comm_kind


def main():
    a = parse()
    if a.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but the launcher started WORLD_SIZE={world} ranks; refusing",
              file=sys.stderr)
        sys.exit(2)
    if a.dry_run:
        dry_run(world, rank, local, a.n)
        return
    dist = None
    dev = 0 if a.share_gpu else local
    if a.share_gpu and a.exchange != "peer":
        raise SystemExit("bench.py: --share-gpu needs --exchange peer (RCCL refuses two ranks on one GPU)")
    if world > 1:
        import torch
        import torch.distributed as dist
        if dev >= torch.cuda.device_count():   # RCCL refuses two ranks on one GPU
            raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} GPUs")
        torch.cuda.set_device(dev)
        dist.init_process_group("gloo" if a.share_gpu else "nccl")
    import gicp
    from gicp import distributed as gd

    src, tgt, Tgt, kw, name = workload(a.n, a.dim)
    params = gicp.default_params(a.dim, fixed_iterations=1, **kw)
    eng = gicp.Engine(dev)
    peer_note, comm_ranks, comm_kind = setup_exchange(eng, gd, rank, world, a.exchange, a.share_gpu)
    t0 = time.perf_counter()
    eng.set_target(tgt, params)
    if world == 1 and a.shard_sim > 1:
        eng.set_source(src, params, shard=a.shard_index, nshards=a.shard_sim)
    else:
        eng.set_source(src, params, shard=rank, nshards=world)
    setup_ms = (time.perf_counter() - t0) * 1e3

    def sync():
        if dist is not None:
            import torch
            dist.barrier()
            torch.cuda.synchronize()
            dist.barrier()

    params.max_iterations = max(1, a.warmup)
    eng.align(None, params)
    params.max_iterations = a.steps
    # the timed run records no HIP events (an event pair costs queue time); the kernel is timed by
    # the separate runs below.  GICP_BENCH_EVENTS=1 keeps the every-8th-launch pairs in the timed run.
    params.timing_stride = 0 if os.environ.get("GICP_BENCH_EVENTS") == "1" else -1
    if not a.warm:
        eng.reset_cache()   # cold start: nothing inherited from the warmup
    sync()
    t1 = time.perf_counter()
    T, res = eng.align(None, params)
    sync()
    elapsed = time.perf_counter() - t1
    warm_elapsed = None
    if not a.warm:   # diagnostic: the same registration again, continuing from the caches it left
        sync()
        t2 = time.perf_counter()
        eng.align(None, params)
        sync()
        warm_elapsed = time.perf_counter() - t2
    params.timing_stride = 0
    # kernel timing runs (not the metric): an event pair around every launch adds queue work, so each
    # run samples every 8th k_corr launch, and the launch cost falls ~4x as the pose converges, so one
    # sample set is biased; 8 identical K-iteration runs with the sampling offset 0..7 time every
    # launch once
    corr_ms_total = 0.0
    timed = 0
    per_iter = np.full(a.steps, np.nan)
    for off in range(8):
        params.timing_offset = off
        if not a.warm:
            eng.reset_cache()   # every timing run starts cold, as the timed run did
        _, res_t = eng.align(None, params)
        corr_ms_total += res_t["corr_kernel_ms_sampled"]
        timed += res_t["corr_samples"]
        t_it = eng.iteration_times()
        got = ~np.isnan(t_it)
        per_iter[:len(t_it)][got] = t_it[got]
    params.timing_offset = 0
    assert timed == a.steps, (timed, a.steps)
    if dist is not None:
        import torch
        t = torch.tensor([elapsed, corr_ms_total, warm_elapsed or 0.0, *per_iter], dtype=torch.float64,
                         device="cpu" if a.share_gpu else f"cuda:{dev}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, corr_ms_total = float(t[0]), float(t[1])
        warm_elapsed = float(t[2]) or None
        per_iter = t[3:].cpu().numpy()
    if dist is not None:   # every rank releases its communicator, then the process group
        eng.close()
        dist.barrier()
        dist.destroy_process_group()
    if rank != 0:
        return
    from gicp.synthetic import rotation_angle_error, translation_error
    rot_err, tr_err = rotation_angle_error(T, Tgt), translation_error(T, Tgt)
    n_shard = a.n / max(world, a.shard_sim)
    corr_avg_ms = corr_ms_total / a.steps
    alg_bytes = bytes_per_point(a.dim) * (n_shard + a.n)
    impl_bytes = IMPL_BYTES_PER_POINT * (n_shard + a.n)
    achieved = alg_bytes / (corr_avg_ms * 1e-3) / 1e9
    n_mov = min(10, a.steps)
    pairs = res["pairs_total"] / a.steps / world   # mean per launch (summed over ranks by the all-reduce)
    traffic, traffic_src, traffic_pp, traffic_note = (measured_traffic(name, a.steps, a.warmup) if world == 1 and
                                                      a.shard_sim <= 1 and not a.warm else
                                                      (None, None, None, "not profiled (multi-rank or diagnostic run)"))
    line = {
        "metric": "GICP iterations/sec (and ms/iter) at N points, 1/2/4/8 GPU; final transform error",
        "value": a.steps / elapsed,
        "unit": "it/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed * 1e3 / a.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32-screen+f64",
        "data": ("synthetic (3-D room scene of SURVEY.md §8(d), area-uniform samples, 5 mm noise)" if a.dim == 3
                 else "synthetic (2-D segment scene of BASELINE.md §3, 0.5 px noise)"),
        "config": {"workload": name, "n_source": a.n, "n_target": a.n, "dim": a.dim,
                   "k": 20 if a.dim == 3 else 6, **kw,
                   "parallelism": (f"dp{world} (source shards; {stats_exchanged(a.dim)} fp64 per iteration summed "
                                   + ("in-kernel over IPC-mapped peer areas, the solve in the same launch)"
                                      if comm_kind == "peer" else "by RCCL all-reduce, then k_solve)"))
                   if world > 1 else "dp1 (one GPU, no collective)"},
        "comm_ranks": comm_ranks,
        "comm": comm_kind,
        "comm_fallback": peer_note,
        "exchange_us": None if comm_kind != "peer" else
        {"mean": res["exchange_us_mean"], "min": res["exchange_us_min"],
         "note": "rank 0's final workgroup per launch of the timed call: its stores into every rank's area until "
                 "every rank's flag arrived (includes waiting for the slower rank)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "traffic_note": traffic_note,
                     "traffic_per_pass": None if not traffic_pp else
                     {k: traffic_pp.get(k) for k in ("first_pass", "moving_mean", "converged_mean", "timed_mean")},
                     "traffic_vs_alg": None if not traffic_pp else
                     {k: round(traffic_pp[k] / alg_bytes, 2) for k in ("first_pass", "moving_mean", "converged_mean")
                      if traffic_pp.get(k)},
                     "kernel": "k_corr", "kernel_avg_ms": corr_avg_ms, "alg_bytes_per_launch": alg_bytes,
                     "alg_bytes_rule": f"SURVEY.md 8(d): {bytes_per_point(a.dim)} B x (N/G + M)",
                     "impl_bytes_per_launch": impl_bytes,
                     "impl_frac": impl_bytes / (corr_avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                     "kernel_timing": "HIP events, every k_corr launch of K timed once (8 identical cold-start "
                                      "K-iteration runs at sampling offsets 0..7, stride 8)",
                     "kernel_note": ("the inner solve is k_solve after the RCCL all-reduce (not in k_corr's time)"
                                     if comm_kind == "rccl" else
                                     "k_corr's final workgroup also runs the one-wave inner solve and pose update "
                                     "(~5 us, inside the timed duration)" +
                                     (", after the in-kernel peer exchange" if comm_kind == "peer" else ""))},
        "passes": {"moving_pass_us": float(np.mean(per_iter[1:1 + n_mov])) * 1e3,
                   "passes_0_9_us": float(np.mean(per_iter[:n_mov])) * 1e3,
                   "converged_pass_us": float(np.mean(per_iter[-n_mov:])) * 1e3,
                   "first_pass_us": float(per_iter[0]) * 1e3,
                   "k_corr_us_per_iteration": [round(float(x) * 1e3, 1) for x in per_iter],
                   "note": "moving = mean k_corr of iterations 1-10 (the pose still moves; rounds 1-3 reported "
                           "iterations 0-9 under this name, now passes_0_9_us), converged = last 10"},
        "warm_start": None if warm_elapsed is None else
        {"value": a.steps / warm_elapsed, "ms_per_step": warm_elapsed * 1e3 / a.steps,
         "note": "diagnostic, not the metric: the same K iterations again, continuing from the caches"},
        "start": "warm (diagnostic)" if a.warm else "cold (caches reset after the warmup)",
        "valu": {"pairs_per_launch": pairs, "tflops": pairs * FLOP_PER_PAIR / (corr_avg_ms * 1e-3) / 1e12,
                 "peak_tflops": FP32_PEAK_TFLOPS,
                 "frac": pairs * FLOP_PER_PAIR / (corr_avg_ms * 1e-3) / 1e12 / FP32_PEAK_TFLOPS},
        "setup_ms": setup_ms,
        "final_error": {"rot_rad": rot_err, "trans": tr_err, "vs": "ground truth after steps+0 iterations"},
        "correspondences": res["correspondences"],
        "ambiguous_last_pass": res["ambiguous"],
    }
    if a.share_gpu:
        line["diagnostic"] = f"{world} ranks sharing GPU 0 (peer exchange protocol timing, not a multi-GPU job)"
        line["cpu_baseline"] = None
        print(json.dumps(line))
        return
    if a.shard_sim > 1 and world == 1:
        line["diagnostic"] = f"shard {a.shard_index} of {a.shard_sim} only, no exchange: one rank of a {a.shard_sim}-GPU job"
        line["cpu_baseline"] = None
        print(json.dumps(line))
        return
    if world == 1 and not a.no_cpu_baseline:
        try:
            its, setup, dt = cpu_baseline(src, tgt, kw, a.cpu_workers)
            line["cpu_baseline"] = {"value": its, "unit": "it/s", "cores": a.cpu_workers, "kind": "port",
                                    "host_nproc": os.cpu_count(),
                                    "sample": f"oracle (NumPy/SciPy cKDTree workers={a.cpu_workers}; host nproc "
                                              f"{os.cpu_count()}, of which this job's share is {a.cpu_workers}) on "
                                              f"the same {name} clouds, 1 outer iteration after {setup:.1f} s "
                                              f"setup (covariances), {dt:.1f} s timed; parity of the 3-D oracle is "
                                              f"pinned by its 2-D instance (reference fixtures) + ground truth"}
            ref = GICP_PY_IT_S.get(a.n)
            line["cpu_baseline"]["reference_gicp_py"] = {
                "value": ref, "unit": "it/s", "cores": 1, "dim": 2,
                "note": ("context only: gicp.py itself (2-D only, 3-D raises) on 2-D segment clouds of the same N, "
                         "1 core of the build container's 8-core Xeon, BASELINE.md §3; the reference cannot run on "
                         "the GPU box") if ref else "no gicp.py timing at this N (BASELINE.md §3: 100k, 1M)"}
        except Exception as e:  # the baseline must never hide the GPU line
            line["cpu_baseline"] = {"value": None, "error": repr(e)}
    else:
        line["cpu_baseline"] = None
    print(json.dumps(line))


if __name__ == "__main__":
    main()
