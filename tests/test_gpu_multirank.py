"""The library's own multi-rank loop on one GPU (config C4's exchange without an 8-GPU node).

Two processes, each with its own context on GPU 0, hold the same clouds and reduce source shards
0 and 1 of 2 (gicp_set_source(shard=rank, nshards=2)).  Their statistics meet through the host
exchange hook (gicp_set_allreduce) summing over a gloo process group -- between k_corr and k_solve
inside gicp_align's device-resident loop, exactly where the RCCL all-reduce sits on an 8-GPU node
(RCCL itself refuses two ranks on one GPU).  Both ranks must end on bit-identical poses (they run
the same device solve on the same sums), equal to the one-process registration within fp64
summation-order rounding.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

gicp = pytest.importorskip("gicp")
from gicp import synthetic as S  # noqa: E402

P3 = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, d, iters, fixed):
    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    src, tgt = np.load(os.path.join(d, "src.npy")), np.load(os.path.join(d, "tgt.npy"))
    p = gicp.default_params(3, **P3)
    eng = gicp.Engine(0)
    calls = [0]

    def allreduce(buf):
        calls[0] += 1
        t = torch.from_numpy(buf.copy())
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()

    eng.set_allreduce(allreduce)
    eng.set_target(tgt, p)
    eng.set_source(src, p, shard=rank, nshards=world)
    # one pass through gicp_iterate: the exchanged statistics are the full sums
    st = eng.iterate(np.eye(4))
    p.max_iterations = iters
    p.fixed_iterations = 1 if fixed else 0
    p.tolerance = 1e-9
    T, res = eng.align(None, p)
    np.savez(os.path.join(d, f"rank{rank}.npz"), T=T, st=st, iters=res["iterations"], loss=res["final_loss"],
             calls=calls[0], corr=res["correspondences"])
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, n, iters, fixed):
    src, tgt, Tgt = S.scene_pair_3d(n)
    np.save(tmp_path / "src.npy", src)
    np.save(tmp_path / "tgt.npy", tgt)
    mp.spawn(_rank, args=(2, _free_port(), str(tmp_path), iters, fixed), nprocs=2, join=True)
    r = [dict(np.load(tmp_path / f"rank{k}.npz")) for k in range(2)]
    eng = gicp.Engine(0)
    try:
        p = gicp.default_params(3, **P3)
        eng.set_target(tgt, p)
        eng.set_source(src, p)
        st1 = eng.iterate(np.eye(4))
        p.max_iterations = iters
        p.fixed_iterations = 1 if fixed else 0
        p.tolerance = 1e-9
        T1, res1 = eng.align(None, p)
    finally:
        eng.close()
    return r, st1, T1, res1, Tgt


def test_two_ranks_one_gpu_1m_30_iterations(tmp_path):
    """C4's protocol at full size: 1M/1M, 30 fixed iterations, two source shards."""
    r, st1, T1, res1, Tgt = _run(tmp_path, 1_000_000, 30, fixed=True)
    assert np.array_equal(r[0]["T"], r[1]["T"]), "ranks disagree: the exchanged sums must give identical solves"
    assert np.array_equal(r[0]["st"], r[1]["st"])
    assert int(r[0]["iters"]) == int(r[1]["iters"]) == 30
    assert int(r[0]["calls"]) == 31   # one exchange per pass: the gicp_iterate pass + 30 in align
    # the sum over the two shards = the one-process pass (summation order differs: fp64 rounding)
    scale = np.maximum(np.abs(st1), 1e-12 * np.abs(st1).max())
    assert np.max(np.abs(r[0]["st"] - st1) / scale) < 1e-9
    assert int(r[0]["corr"]) == int(res1["correspondences"])
    np.testing.assert_allclose(r[0]["T"], T1, rtol=0, atol=1e-9)
    assert S.rotation_angle_error(T1, Tgt) < 1e-4 and S.translation_error(T1, Tgt) < 1e-3


def test_two_ranks_converge_on_the_same_iteration(tmp_path):
    """Convergence on (gicp.py:155-162): both ranks stop at the same iteration as one process."""
    r, _, T1, res1, _ = _run(tmp_path, 20_000, 60, fixed=False)
    assert np.array_equal(r[0]["T"], r[1]["T"])
    assert int(r[0]["iters"]) == int(r[1]["iters"])
    assert abs(int(r[0]["iters"]) - int(res1["iterations"])) <= 1
    np.testing.assert_allclose(r[0]["T"], T1, rtol=0, atol=1e-8)
