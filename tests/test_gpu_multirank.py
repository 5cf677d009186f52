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


def _rank(rank, world, port, d, iters, fixed, exchange="hook"):
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

    if exchange == "hook":
        eng.set_allreduce(allreduce, nranks=world, rank=rank)
    else:   # the in-kernel peer exchange over IPC-mapped areas (gicp_peer_export / gicp_peer_init)
        from gicp import distributed as gd
        err = gd.init_peer(eng, rank, world, timeout=20.0)
        assert err is None, err
    kind = eng.comm_ranks()
    eng.set_target(tgt, p)
    eng.set_source(src, p, shard=rank, nshards=world)
    # one pass through gicp_iterate: the exchanged statistics are the full sums
    st = eng.iterate(np.eye(4))
    p.max_iterations = iters
    p.fixed_iterations = 1 if fixed else 0
    p.tolerance = 1e-9
    T, res = eng.align(None, p)
    np.savez(os.path.join(d, f"rank{rank}.npz"), T=T, st=st, iters=res["iterations"], loss=res["final_loss"],
             calls=calls[0], corr=res["correspondences"], kind=np.array(kind, dtype=object), allow_pickle=True)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def _run(tmp_path, n, iters, fixed, exchange="hook"):
    src, tgt, Tgt = S.scene_pair_3d(n)
    np.save(tmp_path / "src.npy", src)
    np.save(tmp_path / "tgt.npy", tgt)
    mp.spawn(_rank, args=(2, _free_port(), str(tmp_path), iters, fixed, exchange), nprocs=2, join=True)
    r = [dict(np.load(tmp_path / f"rank{k}.npz", allow_pickle=True)) for k in range(2)]
    for k in range(2):   # what each rank's context reported for its exchange
        assert tuple(r[k]["kind"]) == (2, k, exchange), r[k]["kind"]
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


@pytest.mark.parametrize("exchange", ["hook", "peer"])
def test_two_ranks_one_gpu_1m_30_iterations(tmp_path, exchange):
    """C4's protocol at full size: 1M/1M, 30 fixed iterations, two source shards; the statistics meet
    through the host hook (gloo) or in-kernel through the IPC-mapped peer areas (the solve then runs in
    each rank's k_corr launch)."""
    r, st1, T1, res1, Tgt = _run(tmp_path, 1_000_000, 30, fixed=True, exchange=exchange)
    assert np.array_equal(r[0]["T"], r[1]["T"]), "ranks disagree: the exchanged sums must give identical solves"
    assert np.array_equal(r[0]["st"], r[1]["st"])
    assert int(r[0]["iters"]) == int(r[1]["iters"]) == 30
    # one exchange per pass: the gicp_iterate pass + 30 in align (host hook), none through the host (peer)
    assert int(r[0]["calls"]) == (31 if exchange == "hook" else 0)
    # the sum over the two shards = the one-process pass (summation order differs: fp64 rounding)
    scale = np.maximum(np.abs(st1), 1e-12 * np.abs(st1).max())
    assert np.max(np.abs(r[0]["st"] - st1) / scale) < 1e-9
    assert int(r[0]["corr"]) == int(res1["correspondences"])
    np.testing.assert_allclose(r[0]["T"], T1, rtol=0, atol=1e-9)
    assert S.rotation_angle_error(T1, Tgt) < 1e-4 and S.translation_error(T1, Tgt) < 1e-3


@pytest.mark.parametrize("exchange", ["hook", "peer"])
def test_two_ranks_converge_on_the_same_iteration(tmp_path, exchange):
    """Convergence on (gicp.py:155-162): both ranks stop at the same iteration as one process."""
    r, _, T1, res1, _ = _run(tmp_path, 20_000, 60, fixed=False, exchange=exchange)
    assert np.array_equal(r[0]["T"], r[1]["T"])
    assert int(r[0]["iters"]) == int(r[1]["iters"])
    assert abs(int(r[0]["iters"]) - int(res1["iterations"])) <= 1
    np.testing.assert_allclose(r[0]["T"], T1, rtol=0, atol=1e-8)


def _rank_timeout(rank, world, port, d):
    """Rank 1 stops early: rank 0's next exchange must time out inside the kernel (bounded wait), fail
    its call with GICP_E_COMM, and leave the context usable."""
    import torch.distributed as dist
    from gicp import _lib
    from gicp import distributed as gd

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    src, tgt = np.load(os.path.join(d, "src.npy")), np.load(os.path.join(d, "tgt.npy"))
    p = gicp.default_params(3, fixed_iterations=1, **P3)
    eng = gicp.Engine(0)
    out = {}
    assert gd.init_peer(eng, rank, world, timeout=0.5) is None
    eng.set_target(tgt, p)
    eng.set_source(src, p, shard=rank, nshards=world)
    p.max_iterations = 4 if rank == 0 else 2
    try:
        eng.align(None, p)
        out["err"] = 0
    except _lib.GicpError as e:
        out["err"] = e.code
    dist.barrier()
    # the second peer_init probe: rank 1 never joins, so rank 0's probe times out
    if rank == 0:
        eng.peer_close()
        h = eng.peer_export()
        try:
            eng.peer_init(2, 0, [h, h], timeout=0.5)   # rank 1's slot: its own handle is not opened
            out["probe"] = 0
        except _lib.GicpError as e:
            out["probe"] = e.code
        out["kind"] = eng.comm_ranks()[2]
        p.max_iterations = 3   # alone again: the context still registers
        T, res = eng.align(None, p)
        out["after"] = int(res["iterations"])
    np.save(os.path.join(d, f"to{rank}.npy"), np.array(out, dtype=object), allow_pickle=True)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


def test_peer_exchange_times_out_instead_of_hanging(tmp_path):
    src, tgt, _ = S.scene_pair_3d(20_000)
    np.save(tmp_path / "src.npy", src)
    np.save(tmp_path / "tgt.npy", tgt)
    mp.spawn(_rank_timeout, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    r0 = np.load(tmp_path / "to0.npy", allow_pickle=True).item()
    r1 = np.load(tmp_path / "to1.npy", allow_pickle=True).item()
    from gicp import _lib
    assert r1["err"] == 0                       # the rank that stopped first finished its 2 iterations
    assert r0["err"] == _lib.GICP_E_COMM        # its peer's third exchange never came: bounded, reported
    assert r0["probe"] == _lib.GICP_E_COMM and r0["kind"] == "none"
    assert r0["after"] == 3


def _rank_fallback(rank, world, port, d, mode):
    """One rank's peer_init fails (`mode` 'bad_handle': rank 1 is handed its own handle as rank 0's, so its
    IPC open fails; 'skip': rank 1 never calls gicp_peer_init, so rank 0's probe kernel waits and times
    out).  Both ranks must agree on the failure (gd.init_peer returns the same note on each), both end
    with no peer exchange, and both then register through the host hook with bit-identical poses.  Then
    the peer exchange is set up again: the ranks' exchange counters differ after the failed probe (rank 0's
    advanced), and gicp_peer_init must bring them together (the exported counters' maximum)."""
    import torch
    import torch.distributed as dist
    from gicp import _lib
    from gicp import distributed as gd

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    src, tgt = np.load(os.path.join(d, "src.npy")), np.load(os.path.join(d, "tgt.npy"))
    p = gicp.default_params(3, fixed_iterations=1, max_iterations=8, **P3)
    eng = gicp.Engine(0)
    out = {}
    real_init = eng.peer_init
    if rank == 1 and mode == "bad_handle":
        def bad_init(n, r, handles, timeout=10.0):   # rank 0's slot holds rank 1's own area: the open fails
            return real_init(n, r, [handles[1]] + list(handles[1:]), timeout=timeout)
        eng.peer_init = bad_init
    elif rank == 1 and mode == "skip":
        def no_init(n, r, handles, timeout=10.0):
            raise _lib.GicpError(_lib.GICP_E_COMM, "rank 1 skips gicp_peer_init (test)")
        eng.peer_init = no_init
    out["note"] = gd.init_peer(eng, rank, world, timeout=2.0)
    out["kind_after_fail"] = eng.comm_ranks()[2]

    def allreduce(buf):
        t = torch.from_numpy(buf.copy())
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()
    eng.set_allreduce(allreduce, nranks=world, rank=rank)
    out["kind_hook"] = eng.comm_ranks()[2]
    eng.set_target(tgt, p)
    eng.set_source(src, p, shard=rank, nshards=world)
    out["T_hook"], _ = eng.align(None, p)
    # the peer exchange again, now on both ranks
    eng.peer_init = real_init
    eng.set_allreduce(None)
    out["note2"] = gd.init_peer(eng, rank, world, timeout=20.0)
    out["kind_peer"] = eng.comm_ranks()[2]
    out["T_peer"], res = eng.align(None, p)
    out["iters_peer"] = int(res["iterations"])
    np.save(os.path.join(d, f"fb{rank}.npy"), np.array(out, dtype=object), allow_pickle=True)
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["bad_handle", "skip"])
def test_peer_init_failure_is_agreed_and_both_ranks_fall_back(tmp_path, mode):
    src, tgt, _ = S.scene_pair_3d(20_000)
    np.save(tmp_path / "src.npy", src)
    np.save(tmp_path / "tgt.npy", tgt)
    mp.spawn(_rank_fallback, args=(2, _free_port(), str(tmp_path), mode), nprocs=2, join=True)
    r = [np.load(tmp_path / f"fb{k}.npy", allow_pickle=True).item() for k in range(2)]
    assert r[0]["note"] is not None and r[0]["note"] == r[1]["note"], (r[0]["note"], r[1]["note"])
    if mode == "skip":   # rank 0's probe kernel itself timed out (not an IPC open failure)
        assert r[0]["note"].startswith("rank 0") and "probe" in r[0]["note"], r[0]["note"]
    assert r[0]["kind_after_fail"] == r[1]["kind_after_fail"] == "none"
    assert r[0]["kind_hook"] == r[1]["kind_hook"] == "hook"
    assert np.array_equal(r[0]["T_hook"], r[1]["T_hook"])
    assert r[0]["note2"] is None and r[1]["note2"] is None
    assert r[0]["kind_peer"] == r[1]["kind_peer"] == "peer"
    assert r[0]["iters_peer"] == r[1]["iters_peer"] == 8
    assert np.array_equal(r[0]["T_peer"], r[1]["T_peer"])
    # the same registration through either exchange: the same rank-order sums, the same solve
    np.testing.assert_allclose(r[0]["T_peer"], r[0]["T_hook"], rtol=0, atol=1e-12)


def test_peer_exchange_with_an_empty_shard(tmp_path):
    """A shard with no source tile (more ranks than chunks: 2k points are one chunk, rank 1 gets none) still
    takes part in every exchange with one empty workgroup; its zero statistics leave the sums equal to the
    one-process pass, and both ranks end on the same pose."""
    r, st1, T1, res1, _ = _run(tmp_path, 2_000, 10, fixed=True, exchange="peer")
    assert np.array_equal(r[0]["T"], r[1]["T"]) and np.array_equal(r[0]["st"], r[1]["st"])
    scale = np.maximum(np.abs(st1), 1e-12 * np.abs(st1).max())
    assert np.max(np.abs(r[0]["st"] - st1) / scale) < 1e-12
    assert int(r[0]["corr"]) == int(res1["correspondences"])
    np.testing.assert_allclose(r[0]["T"], T1, rtol=0, atol=1e-12)
