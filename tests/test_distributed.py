"""world_size-2 gloo rehearsal of the multi-GPU protocol on CPU: source shards, all-reduce of the
statistics, identical host solve on every rank (the RCCL path in libgicp_hip.so does the same)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import gicp_oracle as O

gicp = pytest.importorskip("gicp")
from gicp import distributed as GD  # noqa: E402
from gicp import synthetic as S  # noqa: E402

P3 = dict(max_distance_correspondence=0.5, max_distance_nearest_neighbors=1.0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _problem(n=3000):
    src, tgt, Tgt = S.scene_pair_3d(n)
    Cs, _ = O.covariances(src, P3["max_distance_nearest_neighbors"])
    Ct, _ = O.covariances(tgt, P3["max_distance_nearest_neighbors"])
    return src, tgt, Cs, Ct, Tgt


def _pass_fn(src, tgt, Cs, Ct, rows):
    """Oracle statistics of the source rows this rank owns (stand-in for the GPU pass)."""
    def f(T):
        s = src[rows]
        moved = O.apply_transformation(s, T)
        idx, _ = O.correspondences(moved, tgt, P3["max_distance_correspondence"])
        R = T[:3, :3]
        W = O.weights(np.einsum("ab,nbc,dc->nad", R, Cs[rows], R), Ct, idx)
        q = np.zeros_like(s)
        q[idx >= 0] = tgt[idx[idx >= 0]]
        return O.stats(s, q, W, idx, T)
    return f


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import torch
    src, tgt, Cs, Ct, _ = _problem()
    n = len(src)
    rows = GD.shard_tiles(n, rank, world)          # interleaved chunks, as the library shards tiles

    def allreduce(st):
        t = torch.from_numpy(st.copy())
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.numpy()

    T, iters, conv, loss = GD.outer_loop(_pass_fn(src, tgt, Cs, Ct, rows), np.eye(4), max_iterations=15,
                                         tolerance=1e-10, allreduce=allreduce)
    np.save(os.path.join(out_dir, f"T{rank}.npy"), np.concatenate([T.ravel(), [iters, conv, loss]]))
    dist.destroy_process_group()


def test_shard_tiles_partition():
    for nt in (1, 7, 64, 1000, 15625):
        for world in (1, 2, 3, 8):
            r = [GD.shard_tiles(nt, k, world) for k in range(world)]
            allt = np.sort(np.concatenate(r))
            assert np.array_equal(allt, np.arange(nt))   # a partition of the tiles
            if nt >= 64 * world:                          # chunks of 64 tiles, round-robin
                assert r[0][0] == 0 and r[min(1, world - 1)][0] == 64 * min(1, world - 1)


def test_two_rank_gloo_matches_single_process(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r0, r1 = (np.load(tmp_path / f"T{k}.npy") for k in range(world))
    assert np.array_equal(r0, r1), "ranks disagree: the all-reduced statistics must give identical solves"
    src, tgt, Cs, Ct, Tgt = _problem()
    T1, iters, conv, loss = GD.outer_loop(_pass_fn(src, tgt, Cs, Ct, np.arange(len(src))), np.eye(4),
                                          max_iterations=15, tolerance=1e-10)
    np.testing.assert_allclose(r0[:16].reshape(4, 4), T1, atol=1e-10)
    assert int(r0[16]) == iters
    # the sparse 3k-point cloud still moves toward the ground truth (2 deg, 19 cm)
    assert S.translation_error(T1, Tgt) < S.translation_error(np.eye(4), Tgt)


def test_sharded_statistics_are_additive():
    src, tgt, Cs, Ct, _ = _problem(1500)
    T = np.eye(4)
    T[:3, 3] = [0.02, 0.01, -0.01]
    full = _pass_fn(src, tgt, Cs, Ct, np.arange(len(src)))(T)
    parts = [_pass_fn(src, tgt, Cs, Ct, GD.shard_tiles(len(src), k, 4))(T) for k in range(4)]
    np.testing.assert_allclose(np.sum(parts, axis=0), full, rtol=1e-12, atol=1e-12 * np.abs(full).max())
