"""Multi-GPU GICP: one process per GPU, source points sharded, statistics all-reduced.

The reference has no parallelism (its only concurrency is a pygame worker
process, robot-visualization.py:151-166,199).  Here the per-iteration work
partitions naturally: every rank holds the whole target (index + covariances)
and the whole source (its covariance neighbourhoods need all points), and
reduces only its shard of source tiles: chunks of 64 Morton-consecutive tiles
dealt round-robin over the ranks (``shard_tiles``).  The one exchange
per iteration is an all-reduce (sum) of the 74 fp64 statistics (26 in 2-D);
every rank then runs the identical host solve and the identical convergence
test, so no pose broadcast is needed.  Inside libgicp_hip.so that all-reduce
is RCCL (``ncclAllReduce`` over xGMI, communicator built by ``init_comm``);
``outer_loop`` states the same protocol in Python with a pluggable reducer.
"""
from __future__ import annotations

import numpy as np

from . import Engine, solve_pose

__all__ = ["init_comm", "init_peer", "shard_tiles", "align", "outer_loop"]


def init_comm(engine: Engine, rank: int, world: int, group=None):
    """Create the library's RCCL communicator: rank 0 makes the id, torch.distributed broadcasts it."""
    if world <= 1:
        return
    import torch.distributed as dist
    uid = [Engine.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0, group=group)
    engine.comm_init(world, rank, uid[0])


def init_peer(engine: Engine, rank: int, world: int, group=None, timeout=10.0):
    """The in-kernel peer exchange (gicp_peer_export / gicp_peer_init): every rank exports its exchange
    area, torch.distributed all-gathers the handles, every rank maps its peers' areas and runs the probe
    exchange.  The outcome is agreed over the group: returns None when every rank has the peer exchange
    on, else the first failure message seen on any rank (and every rank has closed it, so the caller can
    fall back to init_comm on all ranks alike)."""
    if world <= 1:
        return None
    import torch.distributed as dist
    err = None
    try:
        h = engine.peer_export()
    except Exception as e:   # noqa: BLE001 -- reported, and agreed below
        h, err = b"", f"rank {rank}: {e}"
    handles = [None] * world
    dist.all_gather_object(handles, h, group=group)
    if err is None and all(len(x) == len(h) for x in handles):
        try:
            engine.peer_init(world, rank, handles, timeout=timeout)
        except Exception as e:   # noqa: BLE001
            err = f"rank {rank}: {e}"
    elif err is None:
        err = "a rank could not export its exchange area"
    errs = [None] * world
    dist.all_gather_object(errs, err, group=group)
    first = next((e for e in errs if e is not None), None)
    if first is not None:
        engine.peer_close()
    return first


UNIT_TILES = 4      # source tiles per k_corr workgroup (kCorrWaves)
SHARD_CHUNK = 16    # units per shard chunk (kShardChunk, csrc/gicp_internal.h)


def shard_tiles(ntiles: int, rank: int, world: int):
    """Source tiles reduced by `rank` (the split gicp_set_source applies): the cloud's units of
    UNIT_TILES tiles are cut into chunks of SHARD_CHUNK units and rank r takes chunks r, r + world, ...
    (interleaved, so the heavy regions of a registration spread over the ranks)."""
    per = UNIT_TILES * SHARD_CHUNK
    nchunks = -(-ntiles // per)
    return np.concatenate([np.arange(c * per, min(ntiles, (c + 1) * per), dtype=np.int64)
                           for c in range(rank, nchunks, world)] or [np.zeros(0, np.int64)])


def align(engine: Engine, source, target, params, rank: int, world: int, T0=None):
    """Every rank calls this with the same clouds; returns the (identical) pose on every rank."""
    engine.set_target(target, params)
    engine.set_source(source, params, shard=rank, nshards=world)
    return engine.align(T0, params)


def outer_loop(pass_fn, T0, max_iterations=100, tolerance=1e-6, fixed_iterations=False, allreduce=None):
    """gicp.py:116-167 over a statistics provider.

    pass_fn(T) -> this rank's statistics at pose T; allreduce(stats) -> the sum
    over ranks (identity when None).  Returns (T, iterations, converged_at, loss).
    """
    T = np.array(T0, dtype=np.float64)
    last = np.inf
    loss = 0.0
    for it in range(max_iterations):
        st = np.asarray(pass_fn(T), dtype=np.float64)
        if allreduce is not None:
            st = allreduce(st)
        Tn, loss = solve_pose(st, T)
        if not fixed_iterations and abs(last - loss) < tolerance:
            return T, it + 1, it, loss
        last = loss
        T = Tn
    return T, max_iterations, -1, loss
