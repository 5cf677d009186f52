"""Scan-to-scan odometry over a frame stream — the pattern of robot-visualization.py:239-265
(SURVEY.md §8(f) rank 1, config C5), on the device.

Each new scan becomes the target; the previous target, with its index and covariances already on
the GPU, becomes the source (`gicp_target_to_source`, robot-visualization.py:250) — so per frame
only the new scan is uploaded, sorted, tiled and given covariances.  Given the coming scans
(`step(scan, next_scan)` / `run(scans, depth)`), their builds run on their own streams from host
threads while the current pair is registered (`gicp_stage_target` / `gicp_commit_target`, up to
GICP_MAX_STAGED ahead), so setup leaves the critical path (the demo likewise prepares the next scan
while its worker registers, robot-visualization.py:239-252).  A staged scan is copied by the library
before stage_target returns, so the caller may refill its buffer at once (borrow=True skips that copy for
callers that leave their scans untouched until registered).  `gicp(prev, cur)` maps the
previous sensor frame into the current one (p_cur = T p_prev), so the sensor pose advances by
T^-1: `composition='se3'` (default) is that exact SE(d) update; `composition='reference'` is the
demo's first-order update (robot-visualization.py:257-265: translation -T[:2, d], yaw
-atan2(T[1,0], T[0,0]), rotated by the last yaw), kept for trajectory comparisons with the demo.
"""
import math
import time

import numpy as np

from . import Engine, default_params


class Odometry:
    def __init__(self, dim=3, params=None, device=0, composition="se3", init="constant_velocity", borrow=False,
                 **kw):
        if composition not in ("se3", "reference"):
            raise ValueError("composition must be 'se3' or 'reference'")
        if init not in ("identity", "constant_velocity"):
            raise ValueError("init must be 'identity' or 'constant_velocity'")
        self.dim = dim
        self.params = params if params is not None else default_params(dim, **kw)
        self.eng = Engine(device)
        self.composition = composition
        self.init = init
        # borrow=True: staged scans are read by the library in place (GICP_STAGE_BORROW, no copy on this
        # thread); the caller must not modify a scan passed as a coming scan until it has been step()ped
        self.borrow = bool(borrow)
        self.reset()

    def reset(self):
        """Start a new stream (the device context and its buffers are kept)."""
        dim = self.dim
        self._pose = np.eye(dim + 1)         # current sensor -> world (first frame = origin)
        self._poses = [self._pose.copy()]
        self._yaw_xy = (0.0, 0.0, 0.0)       # reference-formula state (x, y, yaw)
        self._pending = []                   # registrations not yet composed into the pose (see _flush)
        self.last_T = None
        self.frames = 0
        if getattr(self, "_staged", None):
            self.eng.cancel_stage()
        self._staged = []                    # the scan objects whose builds are staged, oldest first
        self.timing = {"setup_s": 0.0, "align_s": 0.0, "iterations": 0}

    def _prep(self, scan):
        return np.ascontiguousarray(np.asarray(scan, dtype=np.float64)[:, :self.dim])

    def step(self, scan, next_scan=None, next_scans=()):
        """Add one scan; returns (T, result) of its registration against the previous scan, or
        (None, None) for the first frame.  `next_scan` (or the list `next_scans`, at most
        Engine.MAX_STAGED), if given, is built on the device while this pair is registered; pass the
        same objects as `scan` of the next calls, in order.  By default the library copies a staged scan
        before the call returns, so the caller may reuse the array at once; with borrow=True the library
        reads the caller's array in place (no copy on this thread), and the caller must leave it unchanged
        until that scan has itself been step()ped."""
        t0 = time.perf_counter()
        if self._staged and self._staged[0] is scan:
            try:
                self.eng.commit_target()        # built during an earlier registration
            finally:                            # the library consumed the slot even if its build failed
                self._staged.pop(0)
        else:
            if self._staged:
                self.eng.cancel_stage()
                self._staged = []
            if self.frames > 0:
                self.eng.target_to_source()
            self.eng.set_target(self._prep(scan), self.params)
        coming = list(next_scans) if next_scan is None else [next_scan, *next_scans]
        want = coming[:self.eng.MAX_STAGED]
        n_ok = 0                                # staged builds that are a prefix of the coming scans
        while n_ok < min(len(want), len(self._staged)) and self._staged[n_ok] is want[n_ok]:
            n_ok += 1
        if n_ok < min(len(want), len(self._staged)):   # a different stream than staged: start over, all of it
            self.eng.cancel_stage()
            self._staged = []
        for s in want[len(self._staged):]:
            self.eng.stage_target(self._prep(s), self.params, borrow=self.borrow)
            self._staged.append(s)
        t1 = time.perf_counter()
        self.timing["setup_s"] += t1 - t0
        self.frames += 1
        if self.frames == 1:
            return None, None
        T0 = self.last_T if (self.init == "constant_velocity" and self.last_T is not None) else None
        T, res = self.eng.align(T0, self.params)
        self.timing["align_s"] += time.perf_counter() - t1
        self.timing["iterations"] += res["iterations"]
        self.last_T = T
        self._integrate(T)
        return T, res

    def run(self, scans, depth=2):
        """Register a whole stream, each scan's build started `depth` registrations ahead (1: during the
        previous registration; 2, the default: during the two before it, so a build that takes longer
        than one registration stays off the critical path); yields (T, result) per scan."""
        depth = max(1, min(int(depth), self.eng.MAX_STAGED))
        it = iter(scans)
        window = []
        for s in it:
            window.append(s)
            if len(window) > depth:
                break
        while window:
            cur = window.pop(0)
            nxt = next(it, None)
            if nxt is not None:
                window.append(nxt)
            yield self.step(cur, next_scans=window[:depth])

    def _integrate(self, T):
        # composed when the pose is read (the same compositions in the same order): the stream's loop does not
        # wait on a 4 x 4 inverse per frame
        self._pending.append(T)

    def _flush(self):
        for T in self._pending:
            self._pose, self._yaw_xy = compose(self._pose, T, self.composition, self._yaw_xy)
            self._poses.append(self._pose.copy())
        self._pending = []

    @property
    def pose(self):
        """Current sensor -> world pose."""
        self._flush()
        return self._pose

    @pose.setter
    def pose(self, value):
        """Set the current sensor pose (e.g. a stream that starts from a known pose).  It replaces the
        latest entry of `poses`, and the reference formula's planar state follows it (x, y and the yaw of
        the pose's first two axes), so either composition continues from it."""
        self._flush()
        P = np.asarray(value, dtype=np.float64).copy()
        d = self.dim
        if P.shape != (d + 1, d + 1):
            raise ValueError(f"pose must be {d + 1} x {d + 1}")
        self._pose = P
        self._poses[-1] = P.copy()
        self._yaw_xy = (float(P[0, d]), float(P[1, d]), math.atan2(P[1, 0], P[0, 0]))

    @property
    def poses(self):
        """Sensor poses of every frame so far (the first frame is the origin)."""
        self._flush()
        return self._poses

    @poses.setter
    def poses(self, value):
        self._flush()
        self._poses = [np.asarray(P, dtype=np.float64).copy() for P in value]

    @property
    def yaw_xy(self):
        """The reference formula's planar state (x, y, yaw) (composition='reference')."""
        self._flush()
        return self._yaw_xy

    @yaw_xy.setter
    def yaw_xy(self, value):
        """Set the planar state; with composition='reference' the pose is rebuilt from it, as compose does."""
        self._flush()
        x, y, yaw = (float(v) for v in value)
        self._yaw_xy = (x, y, yaw)
        if self.composition == "reference":
            d = self.dim
            P = np.eye(d + 1)
            c, s = math.cos(yaw), math.sin(yaw)
            P[0, 0], P[0, 1], P[1, 0], P[1, 1] = c, -s, s, c
            P[0, d], P[1, d] = x, y
            self._pose = P


def compose(pose, T, composition="se3", yaw_xy=(0.0, 0.0, 0.0)):
    """Advance the sensor pose by one registration T (p_cur = T p_prev).  Returns (pose, yaw_xy).
    'se3': pose @ T^-1.  'reference': robot-visualization.py:257-265 — translation (-T[0,d], -T[1,d])
    rotated by the last yaw, yaw += -atan2(T[1,0], T[0,0]) — rebuilt as a planar pose."""
    d = T.shape[0] - 1
    if composition == "se3":
        return pose @ np.linalg.inv(T), tuple(yaw_xy)
    x, y, yaw = yaw_xy
    dx, dy = -T[0, d], -T[1, d]
    dyaw = -math.atan2(T[1, 0], T[0, 0])
    x, y = x + dx * math.cos(yaw) - dy * math.sin(yaw), y + dx * math.sin(yaw) + dy * math.cos(yaw)
    yaw += dyaw
    P = np.eye(d + 1)
    c, s = math.cos(yaw), math.sin(yaw)
    P[0, 0], P[0, 1], P[1, 0], P[1, 1] = c, -s, s, c
    P[0, d], P[1, d] = x, y
    return P, (x, y, yaw)
