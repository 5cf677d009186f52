"""Synthetic scan pairs for the GICP engine.

Headless restatements of the reference's demo generators, plus the 3-D scenes
BASELINE.json's configs name.  Nothing here imports the
reference; the generators are re-derived from what the demos do:

* ``robot_scan`` / ``robot_pair`` — the 2-D LiDAR raycaster of
  ``python-implementation/robot-visualization.py:35-120`` driven the way its
  game loop drives it (``:224-237``): rays every ``360 // num_rays`` degrees,
  uniform ±2 px range noise on hits, points in the robot frame.
* ``vis_pair`` — the circle + square pair of ``visualization.py:9-44,169-194``
  (30 circle points, 60 of the 120 square points, motion (150, -50) px and
  pi/3, noise N(0, 2) / N(0, 5), target shuffled and 3 points dropped), seeded.
* ``segment_scene_2d`` — N points on N/200 random segments in a 1000 px box
  (the SURVEY.md §3.3 / BASELINE.md §3 2-D timing cloud).
* ``room_scene`` / ``scene_pair_3d`` — the 40 x 40 x 8 m room with 24 boxes and
  12 spheres of SURVEY.md §8(d) (configs C2/C3/C4), area-uniform samples,
  sigma = 5 mm noise, ground truth 2 deg about normalize(1, 2, 3) and
  t = (0.15, -0.10, 0.05) m.
"""
from __future__ import annotations

import math
import random as _random

import numpy as np

# --------------------------------------------------------------------------
# 2-D robot raycaster (robot-visualization.py:22-27, 35-40)
# --------------------------------------------------------------------------
ROBOT_MAX_RAY_RANGE = 400.0
ROBOT_NOISE = 2.0
# pygame.Rect(x, y, w, h) -> (x, y, w, h); edges walked topleft->topright->
# bottomright->bottomleft->topleft as the demo does (robot-visualization.py:52-57)
ROBOT_RECTS = ((100.0, 250.0, 200.0, 50.0), (400.0, 450.0, 50.0, 200.0))
ROBOT_CIRCLES = ((600.0, 300.0, 50.0), (200.0, 550.0, 75.0))


def _segment_hit(a, b, c, d):
    """Intersection of segment a-b with segment c-d (None if parallel / outside)."""
    (x1, y1), (x2, y2), (x3, y3), (x4, y4) = a, b, c, d
    den = (x1 - x2) * (y3 - y4) - (y1 - y2) * (x3 - x4)
    if den == 0:
        return None
    ta = ((x1 - x3) * (y3 - y4) - (y1 - y3) * (x3 - x4)) / den
    tb = -((x1 - x2) * (y1 - y3) - (y1 - y2) * (x1 - x3)) / den
    if 0 <= ta <= 1 and 0 <= tb <= 1:
        return (x1 + ta * (x2 - x1), y1 + ta * (y2 - y1))
    return None


def _circle_hits(a, b, centre, radius):
    (x1, y1), (x2, y2) = a, b
    dx, dy = x2 - x1, y2 - y1
    fx, fy = x1 - centre[0], y1 - centre[1]
    qa = dx * dx + dy * dy
    qb = 2 * (fx * dx + fy * dy)
    qc = (fx * fx + fy * fy) - radius * radius
    disc = qb * qb - 4 * qa * qc
    if disc < 0:
        return []
    disc = math.sqrt(disc)
    hits = []
    for tt in ((-qb - disc) / (2 * qa), (-qb + disc) / (2 * qa)):
        if 0 <= tt <= 1:
            hits.append((x1 + tt * dx, y1 + tt * dy))
    return hits


def cast_ray(pos, angle_deg, rnd=_random, max_range=ROBOT_MAX_RAY_RANGE, noise=ROBOT_NOISE):
    """Noisy range of the first obstacle hit along ``angle_deg`` or None."""
    x1, y1 = pos
    end = (x1 + max_range * math.cos(math.radians(angle_deg)),
           y1 + max_range * math.sin(math.radians(angle_deg)))
    best = float("inf")
    hit = False
    for (rx, ry, rw, rh) in ROBOT_RECTS:
        corners = ((rx, ry), (rx + rw, ry), (rx + rw, ry + rh), (rx, ry + rh))
        for k in range(4):
            p = _segment_hit((x1, y1), end, corners[k], corners[(k + 1) % 4])
            if p is not None:
                dist = math.hypot(p[0] - x1, p[1] - y1)
                if dist < best:
                    best, hit = dist, True
    for (cx, cy, r) in ROBOT_CIRCLES:
        for p in _circle_hits((x1, y1), end, (cx, cy), r):
            dist = math.hypot(p[0] - x1, p[1] - y1)
            if dist < best:
                best, hit = dist, True
    if not hit:
        return None
    return best + rnd.uniform(-noise, noise)


def robot_scan(x, y, yaw_deg, num_rays=90, rnd=_random):
    """One scan in the robot frame, as robot-visualization.py:222-237 builds it."""
    pts = []
    for angle in range(int(yaw_deg), int(yaw_deg) + 360, 360 // num_rays):
        d = cast_ray((x, y), angle, rnd)
        if d:  # the demo drops a (measure-zero) exact 0.0 range too
            pts.append((d * math.cos(math.radians(angle - yaw_deg)),
                        d * math.sin(math.radians(angle - yaw_deg))))
    return np.asarray(pts, dtype=np.float64).reshape(-1, 2)


# Pose pairs (x, y, yaw_deg) used for the committed robot fixtures.
ROBOT_POSE_PAIRS = (
    ((300.0, 400.0, 0), (310.0, 400.0, 4)),
    ((250.0, 420.0, 30), (255.0, 424.0, 32)),
    ((520.0, 380.0, 90), (520.0, 372.0, 96)),
)


def robot_pair(pair=0, num_rays=90, seed=0):
    """(source, target) = (previous scan, current scan), robot-visualization.py:250-252."""
    rnd = _random.Random(seed)
    a, b = ROBOT_POSE_PAIRS[pair]
    src = robot_scan(*a, num_rays=num_rays, rnd=rnd)
    tgt = robot_scan(*b, num_rays=num_rays, rnd=rnd)
    return src, tgt


# --------------------------------------------------------------------------
# visualization.py pair (visualization.py:9-44, 169-194), seeded
# --------------------------------------------------------------------------
def _square_outline(centre, size, per_side, rnd):
    half = size / 2
    xs = np.linspace(centre[0] - half, centre[0] + half, per_side)
    ys = np.linspace(centre[1] - half, centre[1] + half, per_side)
    outline = ([[x, centre[1] - half] for x in xs] + [[centre[0] + half, y] for y in ys]
               + [[x, centre[1] + half] for x in xs] + [[centre[0] - half, y] for y in ys])
    keep = set(rnd.sample(range(len(outline)), len(outline) // 2))
    return np.array([p for i, p in enumerate(outline) if i in keep])


def _circle_outline(centre, radius, n, rnd):
    out = []
    for _ in range(n):
        a = rnd.uniform(0, 2 * np.pi)
        out.append([centre[0] + radius * np.cos(a), centre[1] + radius * np.sin(a)])
    return np.array(out)


def vis_pair(seed=0):
    """Source (90 pts) and target (87 pts) of the static demo, expected T ~ [R(60 deg) | (150, -50)]."""
    rnd = _random.Random(seed)
    nrs = np.random.RandomState(seed)
    src = np.concatenate([_circle_outline((300, 150), 100, 30, rnd),
                          _square_outline((600, 250), 200, 30, rnd)])
    ang = np.pi / 3
    rot = np.array([[np.cos(ang), -np.sin(ang)], [np.sin(ang), np.cos(ang)]])
    tgt = src @ rot.T + np.array([150, -50])
    src = src + nrs.normal(0, 2, src.shape)
    tgt = tgt + nrs.normal(0, 5, tgt.shape)
    nrs.shuffle(tgt)
    return src, tgt[: len(tgt) - 3]


# --------------------------------------------------------------------------
# 2-D segment scene (BASELINE.md §3 timing cloud)
# --------------------------------------------------------------------------
def rot2(theta):
    c, s = math.cos(theta), math.sin(theta)
    return np.array([[c, -s], [s, c]])


def segment_scene_2d(n, seed=0, theta=0.02, t=(2.0, -1.0), sigma=0.5, box=1000.0):
    """(source, target, T_gt) with target ~= T_gt(source); n points each on n/200 segments."""
    rng = np.random.default_rng(seed)
    nseg = max(1, n // 200)
    a = rng.uniform(0, box, (nseg, 2))
    b = rng.uniform(0, box, (nseg, 2))

    def sample(m):
        k = rng.integers(0, nseg, m)
        u = rng.random(m)[:, None]
        return a[k] + u * (b[k] - a[k])

    T = np.eye(3)
    T[:2, :2] = rot2(theta)
    T[:2, 2] = t
    tgt = sample(n) + rng.normal(0, sigma, (n, 2))
    src_w = sample(n)
    src = (src_w - T[:2, 2]) @ T[:2, :2] + rng.normal(0, sigma, (n, 2))
    return src, tgt, T


# --------------------------------------------------------------------------
# 3-D room scene
# --------------------------------------------------------------------------
def axis_angle(axis, angle):
    axis = np.asarray(axis, dtype=np.float64)
    axis = axis / np.linalg.norm(axis)
    k = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + math.sin(angle) * k + (1 - math.cos(angle)) * (k @ k)


def gt_transform_3d(deg=2.0, axis=(1, 2, 3), t=(0.15, -0.10, 0.05)):
    T = np.eye(4)
    T[:3, :3] = axis_angle(axis, math.radians(deg))
    T[:3, 3] = t
    return T


class Scene3D:
    """Rectangles (origin, edge1, edge2) and spheres (centre, radius)."""

    def __init__(self, rects, spheres):
        self.rects = np.asarray(rects, dtype=np.float64).reshape(-1, 3, 3)
        self.spheres = np.asarray(spheres, dtype=np.float64).reshape(-1, 4)

    def areas(self):
        ra = np.linalg.norm(np.cross(self.rects[:, 1], self.rects[:, 2]), axis=1)
        sa = 4 * np.pi * self.spheres[:, 3] ** 2
        return np.concatenate([ra, sa])

    def sample(self, n, rng):
        """n area-uniform surface points."""
        area = self.areas()
        prim = rng.choice(len(area), size=n, p=area / area.sum())
        out = np.empty((n, 3))
        nr = len(self.rects)
        isr = prim < nr
        ids = prim[isr]
        uv = rng.random((len(ids), 2))
        r = self.rects[ids]
        out[isr] = r[:, 0] + uv[:, :1] * r[:, 1] + uv[:, 1:] * r[:, 2]
        ids = prim[~isr] - nr
        d = rng.normal(size=(len(ids), 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        s = self.spheres[ids]
        out[~isr] = s[:, :3] + s[:, 3:] * d
        return out


def _box_faces(centre, half, yaw):
    rz = axis_angle((0, 0, 1), yaw)
    ex, ey, ez = (rz[:, i] * half[i] for i in range(3))
    faces = []
    for (u, v, w) in ((ex, ey, ez), (ey, ez, ex), (ez, ex, ey)):
        for sgn in (-1, 1):
            o = centre + sgn * w - u - v
            faces.append((o, 2 * u, 2 * v))
    return faces


def room_scene(seed=42, size=(40.0, 40.0, 8.0), n_boxes=24, n_spheres=12):
    rng = np.random.default_rng(seed)
    lx, ly, lz = size
    x0, y0 = -lx / 2, -ly / 2
    X, Y, Z = np.eye(3)
    rects = [
        (np.array([x0, y0, 0.0]), lx * X, ly * Y),          # floor
        (np.array([x0, y0, lz]), lx * X, ly * Y),           # ceiling
        (np.array([x0, y0, 0.0]), lx * X, lz * Z),          # wall y = y0
        (np.array([x0, -y0, 0.0]), lx * X, lz * Z),         # wall y = -y0
        (np.array([x0, y0, 0.0]), ly * Y, lz * Z),          # wall x = x0
        (np.array([-x0, y0, 0.0]), ly * Y, lz * Z),         # wall x = -x0
    ]
    for _ in range(n_boxes):
        half = rng.uniform(0.25, 1.5, 3)
        c = np.array([rng.uniform(x0 + 2, -x0 - 2), rng.uniform(y0 + 2, -y0 - 2), half[2]])
        rects.extend(_box_faces(c, half, rng.uniform(0, np.pi)))
    spheres = []
    for _ in range(n_spheres):
        r = rng.uniform(0.5, 2.0)
        spheres.append((rng.uniform(x0 + 3, -x0 - 3), rng.uniform(y0 + 3, -y0 - 3),
                        rng.uniform(r, lz - r), r))
    return Scene3D(rects, spheres)


def scene_pair_3d(n_src, n_tgt=None, sigma=0.005, T_gt=None, scene=None):
    """(source, target, T_gt) with target ~= T_gt(source), SURVEY.md §8(d) C2/C3."""
    n_tgt = n_src if n_tgt is None else n_tgt
    scene = room_scene() if scene is None else scene
    T_gt = gt_transform_3d() if T_gt is None else T_gt
    rt = np.random.default_rng(1)
    tgt = scene.sample(n_tgt, rt)
    tgt += rt.normal(0, sigma, tgt.shape)
    rs = np.random.default_rng(0)
    src_w = scene.sample(n_src, rs)
    src = (src_w - T_gt[:3, 3]) @ T_gt[:3, :3] + rs.normal(0, sigma, src_w.shape)
    return src, tgt, T_gt


def transform_points(points, T):
    """x -> R x + t for (d+1)x(d+1) homogeneous T."""
    d = T.shape[0] - 1
    return np.asarray(points)[:, :d] @ T[:d, :d].T + T[:d, d]


def rotation_angle_error(Ta, Tb):
    """Geodesic angle (rad) between the rotation parts of two transforms."""
    d = Ta.shape[0] - 1
    Rr = Ta[:d, :d].T @ Tb[:d, :d]
    if d == 2:
        return abs(math.atan2(Rr[1, 0], Rr[0, 0]))
    c = (np.trace(Rr) - 1) / 2
    return math.acos(max(-1.0, min(1.0, c)))


def translation_error(Ta, Tb):
    d = Ta.shape[0] - 1
    return float(np.linalg.norm(Ta[:d, d] - Tb[:d, d]))


# ----------------------------------------------------------------------------- C5: LiDAR stream
# a spinning LiDAR (64 beams, elevation -25..+15 deg, 1563 azimuths ~ 100k rays,
# 100 m range, uniform +-0.02 m range noise mirroring robot-visualization.py:74) moving through the
# C2 room; each frame is registered against the previous one (robot-visualization.py:239-265).

def lidar_scene(radius=14.0, clearance=2.5, seed=42):
    """The C2 room without the obstacles that block the circular sensor path (centre 0, `radius`)."""
    sc = room_scene(seed=seed)
    keep = []
    for k in range(6, len(sc.rects), 6):     # boxes are 6 faces each after the 6 room rectangles
        c = (sc.rects[k:k + 6, 0] + 0.5 * (sc.rects[k:k + 6, 1] + sc.rects[k:k + 6, 2])).mean(axis=0)
        if abs(math.hypot(c[0], c[1]) - radius) > clearance + 1.5:
            keep.extend(range(k, k + 6))
    rects = np.concatenate([sc.rects[:6], sc.rects[keep]]) if keep else sc.rects[:6]
    sph = [s for s in sc.spheres if abs(math.hypot(s[0], s[1]) - radius) > clearance + s[3]]
    return Scene3D(rects, np.asarray(sph).reshape(-1, 4))


def lidar_trajectory(frames, seed=7, radius=14.0, step=0.5, yaw_step_deg=0.5, height=1.8, along_path=False):
    """Sensor-to-world poses (4x4) on a circle of `radius`: per frame ~`step` m
    along the circle and ~`yaw_step_deg` of yaw, both jittered by +-10 % from rng(seed).  A 0.5 m /
    0.5 deg frame cannot follow a circle that fits the 40 m room (0.5 deg per 0.5 m is a 57 m
    radius), so the sensor's yaw turns at its own rate; `along_path=True` instead keeps it looking
    along the path (yaw step = step / radius)."""
    rng = np.random.default_rng(seed)
    poses = []
    ang, yaw = 0.0, math.pi / 2
    for _ in range(frames):
        T = np.eye(4)
        T[:3, :3] = axis_angle((0, 0, 1), ang + math.pi / 2 if along_path else yaw)
        T[:3, 3] = (radius * math.cos(ang), radius * math.sin(ang), height)
        poses.append(T)
        ang += step / radius * (1.0 + 0.2 * (rng.random() - 0.5))
        if not along_path:
            yaw += math.radians(yaw_step_deg) * (1.0 + 0.2 * (rng.random() - 0.5))
    return np.asarray(poses)


def lidar_dirs(beams=64, azimuths=1563, elev=(-25.0, 15.0)):
    el = np.radians(np.linspace(elev[0], elev[1], beams))
    az = np.radians(np.arange(azimuths) * 360.0 / azimuths)
    ce, se = np.cos(el)[:, None], np.sin(el)[:, None]
    d = np.stack([ce * np.cos(az)[None, :], ce * np.sin(az)[None, :], np.broadcast_to(se, (beams, azimuths))], -1)
    return d.reshape(-1, 3)


def lidar_scan(scene, pose, dirs, rng, max_range=100.0, noise=0.02, xp=None, device=None):
    """Points (sensor frame) where the rays `dirs` (sensor frame) from `pose` first hit `scene`.
    `xp`: None for NumPy, or the `torch` module (then computed on `device`, returned as NumPy)."""
    if xp is None:
        return _lidar_scan_np(scene, pose, dirs, rng, max_range, noise)
    return _lidar_scan_torch(xp, scene, pose, dirs, rng, max_range, noise, device)


def _lidar_scan_np(scene, pose, dirs, rng, max_range, noise):
    R, o = pose[:3, :3], pose[:3, 3]
    D = dirs @ R.T                                            # world directions
    best = np.full(len(D), np.inf)
    for p0, e1, e2 in scene.rects:
        n = np.cross(e1, e2)
        dn = D @ n
        with np.errstate(divide="ignore", invalid="ignore"):
            t = ((p0 - o) @ n) / dn
        h = o + t[:, None] * D - p0
        a = (h @ e1) / (e1 @ e1)
        b = (h @ e2) / (e2 @ e2)
        ok = (t > 1e-6) & (a >= 0) & (a <= 1) & (b >= 0) & (b <= 1)
        best = np.where(ok & (t < best), t, best)
    for cx, cy, cz, r in scene.spheres:
        oc = o - np.array([cx, cy, cz])
        bq = D @ oc
        disc = bq * bq - (oc @ oc - r * r)
        sq = np.sqrt(np.maximum(disc, 0))
        for t in (-bq - sq, -bq + sq):
            ok = (disc >= 0) & (t > 1e-6) & (t < best)
            best = np.where(ok, t, best)
    hit = best < max_range
    rng_ = best[hit] + rng.uniform(-noise, noise, hit.sum())
    return dirs[hit] * rng_[:, None]


def _lidar_scan_torch(torch, scene, pose, dirs, rng, max_range, noise, device):
    f = lambda a: torch.as_tensor(np.asarray(a, dtype=np.float64), device=device)
    R, o = f(pose[:3, :3]), f(pose[:3, 3])
    dt = f(dirs)
    D = dt @ R.T
    rects = f(scene.rects)
    p0, e1, e2 = rects[:, 0], rects[:, 1], rects[:, 2]
    n = torch.linalg.cross(e1, e2)
    dn = D @ n.T                                              # rays x rects
    t = ((p0 - o) * n).sum(1)[None, :] / dn
    hx = o[None, None, :] + t[..., None] * D[:, None, :] - p0[None]
    a = (hx * e1[None]).sum(-1) / (e1 * e1).sum(1)[None]
    b = (hx * e2[None]).sum(-1) / (e2 * e2).sum(1)[None]
    ok = (t > 1e-6) & (a >= 0) & (a <= 1) & (b >= 0) & (b <= 1)
    best = torch.where(ok, t, torch.full_like(t, float("inf"))).min(1).values
    if len(scene.spheres):
        sp = f(scene.spheres)
        oc = o[None, :] - sp[:, :3]                            # spheres x 3
        bq = D @ oc.T                                          # rays x spheres
        disc = bq * bq - ((oc * oc).sum(1) - sp[:, 3] ** 2)[None]
        sq = torch.sqrt(torch.clamp(disc, min=0))
        for tt in (-bq - sq, -bq + sq):
            ok = (disc >= 0) & (tt > 1e-6)
            best = torch.minimum(best, torch.where(ok, tt, torch.full_like(tt, float("inf"))).min(1).values)
    best = best.cpu().numpy()
    hit = best < max_range
    rng_ = best[hit] + rng.uniform(-noise, noise, hit.sum())
    return dirs[hit] * rng_[:, None]


def lidar_stream(frames, beams=64, azimuths=1563, seed=7, xp=None, device=None, **traj):
    """Generator of (scan_k, pose_k) for k = 0..frames-1 (scans in sensor coordinates); `traj`:
    lidar_trajectory keywords (step, yaw_step_deg, along_path)."""
    scene = lidar_scene()
    poses = lidar_trajectory(frames, seed=seed, **traj)
    dirs = lidar_dirs(beams, azimuths)
    rng = np.random.default_rng(seed + 1)
    for k in range(frames):
        yield lidar_scan(scene, poses[k], dirs, rng, xp=xp, device=device), poses[k]
