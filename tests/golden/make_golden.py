"""Capture golden vectors from the reference ``gicp.py`` (run in the build container ONLY).

The reference (``/root/reference/python-implementation/gicp.py``) is imported
unchanged, never copied: this script drives it on seeded synthetic inputs and
stores inputs + outputs as ``.npz`` fixtures next to itself.  The GPU box never
sees the reference; the fixtures are the only thing that travels.

What each fixture holds:

* inputs ``source``, ``target`` and the ``gicp()`` keyword arguments;
* the full 7-tuple ``gicp()`` returns (gicp.py:174);
* per outer iteration, read out of the reference's own ``fmin_cg`` call
  (gicp.py:148-154) by wrapping ``fmin_cg`` and reading the closure of the
  loss lambda: ``x0``, ``xopt``, ``fopt``, ``nfev``, ``ngev``, ``warnflag``,
  the corresponding target points ``q`` and the weight matrices ``W``
  (gicp.py:124-145), and the correspondence index ``idx`` recovered from
  ``q`` (-1 where the reference rejected the point, gicp.py:136-138);
* ``ens_T``: the distinct final transforms over runs whose source was
  perturbed by 1e-9 and 1e-7 relative noise, plus the unperturbed run (the
  reference's endpoint ensemble, SURVEY.md §8(c) grading rule).

Run:  ``PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py``
"""
from __future__ import annotations

import contextlib
import io
import os
import sys
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF_DIR = "/root/reference/python-implementation"
sys.path.insert(0, os.path.join(HERE, "..", "..", "generalized-icp_amd"))

from gicp import synthetic as S  # noqa: E402


def _ref():
    sys.dont_write_bytecode = True
    if REF_DIR not in sys.path:
        sys.path.insert(0, REF_DIR)
    import gicp as ref  # the reference module (shadowing is fine: separate process)
    return ref


def _load_ref_module():
    """Import the reference gicp.py under a private name (our package is also `gicp`)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ref_gicp", os.path.join(REF_DIR, "gicp.py"))
    mod = importlib.util.module_from_spec(spec)
    sys.dont_write_bytecode = True
    spec.loader.exec_module(mod)
    return mod


def run_reference(src, tgt, kwargs, record=True):
    ref = _load_ref_module()
    real_cg = ref.fmin_cg
    recs = []

    def spy(f, x0, fprime, **kw):
        cells = dict(zip(f.__code__.co_freevars, (c.cell_contents for c in f.__closure__)))
        out = real_cg(f, x0, fprime=fprime, **kw)
        if record:
            recs.append(dict(x0=np.array(x0, dtype=np.float64), xopt=np.array(out[0]), fopt=float(out[1]),
                             nfev=int(out[2]), ngev=int(out[3]), warnflag=int(out[4]),
                             q=np.array(cells["corresponding_target_points"]),
                             W=np.array(cells["weight_matrices"])))
        return out

    ref.fmin_cg = spy
    with contextlib.redirect_stdout(io.StringIO()) as buf:
        res = ref.gicp(src, tgt, **kwargs)
    return res, recs, buf.getvalue()


def recover_idx(q, W, tgt):
    idx = np.full(len(q), -1, dtype=np.int64)
    for i in range(len(q)):
        if not np.any(W[i]):
            continue
        m = np.nonzero(np.all(tgt == q[i], axis=1))[0]
        idx[i] = m[0] if len(m) else -2
    return idx


def _final_T(args):
    src, tgt, kwargs = args
    res, _, _ = run_reference(src, tgt, kwargs, record=False)
    return res[0]


def ensemble(src, tgt, kwargs, n_per_level=16, levels=(1e-9, 1e-7), seed=1234, pool=None):
    rng = np.random.default_rng(seed)
    jobs = []
    for eps in levels:
        for _ in range(n_per_level):
            jobs.append((src + eps * np.abs(src) * rng.standard_normal(src.shape), tgt, kwargs))
    Ts = list(pool.map(_final_T, jobs)) if pool is not None else [_final_T(j) for j in jobs]
    return Ts


def dedupe(Ts, tol=1e-9):
    out = []
    for T in Ts:
        if not any(np.max(np.abs(T - U)) <= tol for U in out):
            out.append(T)
    return np.stack(out)


def capture(name, src, tgt, kwargs, pool, ens=16, keep_iters=None):
    res, recs, log = run_reference(src, tgt, kwargs)
    T, all_T, init_src_cov, tgt_cov, hw_s, hw_t, all_src_cov = res
    n_it = len(recs)
    keep = n_it if keep_iters is None else min(n_it, keep_iters)
    d = dict(
        source=np.asarray(src, dtype=np.float64), target=np.asarray(tgt, dtype=np.float64),
        max_iterations=kwargs.get("max_iterations", 100), tolerance=kwargs.get("tolerance", 1e-6),
        max_distance_correspondence=kwargs.get("max_distance_correspondence", 150),
        max_distance_nearest_neighbors=kwargs.get("max_distance_nearest_neighbors", 50),
        T=T, all_T=np.stack(all_T), init_src_cov=init_src_cov, tgt_cov=tgt_cov,
        hw_src=np.stack(hw_s) if hw_s else np.zeros((0, 5, 2)),
        hw_tgt=np.stack(hw_t) if hw_t else np.zeros((0, 5, 2)),
        all_src_cov=np.stack(all_src_cov[:keep]),
        n_iter=n_it, converged=int("Converged" in log), log=np.array(log),
        x0=np.stack([r["x0"] for r in recs]), xopt=np.stack([r["xopt"] for r in recs]),
        fopt=np.array([r["fopt"] for r in recs]), nfev=np.array([r["nfev"] for r in recs]),
        ngev=np.array([r["ngev"] for r in recs]), warnflag=np.array([r["warnflag"] for r in recs]),
        q=np.stack([r["q"] for r in recs[:keep]]), W=np.stack([r["W"] for r in recs[:keep]]),
        idx=np.stack([recover_idx(r["q"], r["W"], np.asarray(tgt)) for r in recs[:keep]]),
        versions=np.array(f"numpy {np.__version__}; scipy {__import__('scipy').__version__}"),
    )
    Ts = [T] + (ensemble(np.asarray(src), np.asarray(tgt), kwargs, n_per_level=ens, pool=pool) if ens else [])
    d["ens_T"] = dedupe(Ts)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **d)
    print(f"{name}: N={len(src)} M={len(tgt)} iters={n_it} conv={d['converged']} "
          f"ensemble={len(d['ens_T'])} T=[{T[0,2]:.4f},{T[1,2]:.4f},{np.degrees(np.arctan2(T[1,0],T[0,0])):.4f}deg]",
          flush=True)


def main():
    robot_kw = dict(max_distance_nearest_neighbors=200, tolerance=1)  # robot-visualization.py:157-162
    with Pool(6) as pool:
        for pair in range(3):
            for rays in (90, 360):
                src, tgt = S.robot_pair(pair, rays)
                capture(f"robot_p{pair}_r{rays}", src, tgt, robot_kw, pool)
        for seed in range(6):
            src, tgt = S.vis_pair(seed)
            capture(f"vis_s{seed}", src, tgt, {}, pool)
        src, tgt, _ = S.segment_scene_2d(2000, seed=0)
        capture("segment_2k", src, tgt, dict(max_distance_correspondence=20, max_distance_nearest_neighbors=25),
                pool, ens=4, keep_iters=3)


if __name__ == "__main__":
    main()
