"""ctypes binding of libgicp_hip.so (include/gicp_hip.h).

The shared library is built in-tree (``make -C generalized-icp_amd/csrc`` or
``__graft_entry__.build()``) and loaded from this directory.  There is no CPU
fallback: if the library is missing the import of the engine fails loudly.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# GICP_LIB_VARIANT=stamps loads the diagnostic build with in-kernel phase timers (make STAMPS=1)
_VARIANT = os.environ.get("GICP_LIB_VARIANT", "")
LIB_PATH = os.path.join(HERE, f"libgicp_hip_{_VARIANT}.so" if _VARIANT else "libgicp_hip.so")

GICP_OK = 0
GICP_E_INVALID = -1
GICP_E_HIP = -2
GICP_E_STATE = -3
GICP_E_COMM = -4
GICP_E_NOMEM = -5
COMM_ID_BYTES = 128
PEER_HANDLE_BYTES = 72
GICP_STAGE_BORROW = 1
MAX_PEERS = 16
PASS_INFO = 6
GRAPH_K = 20

# gicp_params.cov_model (include/gicp_hip.h GICP_COV_*)
COV_MODELS = {"plane_to_plane": 0, "gicp": 0, "point_to_point": 1, "icp": 1, "point_to_plane": 2}
# gicp_result.stop_reason (GICP_STOP_*)
STOP_REASONS = {0: "none", 1: "loss", 2: "transform", 3: "abs_mse", 4: "rel_mse"}


class Params(C.Structure):
    """gicp_params (include/gicp_hip.h) — gicp.py:78 keyword arguments + its constants."""
    _fields_ = [
        ("max_iterations", C.c_int32),
        ("k_neighbors", C.c_int32),
        ("tolerance", C.c_double),
        ("max_distance_correspondence", C.c_double),
        ("max_distance_nearest_neighbors", C.c_double),
        ("epsilon", C.c_double),
        ("ratio", C.c_double),
        ("fixed_iterations", C.c_int32),
        ("min_neighbors", C.c_int32),
        ("timing_stride", C.c_int32),
        ("timing_offset", C.c_int32),
        ("cov_model", C.c_int32),
        ("transformation_epsilon", C.c_double),
        ("rotation_epsilon", C.c_double),
        ("euclidean_fitness_epsilon", C.c_double),
        ("mse_relative_epsilon", C.c_double),
    ]


class Result(C.Structure):
    _fields_ = [
        ("iterations", C.c_int32),
        ("converged", C.c_int32),
        ("converged_at", C.c_int32),
        ("ambiguous", C.c_int32),
        ("final_loss", C.c_double),
        ("correspondences", C.c_int64),
        ("wall_ms", C.c_double),
        ("corr_kernel_ms", C.c_double),
        ("reduce_ms", C.c_double),
        ("pairs_evaluated", C.c_int64),
        ("stop_reason", C.c_int32),
        ("pad", C.c_int32),
        ("mse", C.c_double),
        ("pairs_total", C.c_double),
        ("corr_kernel_ms_sampled", C.c_double),
        ("corr_samples", C.c_int32),
        ("pad2", C.c_int32),
        ("exchange_us_mean", C.c_double),
        ("exchange_us_min", C.c_double),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class Debug(C.Structure):
    _fields_ = [
        ("index", C.POINTER(C.c_int64)),
        ("weight", C.POINTER(C.c_double)),
        ("distance", C.POINTER(C.c_double)),
        ("want_top_weights", C.c_int32),
    ]


class Trace(C.Structure):
    """gicp_trace (include/gicp_hip.h): per-iteration rows of gicp_align_trace."""
    _fields_ = [
        ("capacity", C.c_int32),
        ("top_k", C.c_int32),
        ("poses", C.POINTER(C.c_double)),
        ("losses", C.POINTER(C.c_double)),
        ("top_src", C.POINTER(C.c_int64)),
        ("top_tgt", C.POINTER(C.c_int64)),
        ("top_det", C.POINTER(C.c_double)),
    ]


# every entry point include/gicp_hip.h declares: name -> (restype, argtypes)
_VP = C.c_void_p
_DP = C.POINTER(C.c_double)
SIGNATURES = {
    "gicp_version": (C.c_int, []),
    "gicp_stats_size": (C.c_int, [C.c_int]),
    "gicp_default_params": (None, [C.c_int, C.POINTER(Params)]),
    "gicp_strerror": (C.c_char_p, [C.c_int]),
    "gicp_create": (C.c_int, [C.POINTER(_VP), C.c_int]),
    "gicp_destroy": (None, [_VP]),
    "gicp_last_error": (C.c_char_p, [_VP]),
    "gicp_comm_unique_id": (C.c_int, [C.c_char_p]),
    "gicp_comm_init": (C.c_int, [_VP, C.c_int, C.c_int, C.c_char_p]),
    "gicp_comm_ranks": (C.c_int, [_VP, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "gicp_set_target": (C.c_int, [_VP, _DP, C.c_int64, C.c_int, C.POINTER(Params)]),
    "gicp_set_source": (C.c_int, [_VP, _DP, C.c_int64, C.c_int, C.POINTER(Params), C.c_int, C.c_int]),
    "gicp_target_to_source": (C.c_int, [_VP, C.c_int, C.c_int]),
    "gicp_get_covariances": (C.c_int, [_VP, C.c_int, _DP]),
    "gicp_get_neighbor_counts": (C.c_int, [_VP, C.c_int, C.POINTER(C.c_int32)]),
    "gicp_iterate": (C.c_int, [_VP, _DP, _DP, C.POINTER(Debug)]),
    "gicp_solve_pose": (C.c_int, [C.c_int, _DP, _DP, _DP, _DP]),
    "gicp_cg_inner_2d": (C.c_int, [_DP, _DP, _DP, _DP, _DP, C.POINTER(C.c_int32)]),
    "gicp_pass_info": (C.c_int, [_VP, _DP]),
    "gicp_top_weights": (C.c_int, [_VP, C.c_int, C.POINTER(C.c_int64), C.POINTER(C.c_int64), _DP]),
    "gicp_align": (C.c_int, [_VP, _DP, C.POINTER(Params), _DP, C.POINTER(Result)]),
    "gicp_align_trace": (C.c_int, [_VP, _DP, C.POINTER(Params), _DP, C.POINTER(Result), C.POINTER(Trace)]),
    "gicp_reset_cache": (C.c_int, [_VP]),
    "gicp_stage_target": (C.c_int, [_VP, _DP, C.c_int64, C.c_int, C.POINTER(Params)]),
    "gicp_stage_target_ex": (C.c_int, [_VP, _DP, C.c_int64, C.c_int, C.POINTER(Params), C.c_int]),
    "gicp_commit_target": (C.c_int, [_VP, C.c_int, C.c_int]),
    "gicp_cancel_stage": (C.c_int, [_VP]),
    "gicp_get_graph": (C.c_int, [_VP, C.POINTER(C.c_int64), _DP]),
    "gicp_iteration_times": (C.c_int, [_VP, C.POINTER(C.c_float), C.c_int]),
    "gicp_set_allreduce": (C.c_int, [_VP, C.c_void_p, C.c_void_p]),
    "gicp_set_allreduce_ranks": (C.c_int, [_VP, C.c_void_p, C.c_void_p, C.c_int, C.c_int]),
    "gicp_peer_export": (C.c_int, [_VP, C.c_char_p]),
    "gicp_peer_init": (C.c_int, [_VP, C.c_int, C.c_int, C.c_char_p, C.c_double]),
    "gicp_peer_close": (C.c_int, [_VP]),
    "gicp_build_info": (C.c_char_p, []),
    "gicp_rotated_covariances": (C.c_int, [_VP, C.c_int, _DP, _DP]),
}

# gicp_allreduce_fn: int (*)(double* buf, int n, void* user)
ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, _DP, C.c_int, C.c_void_p)

_lib = None

# the sources gicp_build_info()'s hash covers, in the Makefile's HASH_SRCS order
HASH_SRCS = ("csrc/gicp_kernels.hip", "csrc/gicp_capi.cpp", "csrc/gicp_solver.cpp", "csrc/gicp_cg.cpp", "csrc/gicp_internal.h",
             "csrc/gicp_solver.h", "csrc/gicp_solve_dev.h", "../include/gicp_hip.h")


def source_hash():
    """First 16 hex digits of sha256 over the library's sources as they lie in this tree (the same
    bytes the Makefile hashes into gicp_build_info())."""
    import hashlib
    h = hashlib.sha256()
    pkg = os.path.dirname(HERE)
    for f in HASH_SRCS:
        with open(os.path.normpath(os.path.join(pkg, f)), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info():
    """gicp_build_info() of the loaded library as a dict (src, git, built, arch)."""
    raw = load().gicp_build_info().decode()
    return dict(kv.split("=", 1) for kv in raw.split(";") if "=" in kv)


def load():
    """Load libgicp_hip.so (raises if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libgicp_hip.so not found at {LIB_PATH}; build it with "
                          "`make -C generalized-icp_amd/csrc` (there is no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class GicpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def check(rc, ctx=None, what=""):
    if rc == GICP_OK:
        return
    lib = load()
    msg = lib.gicp_last_error(ctx).decode() if ctx else lib.gicp_strerror(rc).decode()
    if rc == GICP_E_INVALID:
        raise ValueError(f"{what}: {msg}")
    raise GicpError(rc, f"{what}: {msg}")


def dptr(a):
    return a.ctypes.data_as(_DP)
