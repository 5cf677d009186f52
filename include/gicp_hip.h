/*
 * gicp_hip.h — C-ABI of libgicp_hip.so, the MI355X (gfx950) GICP engine.
 *
 * The drop-in boundary for the reference's only public surface,
 *   gicp(source_points, target_points, max_iterations=100, tolerance=1e-6,
 *        max_distance_correspondence=150, max_distance_nearest_neighbors=50)
 *   (/root/reference/python-implementation/gicp.py:78, returns gicp.py:174)
 * and apply_transformation(cloud, T) (gicp.py:176-177).  The Python module
 * generalized-icp_amd/gicp/__init__.py binds these entry points with ctypes
 * and restores the reference's signature and 7-tuple; INTEGRATION.md shows
 * the binding.
 *
 * Conventions
 *   - Host buffers are caller-owned, fp64, row-major (N x dim); device
 *     buffers are library-owned.  No torch / HIP types cross this boundary.
 *   - Every int-returning call returns GICP_OK (0) or a negative GICP_E_*;
 *     gicp_last_error() then describes the failure.  No C++ exception
 *     crosses the boundary.
 *   - HIP is initialised lazily inside gicp_create(), never at load time, so
 *     the library is safe to load before fork() (robot-visualization.py:199
 *     runs gicp() in a forked worker).
 *   - One context = one GPU = one host thread; one process per GPU.  Ranks
 *     of a multi-GPU job share the per-iteration statistics through an RCCL
 *     all-reduce (gicp_comm_init) -- or a host reducer (gicp_set_allreduce) --
 *     between the correspondence pass and the pose solve; every rank then runs
 *     the same device solve (k_solve) on bit-identical sums, so no pose
 *     broadcast is needed.
 */
#ifndef GICP_HIP_H
#define GICP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GICP_OK 0
#define GICP_E_INVALID (-1)   /* bad argument (shape, dim, NULL, range) */
#define GICP_E_HIP (-2)       /* HIP runtime failure */
#define GICP_E_STATE (-3)     /* call out of order (e.g. align before set_target) */
#define GICP_E_COMM (-4)      /* RCCL failure */
#define GICP_E_NOMEM (-5)     /* host or device allocation failed */

#define GICP_COMM_ID_BYTES 128
#define GICP_MAX_STATS 74     /* statistics per pass, dim 3 (dim 2: 26); a multi-GPU exchange carries these
                                 plus the GICP_PASS_INFO diagnostics: 80 fp64 (dim 2: 32) */

typedef struct gicp_ctx gicp_ctx;

/* Keyword arguments of gicp() (gicp.py:78) and the constants gicp.py
 * hard-codes (epsilon gicp.py:5, 0.1 ratio gicp.py:11, k = 6 gicp.py:24). */
typedef struct gicp_params {
    int32_t max_iterations;                 /* gicp.py:78, default 100 */
    int32_t k_neighbors;                    /* 0 -> 6 for dim 2 (gicp.py:24), 20 for dim 3 */
    double tolerance;                       /* |delta loss| < tolerance stops, gicp.py:155-162 */
    double max_distance_correspondence;     /* d_c, inclusive (gicp.py:136), default 150 */
    double max_distance_nearest_neighbors;  /* d_n, strict (KDTree distance_upper_bound, gicp.py:24), default 50 */
    double epsilon;                         /* 100 (gicp.py:5) */
    double ratio;                           /* 0.1 (gicp.py:11) */
    int32_t fixed_iterations;               /* 1: never stop on tolerance (benchmark mode) */
    int32_t min_neighbors;                  /* 0 -> dim (2-D: > 1 neighbour, gicp.py:27) */
    int32_t timing_stride;                  /* gicp_align times every n-th correspondence launch with HIP
                                               events (0 -> 8; 1 = every launch, adds queue work;
                                               < 0: no events, corr_kernel_ms 0) ... */
    int32_t timing_offset;                  /* ... starting at launch timing_offset (< stride) */
    /* --- additions beyond gicp.py; zero = the reference's behaviour --- */
    int32_t cov_model;                      /* GICP_COV_* : which covariances weight a correspondence
                                               (presentation/main.typ:446-455) */
    double transformation_epsilon;          /* > 0: PCL-style stop when the iteration's increment has
                                               |dt|^2 <= this and cos(angle) >= rotation threshold
                                               (presentation/main.typ:773-776) */
    double rotation_epsilon;                /* cosine threshold of that test; 0 -> 1 - transformation_epsilon
                                               (PCL's default when its rotation epsilon is unset) */
    double euclidean_fitness_epsilon;       /* > 0: stop when |MSE - previous MSE| < this, MSE = mean squared
                                               correspondence distance of the pass (presentation/main.typ:776) */
    double mse_relative_epsilon;            /* > 0: stop when |MSE - previous| / previous < this (PCL: 1e-5) */
} gicp_params;

/* gicp_params.cov_model (the GICP paper's three instances, presentation/main.typ:446-455) */
#define GICP_COV_PLANE_TO_PLANE 0   /* W = inv(R C_s R^T + C_t), both surface covariances (gicp.py:143-145) */
#define GICP_COV_POINT_TO_POINT 1   /* C_s = 0, C_t = I: W = I (standard ICP) */
#define GICP_COV_POINT_TO_PLANE 2   /* C_s = 0, C_t = P^-1: W = n_t n_t^T (projection on the target normal) */

/* gicp_result.stop_reason */
#define GICP_STOP_NONE 0            /* max_iterations reached (or fixed_iterations) */
#define GICP_STOP_LOSS 1            /* |delta loss| < tolerance, gicp.py:160 (the update is NOT applied) */
#define GICP_STOP_TRANSFORM 2       /* transformation_epsilon test (the update IS applied, as PCL does) */
#define GICP_STOP_ABS_MSE 3         /* euclidean_fitness_epsilon test (update applied) */
#define GICP_STOP_REL_MSE 4         /* mse_relative_epsilon test (update applied) */

/* What gicp_align() reports (the reference only prints "Converged at iteration", gicp.py:161). */
typedef struct gicp_result {
    int32_t iterations;        /* outer iterations executed (each = correspondences + solve) */
    int32_t converged;         /* 1 if a stopping criterion ended the loop (which: stop_reason) */
    int32_t converged_at;      /* iteration index printed by gicp.py:161, -1 if none */
    int32_t ambiguous;         /* points re-resolved in fp64 in the last pass (diagnostic) */
    double final_loss;         /* min_loss of the last inner solve */
    int64_t correspondences;   /* accepted correspondences in the last pass, all ranks */
    double wall_ms;            /* host wall time of the iteration loop */
    double corr_kernel_ms;     /* correspondence-kernel time: mean HIP-event duration of the sampled launches
                                  (gicp_params.timing_stride / timing_offset) x iterations executed */
    double reduce_ms;          /* sum of HIP-event durations of partial-reduce + all-reduce */
    int64_t pairs_evaluated;   /* source x target distance evaluations in the last pass (if counted) */
    int32_t stop_reason;       /* GICP_STOP_* */
    int32_t pad;
    double mse;                /* mean squared correspondence distance of the last pass */
    double pairs_total;        /* distance pairs screened over all passes of this call, all ranks */
    double corr_kernel_ms_sampled;  /* sum of the event-timed correspondence launches ... */
    int32_t corr_samples;           /* ... and how many there were */
    int32_t pad2;
    double exchange_us_mean;        /* peer exchange (gicp_peer_init): mean / minimum time the final workgroup spent */
    double exchange_us_min;         /* in the exchange per launch of this call (its stores to every rank's arrival) */
} gicp_result;

/* Optional caller-allocated per-point outputs of one pass, ORIGINAL source
 * order, this rank's shard only (other rows untouched).  Any pointer may be NULL. */
typedef struct gicp_debug {
    int64_t* index;      /* [N] target index of the correspondence, -1 if rejected (gicp.py:136-138) */
    double* weight;      /* [N, dim, dim] W_i = inv(R C_s R^T + C_t), zeros if rejected (gicp.py:143-145) */
    double* distance;    /* [N] fp64 distance to the nearest target point (gicp.py:133) */
    int32_t want_top_weights;  /* 1: the pass also keeps det(W) on the device for gicp_top_weights */
} gicp_debug;

/* ---- library ------------------------------------------------------------ */
int gicp_version(void);                          /* 100 * major + minor */
int gicp_stats_size(int dim);                    /* 26 (dim 2) or 74 (dim 3) */
void gicp_default_params(int dim, gicp_params* out);
const char* gicp_strerror(int code);

/* ---- context ------------------------------------------------------------ */
int gicp_create(gicp_ctx** out, int device);     /* lazily initialises HIP on `device` */
void gicp_destroy(gicp_ctx* ctx);
const char* gicp_last_error(const gicp_ctx* ctx);

/* ---- multi-GPU: one process per GPU, RCCL over xGMI ---------------------- */
int gicp_comm_unique_id(char out[GICP_COMM_ID_BYTES]);   /* rank 0, then broadcast out-of-band */
int gicp_comm_init(gicp_ctx* ctx, int nranks, int rank, const char id[GICP_COMM_ID_BYTES]);
/* The exchange this context's statistics go through, read back from the communicator itself
 * (ncclCommCount / ncclCommUserRank): *nranks = 1 and *rank = 0 without one; with a host hook
 * (gicp_set_allreduce_ranks) the values it was given, else 1 / 0; with the peer exchange
 * (gicp_peer_init) its nranks / rank.  *kind: 0 none, 1 RCCL, 2 host hook, 3 peer exchange.  Any
 * output may be NULL. */
int gicp_comm_ranks(gicp_ctx* ctx, int* nranks, int* rank, int* kind);

/* In-kernel peer exchange (replaces the collective on the per-iteration path).  Every rank
 * exports one small exchange area of its own device memory (fine-grained, uncached) as an IPC handle
 * (gicp_peer_export), the handles are all-gathered out of band, and gicp_peer_init maps the peers' areas.
 * From then on the final workgroup of each correspondence launch writes this rank's statistics into its
 * slot of every rank's area, raises the exchange's sequence number there, waits (bounded by `timeout_s`)
 * until every rank's slot of this exchange has arrived in its own area, sums them in rank order -- the
 * same bits on every rank -- and runs the pose solve in the same launch: no collective and no second kernel
 * per iteration.  The sequence number counts the exchanges that happen (launches that exit at once after
 * convergence take none) and lives on the device; an exported handle carries this rank's current number
 * after the 64-byte IPC handle, and gicp_peer_init starts every rank at the maximum, so the ranks agree
 * again after a timed-out exchange.  gicp_peer_init is collective (every rank, same order of calls) and
 * proves the path with one probe exchange before it returns.  It first closes this context's previous peer
 * exchange; on success it replaces RCCL / the host hook, on failure (GICP_E_COMM) the context is left with
 * no peer exchange and its RCCL communicator / hook as they were.  A timed-out exchange inside gicp_align
 * fails the call with GICP_E_COMM.  `handles` holds nranks x GICP_PEER_HANDLE_BYTES bytes in rank order
 * (this rank's entry is not opened).  Ranks of one GPU (several processes) and of several GPUs (xGMI) use
 * the same protocol.  gicp_comm_ranks reports kind 3. */
#define GICP_PEER_HANDLE_BYTES 72
#define GICP_MAX_PEERS 16
int gicp_peer_export(gicp_ctx* ctx, char handle[GICP_PEER_HANDLE_BYTES]);
int gicp_peer_init(gicp_ctx* ctx, int nranks, int rank, const char* handles, double timeout_s);
int gicp_peer_close(gicp_ctx* ctx);   /* back to no exchange (RCCL / hook as set before are dropped by init) */

/* Build provenance of this library: "src=<first 16 hex of sha256 over the sources>;git=<rev>;built=<date
 * time>;arch=gfx950".  The source hash covers csrc/{gicp_kernels.hip, gicp_capi.cpp, gicp_solver.cpp,
 * gicp_internal.h, gicp_solver.h, gicp_solve_dev.h} and include/gicp_hip.h, concatenated in that order, so
 * a caller can prove the loaded library was compiled from the sources beside it. */
const char* gicp_build_info(void);

/* ---- clouds -------------------------------------------------------------- */
/* Target cloud (gicp.py:101,104): builds the tile index and the per-point
 * surface covariances once; reusable across gicp_align calls. */
int gicp_set_target(gicp_ctx* ctx, const double* xyz, int64_t M, int dim, const gicp_params* p);
/* Source cloud (gicp.py:100,111): the whole cloud is uploaded and indexed (its
 * covariance neighbourhoods need every point); this rank reduces only the
 * source tiles of shard `shard` of `nshards`: the cloud's Morton-ordered
 * tiles in chunks of 64, dealt round-robin (chunks shard, shard + nshards, ...;
 * gicp/distributed.py shard_tiles states the same split), and computes the
 * covariances of those tiles only (with nshards > 1, gicp_get_covariances /
 * gicp_rotated_covariances of the source give NaN rows for the other shards'
 * points: merge them across ranks). */
int gicp_set_source(gicp_ctx* ctx, const double* xyz, int64_t N, int dim, const gicp_params* p,
                    int shard, int nshards);
/* Promote the current target (index + covariances) to be the next source,
 * as robot-visualization.py:250 swaps scans; then set a new target. */
int gicp_target_to_source(gicp_ctx* ctx, int shard, int nshards);

/* Pipelined frame stream (robot-visualization.py:239-252): build the NEXT
 * targets -- pinned copy, upload, Morton sort, tiling, covariances, neighbour graph -- each on its own
 * stream from a host thread while the current target is registered (gicp_align on the library's stream
 * runs concurrently).  Up to GICP_MAX_STAGED builds may be pending; commits take them in staging
 * order.  `xyz` is copied into a pinned buffer of the slot before gicp_stage_target returns: the caller may
 * reuse or refill it at once.
 * gicp_commit_target waits for the oldest build, then promotes: current target -> source (as
 * gicp_target_to_source), staged cloud -> target.  gicp_cancel_stage waits for and drops them all. */
#define GICP_MAX_STAGED 2
int gicp_stage_target(gicp_ctx* ctx, const double* xyz, int64_t M, int dim, const gicp_params* p);
/* gicp_stage_target with flags.  GICP_STAGE_BORROW: no copy -- the build reads the caller's `xyz` on its
 * own thread, so the caller must keep that buffer alive and unmodified until the staged target is committed
 * (gicp_commit_target) or dropped (gicp_cancel_stage); for callers that own their frames (a stream held in
 * memory), it saves the ~0.06 ms copy of a 100k frame on the calling thread. */
#define GICP_STAGE_BORROW 1
int gicp_stage_target_ex(gicp_ctx* ctx, const double* xyz, int64_t M, int dim, const gicp_params* p, int flags);
int gicp_commit_target(gicp_ctx* ctx, int shard, int nshards);
int gicp_cancel_stage(gicp_ctx* ctx);

/* Surface covariances C = a I - m m^T of the last set_target/set_source,
 * original order, [n, dim, dim] (gicp.py:104 target_cov_matrices, :111
 * initial_source_cov_matrices).  which: 0 = target, 1 = source. */
int gicp_get_covariances(gicp_ctx* ctx, int which, double* out);
/* The target's neighbour graph (built by gicp_set_target unless GICP_NO_GRAPH=1):
 * index[M][GICP_GRAPH_K] original indices of up to GICP_GRAPH_K other target points (-1 pads),
 * radius[M] such that every target within distance < radius[i] of point i is in row i (0: the
 * row certifies nothing).  Original order.  Either output may be NULL. */
#define GICP_GRAPH_K 20
int gicp_get_graph(gicp_ctx* ctx, int64_t* index, double* radius);
/* Neighbour count (incl. self, < d_n, capped at k) per point, original order. */
int gicp_get_neighbor_counts(gicp_ctx* ctx, int which, int32_t* out);

/* ---- the hot path -------------------------------------------------------- */
/* One pass at pose T ((dim+1)^2, row-major): correspondences + Mahalanobis
 * weights + normal-equation statistics (gicp.py:119-145 plus everything
 * loss()/grad_loss() need, gicp.py:52-76).  `stats` receives
 * gicp_stats_size(dim) doubles, summed over all ranks when a communicator is
 * set.  Layout: see DESIGN.md §4 (A, B, C, gR, gt, c0, count). */
int gicp_iterate(gicp_ctx* ctx, const double* T, double* stats, gicp_debug* dbg);

/* Per-pass diagnostics of the last gicp_iterate / gicp_align pass, summed over ranks:
 * out[0] ambiguous lanes re-resolved in fp64, out[1] distance pairs screened, out[2] candidate-list
 * rebuilds, out[3] sum of squared correspondence distances |q - (R s + t)|^2 (PCL's MSE numerator),
 * out[4] points whose nearest target the graph descent proved, out[5] source tiles that walked. */
#define GICP_PASS_INFO 6
int gicp_pass_info(gicp_ctx* ctx, double out[GICP_PASS_INFO]);

/* The drop-in's visualisation extras (gicp.py:169-172) without copying per-point arrays: the k
 * accepted source points of the last gicp_iterate pass with the largest det(W) (W as in
 * gicp_debug.weight; rejected points have det 0), ascending by det as np.argsort(...)[-k:] yields
 * them, ties broken towards the larger original index (the last k of a stable argsort).  Needs a
 * preceding gicp_iterate whose gicp_debug had want_top_weights = 1.  src_out[k]: original source
 * indices; tgt_out[k]: their matched target indices (-1 if rejected); det_out[k]: det(W).  Any
 * output may be NULL.  1 <= k <= 16; slots beyond the shard's point count are -1 / 0.  The pass
 * itself computes the top-k for the k of the previous call (default 5), so that call returns without
 * touching the device; another k costs one more launch and stream sync. */
int gicp_top_weights(gicp_ctx* ctx, int k, int64_t* src_out, int64_t* tgt_out, double* det_out);

/* Host solve of the inner problem (gicp.py:148-154): minimise
 * c0 - 2 g^T dz + dz^T H dz over SE(dim), dz = z(T) - z(T_k), starting at T_k.
 * Pure host code, no GPU needed.  Writes T_out and the minimum. */
int gicp_solve_pose(int dim, const double* stats, const double* T_k, double* T_out, double* loss_out);

/* 2-D inner solve of gicp.py:148-154 as the reference runs it: scipy.optimize.fmin_cg (SciPy 1.15.3:
 * Polak-Ribiere+ CG, gtol 1e-5, maxiter 600, Wolfe line search dcsrch then wolfe2, c1 1e-4, c2 0.4),
 * restated natively (csrc/gicp_cg.cpp), on the closed form of the loss from one pass's 2-D statistics
 * (gicp_iterate's 26 values at pose T_k, 3x3): minimises over the offset x = (tx, ty, theta) from x0
 * (gicp.py:151).  Writes xopt[3], *fopt (gicp.py:153-154; may be NULL) and counts[4] = {nfev, ngev,
 * warnflag, iterations} (may be NULL).  Pure host code, no GPU needed.  Replaces the reference's
 * fmin_cg call at gicp.py:152 (the fast mode's host inner solve). */
int gicp_cg_inner_2d(const double* stats, const double* T_k, const double* x0, double* xopt, double* fopt,
                     int32_t* counts);

/* The whole outer loop (gicp.py:116-167) on the GPU: per iteration the correspondence pass
 * (k_corr), the statistics exchange when sharded, the pose solve + convergence test (k_solve). */
int gicp_align(gicp_ctx* ctx, const double* T0, const gicp_params* p, double* T_out, gicp_result* res);

/* What the drop-in's 7-tuple needs from each iteration of that loop (gicp.py:108,121,154,167-172),
 * recorded on the device while it runs and copied out once at the end.  Caller-allocated; row k is
 * iteration k (rows >= gicp_result.iterations are untouched).  Any array may be NULL. */
typedef struct gicp_trace {
    int32_t capacity;   /* rows the arrays hold: >= gicp_params.max_iterations */
    int32_t top_k;      /* 0: no top-k rows; 1..16: the pass's k largest det(W) (gicp_top_weights order) */
    double* poses;      /* [capacity][(dim+1)^2] the pose iteration k's pass ran at (T_k, row-major) */
    double* losses;     /* [capacity] min_loss of iteration k's inner solve (gicp.py:154) */
    int64_t* top_src;   /* [capacity][top_k] original source indices (-1 pads) */
    int64_t* top_tgt;   /* [capacity][top_k] their matched target indices (-1: rejected) */
    double* top_det;    /* [capacity][top_k] det(W) */
} gicp_trace;
/* gicp_align plus the trace (trace = NULL is gicp_align).  With top_k the pass also records det(W)
 * on the device and two small launches per iteration select the rows (gicp.py:170-172); with a
 * shard (nshards > 1) the rows cover this rank's shard only -- merge them across ranks by
 * (det, source index). */
int gicp_align_trace(gicp_ctx* ctx, const double* T0, const gicp_params* p, double* T_out, gicp_result* res,
                     gicp_trace* trace);

/* Drop every pose-dependent cache of the current clouds (candidate lists, nearest-neighbour
 * certificates, last matches, seed tiles): the next pass starts cold, as after a fresh
 * gicp_set_source.  Results never depend on the caches (they are exact); only the time does. */
int gicp_reset_cache(gicp_ctx* ctx);

/* Per-iteration correspondence-kernel time (ms, HIP events) of the last gicp_align: out[i] for
 * iteration i, -1 where that launch was not sampled (gicp_params.timing_stride / timing_offset).
 * Returns the number of iterations written (<= n), or a negative GICP_E_*. */
int gicp_iteration_times(gicp_ctx* ctx, float* out, int n);

/* Host statistics exchange, for a job whose ranks talk over something other than RCCL (e.g. a
 * gloo process group, or ranks sharing one GPU, which RCCL refuses).  When set, every pass
 * copies its statistics (n = gicp_stats_size(dim) + GICP_PASS_INFO doubles) to a host buffer,
 * calls fn(buf, n, user), which must replace buf by the sum over ranks and return 0, and copies
 * the sum back before the pose solve -- in gicp_iterate and inside gicp_align's loop (which then
 * synchronises once per iteration).  Replaces an RCCL communicator on the same context.
 * fn = NULL removes the hook. */
typedef int (*gicp_allreduce_fn)(double* buf, int n, void* user);
int gicp_set_allreduce(gicp_ctx* ctx, gicp_allreduce_fn fn, void* user);
/* gicp_set_allreduce that also records the job's (nranks, rank), which gicp_comm_ranks then reports
 * for the hook (e.g. the device threads of one gicp(devices=[...]) call). */
int gicp_set_allreduce_ranks(gicp_ctx* ctx, gicp_allreduce_fn fn, void* user, int nranks, int rank);

/* The source covariances rotated by R (dim x dim, row-major): R C_s R^T = a I - (R m)(R m)^T per
 * point, computed on the device (gicp.py:120-121 all_source_cov_matrices, rotated instead of
 * recomputed), ORIGINAL order, [n, dim, dim].  which: 0 = target, 1 = source. */
int gicp_rotated_covariances(gicp_ctx* ctx, int which, const double* R, double* out);

#ifdef __cplusplus
}
#endif
#endif /* GICP_HIP_H */
