// gicp_capi.cpp — the C-ABI of libgicp_hip.so (include/gicp_hip.h).
//
// Owns one GPU per context: device copies of both clouds (Morton-sorted tile index,
// per-point surface covariances), the per-iteration workspace, an optional RCCL
// communicator for the statistics all-reduce, and the outer loop of gicp.py:116-167.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <cmath>
#include <cstdio>
#include <cstddef>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <thread>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>

#include "../../include/gicp_hip.h"
#include "gicp_internal.h"

namespace gicp {
hipError_t launch_morton(const double*, int64_t, int, const DevCloud&, uint32_t*, int32_t*, hipStream_t);
hipError_t launch_build_tiles(const double*, int, int32_t*, TileInfo*, TileBox*, int, double*, float4*, int32_t*,
                              unsigned*, hipStream_t);
hipError_t launch_build_blocks(const TileInfo*, int, BlockInfo*, int, int, hipStream_t);
hipError_t launch_knn_cov(const CovArgs&, int, int, bool, hipStream_t);
hipError_t launch_corr(const CorrArgs&, int, int, hipStream_t);
hipError_t launch_solve(IterState*, int, hipStream_t, double*);
hipError_t launch_peer_probe(const PeerArgs&, double*, hipStream_t);
hipError_t launch_reset_tiles(int32_t*, int32_t*, float*, int32_t*, int, int32_t*, int64_t, hipStream_t);
hipError_t launch_graph_pack(const GraphArgs&, hipStream_t);
hipError_t launch_rotate_cov(const double4*, const int32_t*, int64_t, int, const double*, double*, hipStream_t);
hipError_t launch_top_weights(const double*, const int64_t*, const int32_t*, int64_t, int, double*, int64_t*, int, double*, int64_t*,
                              int64_t*, hipStream_t);
int corr_grid(int q_tiles, int shard, int nshards);
int solve_pose(int d, const double* st, const double* Tk, double* Tout, double* loss_out);
}  // namespace gicp

using namespace gicp;

namespace {

struct Fail {
    int code;
    std::string msg;
};

// a failing HIP call is reported to the caller (the exception) and its error cleared from HIP's
// per-thread last error here, so it cannot fail a later call's first launch check
#define HIPCHK(x)                                                                                  \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            (void)hipGetLastError();                                                               \
            throw Fail{GICP_E_HIP, std::string(#x) + ": " + hipGetErrorString(e_)};               \
        }                                                                                          \
    } while (0)

// a HIP call whose failure is deliberately ignored (teardown): its error must not linger either
inline void quiet(hipError_t e) {
    if (e != hipSuccess) (void)hipGetLastError();
}

template <class T>
void dalloc(T*& p, size_t n) {
    if (p) {
        quiet(hipFree(p));
        p = nullptr;
    }
    if (n == 0) n = 1;
    HIPCHK(hipMalloc(reinterpret_cast<void**>(&p), n * sizeof(T)));
}
template <class T>
void dfree(T*& p) {
    if (p) quiet(hipFree(p));
    p = nullptr;
}
// grow-only device buffer: reallocates (contents dropped) only when n exceeds the capacity, with
// headroom, so a stream of similar-sized clouds allocates once
template <class T>
void dreserve(T*& p, size_t& cap, size_t n) {
    if (n <= cap && p) return;
    const size_t want = std::max<size_t>({n, (size_t)(cap * 1.125), 1});
    dalloc(p, want);
    cap = want;
}

// A few persistent host threads for the tiling (spawning threads per cloud costs tens of us each,
// which a 100k-point frame of a stream cannot afford).  run(n, fn) calls fn(0 .. n-1) on the workers
// and the calling thread and returns when all are done; one caller at a time.
class WorkerPool {
public:
    explicit WorkerPool(int workers) {
        for (int i = 0; i < workers; ++i) th_.emplace_back([this] { loop(); });
    }
    ~WorkerPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    void run(int tasks, std::function<void(int)> fn) {
        std::unique_lock<std::mutex> lk(m_);
        job_ = std::move(fn);
        ntasks_ = tasks;
        next_ = done_ = 0;
        ++gen_;
        lk.unlock();
        cv_.notify_all();
        work();
        lk.lock();
        done_cv_.wait(lk, [&] { return done_ == ntasks_ && active_ == 0; });
    }

private:
    void work() {
        for (;;) {
            int k;
            {
                std::lock_guard<std::mutex> g(m_);
                if (next_ >= ntasks_) return;
                k = next_++;
            }
            job_(k);
            std::lock_guard<std::mutex> g(m_);
            if (++done_ == ntasks_) done_cv_.notify_all();
        }
    }
    void loop() {
        std::unique_lock<std::mutex> lk(m_);
        long seen = 0;
        for (;;) {
            cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            ++active_;
            lk.unlock();
            work();
            lk.lock();
            if (--active_ == 0) done_cv_.notify_all();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_cv_;
    std::function<void(int)> job_;
    int ntasks_ = 0, next_ = 0, done_ = 0, active_ = 0;
    long gen_ = 0;
    bool stop_ = false;
};

// One indexed cloud on the device.
struct Cloud {
    int dim = 0;
    int64_t n = 0;
    int ntiles = 0, nblocks = 0, level = 0, bits = 0;   // level: tile extent-cap step k (cap 2^(1 + k/4) cells)
    double lo[3] = {0, 0, 0};
    double scale = 1.0;
    float rho = 0.f;
    double* xyz64 = nullptr;
    float4* rel32 = nullptr;
    double4* cov = nullptr;
    int32_t* perm = nullptr;
    int32_t* inv = nullptr;
    int32_t* ncount = nullptr;
    TileInfo* tiles = nullptr;
    BlockInfo* blocks = nullptr;
    uint32_t* tile_code = nullptr;
    TileBox* boxes = nullptr;         // the walk's compact tile records (k_build_tiles)
    int32_t* seed_tab = nullptr;      // Morton seed lookup (DevCloud::seed_tab), built on the host
    int seed_shift = 0;
    uint4* nbq = nullptr;             // neighbour graph (targets only): packed rows (line A)
    uint4* nbx = nullptr;             // ... their last entries
    int32_t* nbi = nullptr;           // ... and their sorted indices
    bool graph_ready = false;
    bool cov_ready = false;
    int cov_shard = 0, cov_nshards = 1;  // whose tiles' covariances were computed (build_cloud)

    size_t cap_xyz = 0, cap_rel = 0, cap_cov = 0, cap_perm = 0, cap_inv = 0, cap_cnt = 0;
    size_t cap_tiles = 0, cap_blocks = 0, cap_tcode = 0, cap_nbq = 0, cap_nbx = 0, cap_nbi = 0, cap_boxes = 0, cap_seed = 0;
    void reserve_points(int64_t np) {
        dreserve(xyz64, cap_xyz, (size_t)np * 4);
        dreserve(rel32, cap_rel, (size_t)np);
        dreserve(cov, cap_cov, (size_t)np);
        dreserve(perm, cap_perm, (size_t)np);
        dreserve(inv, cap_inv, (size_t)np);
        dreserve(ncount, cap_cnt, (size_t)np);
    }
    void reserve_tiles(int nt, int nb) {
        dreserve(tiles, cap_tiles, (size_t)nt);
        dreserve(blocks, cap_blocks, (size_t)nb + (nb + kBlockTiles - 1) / kBlockTiles);   // + super-blocks
        dreserve(tile_code, cap_tcode, (size_t)nt);
        dreserve(boxes, cap_boxes, (size_t)nt);
    }
    void release() {
        dfree(xyz64);
        dfree(rel32);
        dfree(cov);
        dfree(perm);
        dfree(inv);
        dfree(ncount);
        dfree(tiles);
        dfree(blocks);
        dfree(tile_code);
        dfree(boxes);
        dfree(seed_tab);
        dfree(nbq);
        dfree(nbx);
        dfree(nbi);
        cap_xyz = cap_rel = cap_cov = cap_perm = cap_inv = cap_cnt = cap_tiles = cap_blocks = cap_tcode = 0;
        cap_nbq = cap_nbx = cap_nbi = cap_boxes = cap_seed = 0;
        n = 0;
        cov_ready = false;
        graph_ready = false;
    }
    DevCloud view() const {
        DevCloud v{};
        v.xyz64 = xyz64;
        v.rel32 = rel32;
        v.cov = cov;
        v.perm = perm;
        v.tiles = tiles;
        v.blocks = blocks;
        v.tile_code = tile_code;
        v.boxes = boxes;
        v.seed_tab = seed_tab;
        v.seed_shift = seed_shift;
        v.nbq = graph_ready ? nbq : nullptr;
        v.nbx = graph_ready ? nbx : nullptr;
        v.nbi = graph_ready ? nbi : nullptr;
        v.n = n;
        v.ntiles = ntiles;
        v.nblocks = nblocks;
        for (int a = 0; a < 3; ++a) v.lo[a] = lo[a];
        v.scale = scale;
        v.bits = bits;
        v.dim = dim;
        return v;
    }
};

// Scratch of one cloud build (grow-only): the synchronous builds and the staged one (which runs on
// its own stream and host thread while the current target is registered) each own one.
struct BuildScratch {
    double* s_in = nullptr;
    uint32_t *s_codes = nullptr, *s_codes2 = nullptr;
    int32_t* s_idx = nullptr;
    unsigned char* s_sort = nullptr;
    float4* g_nb = nullptr;           // graph build scratch
    float2* g_nbh = nullptr;
    int32_t* d_amb = nullptr;         // covariance-kernel diagnostics counter
    size_t cap_in = 0, cap_codes = 0, cap_codes2 = 0, cap_idx = 0, cap_sort = 0, cap_gnb = 0, cap_gnbh = 0;
    int cap_k_hint[4] = {0, 0, 0, 0};  // last tile extent-cap step per dimension (tiling warm start)
    double* h_pinned = nullptr;       // pinned host copy of the input (staged builds)
    size_t cap_pinned = 0;
    std::unique_ptr<WorkerPool> pool;  // tiling threads (lazily started)
    WorkerPool& workers() {
        if (!pool) {
            const unsigned hc = std::max(1u, std::thread::hardware_concurrency());
            pool.reset(new WorkerPool((int)std::min(7u, hc > 1 ? hc - 1 : 0u)));
        }
        return *pool;
    }
    void release() {
        dfree(s_in);
        dfree(s_codes);
        dfree(s_codes2);
        dfree(s_idx);
        dfree(s_sort);
        dfree(g_nb);
        dfree(g_nbh);
        dfree(d_amb);
        if (h_pinned) quiet(hipHostFree(h_pinned));
        h_pinned = nullptr;
        pool.reset();
        cap_in = cap_codes = cap_codes2 = cap_idx = cap_sort = cap_gnb = cap_gnbh = cap_pinned = 0;
    }
};

}  // namespace

struct gicp_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::string err;
    Cloud tgt, src;
    gicp_params ptgt{}, psrc{};
    int shard = 0, nshards = 1, q_begin = 0, q_end = 0;
    int32_t* d_hint = nullptr;
    double* d_partials = nullptr;
    size_t partials_cap = 0;
    IterState* d_state = nullptr;
    IterState* h_state = nullptr;     // pinned mirror
    uint32_t* d_tickets = nullptr;
    double* d_gpart = nullptr;
    double h_stats[80];
    int32_t* d_amb = nullptr;
    int64_t* d_dbg_idx = nullptr;
    double* d_dbg_w = nullptr;
    double* d_dbg_dist = nullptr;
    double* d_dbg_det = nullptr;      // det(W) per source point (gicp_top_weights)
    size_t dbg_cap = 0;
    bool top_ready = false;           // the last pass recorded det(W)
    // the top-k of that pass, computed inside the pass (same stream sync) for k = top_k_pref, the k the
    // last gicp_top_weights call asked for: [0, 16) source, [16, 32) target indices, then 16 det values
    int top_k_pref = 5, top_cached_k = 0;
    int64_t* h_top = nullptr;         // pinned, 32 int64 + 16 double
    double* d_top_v = nullptr;        // top-k scratch: stage-1 candidates and outputs
    int64_t* d_top_i = nullptr;
    int64_t* d_top_tgt = nullptr;     // [N] sorted order: target of each correspondence (with det(W))
    int64_t* d_top_out = nullptr;
    // per-source-tile candidate lists
    int32_t* d_list = nullptr;
    int32_t* d_list_len = nullptr;
    int32_t* d_list_pass = nullptr;
    float* d_list_rcert = nullptr;
    double* d_poses = nullptr;
    // per-source-point nearest-neighbour certificates
    int32_t* d_cert_j = nullptr;
    float* d_cert_gap = nullptr;
    int32_t* d_cert_pass = nullptr;
    size_t cap_cj = 0, cap_cg = 0, cap_cp = 0;
    bool use_certs = true;            // GICP_NO_CERTS=1: every pass walks every lane
    bool use_graph = true;            // GICP_NO_GRAPH=1: no target neighbour graph, no graph descent
    bool fuse_solve = true;           // GICP_FUSE_SOLVE=0: the solve as its own k_solve launch even with no exchange
    int unit_map = 0;                 // k_corr workgroup -> unit map (CorrArgs::unit_map, GICP_UNIT_MAP)
    int moving_map = 8;               // ... for the first moving_iters iterations of an align (GICP_MOVING_MAP)
    int moving_iters = 5;             // (GICP_MOVING_ITERS)
    int src_tile = kTile;             // source points per tile at most: 64, 32 or 16 (GICP_SRC_TILE)
    double kappa_frac = 0.002;        // certificate gap resolved by the walk, fraction of d_c (GICP_CERT_KAPPA)
    int sparse_max = 4;               // CorrArgs::sparse_max (GICP_SPARSE_WALK; 0: sparse waves walk like the rest)
    int sparse_amb = 2;               // CorrArgs::sparse_amb (GICP_SPARSE_AMB; 0: every fp64 re-resolution wave-wide)
    // cloud-build scratch (synchronous builds) and per-source-tile arrays, grow-only (a frame stream
    // allocates once)
    BuildScratch bs;
    // staged targets (gicp_stage_target / gicp_commit_target): a ring of GICP_MAX_STAGED slots, each
    // built into its own cloud on its own stream by a host thread while the current target is
    // registered; commits take them in staging order
    // Each slot owns a persistent build thread (started on first use): a thread per staged frame cost
    // tens of microseconds of the caller's time per frame.  state: 0 idle, 1 build queued or running,
    // 2 built (rc / err hold the outcome); the caller waits for state != 1 before it takes the slot.
    struct Staged {
        Cloud cl;
        BuildScratch bs;
        hipStream_t stream = nullptr;
        std::thread th;
        std::mutex m;
        std::condition_variable cv;
        int state = 0;
        bool quit = false;
        const double* xyz = nullptr;   // the slot's pinned copy, or the caller's buffer (GICP_STAGE_BORROW)
        int64_t M = 0;
        int dim = 0;
        bool graph = false;
        int device = 0;
        gicp_params p{};
        int rc = GICP_OK;
        std::string err;
        void wait_idle() {
            std::unique_lock<std::mutex> lk(m);
            cv.wait(lk, [&] { return state != 1; });
        }
        void stop() {
            if (!th.joinable()) return;
            {
                std::lock_guard<std::mutex> g(m);
                quit = true;
            }
            cv.notify_all();
            th.join();
        }
    };
    Staged stg[GICP_MAX_STAGED];
    int stg_head = 0, stg_count = 0;
    size_t cap_hint = 0, cap_list = 0, cap_llen = 0, cap_lpass = 0, cap_lrc = 0;
    int pass = 0;
    bool use_lists = true;
    double skin_frac = 0.2;           // candidate-list skin as a fraction of d_c (GICP_SKIN)
    double skin_gain = 1.0;           // adaptive skin: multiple of the tile's last displacement (GICP_SKIN_GAIN)
    double last_rebuilds = 0.0;
    ncclComm_t comm = nullptr;
    int nranks = 1, rank = 0;
    gicp_allreduce_fn hook = nullptr;  // host statistics exchange (gicp_set_allreduce)
    void* hook_user = nullptr;
    double* h_xchg = nullptr;         // pinned exchange buffer of the hook
    // in-kernel peer exchange (gicp_peer_export / gicp_peer_init)
    double* d_peer_area = nullptr;    // this rank's exchange area (uncached device memory, IPC-exported)
    void* peer_open[kMaxPeers] = {};  // the peers' areas as opened here (closed by gicp_peer_close)
    PeerArgs peer{};                  // n > 1 while the peer exchange is on
    uint64_t* d_peer_ctr = nullptr;   // the device's exchange counter (PeerArgs::ctr)
    double peer_timeout_s = 10.0;
    double* d_probe = nullptr;
    double** d_peer_ptrs = nullptr;   // device copy of the areas' addresses (PeerArgs::area)
    std::vector<float> iter_ms;       // sampled k_corr time per iteration of the last align (-1: not sampled)
    double* d_rot = nullptr;          // gicp_rotated_covariances output
    size_t cap_rot = 0;
    // gicp_align_trace: per-iteration rows recorded on the device ([iter][(d+1)^2 + 1] pose + loss;
    // top-k rows [iter][16] source, target, det), copied out once after the loop
    double* d_hist = nullptr;
    size_t cap_hist = 0;
    int64_t* d_trace_top = nullptr;   // [iter][16] source, then [iter][16] target
    double* d_trace_det = nullptr;    // [iter][16]
    size_t cap_ttop = 0, cap_tdet = 0;
    unsigned long long* d_tail = nullptr;   // GICP_TAIL diagnostic build: [iter][kTailWords] (on this context's device)
    size_t cap_tail = 0;
    static constexpr int kMaxBatch = 64;
    hipEvent_t ev[2 * kMaxBatch] = {};
    int batch_hint = 0;               // iterations the last converging align ran: its first batch next time
    // diagnostics of the last pass
    double last_amb = 0.0, last_pairs = 0.0, last_sq = 0.0, last_gproved = 0.0, last_walked = 0.0;
    float last_corr_ms = 0.f, last_reduce_ms = 0.f;
    bool timing = false;
};

namespace {

void default_params(int dim, gicp_params* p) {
    std::memset(p, 0, sizeof(*p));
    p->max_iterations = 100;
    p->k_neighbors = dim == 2 ? 6 : 20;
    p->tolerance = 1e-6;
    p->max_distance_correspondence = 150.0;
    p->max_distance_nearest_neighbors = 50.0;
    p->epsilon = 100.0;
    p->ratio = 0.1;
    p->fixed_iterations = 0;
    p->min_neighbors = dim;
}

gicp_params resolve(int dim, const gicp_params* in) {
    gicp_params p;
    default_params(dim, &p);
    if (!in) return p;
    p = *in;
    if (p.k_neighbors <= 0) p.k_neighbors = dim == 2 ? 6 : 20;
    if (p.min_neighbors <= 0) p.min_neighbors = dim;
    if (p.epsilon == 0.0) p.epsilon = 100.0;
    if (p.cov_model < GICP_COV_PLANE_TO_PLANE || p.cov_model > GICP_COV_POINT_TO_PLANE)
        throw Fail{GICP_E_INVALID, "cov_model must be GICP_COV_PLANE_TO_PLANE, _POINT_TO_POINT or _POINT_TO_PLANE"};
    if (p.rotation_epsilon <= 0.0 && p.transformation_epsilon > 0.0) p.rotation_epsilon = 1.0 - p.transformation_epsilon;
    return p;
}

// fp32-screen error bound: E bounds the error of one coordinate difference
Margin make_margin(int dim, float rho_q, float rho_db, double dmax) {
    const double E = std::ldexp(8.0 * rho_q + 3.0 * rho_db + 3.0 * dmax, -23) + 1e-30;
    Margin m;
    m.a = (float)(2.0 * std::sqrt((double)dim) * E);
    m.b = (float)(dim * E * E);
    m.c = (float)std::ldexp(1.0, -16);
    return m;
}
float screen_bound(const Margin& m, double d) {
    const double d2 = d * d;
    const double b = d2 + 2.0 * (m.a * d + m.b + m.c * d2);
    return (float)(b * (1.0 + 1e-6)) + 1e-30f;
}

// Cut the Morton-sorted points into tiles: runs of <= 64 consecutive points whose bounding box (in
// Morton grid cells) stays within an extent cap E.  E is the smallest cap (steps of 2^(1/4)) whose
// tile count stays <= 1.35x the minimum ceil(n/64): tiles are as compact as that budget allows, and
// the cap bounds the largest tile, which sets both the widest query wave and the loosest box.
void build_tile_table(const std::vector<uint32_t>& codes, int dim, int bits, std::vector<int32_t>& start,
                      std::vector<int32_t>& count, std::vector<uint32_t>& first_code, int& cap_out, int k_hint,
                      WorkerPool& pool, int maxp = kTile) {
    const int64_t n = (int64_t)codes.size();
    static const double budget = [] {   // GICP_TILE_BUDGET: tile-count budget over ceil(n / 64)
        const char* e = std::getenv("GICP_TILE_BUDGET");
        const double b = e ? std::atof(e) : 1.35;
        return b >= 1.0 ? b : 1.35;
    }();
    const int64_t target = (int64_t)(budget * std::ceil(n / (double)maxp)) + 2;   // (maxp <= 64 points a tile)
    // decode the grid coordinates once
    auto compact3 = [](uint32_t x) {   // inverse of the kernels' spread3
        x &= 0x09249249u;
        x = (x | (x >> 2)) & 0x030C30C3u;
        x = (x | (x >> 4)) & 0x0300F00Fu;
        x = (x | (x >> 8)) & 0x030000FFu;
        x = (x | (x >> 16)) & 0x000003FFu;
        return x;
    };
    auto compact2 = [](uint32_t x) {
        x &= 0x55555555u;
        x = (x | (x >> 1)) & 0x33333333u;
        x = (x | (x >> 2)) & 0x0F0F0F0Fu;
        x = (x | (x >> 4)) & 0x00FF00FFu;
        x = (x | (x >> 8)) & 0x0000FFFFu;
        return x;
    };
    std::vector<uint16_t> g((size_t)n * dim);
    constexpr int kSeg = 16;   // fixed segments (independent of the host's core count: deterministic)
    pool.run(kSeg, [&](int k) {
        for (int64_t i = n * k / kSeg; i < n * (k + 1) / kSeg; ++i) {
            const uint32_t c = codes[i];
            for (int a = 0; a < dim; ++a)
                g[(size_t)i * dim + a] = (uint16_t)(dim == 3 ? compact3(c >> a) : compact2(c >> a));
        }
    });
    // greedy cut of points [b, e) (a forced break at b); appends (start, count) pairs if `out`
    auto cut_seg = [&](int64_t b, int64_t e, int E, std::vector<int32_t>* out) -> int64_t {
        int64_t nt = 0, i0 = b;
        int lo0 = 0, lo1 = 0, lo2 = 0, hi0 = 0, hi1 = 0, hi2 = 0;
        const uint16_t* gp = g.data();
        for (int64_t i = b; i < e; ++i) {
            const int v0 = gp[i * dim], v1 = gp[i * dim + 1], v2 = dim == 3 ? gp[i * dim + 2] : 0;
            if (i > i0) {
                const int n0 = std::min(lo0, v0), x0 = std::max(hi0, v0);
                const int n1 = std::min(lo1, v1), x1 = std::max(hi1, v1);
                const int n2 = std::min(lo2, v2), x2 = std::max(hi2, v2);
                if (i - i0 < maxp && x0 - n0 <= E && x1 - n1 <= E && x2 - n2 <= E) {
                    lo0 = n0, hi0 = x0, lo1 = n1, hi1 = x1, lo2 = n2, hi2 = x2;
                    continue;
                }
                ++nt;
                if (out) {
                    out->push_back((int32_t)i0);
                    out->push_back((int32_t)(i - i0));
                }
                i0 = i;
            }
            lo0 = hi0 = v0, lo1 = hi1 = v1, lo2 = hi2 = v2;
        }
        if (e > i0) {
            ++nt;
            if (out) {
                out->push_back((int32_t)i0);
                out->push_back((int32_t)(e - i0));
            }
        }
        return nt;
    };
    // the 16 segments are cut concurrently on the pool
    std::vector<std::vector<int32_t>> seg_out(kSeg);
    auto cut = [&](int E, bool emit) -> int64_t {
        int64_t nt_seg[kSeg] = {};
        pool.run(kSeg, [&](int k) {
            if (emit) seg_out[k].clear();
            nt_seg[k] = cut_seg(n * k / kSeg, n * (k + 1) / kSeg, E, emit ? &seg_out[k] : nullptr);
        });
        int64_t nt = 0;
        for (int k = 0; k < kSeg; ++k) nt += nt_seg[k];
        if (emit)
            for (int k = 0; k < kSeg; ++k)
                for (size_t j = 0; j < seg_out[k].size(); j += 2) {
                    start.push_back(seg_out[k][j]);
                    count.push_back(seg_out[k][j + 1]);
                    first_code.push_back(codes[seg_out[k][j]]);
                }
        return nt;
    };
    // smallest cap on the grid E_k = 2 * 2^(k/4) meeting the budget (the count falls as E grows):
    // a short walk from the previous cloud's k when given (a frame stream changes little), else a
    // binary search over k
    auto cap_of = [](int k) { return (int)(2.0 * std::pow(2.0, k / 4.0)); };
    const int kmax = 4 * (bits - 1);   // cap_of(kmax) = 2^bits: one Morton run per tile
    int klo = 0, khi = kmax;
    if (k_hint > 0 && k_hint < kmax) {   // walk from the hint: usually hint feasible, hint-1 not
        if (cut(cap_of(k_hint), false) <= target) {
            khi = k_hint;
            klo = k_hint - 1;
            if (cut(cap_of(klo), false) <= target) {
                khi = klo;
                klo = 0;
            } else {
                klo = k_hint;
            }
        } else {
            klo = k_hint + 1;
        }
    }
    while (klo < khi) {
        const int km = (klo + khi) / 2;
        if (cut(cap_of(km), false) <= target) khi = km;
        else klo = km + 1;
    }
    const int E = cap_of(klo);
    cap_out = klo;
    start.clear();
    count.clear();
    first_code.clear();
    cut(E, true);
}

// Build the device index of a cloud and the per-point covariances of all its tiles (a source shard
// is a set of interleaved chunks, and the whole-cloud pass costs ~1 ms at 1M points).
// Tiles of shard `shard` of `nshards` (the k_corr split: chunks of kShardChunk units of kCorrWaves tiles, dealt
// round-robin), or all of them when nshards = 1.
int shard_tile_count(int ntiles, int shard, int nshards) {
    if (nshards <= 1) return ntiles;
    constexpr int kChunkTiles = kShardChunk * kCorrWaves;
    const int nchunks = (ntiles + kChunkTiles - 1) / kChunkTiles;
    int mine = 0;
    for (int c = shard; c < nchunks; c += nshards) mine += std::min(kChunkTiles, ntiles - c * kChunkTiles);
    return mine;
}

// cov_shard / cov_nshards: the covariances are computed for that shard's tiles only (a sharded source: every
// rank needs the whole cloud's index for the neighbourhoods, but only its own tiles' covariances); the other
// rows read NaN.
// tile_points: points per tile at most (64; a source may take 32 or 16: GICP_SRC_TILE)
void build_cloud(Cloud& cl, const double* xyz, int64_t n, int dim, const gicp_params& p, bool graph,
                 BuildScratch& bs, hipStream_t st, bool staged = false, int cov_shard = 0, int cov_nshards = 1,
                 int tile_points = kTile) {
    if (!xyz || n <= 0 || (dim != 2 && dim != 3)) throw Fail{GICP_E_INVALID, "cloud must be a non-empty N x 2 or N x 3 array"};
    if (n > (int64_t)0x7FFFFFFF - 64) throw Fail{GICP_E_INVALID, "cloud too large (> 2^31 points)"};
    const bool verbose = std::getenv("GICP_VERBOSE") && std::getenv("GICP_VERBOSE")[0] == '1';
    auto tprev = std::chrono::steady_clock::now();
    std::string tlog;
    auto tick = [&](const char* what) {
        if (!verbose) return;
        HIPCHK(hipStreamSynchronize(st));
        const auto t = std::chrono::steady_clock::now();
        char b[64];
        std::snprintf(b, sizeof b, " %s %.1f", what, std::chrono::duration<double, std::milli>(t - tprev).count());
        tlog += b;
        tprev = t;
    };
    cl.n = 0;   // buffers are kept (grow-only) and reused
    cl.cov_ready = false;
    cl.graph_ready = false;
    cl.dim = dim;
    cl.bits = dim == 3 ? 10 : 16;
    // one fused, branch-free pass: bounds and the finiteness test (v - v is NaN for NaN and +-inf)
    double mn[3] = {0, 0, 0}, mx[3] = {0, 0, 0};
    bool finite = true;
    auto scan = [&](auto D_) {
        constexpr int D = decltype(D_)::value;
        double lo[D], hi[D], acc[D];
        for (int a = 0; a < D; ++a) lo[a] = hi[a] = xyz[a], acc[a] = 0.0;
        for (int64_t i = 0; i < n; ++i)
            for (int a = 0; a < D; ++a) {
                const double v = xyz[i * D + a];
                lo[a] = v < lo[a] ? v : lo[a];
                hi[a] = v > hi[a] ? v : hi[a];
                acc[a] += v - v;
            }
        for (int a = 0; a < D; ++a) {
            mn[a] = lo[a], mx[a] = hi[a];
            finite = finite && acc[a] == 0.0 && std::isfinite(lo[a]) && std::isfinite(hi[a]);
        }
    };
    if (dim == 3) scan(std::integral_constant<int, 3>{});
    else scan(std::integral_constant<int, 2>{});
    if (!finite) throw Fail{GICP_E_INVALID, "cloud contains non-finite coordinates"};
    double ext = 0.0;
    for (int a = 0; a < dim; ++a) ext = std::max(ext, mx[a] - mn[a]);
    ext = ext * (1.0 + 1e-9) + 1e-12 * (1.0 + std::fabs(mn[0]));
    for (int a = 0; a < 3; ++a) cl.lo[a] = a < dim ? mn[a] : 0.0;
    cl.scale = std::ldexp(1.0, cl.bits) / ext;
    tick("host-scan");

    {
        cl.reserve_points(n);
        dreserve(bs.s_in, bs.cap_in, (size_t)n * dim);
        dreserve(bs.s_codes, bs.cap_codes, (size_t)n);
        dreserve(bs.s_codes2, bs.cap_codes2, (size_t)n);
        dreserve(bs.s_idx, bs.cap_idx, (size_t)n);
        if (!bs.d_amb) {
            dalloc(bs.d_amb, 4);
            HIPCHK(hipMemsetAsync(bs.d_amb, 0, sizeof(int32_t) * 4, st));
        }
        double* d_in = bs.s_in;
        uint32_t *d_codes = bs.s_codes, *d_codes_s = bs.s_codes2;
        int32_t* d_idx = bs.s_idx;
        // (a staged build passes its pinned copy: the H2D copy is then asynchronous)
        HIPCHK(hipMemcpyAsync(d_in, xyz, sizeof(double) * n * dim, hipMemcpyHostToDevice, st));
        DevCloud fr = cl.view();
        HIPCHK(launch_morton(d_in, n, dim, fr, d_codes, d_idx, st));
        size_t tmp_bytes = 0;
        const unsigned end_bit = (unsigned)(dim * cl.bits);
        HIPCHK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, d_codes, d_codes_s, d_idx, cl.perm, (size_t)n, 0, end_bit,
                                         st));
        dreserve(bs.s_sort, bs.cap_sort, tmp_bytes + 16);
        HIPCHK(rocprim::radix_sort_pairs((void*)bs.s_sort, tmp_bytes, d_codes, d_codes_s, d_idx, cl.perm, (size_t)n, 0,
                                         end_bit, st));
        tick("upload+sort");
        std::vector<uint32_t> codes(n);
        HIPCHK(hipMemcpyAsync(codes.data(), d_codes_s, sizeof(uint32_t) * n, hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        tick("codes-d2h");
        std::vector<int32_t> tstart, tcount;
        std::vector<uint32_t> tcode;
        // (the extent-cap hint is kept for full-size tiles, the stream's case)
        build_tile_table(codes, dim, cl.bits, tstart, tcount, tcode, cl.level,
                         tile_points == kTile ? bs.cap_k_hint[dim & 3] : 0, bs.workers(), tile_points);
        if (tile_points == kTile) bs.cap_k_hint[dim & 3] = cl.level;
        tick("tiling");
        cl.ntiles = (int)tstart.size();
        cl.nblocks = (cl.ntiles + kBlockTiles - 1) / kBlockTiles;
        std::vector<TileInfo> ti(cl.ntiles);
        std::memset(ti.data(), 0, sizeof(TileInfo) * ti.size());
        for (int t = 0; t < cl.ntiles; ++t) {
            ti[t].start = tstart[t];
            ti[t].count = tcount[t];
        }
        cl.reserve_tiles(cl.ntiles, cl.nblocks);
        cl.n = n;
        unsigned* d_rho = reinterpret_cast<unsigned*>(d_codes);  // reuse scratch
        HIPCHK(hipMemsetAsync(d_rho, 0, sizeof(unsigned), st));
        HIPCHK(hipMemcpyAsync(cl.tiles, ti.data(), sizeof(TileInfo) * cl.ntiles, hipMemcpyHostToDevice, st));
        HIPCHK(hipMemcpyAsync(cl.tile_code, tcode.data(), sizeof(uint32_t) * cl.ntiles, hipMemcpyHostToDevice, st));
        // Morton seed lookup (DevCloud::seed_tab): 2^sb buckets of the code's top bits, about 4 per tile
        std::vector<int32_t> seed;
        {
            const int code_bits = dim * cl.bits;
            int sb = 2;
            while ((1 << sb) < 4 * cl.ntiles && sb < 20) ++sb;
            sb = std::min(sb, code_bits);
            cl.seed_shift = code_bits - sb;
            const size_t nb = (size_t)1 << sb;
            seed.resize(nb + 1);
            int t = 0;   // last tile whose first code <= p << shift (0 if none)
            for (size_t p = 0; p < nb; ++p) {
                const uint64_t lim = (uint64_t)p << cl.seed_shift;
                while (t + 1 < cl.ntiles && (uint64_t)tcode[t + 1] <= lim) ++t;
                seed[p] = t;
            }
            seed[nb] = cl.ntiles - 1;
            dreserve(cl.seed_tab, cl.cap_seed, nb + 1);
            HIPCHK(hipMemcpyAsync(cl.seed_tab, seed.data(), sizeof(int32_t) * (nb + 1), hipMemcpyHostToDevice, st));
        }
        HIPCHK(launch_build_tiles(d_in, dim, cl.perm, cl.tiles, cl.boxes, cl.ntiles, cl.xyz64, cl.rel32, cl.inv, d_rho, st));
        HIPCHK(launch_build_blocks(cl.tiles, cl.ntiles, cl.blocks, cl.nblocks, dim, st));
        unsigned rho_bits = 0;
        HIPCHK(hipMemcpyAsync(&rho_bits, d_rho, sizeof(unsigned), hipMemcpyDeviceToHost, st));
        HIPCHK(hipStreamSynchronize(st));
        std::memcpy(&cl.rho, &rho_bits, sizeof(float));
        tick("tiles");

        // surface covariances (gicp.py:19-35), of this rank's tiles when sharded
        const int qb = 0, qe = shard_tile_count(cl.ntiles, cov_shard, cov_nshards);
        CovArgs ca{};
        ca.cl = cl.view();
        ca.q_begin = qb;
        ca.q_end = qe;
        ca.sh_n = cov_nshards;
        ca.sh_r = cov_shard;
        if (cov_nshards > 1) HIPCHK(hipMemsetAsync(cl.cov, 0xFF, sizeof(double4) * n, st));   // NaN: not computed
        const double dn = p.max_distance_nearest_neighbors;
        ca.mg = make_margin(dim, cl.rho, cl.rho, dn);
        ca.search2 = screen_bound(ca.mg, dn);
        ca.dn2 = dn * dn;
        ca.eps_a = p.epsilon;
        ca.m_scale = std::sqrt(p.epsilon * (1.0 - p.ratio));
        ca.min_nb = p.min_neighbors;
        ca.cov_out = cl.cov;
        ca.count_out = cl.ncount;
        ca.amb_counter = bs.d_amb;
        // waves per query tile: a synchronous build of a small cloud is split by sub-tile (the walk of its
        // longest wave bounds it); a staged build keeps one wave per tile -- it runs beside a registration,
        // whose k_corr the split's idle lanes would slow (C5, 500 frames: 1050 vs 960 frames/s) -- and so
        // does a cloud whose tiles alone fill the GPU (GICP_BUILD_SPLIT = 1 / 4 forces either)
        static const int split_env = [] {
            const char* e = std::getenv("GICP_BUILD_SPLIT");
            return e ? std::atoi(e) : 0;
        }();
        ca.split = split_env == 1 || split_env == kSub ? split_env : (!staged && cl.ntiles <= 8192 ? kSub : 1);
        // the target neighbour graph (k_corr's graph descent) comes out of the covariances'
        // own two walks (k_knn_cov<D, K, true>), then one pass packs the rows
        GraphArgs ga{};
        if (graph) {
            dreserve(cl.nbq, cl.cap_nbq, (size_t)n * 8);
            dreserve(cl.nbx, cl.cap_nbx, (size_t)n * 3);
            dreserve(cl.nbi, cl.cap_nbi, (size_t)n * kGraphK);
            dreserve(bs.g_nb, bs.cap_gnb, (size_t)n * kGraphK);   // unpacked rows (scratch)
            dreserve(bs.g_nbh, bs.cap_gnbh, (size_t)n);
            ga.cl = cl.view();
            ga.split = ca.split;
            ga.mg = ca.mg;
            ga.search2 = ca.search2;
            ga.nb = bs.g_nb;
            ga.nbh = bs.g_nbh;
            ga.nbq = cl.nbq;
            ga.nbx = cl.nbx;
            ga.nbi = cl.nbi;
            ca.g_nb = bs.g_nb;
            ca.g_nbh = bs.g_nbh;
        }
        HIPCHK(hipMemsetAsync(cl.ncount, 0, sizeof(int32_t) * n, st));
        hipError_t e = launch_knn_cov(ca, dim, p.k_neighbors, graph, st);
        if (e == hipErrorInvalidValue) throw Fail{GICP_E_INVALID, "unsupported k_neighbors for this dim (2-D: 6, 10; 3-D: 10, 20)"};
        HIPCHK(e);
        if (graph) HIPCHK(launch_graph_pack(ga, st));
        HIPCHK(hipStreamSynchronize(st));
        cl.cov_ready = true;
        cl.cov_shard = cov_shard;
        cl.cov_nshards = cov_nshards;
        cl.graph_ready = graph;
        tick(graph ? "covariances+graph" : "covariances");
        if (verbose)
            std::fprintf(stderr, "[gicp] cloud n=%lld tiles=%d (%.2fx min) extent cap=%d cells rho=%.4f | ms:%s\n",
                         (long long)n, cl.ntiles, cl.ntiles / std::ceil(n / 64.0), cl.level, cl.rho, tlog.c_str());
    }
}

// Per-source-tile state that refers to target tiles (hints, candidate lists, heavy schedule):
// reset whenever either cloud changes.
void reset_tile_state(gicp_ctx* c) {
    const int nt = std::max(1, c->src.ntiles);
    if (!c->d_hint) return;
    // hints -1, lists empty, certificates none (cert_pass -1) and no last match (cert_j -1: k_corr's per-lane
    // search cap) -- one launch (five memsets were five queue operations, ~40 us of a C5 frame)
    HIPCHK(launch_reset_tiles(c->d_hint, c->d_list_len, c->d_list_rcert, c->d_cert_pass, nt, c->d_cert_j,
                              c->d_cert_j ? std::max<int64_t>(1, c->src.n) : 0, c->stream));
    c->pass = 0;
}

void set_shard(gicp_ctx* c, int shard, int nshards) {
    if (nshards < 1 || shard < 0 || shard >= nshards) throw Fail{GICP_E_INVALID, "bad shard / nshards"};
    if (c->src.cov_nshards > 1 && (c->src.cov_nshards != nshards || c->src.cov_shard != shard))
        throw Fail{GICP_E_INVALID, "the source's covariances were computed for another shard"};
    c->shard = shard;
    c->nshards = nshards;
    c->q_begin = 0;   // k_corr maps this rank's units onto the cloud's (interleaved chunks)
    c->q_end = c->src.ntiles;
    const int nt = std::max(1, c->src.ntiles);
    dreserve(c->d_hint, c->cap_hint, nt);
    dreserve(c->d_list, c->cap_list, (size_t)nt * kListMax);
    dreserve(c->d_list_len, c->cap_llen, nt);
    dreserve(c->d_list_pass, c->cap_lpass, nt);
    dreserve(c->d_list_rcert, c->cap_lrc, nt);
    if (!c->d_poses) dalloc(c->d_poses, (size_t)kPoseRing * 12);
    dreserve(c->d_cert_j, c->cap_cj, (size_t)std::max<int64_t>(1, c->src.n));
    dreserve(c->d_cert_gap, c->cap_cg, (size_t)std::max<int64_t>(1, c->src.n));
    dreserve(c->d_cert_pass, c->cap_cp, nt);
    reset_tile_state(c);
}

void ensure_workspace(gicp_ctx* c) {
    const int nsx = nstat_ext(3);
    const int grid = std::max(1, corr_grid(c->src.ntiles, c->shard, c->nshards));
    if ((grid + kGroupWG - 1) / kGroupWG > kMaxGroups) throw Fail{GICP_E_INVALID, "source shard too large"};
    const size_t need = (size_t)grid * nsx;
    if (need > c->partials_cap) {
        dalloc(c->d_partials, need);
        c->partials_cap = need;
    }
    if (!c->d_state) {
        dalloc(c->d_state, 1);
        HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->h_state), sizeof(IterState)));
        std::memset(c->h_state, 0, sizeof(IterState));
        dalloc(c->d_tickets, (size_t)(kMaxGroups + 1) * kTicketStride);
        HIPCHK(hipMemsetAsync(c->d_tickets, 0, sizeof(uint32_t) * (kMaxGroups + 1) * kTicketStride, c->stream));
        dalloc(c->d_gpart, (size_t)kMaxGroups * nsx);
    }
}

// The largest double x with sqrt(x) <= dc (sqrt correctly rounded, as on the device), so the accept
// test of gicp.py:136, !(distance > d_c) with distance = sqrt(d2), is exactly d2 <= accept_d2_max(d_c)
double accept_d2_max(double dc) {
    if (!(dc >= 0.0) || std::isinf(dc)) return dc;   // d_c = +inf accepts everything; NaN nothing
    double x = dc * dc;
    while (std::sqrt(x) > dc) x = std::nextafter(x, 0.0);
    while (std::sqrt(std::nextafter(x, INFINITY)) <= dc) x = std::nextafter(x, INFINITY);
    return x;
}

// kernel arguments of a pass (the pose comes from the device state)
CorrArgs corr_args(gicp_ctx* c, int single_pass) {
    const int d = c->src.dim;
    CorrArgs a{};
    a.src = c->src.view();
    a.tgt = c->tgt.view();
    a.q_begin = c->q_begin;
    a.q_end = c->q_end;
    a.sh_skip = (c->nshards - 1) * kShardChunk;
    a.sh_first = c->shard * kShardChunk;
    a.unit_map = c->unit_map;
    a.state = c->d_state;
    a.tickets = c->d_tickets;
    a.gpart = c->d_gpart;
    a.single_pass = single_pass;
    const double dc = c->psrc.max_distance_correspondence;
    a.dc = dc;
    a.dc2_max = accept_d2_max(dc);
    // with certificates the screen reaches kappa past d_c, so an empty lane's radius outlasts small moves
    const double kappa = c->use_certs ? c->kappa_frac * dc : 0.0;
    a.mg = make_margin(d, c->src.rho, c->tgt.rho, dc + kappa);
    a.search2 = screen_bound(a.mg, dc + kappa);
    a.kappa = (float)kappa;
    a.empty_r = (float)dc * (1.0f + 1e-6f);
    if (c->use_certs) {
        a.cert_j = c->d_cert_j;
        a.cert_gap = c->d_cert_gap;
    }
    a.cert_pass = c->d_cert_pass;   // always valid: k_corr reads it (and hint) unconditionally, with the tile metadata
    a.hint = c->d_hint;
    a.partials = c->d_partials;
    a.count_pairs = 1;
    a.list = c->d_list;
    a.list_len = c->d_list_len;
    a.list_rcert = c->d_list_rcert;
    a.list_pass = c->d_list_pass;
    a.poses = c->d_poses;
    a.pass = ++c->pass;
    a.use_lists = c->use_lists ? 1 : 0;
    a.sparse_max = c->sparse_max;
    a.sparse_amb = c->sparse_amb;
    a.skin = (float)(c->skin_frac * dc);
    a.skin_gain = (float)c->skin_gain;
    a.skin_max = (float)dc;
    a.gap_slack = (float)std::ldexp(std::sqrt((double)a.search2) + 2.0 * c->tgt.rho + 2.0 * c->src.rho, -19);
    a.cov_model = c->psrc.cov_model;
    a.pl_inv = 1.0 / (c->ptgt.epsilon * (1.0 - c->ptgt.ratio));   // target m = sqrt(eps (1 - ratio)) n
    if (c->peer.n > 1) a.peer = c->peer;   // (the exchange's sequence number is counted on the device)
    return a;
}

void allreduce_stats(gicp_ctx* c) {
    const int nsx = nstat_ext(c->src.dim);
    if (c->peer.n > 1) return;   // summed inside k_corr
    if (c->hook) {   // host exchange: statistics out, the caller's sum over ranks back in
        HIPCHK(hipMemcpyAsync(c->h_xchg, c->d_state->stats, sizeof(double) * nsx, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        if (c->hook(c->h_xchg, nsx, c->hook_user) != 0) throw Fail{GICP_E_COMM, "host all-reduce hook failed"};
        HIPCHK(hipMemcpyAsync(c->d_state->stats, c->h_xchg, sizeof(double) * nsx, hipMemcpyHostToDevice, c->stream));
        return;
    }
    if (!c->comm) return;
    ncclResult_t r = ncclAllReduce(c->d_state->stats, c->d_state->stats, nsx, ncclFloat64, ncclSum, c->comm, c->stream);
    if (r != ncclSuccess) throw Fail{GICP_E_COMM, std::string("ncclAllReduce: ") + ncclGetErrorString(r)};
}

#if defined(GICP_STAMPS) || defined(GICP_TIMELINE)
// Diagnostic build: per wave 8 phase-cycle slots (7 = rows scanned) + 8 event counters.
void print_stamps(const unsigned long long* d_stamps, size_t nst) {
    constexpr int W = 20;
    std::vector<unsigned long long> hs(nst);
    HIPCHK(hipMemcpy(hs.data(), d_stamps, nst * 8, hipMemcpyDeviceToHost));
    if (const char* f = std::getenv("GICP_STAMPS_DUMP")) {   // raw [waves][20] u64 for offline analysis
        static int seq = 0;
        const std::string path = std::string(f) + "." + std::to_string(seq++);
        if (FILE* fp = std::fopen(path.c_str(), "wb")) {
            std::fwrite(hs.data(), 8, hs.size(), fp);
            std::fclose(fp);
        }
    }
    std::vector<std::pair<double, size_t>> byc;
    double tot[W] = {0}, all = 0;
    for (size_t w = 0; w < nst / W; ++w) {
        double r = 0;
        for (int k = 0; k < 7; ++k) r += (double)hs[w * W + k];
        if (r <= 0) continue;
        byc.push_back({r, w});
        all += r;
        for (int k = 0; k < W; ++k) tot[k] += (double)hs[w * W + k];
    }
    if (byc.empty()) return;
    std::sort(byc.begin(), byc.end());
    const size_t nw = byc.size(), n1 = std::max<size_t>(1, nw / 100);
    static const char* nm[W] = {"setup", "trav", "stage", "scan", "fb", "epi", "red", "rows",
                                "visits", "scanned", "chunks", "list", "listlen", "blktests", "candblk", "fbtiles",
                                "t0", "t1", "hwid", "xcc"};
    auto row = [&](const char* tag, size_t b, size_t e) {
        double m[W] = {0};
        for (size_t i = b; i < e; ++i)
            for (int k = 0; k < W; ++k) m[k] += (double)hs[byc[i].second * W + k] / (double)(e - b);
        std::fprintf(stderr, "[stamps] %-9s", tag);
        for (int k = 0; k < 16; ++k) std::fprintf(stderr, " %s %.6g", nm[k], m[k]);
        std::fprintf(stderr, "\n");
    };
    row("all", 0, nw);
    row("median1%", nw / 2 - n1 / 2, nw / 2 - n1 / 2 + n1);
    row("slowest1%", nw - n1, nw);
    for (size_t i = nw - std::min<size_t>(nw, 4); i < nw; ++i) {
        char tag[32];
        std::snprintf(tag, sizeof tag, "w%zu", byc[i].second);
        row(tag, i, i + 1);
    }
    std::fprintf(stderr, "[stamps] wave cycles p50 %.0f p90 %.0f p99 %.0f p999 %.0f max %.0f\n", byc[nw / 2].first,
                 byc[nw * 9 / 10].first, byc[nw * 99 / 100].first, byc[nw * 999 / 1000].first, byc.back().first);
    std::fprintf(stderr, "[stamps] waves %zu, mean cycles/wave %.0f:", nw, all / (double)nw);
    for (int k = 0; k < 7; ++k) std::fprintf(stderr, " %s %.1f%%", nm[k], 100.0 * tot[k] / std::max(1.0, all));
    std::fprintf(stderr, "\n");
}
#endif

// per-point debug outputs of a pass (gicp_debug) and the det(W) record of the top-k, grow-only
void ensure_dbg(gicp_ctx* c) {
    const size_t n = (size_t)c->src.n;
    if (c->dbg_cap < n) {
        dalloc(c->d_dbg_idx, n);
        dalloc(c->d_dbg_w, n * 9);
        dalloc(c->d_dbg_dist, n);
        dalloc(c->d_dbg_det, n);
        dalloc(c->d_top_tgt, n);
        c->dbg_cap = n;
    }
}

constexpr int kTopBlocks = 256;   // stage-1 blocks of the top-k of det(W)

void ensure_top_scratch(gicp_ctx* c) {
    if (!c->d_top_v) {
        dalloc(c->d_top_v, (size_t)kTopBlocks * 16 + 16);
        dalloc(c->d_top_i, (size_t)kTopBlocks * 16);
        dalloc(c->d_top_out, 32);
    }
}

// Top-k of the last pass's det(W) (k_top1 / k_top2) and its copy into the pinned c->h_top, enqueued on
// the library's stream (the caller synchronises).
void top_enqueue(gicp_ctx* c, int k) {
    ensure_top_scratch(c);
    if (!c->h_top) HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->h_top), sizeof(int64_t) * 32 + sizeof(double) * 16));
    double* ov = c->d_top_v + (size_t)kTopBlocks * 16;
    HIPCHK(launch_top_weights(c->d_dbg_det, c->d_top_tgt, c->src.perm, c->src.n, k, c->d_top_v, c->d_top_i, kTopBlocks,
                              ov, c->d_top_out, c->d_top_out + 16, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_top, c->d_top_out, sizeof(int64_t) * 32, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipMemcpyAsync(c->h_top + 32, ov, sizeof(double) * 16, hipMemcpyDeviceToHost, c->stream));
}

// One pass at pose T: statistics (all-reduced) into c->h_stats.
void run_pass(gicp_ctx* c, const double* T, gicp_debug* dbg) {
    if (!c->tgt.n || !c->src.n) throw Fail{GICP_E_STATE, "set_target and set_source first"};
    if (c->tgt.dim != c->src.dim) throw Fail{GICP_E_INVALID, "source and target dimensions differ"};
    const int d = c->src.dim, n1 = d + 1;
    for (int k = 0; k < n1 * n1; ++k)
        if (!std::isfinite(T[k])) throw Fail{GICP_E_INVALID, "pose contains non-finite values"};
    ensure_workspace(c);
    hipStream_t st = c->stream;
    IterState& hs = *c->h_state;
    std::memset(&hs, 0, offsetof(IterState, stats));
    for (int k = 0; k < n1 * n1; ++k) hs.T[k] = T[k];
    hs.converged_at = -1;
    HIPCHK(hipMemcpyAsync(c->d_state, &hs, offsetof(IterState, stats), hipMemcpyHostToDevice, st));
    CorrArgs a = corr_args(c, 1);
    c->top_ready = false;
    if (dbg && (dbg->index || dbg->weight || dbg->distance || dbg->want_top_weights)) {
        ensure_dbg(c);
        a.dbg_index = dbg->index ? c->d_dbg_idx : nullptr;
        a.dbg_weight = dbg->weight ? c->d_dbg_w : nullptr;
        a.dbg_dist = dbg->distance ? c->d_dbg_dist : nullptr;
        if (dbg->want_top_weights) {   // rows of other shards stay NaN (never selected); one shard writes every row
            if (c->nshards > 1) HIPCHK(hipMemsetAsync(c->d_dbg_det, 0xFF, sizeof(double) * c->src.n, st));
            a.dbg_det = c->d_dbg_det;
            a.top_tgt = c->d_top_tgt;
        }
    }
    const int nsx = nstat_ext(d);
    const int grid = corr_grid(c->src.ntiles, c->shard, c->nshards);
#if defined(GICP_STAMPS) || defined(GICP_TIMELINE)
    static unsigned long long* d_stamps = nullptr;
    static size_t stamps_cap = 0;
    const size_t nst = (size_t)std::max(1, grid) * kCorrWaves * 20;
    if (nst > stamps_cap) {
        dalloc(d_stamps, nst);
        stamps_cap = nst;
    }
    HIPCHK(hipMemsetAsync(d_stamps, 0, nst * 8, st));
    a.stamps = d_stamps;
#endif
    if (grid > 0) {
        HIPCHK(launch_corr(a, d, grid, st));
    } else if (a.peer.n > 1) {   // no tile in this shard: one empty workgroup still takes part in the exchange
        a.q_end = 0;
        HIPCHK(launch_corr(a, d, 1, st));
    } else {
        HIPCHK(hipMemsetAsync(c->d_state->stats, 0, sizeof(double) * nsx, st));
    }
    allreduce_stats(c);
    HIPCHK(hipMemcpyAsync(c->h_stats, c->d_state->stats, sizeof(double) * nsx, hipMemcpyDeviceToHost, st));
    c->top_cached_k = 0;
    if (a.dbg_det && c->src.n > 0) {   // the top-k in the same stream sync as the pass
        top_enqueue(c, c->top_k_pref);
        c->top_cached_k = c->top_k_pref;
    }
    if (dbg) {
        const size_t n = (size_t)c->src.n;
        if (dbg->index) HIPCHK(hipMemcpyAsync(dbg->index, c->d_dbg_idx, sizeof(int64_t) * n, hipMemcpyDeviceToHost, st));
        if (dbg->weight)
            HIPCHK(hipMemcpyAsync(dbg->weight, c->d_dbg_w, sizeof(double) * n * d * d, hipMemcpyDeviceToHost, st));
        if (dbg->distance)
            HIPCHK(hipMemcpyAsync(dbg->distance, c->d_dbg_dist, sizeof(double) * n, hipMemcpyDeviceToHost, st));
    }
    HIPCHK(hipStreamSynchronize(st));
    if (a.peer.n > 1) {
        int fail = 0;
        HIPCHK(hipMemcpy(&fail, &c->d_state->solve_fail, sizeof(int), hipMemcpyDeviceToHost));
        if (fail == 2) throw Fail{GICP_E_COMM, "peer exchange timed out (a rank did not arrive)"};
    }
#if defined(GICP_STAMPS) || defined(GICP_TIMELINE)
    print_stamps(d_stamps, nst);
#endif
    const int ns = nstat(d);
    c->last_amb = c->h_stats[ns];
    c->last_pairs = c->h_stats[ns + 1];
    c->last_rebuilds = c->h_stats[ns + 2];
    c->last_sq = c->h_stats[ns + 3];
    c->last_gproved = c->h_stats[ns + 4];
    c->last_walked = c->h_stats[ns + 5];
    c->top_ready = a.dbg_det != nullptr;
}

}  // namespace

namespace {
// drop the peer exchange: unmap the peers' areas (this rank's own area stays, re-exportable)
void close_peers(gicp_ctx* c) {
    bool any = c->peer.n > 1;
    for (void* p : c->peer_open) any = any || p != nullptr;
    if (any) quiet(hipStreamSynchronize(c->stream));   // no launch of ours still uses the mappings
    for (auto& p : c->peer_open) {
        if (p) quiet(hipIpcCloseMemHandle(p));
        p = nullptr;
    }
    c->peer = PeerArgs{};
}

int guard_impl(gicp_ctx* c, const char* where, const std::function<void()>& body) {
    try {
        if (c) HIPCHK(hipSetDevice(c->device));
        body();
        return GICP_OK;
    } catch (const Fail& f) {
        if (c) c->err = std::string(where) + ": " + f.msg;
        return f.code;
    } catch (const std::bad_alloc&) {
        if (c) c->err = std::string(where) + ": out of host memory";
        return GICP_E_NOMEM;
    } catch (...) {
        if (c) c->err = std::string(where) + ": unknown error";
        return GICP_E_INVALID;
    }
}
}  // namespace

extern "C" {

int gicp_version(void) { return 100; }

int gicp_stats_size(int dim) { return (dim == 2 || dim == 3) ? nstat(dim == 2 ? 2 : 3) : GICP_E_INVALID; }

void gicp_default_params(int dim, gicp_params* out) {
    if (out) default_params(dim == 2 ? 2 : 3, out);
}

const char* gicp_strerror(int code) {
    switch (code) {
        case GICP_OK: return "ok";
        case GICP_E_INVALID: return "invalid argument";
        case GICP_E_HIP: return "HIP runtime error";
        case GICP_E_STATE: return "call out of order";
        case GICP_E_COMM: return "RCCL error";
        case GICP_E_NOMEM: return "out of memory";
        default: return "unknown error";
    }
}

int gicp_create(gicp_ctx** out, int device) {
    if (!out) return GICP_E_INVALID;
    *out = nullptr;
    gicp_ctx* c = new (std::nothrow) gicp_ctx();
    if (!c) return GICP_E_NOMEM;
    c->device = device;
    if (const char* e = std::getenv("GICP_NO_LISTS")) c->use_lists = !(e[0] == '1');
    if (const char* e = std::getenv("GICP_SKIN")) c->skin_frac = std::max(0.0, std::atof(e));
    if (const char* e = std::getenv("GICP_SKIN_GAIN")) c->skin_gain = std::max(0.0, std::atof(e));
    if (const char* e = std::getenv("GICP_NO_CERTS")) c->use_certs = !(e[0] == '1');
    if (const char* e = std::getenv("GICP_NO_GRAPH")) c->use_graph = !(e[0] == '1');
    if (const char* e = std::getenv("GICP_FUSE_SOLVE")) c->fuse_solve = !(e[0] == '0');
    if (const char* e = std::getenv("GICP_UNIT_MAP")) c->unit_map = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("GICP_MOVING_MAP")) c->moving_map = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("GICP_MOVING_ITERS")) c->moving_iters = std::max(0, std::atoi(e));
    if (const char* e = std::getenv("GICP_SRC_TILE")) {
        const int v = std::atoi(e);
        c->src_tile = v == 16 || v == 32 ? v : kTile;
    }
    if (const char* e = std::getenv("GICP_CERT_KAPPA")) c->kappa_frac = std::max(0.0, std::atof(e));
    if (const char* e = std::getenv("GICP_SPARSE_WALK")) c->sparse_max = std::max(0, std::min(64, std::atoi(e)));
    if (const char* e = std::getenv("GICP_SPARSE_AMB")) c->sparse_amb = std::max(0, std::min(64, std::atoi(e)));
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) {
        delete c;
        return GICP_E_HIP;
    }
    if (device < 0 || device >= ndev) {
        delete c;
        return GICP_E_INVALID;
    }
    const int rc = guard_impl(c, "gicp_create", [&] {
        HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        for (auto& e : c->ev) HIPCHK(hipEventCreate(&e));
    });
    if (rc != GICP_OK) {
        gicp_destroy(c);
        return rc;
    }
    *out = c;
    return GICP_OK;
}

void gicp_destroy(gicp_ctx* c) {
    if (!c) return;
    for (auto& g : c->stg) g.stop();             // staged builds still running finish first
    quiet(hipSetDevice(c->device));
    if (c->stream) quiet(hipStreamSynchronize(c->stream));
    if (c->comm) ncclCommDestroy(c->comm);
    for (auto& p : c->peer_open)
        if (p) quiet(hipIpcCloseMemHandle(p));
    if (c->d_peer_area) quiet(hipFree(c->d_peer_area));
    dfree(c->d_probe);
    dfree(c->d_peer_ptrs);
    dfree(c->d_peer_ctr);
    c->tgt.release();
    c->src.release();
    dfree(c->d_hint);
    dfree(c->d_partials);
    dfree(c->d_state);
    dfree(c->d_tickets);
    dfree(c->d_gpart);
    dfree(c->d_dbg_idx);
    dfree(c->d_dbg_w);
    dfree(c->d_dbg_dist);
    dfree(c->d_dbg_det);
    dfree(c->d_top_tgt);
    dfree(c->d_cert_j);
    dfree(c->d_cert_gap);
    dfree(c->d_cert_pass);
    dfree(c->d_top_v);
    dfree(c->d_top_i);
    dfree(c->d_top_out);
    dfree(c->d_list);
    dfree(c->d_list_len);
    dfree(c->d_list_pass);
    dfree(c->d_list_rcert);
    dfree(c->d_poses);
    c->bs.release();
    for (auto& g : c->stg) {
        g.bs.release();
        g.cl.release();
        if (g.stream) quiet(hipStreamDestroy(g.stream));
    }
    if (c->h_state) quiet(hipHostFree(c->h_state));
    if (c->h_top) quiet(hipHostFree(c->h_top));
    if (c->h_xchg) quiet(hipHostFree(c->h_xchg));
    dfree(c->d_rot);
    dfree(c->d_hist);
    dfree(c->d_trace_top);
    dfree(c->d_trace_det);
    dfree(c->d_tail);
    for (auto& e : c->ev)
        if (e) quiet(hipEventDestroy(e));
    if (c->stream) quiet(hipStreamDestroy(c->stream));
    delete c;
}

const char* gicp_last_error(const gicp_ctx* c) { return c ? c->err.c_str() : "null context"; }

int gicp_comm_unique_id(char out[GICP_COMM_ID_BYTES]) {
    if (!out) return GICP_E_INVALID;
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return GICP_E_COMM;
    static_assert(sizeof(id) == GICP_COMM_ID_BYTES, "ncclUniqueId size");
    std::memcpy(out, &id, sizeof(id));
    return GICP_OK;
}

int gicp_comm_init(gicp_ctx* c, int nranks, int rank, const char id[GICP_COMM_ID_BYTES]) {
    if (!c || !id || nranks < 1 || rank < 0 || rank >= nranks) return GICP_E_INVALID;
    return guard_impl(c, "gicp_comm_init", [&] {
        if (c->comm) {
            ncclCommDestroy(c->comm);
            c->comm = nullptr;
        }
        c->hook = nullptr;   // one exchange per context
        close_peers(c);
        // a one-rank communicator is created too: the all-reduce then runs (as an identity) on the
        // same stream path as a multi-GPU job, which is how the one-GPU tests exercise it
        ncclUniqueId uid;
        std::memcpy(&uid, id, sizeof(uid));
        ncclResult_t r = ncclCommInitRank(&c->comm, nranks, uid, rank);
        if (r != ncclSuccess) throw Fail{GICP_E_COMM, std::string("ncclCommInitRank: ") + ncclGetErrorString(r)};
        c->nranks = nranks;
        c->rank = rank;
    });
}

int gicp_comm_ranks(gicp_ctx* c, int* nranks, int* rank, int* kind) {
    if (!c) return GICP_E_INVALID;
    return guard_impl(c, "gicp_comm_ranks", [&] {
        int n = 1, r = 0, k = 0;
        if (c->peer.n > 1) {
            n = c->peer.n;
            r = c->peer.rank;
            k = 3;
        } else if (c->comm) {
            ncclResult_t e = ncclCommCount(c->comm, &n);
            if (e == ncclSuccess) e = ncclCommUserRank(c->comm, &r);
            if (e != ncclSuccess) throw Fail{GICP_E_COMM, std::string("ncclCommCount: ") + ncclGetErrorString(e)};
            k = 1;
        } else if (c->hook) {
            n = c->nranks;
            r = c->rank;
            k = 2;
        }
        if (nranks) *nranks = n;
        if (rank) *rank = r;
        if (kind) *kind = k;
    });
}

int gicp_set_target(gicp_ctx* c, const double* xyz, int64_t M, int dim, const gicp_params* p) {
    if (!c) return GICP_E_INVALID;
    return guard_impl(c, "gicp_set_target", [&] {
        c->ptgt = resolve(dim, p);
        c->top_ready = false;
        build_cloud(c->tgt, xyz, M, dim, c->ptgt, c->use_graph && c->use_certs, c->bs, c->stream);
        if (c->src.n) reset_tile_state(c);
    });
}

int gicp_set_source(gicp_ctx* c, const double* xyz, int64_t N, int dim, const gicp_params* p, int shard,
                    int nshards) {
    if (!c) return GICP_E_INVALID;
    return guard_impl(c, "gicp_set_source", [&] {
        if (nshards < 1 || shard < 0 || shard >= nshards) throw Fail{GICP_E_INVALID, "bad shard / nshards"};
        c->psrc = resolve(dim, p);
        c->top_ready = false;
        build_cloud(c->src, xyz, N, dim, c->psrc, false, c->bs, c->stream, false, shard, nshards, c->src_tile);
        set_shard(c, shard, nshards);
        HIPCHK(hipStreamSynchronize(c->stream));
    });
}

int gicp_target_to_source(gicp_ctx* c, int shard, int nshards) {
    if (!c) return GICP_E_INVALID;
    return guard_impl(c, "gicp_target_to_source", [&] {
        if (!c->tgt.n) throw Fail{GICP_E_STATE, "no target to promote"};
        std::swap(c->src, c->tgt);   // the old source's buffers are kept for the next target
        c->top_ready = false;
        c->tgt.n = 0;
        c->tgt.cov_ready = false;
        c->psrc = c->ptgt;
        set_shard(c, shard, nshards);   // (its resets are stream-ordered before the next registration: no host sync)
    });
}

int gicp_get_covariances(gicp_ctx* c, int which, double* out) {
    if (!c || !out || (which != 0 && which != 1)) return GICP_E_INVALID;
    return guard_impl(c, "gicp_get_covariances", [&] {
        Cloud& cl = which == 0 ? c->tgt : c->src;
        if (!cl.n || !cl.cov_ready) throw Fail{GICP_E_STATE, "cloud not set"};
        // a I - m m^T expanded on the device in original order (k_rotate_cov with R = I: R m = m
        // exactly), then one copy of the n x d x d result
        const int d = cl.dim;
        const double I[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        const double I2[4] = {1, 0, 0, 1};
        const size_t m = (size_t)cl.n * d * d;
        dreserve(c->d_rot, c->cap_rot, m);
        HIPCHK(launch_rotate_cov(cl.cov, cl.perm, cl.n, d, d == 3 ? I : I2, c->d_rot, c->stream));
        HIPCHK(hipMemcpyAsync(out, c->d_rot, sizeof(double) * m, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    });
}

int gicp_get_graph(gicp_ctx* c, int64_t* index, double* radius) {
    if (!c) return GICP_E_INVALID;
    static_assert(GICP_GRAPH_K == kGraphK, "graph width");
    return guard_impl(c, "gicp_get_graph", [&] {
        Cloud& cl = c->tgt;
        if (!cl.n || !cl.graph_ready) throw Fail{GICP_E_STATE, "no target graph (set_target first; GICP_NO_GRAPH unset)"};
        const int64_t n = cl.n;
        std::vector<uint4> nbq((size_t)n * 8);
        std::vector<int32_t> nbi((size_t)n * kGraphK), perm(n);
        HIPCHK(hipMemcpyAsync(nbq.data(), cl.nbq, sizeof(uint4) * n * 8, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(nbi.data(), cl.nbi, sizeof(int32_t) * n * kGraphK, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(perm.data(), cl.perm, sizeof(int32_t) * n, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (int64_t i = 0; i < n; ++i) {
            const int64_t o = perm[i];
            if (radius) {
                float r;
                std::memcpy(&r, &nbq[(size_t)i * 8].x, sizeof(float));
                radius[o] = r;
            }
            if (index)
                for (int k = 0; k < kGraphK; ++k) {
                    const int t = nbi[(size_t)i * kGraphK + k];
                    index[o * kGraphK + k] = t >= 0 ? (int64_t)perm[t] : -1;
                }
        }
    });
}

int gicp_get_neighbor_counts(gicp_ctx* c, int which, int32_t* out) {
    if (!c || !out || (which != 0 && which != 1)) return GICP_E_INVALID;
    return guard_impl(c, "gicp_get_neighbor_counts", [&] {
        Cloud& cl = which == 0 ? c->tgt : c->src;
        if (!cl.n) throw Fail{GICP_E_STATE, "cloud not set"};
        std::vector<int32_t> cnt(cl.n), perm(cl.n);
        HIPCHK(hipMemcpyAsync(cnt.data(), cl.ncount, sizeof(int32_t) * cl.n, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipMemcpyAsync(perm.data(), cl.perm, sizeof(int32_t) * cl.n, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        for (int64_t i = 0; i < cl.n; ++i) out[perm[i]] = cnt[i];
    });
}

int gicp_iterate(gicp_ctx* c, const double* T, double* stats, gicp_debug* dbg) {
    if (!c || !T || !stats) return GICP_E_INVALID;
    return guard_impl(c, "gicp_iterate", [&] {
        run_pass(c, T, dbg);
        std::memcpy(stats, c->h_stats, sizeof(double) * nstat(c->src.dim));
    });
}

int gicp_pass_info(gicp_ctx* c, double out[GICP_PASS_INFO]) {
    if (!c || !out) return GICP_E_INVALID;
    out[0] = c->last_amb;
    out[1] = c->last_pairs;
    out[2] = c->last_rebuilds;
    out[3] = c->last_sq;
    out[4] = c->last_gproved;
    out[5] = c->last_walked;
    return GICP_OK;
}

int gicp_top_weights(gicp_ctx* c, int k, int64_t* src_out, int64_t* tgt_out, double* det_out) {
    if (!c || k < 1 || k > 16) return GICP_E_INVALID;
    return guard_impl(c, "gicp_top_weights", [&] {
        if (!c->top_ready) throw Fail{GICP_E_STATE, "no pass with want_top_weights since the last cloud change"};
        if (c->top_cached_k != k) {   // not computed with the pass: now (and for this k from the next pass on)
            top_enqueue(c, k);
            HIPCHK(hipStreamSynchronize(c->stream));
            c->top_cached_k = c->top_k_pref = k;
        }
        const double* hv = reinterpret_cast<const double*>(c->h_top + 32);
        for (int r = 0; r < k; ++r) {
            if (src_out) src_out[r] = c->h_top[r];
            if (tgt_out) tgt_out[r] = c->h_top[16 + r];
            if (det_out) det_out[r] = hv[r];
        }
    });
}

int gicp_solve_pose(int dim, const double* stats, const double* T_k, double* T_out, double* loss_out) {
    if ((dim != 2 && dim != 3) || !stats || !T_k || !T_out) return GICP_E_INVALID;
    try {
        return solve_pose(dim, stats, T_k, T_out, loss_out) == 0 ? GICP_OK : GICP_E_INVALID;
    } catch (...) {
        return GICP_E_INVALID;
    }
}

int gicp_align(gicp_ctx* c, const double* T0, const gicp_params* p, double* T_out, gicp_result* res) {
    return gicp_align_trace(c, T0, p, T_out, res, nullptr);
}

int gicp_align_trace(gicp_ctx* c, const double* T0, const gicp_params* p, double* T_out, gicp_result* res,
                     gicp_trace* trace) {
    if (!c || !T_out) return GICP_E_INVALID;
    return guard_impl(c, "gicp_align", [&] {
        if (!c->tgt.n || !c->src.n) throw Fail{GICP_E_STATE, "set_target and set_source first"};
        if (c->tgt.dim != c->src.dim) throw Fail{GICP_E_INVALID, "source and target dimensions differ"};
        const int d = c->src.dim, n1 = d + 1;
        gicp_params prm = p ? resolve(d, p) : c->psrc;
        c->psrc.max_distance_correspondence = prm.max_distance_correspondence;
        c->psrc.cov_model = prm.cov_model;
        ensure_workspace(c);
        hipStream_t st = c->stream;
        // per-iteration trace rows (gicp_trace): pose + loss from k_solve, top-k rows after k_corr
        const int HS = n1 * n1 + 1;
        const int tk = trace ? trace->top_k : 0;
        if (trace) {
            if (trace->capacity < std::max(0, prm.max_iterations))
                throw Fail{GICP_E_INVALID, "gicp_trace.capacity < max_iterations"};
            if (tk < 0 || tk > 16) throw Fail{GICP_E_INVALID, "gicp_trace.top_k must be 0..16"};
            const size_t rows = (size_t)std::max(1, prm.max_iterations);
            dreserve(c->d_hist, c->cap_hist, rows * HS);
            if (tk > 0) {
                ensure_dbg(c);
                ensure_top_scratch(c);
                dreserve(c->d_trace_top, c->cap_ttop, rows * 32);
                dreserve(c->d_trace_det, c->cap_tdet, rows * 16);
                // rows of other shards stay NaN (never selected); one shard writes every row
                if (c->nshards > 1) HIPCHK(hipMemsetAsync(c->d_dbg_det, 0xFF, sizeof(double) * c->src.n, st));
            }
        }
        c->top_ready = false;
        // device state: T0, last_loss = inf (gicp.py:106-110)
        IterState& hs = *c->h_state;
        std::memset(&hs, 0, offsetof(IterState, stats));
        for (int k = 0; k < n1 * n1; ++k) hs.T[k] = T0 ? T0[k] : ((k % (n1 + 1)) == 0 ? 1.0 : 0.0);
        for (int k = 0; k < n1 * n1; ++k)
            if (!std::isfinite(hs.T[k])) throw Fail{GICP_E_INVALID, "T0 contains non-finite values"};
        hs.last_loss = INFINITY;
        hs.tol = prm.tolerance;
        hs.fixed = prm.fixed_iterations ? 1 : 0;
        hs.trans_eps = prm.transformation_epsilon;
        hs.rot_cos = prm.rotation_epsilon;
        hs.fit_eps = prm.euclidean_fitness_epsilon;
        hs.rel_eps = prm.mse_relative_epsilon;
        hs.prev_mse = INFINITY;
        hs.pairs_total = 0.0;
        hs.converged_at = -1;
        HIPCHK(hipMemcpyAsync(c->d_state, &hs, offsetof(IterState, stats), hipMemcpyHostToDevice, st));   // (xchg_* = 0)
        const int grid = corr_grid(c->src.ntiles, c->shard, c->nshards);
        const bool timing = res != nullptr && prm.timing_stride >= 0;   // < 0: no timing events
        const auto t0 = std::chrono::steady_clock::now();
        double corr_ms = 0.0;
        int enq = 0, samples = 0;
        // Timing events are recorded around every kEvStride-th k_corr only: an event pair around
        // every launch inserts a few microseconds of queue work per iteration.
        const int kEvStride = prm.timing_stride > 0 ? std::min(prm.timing_stride, (int)gicp_ctx::kMaxBatch) : 8;
        const int kEvOffset = std::max(0, prm.timing_offset) % kEvStride;
        c->iter_ms.assign((size_t)std::max(0, prm.max_iterations), -1.f);
#ifdef GICP_TAIL
        // diagnostic build: one tail record per iteration (gicp_internal.h kTailWords), dumped raw to
        // $GICP_TAIL_DUMP.<call> after the loop
        static std::atomic<int> tail_seq{0};   // dump file counter (process-wide)
        const char* tail_path = std::getenv("GICP_TAIL_DUMP");
        const size_t ntail = (size_t)std::max(1, prm.max_iterations) * kTailWords;
        unsigned long long* d_tail = nullptr;
        if (tail_path) {   // the context's own buffer, on its device
            dreserve(c->d_tail, c->cap_tail, ntail);
            d_tail = c->d_tail;
            std::vector<unsigned long long> init(ntail, 0ull);
            for (size_t k = 0; k < ntail; k += kTailWords) init[k] = ~0ull;
            HIPCHK(hipMemcpyAsync(d_tail, init.data(), ntail * 8, hipMemcpyHostToDevice, st));
            HIPCHK(hipStreamSynchronize(st));
        }
#endif
        // Iterations are enqueued in batches with no host sync inside a batch: each is k_corr (pose
        // from the device state, statistics reduced in-launch) [+ RCCL all-reduce] + k_solve.
        // After convergence the remaining launches of a batch exit at once.
        // A host exchange synchronises every iteration anyway: batches of one, so the loop stops at the
        // converged iteration without launching more.  Otherwise the first batch is as long as the last
        // converging align on this context ran (a sequence of similar registrations -- odometry frames --
        // then pays one host sync per call instead of two or three; a shorter registration pays a few
        // launches that exit at once), later batches 8.
        const int first_batch = std::max(8, std::min((int)gicp_ctx::kMaxBatch, c->batch_hint));
        while (enq < prm.max_iterations) {
            const int B = std::min(prm.max_iterations - enq,
                                   c->hook ? 1 : prm.fixed_iterations ? (int)gicp_ctx::kMaxBatch
                                                                      : enq == 0 ? first_batch : 8);
            for (int b = 0; b < B; ++b) {
                const int it = enq + b;
                CorrArgs a = corr_args(c, 0);
                if (it < c->moving_iters) a.unit_map = c->moving_map;
#ifdef GICP_TAIL
                if (tail_path) a.tail = d_tail + (size_t)it * kTailWords;
#endif
                if (tk > 0) {   // det(W) of every point, for this iteration's top-k rows (gicp.py:170)
                    a.dbg_det = c->d_dbg_det;
                    a.top_tgt = c->d_top_tgt;
                }
                // k_corr's final workgroup runs the solve too whenever it holds the sums the solve needs: with
                // no exchange (one rank, or bench.py --shard-sim's lone shard: the peer-exchange launch shape
                // without the exchange) and with the in-kernel peer exchange; RCCL and the host hook sit
                // between k_corr and k_solve
                const bool peer = a.peer.n > 1;
                const bool fuse = c->fuse_solve && (peer || (grid > 0 && !c->hook && !c->comm));
                double* const hist = trace ? c->d_hist + (size_t)it * HS : nullptr;
                if (fuse) {
                    a.fuse_solve = 1;
                    a.hist = hist;
                }
                const bool ev = timing && it % kEvStride == kEvOffset;
                if (ev) HIPCHK(hipEventRecord(c->ev[2 * b], st));
                if (grid > 0) {
                    HIPCHK(launch_corr(a, d, grid, st));
                } else if (peer) {   // no tile in this shard: one empty workgroup takes part in the exchange
                    a.q_end = 0;
                    HIPCHK(launch_corr(a, d, 1, st));
                } else {
                    HIPCHK(hipMemsetAsync(c->d_state->stats, 0, sizeof(double) * nstat_ext(d), st));
                }
                if (ev) HIPCHK(hipEventRecord(c->ev[2 * b + 1], st));
                if (tk > 0)   // launched after convergence too (the pass exited at once): rows >= iter are ignored
                    HIPCHK(launch_top_weights(c->d_dbg_det, c->d_top_tgt, c->src.perm, c->src.n, tk, c->d_top_v,
                                              c->d_top_i, kTopBlocks, c->d_trace_det + (size_t)it * 16,
                                              c->d_trace_top + (size_t)it * 32, c->d_trace_top + (size_t)it * 32 + 16,
                                              st));
                if (!fuse) {
                    allreduce_stats(c);
                    HIPCHK(launch_solve(c->d_state, d, st, hist));
                }
            }
            enq += B;
            HIPCHK(hipMemcpyAsync(&hs, c->d_state, sizeof(IterState), hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            if (timing)
                for (int b = 0; b < B; ++b) {
                    if ((enq - B + b) % kEvStride != kEvOffset) continue;
                    if (enq - B + b >= hs.iter) break;   // launched after convergence: exited at once
                    float ms = 0.f;
                    HIPCHK(hipEventElapsedTime(&ms, c->ev[2 * b], c->ev[2 * b + 1]));
                    c->iter_ms[enq - B + b] = ms;
                    corr_ms += ms;
                    ++samples;
                }
            if (hs.converged) break;
        }
        const auto t1 = std::chrono::steady_clock::now();
        if (!prm.fixed_iterations && hs.converged) c->batch_hint = hs.iter;
        c->iter_ms.resize((size_t)std::max(0, std::min(hs.iter, prm.max_iterations)));
#ifdef GICP_TAIL
        if (tail_path) {
            std::vector<unsigned long long> h(ntail);
            HIPCHK(hipMemcpyAsync(h.data(), d_tail, ntail * 8, hipMemcpyDeviceToHost, st));
            HIPCHK(hipStreamSynchronize(st));
            const std::string path = std::string(tail_path) + "." + std::to_string(tail_seq++);
            if (FILE* fp = std::fopen(path.c_str(), "wb")) {
                std::fwrite(h.data(), 8, h.size(), fp);
                std::fclose(fp);
            }
        }
#endif
        if (trace && hs.iter > 0) {   // the rows of the iterations executed, in one copy per array
            const int ni = std::min(hs.iter, prm.max_iterations);
            std::vector<double> hist((size_t)ni * HS);
            HIPCHK(hipMemcpyAsync(hist.data(), c->d_hist, sizeof(double) * hist.size(), hipMemcpyDeviceToHost, st));
            std::vector<int64_t> ttop;
            std::vector<double> tdet;
            if (tk > 0) {
                ttop.resize((size_t)ni * 32);
                tdet.resize((size_t)ni * 16);
                HIPCHK(hipMemcpyAsync(ttop.data(), c->d_trace_top, sizeof(int64_t) * ttop.size(), hipMemcpyDeviceToHost, st));
                HIPCHK(hipMemcpyAsync(tdet.data(), c->d_trace_det, sizeof(double) * tdet.size(), hipMemcpyDeviceToHost, st));
            }
            HIPCHK(hipStreamSynchronize(st));
            for (int k = 0; k < ni; ++k) {
                if (trace->poses) std::memcpy(trace->poses + (size_t)k * n1 * n1, &hist[(size_t)k * HS], sizeof(double) * n1 * n1);
                if (trace->losses) trace->losses[k] = hist[(size_t)k * HS + n1 * n1];
                for (int r = 0; r < tk; ++r) {
                    if (trace->top_src) trace->top_src[(size_t)k * tk + r] = ttop[(size_t)k * 32 + r];
                    if (trace->top_tgt) trace->top_tgt[(size_t)k * tk + r] = ttop[(size_t)k * 32 + 16 + r];
                    if (trace->top_det) trace->top_det[(size_t)k * tk + r] = tdet[(size_t)k * 16 + r];
                }
            }
        }
        if (hs.solve_fail == 2) throw Fail{GICP_E_COMM, "peer exchange timed out (a rank did not arrive)"};
        if (hs.solve_fail) throw Fail{GICP_E_INVALID, "pose solve failed (degenerate statistics)"};
        std::memcpy(T_out, hs.T, sizeof(double) * n1 * n1);
        if (res) {
            gicp_result r;
            std::memset(&r, 0, sizeof(r));
            const int ns = nstat(d);
            r.iterations = hs.iter;
            r.converged = hs.converged;
            r.converged_at = hs.converged ? hs.converged_at : -1;
            r.final_loss = hs.loss;
            r.correspondences = (int64_t)hs.stats_solved[ns - 1];
            r.ambiguous = (int32_t)hs.stats_solved[ns];
            r.pairs_evaluated = (int64_t)hs.stats_solved[ns + 1];
            c->last_amb = hs.stats_solved[ns];
            c->last_pairs = hs.stats_solved[ns + 1];
            c->last_rebuilds = hs.stats_solved[ns + 2];
            c->last_sq = hs.stats_solved[ns + 3];
            c->last_gproved = hs.stats_solved[ns + 4];
            c->last_walked = hs.stats_solved[ns + 5];
            r.wall_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
            // kernel time of the iterations actually executed (after convergence launches exit at once)
            r.corr_kernel_ms = samples ? corr_ms / samples * hs.iter : 0.0;
            r.reduce_ms = 0.0;
            r.stop_reason = hs.converged ? hs.stop_reason : GICP_STOP_NONE;
            r.pairs_total = hs.pairs_total;
            r.corr_kernel_ms_sampled = corr_ms;
            r.corr_samples = samples;
            r.mse = hs.mse;
            if (hs.xchg_n > 0.0) {   // wall-clock ticks -> us
                int khz = 0;
                HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
                const double us = 1e3 / (khz > 0 ? khz : 100000);
                r.exchange_us_mean = hs.xchg_sum / hs.xchg_n * us;
                r.exchange_us_min = hs.xchg_min * us;
            }
            *res = r;
        }
    });
}

namespace {
// the slot's build thread: waits for a queued build, runs it on the slot's stream, reports state 2
void staged_worker(gicp_ctx::Staged* gp) {
    for (;;) {
        {
            std::unique_lock<std::mutex> lk(gp->m);
            gp->cv.wait(lk, [&] { return gp->quit || gp->state == 1; });
            if (gp->state != 1) return;   // quit with nothing queued
        }
        int rc = GICP_OK;
        std::string err;
        try {
            HIPCHK(hipSetDevice(gp->device));
            build_cloud(gp->cl, gp->xyz, gp->M, gp->dim, gp->p, gp->graph, gp->bs, gp->stream, true);
        } catch (const Fail& f) {
            rc = f.code;
            err = f.msg;
        } catch (const std::bad_alloc&) {
            rc = GICP_E_NOMEM;
            err = "out of host memory";
        } catch (...) {
            rc = GICP_E_INVALID;
            err = "unknown error";
        }
        {
            std::lock_guard<std::mutex> g(gp->m);
            gp->rc = rc;
            gp->err = err;
            gp->state = 2;
        }
        gp->cv.notify_all();
    }
}
}  // namespace

int gicp_stage_target(gicp_ctx* c, const double* xyz, int64_t M, int dim, const gicp_params* p) {
    return gicp_stage_target_ex(c, xyz, M, dim, p, 0);
}

int gicp_stage_target_ex(gicp_ctx* c, const double* xyz, int64_t M, int dim, const gicp_params* p, int flags) {
    if (!c) return GICP_E_INVALID;
    return guard_impl(c, "gicp_stage_target", [&] {
        if (c->stg_count >= GICP_MAX_STAGED)
            throw Fail{GICP_E_STATE, "GICP_MAX_STAGED staged targets are pending (gicp_commit_target or gicp_cancel_stage first)"};
        if (!xyz || M <= 0 || (dim != 2 && dim != 3)) throw Fail{GICP_E_INVALID, "cloud must be a non-empty N x 2 or N x 3 array"};
        if (flags & ~GICP_STAGE_BORROW) throw Fail{GICP_E_INVALID, "unknown gicp_stage_target_ex flags"};
        gicp_ctx::Staged& g = c->stg[(c->stg_head + c->stg_count) % GICP_MAX_STAGED];
        g.wait_idle();   // (a slot is only reused after its commit or cancel; a build never runs here)
        const gicp_params prm = resolve(dim, p);
        if (!g.stream) HIPCHK(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking));
        const double* src = xyz;
        if (!(flags & GICP_STAGE_BORROW)) {
            const size_t need = (size_t)M * dim;
            if (need > g.bs.cap_pinned) {   // grow-only pinned staging buffer (allocated here, not in the worker)
                if (g.bs.h_pinned) HIPCHK(hipHostFree(g.bs.h_pinned));
                g.bs.h_pinned = nullptr;
                g.bs.cap_pinned = 0;
                const size_t cap = need + need / 8;
                HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&g.bs.h_pinned), sizeof(double) * cap));
                g.bs.cap_pinned = cap;
            }
            // the caller's scan is copied into the slot's pinned buffer before this call returns (the caller
            // may refill its buffer at once): 16 fixed chunks on the calling thread's tiling pool (a 100k-point
            // frame, 2.4 MB, in ~0.06 ms instead of one thread's ~0.3 ms)
            const size_t total = sizeof(double) * need;
            char* dst = reinterpret_cast<char*>(g.bs.h_pinned);
            const char* srcb = reinterpret_cast<const char*>(xyz);
            constexpr int kChunks = 16;
            c->bs.workers().run(kChunks, [&](int k) {
                const size_t b0 = total * k / kChunks, b1 = total * (k + 1) / kChunks;
                std::memcpy(dst + b0, srcb + b0, b1 - b0);
            });
            src = g.bs.h_pinned;
        }
        if (!g.th.joinable()) g.th = std::thread(staged_worker, &g);
        {
            std::lock_guard<std::mutex> lk(g.m);
            g.xyz = src;
            g.M = M;
            g.dim = dim;
            g.graph = c->use_graph && c->use_certs;
            g.device = c->device;
            g.p = prm;
            g.rc = GICP_OK;
            g.err.clear();
            g.state = 1;
        }
        g.cv.notify_all();
        ++c->stg_count;
    });
}

int gicp_commit_target(gicp_ctx* c, int shard, int nshards) {
    if (!c) return GICP_E_INVALID;
    return guard_impl(c, "gicp_commit_target", [&] {
        if (!c->stg_count) throw Fail{GICP_E_STATE, "no staged target (gicp_stage_target first)"};
        gicp_ctx::Staged& g = c->stg[c->stg_head];
        g.wait_idle();
        c->stg_head = (c->stg_head + 1) % GICP_MAX_STAGED;
        --c->stg_count;
        {
            std::lock_guard<std::mutex> lk(g.m);
            g.state = 0;
            g.xyz = nullptr;
        }
        if (g.rc != GICP_OK) throw Fail{g.rc, "staged build: " + g.err};
        if (nshards < 1 || shard < 0 || shard >= nshards) throw Fail{GICP_E_INVALID, "bad shard / nshards"};
        // the current target (index + covariances) becomes the source, as robot-visualization.py:250
        // swaps scans, and the staged cloud the target; the old source's buffers wait in the slot
        if (c->tgt.n) {
            std::swap(c->src, c->tgt);
            c->psrc = c->ptgt;
        }
        std::swap(c->tgt, g.cl);
        g.cl.n = 0;
        g.cl.cov_ready = false;
        g.cl.graph_ready = false;
        c->ptgt = g.p;
        c->top_ready = false;
        if (c->src.n) set_shard(c, shard, nshards);   // (stream-ordered resets: no host sync)
    });
}

int gicp_cancel_stage(gicp_ctx* c) {
    if (!c) return GICP_E_INVALID;
    for (auto& g : c->stg) {
        g.wait_idle();
        std::lock_guard<std::mutex> lk(g.m);
        g.state = 0;
        g.xyz = nullptr;
    }
    c->stg_head = c->stg_count = 0;
    return GICP_OK;
}

int gicp_reset_cache(gicp_ctx* c) {
    if (!c) return GICP_E_INVALID;
    return guard_impl(c, "gicp_reset_cache", [&] {
        reset_tile_state(c);
        HIPCHK(hipStreamSynchronize(c->stream));
    });
}

int gicp_iteration_times(gicp_ctx* c, float* out, int n) {
    if (!c || (!out && n > 0) || n < 0) return GICP_E_INVALID;
    const int m = std::min(n, (int)c->iter_ms.size());
    for (int i = 0; i < m; ++i) out[i] = c->iter_ms[i];
    return m;
}

int gicp_set_allreduce(gicp_ctx* c, gicp_allreduce_fn fn, void* user) {
    return gicp_set_allreduce_ranks(c, fn, user, 1, 0);
}

int gicp_set_allreduce_ranks(gicp_ctx* c, gicp_allreduce_fn fn, void* user, int nranks, int rank) {
    if (!c || nranks < 1 || rank < 0 || rank >= nranks) return GICP_E_INVALID;
    return guard_impl(c, "gicp_set_allreduce", [&] {
        if (fn) close_peers(c);
        if (fn && !c->h_xchg) HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&c->h_xchg), sizeof(double) * 80));
        if (fn && c->comm) {   // one exchange per context: the hook replaces the communicator
            HIPCHK(hipStreamSynchronize(c->stream));
            ncclCommDestroy(c->comm);
            c->comm = nullptr;
        }
        c->hook = fn;
        c->hook_user = fn ? user : nullptr;
        if (!c->comm) {   // what gicp_comm_ranks reports for the hook
            c->nranks = fn ? nranks : 1;
            c->rank = fn ? rank : 0;
        }
    });
}

int gicp_peer_export(gicp_ctx* c, char handle[GICP_PEER_HANDLE_BYTES]) {
    if (!c || !handle) return GICP_E_INVALID;
    return guard_impl(c, "gicp_peer_export", [&] {
        static_assert(sizeof(hipIpcMemHandle_t) + sizeof(uint64_t) == GICP_PEER_HANDLE_BYTES, "IPC handle + counter");
        if (!c->d_peer_area) {   // uncached: peers' stores and this rank's polling meet in memory
            HIPCHK(hipExtMallocWithFlags(reinterpret_cast<void**>(&c->d_peer_area), sizeof(double) * kPeerAreaDoubles,
                                         hipDeviceMallocUncached));
            HIPCHK(hipMemset(c->d_peer_area, 0, sizeof(double) * kPeerAreaDoubles));
            HIPCHK(hipDeviceSynchronize());
        }
        if (!c->d_peer_ctr) {
            dalloc(c->d_peer_ctr, 1);
            HIPCHK(hipMemset(c->d_peer_ctr, 0, sizeof(uint64_t)));
        }
        hipIpcMemHandle_t h;
        HIPCHK(hipIpcGetMemHandle(&h, c->d_peer_area));
        uint64_t seq = 0;   // this rank's exchange counter (its launches have finished: stream sync)
        HIPCHK(hipStreamSynchronize(c->stream));
        HIPCHK(hipMemcpy(&seq, c->d_peer_ctr, sizeof(seq), hipMemcpyDeviceToHost));
        std::memcpy(handle, &h, sizeof(h));
        std::memcpy(handle + sizeof(h), &seq, sizeof(seq));
    });
}

int gicp_peer_init(gicp_ctx* c, int nranks, int rank, const char* handles, double timeout_s) {
    if (!c || !handles || nranks < 2 || nranks > GICP_MAX_PEERS || rank < 0 || rank >= nranks || !(timeout_s > 0.0))
        return GICP_E_INVALID;
    return guard_impl(c, "gicp_peer_init", [&] {
        if (!c->d_peer_area || !c->d_peer_ctr) throw Fail{GICP_E_STATE, "gicp_peer_export first"};
        close_peers(c);
        PeerArgs p{};
        p.n = nranks;
        p.rank = rank;
        p.own = c->d_peer_area;
        p.ctr = c->d_peer_ctr;
        // every rank starts at the largest counter any rank exported: above every flag left in any area
        uint64_t seq0 = 0;
        for (int r = 0; r < nranks; ++r) {
            uint64_t v = 0;
            std::memcpy(&v, handles + (size_t)r * GICP_PEER_HANDLE_BYTES + sizeof(hipIpcMemHandle_t), sizeof(v));
            seq0 = std::max(seq0, v);
        }
        HIPCHK(hipMemcpy(c->d_peer_ctr, &seq0, sizeof(seq0), hipMemcpyHostToDevice));
        double* area[kMaxPeers] = {};
        try {
            for (int r = 0; r < nranks; ++r) {
                if (r == rank) {
                    area[r] = c->d_peer_area;
                    continue;
                }
                hipIpcMemHandle_t h;
                std::memcpy(&h, handles + (size_t)r * GICP_PEER_HANDLE_BYTES, sizeof(h));
                void* ptr = nullptr;
                const hipError_t e = hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess);
                if (e != hipSuccess) {
                    (void)hipGetLastError();
                    throw Fail{GICP_E_COMM, std::string("hipIpcOpenMemHandle(rank ") + std::to_string(r) + "): " +
                                                hipGetErrorString(e)};
                }
                c->peer_open[r] = ptr;
                area[r] = static_cast<double*>(ptr);
            }
            if (!c->d_peer_ptrs) dalloc(c->d_peer_ptrs, kMaxPeers);
            HIPCHK(hipMemcpy(c->d_peer_ptrs, area, sizeof(area), hipMemcpyHostToDevice));
            p.area = c->d_peer_ptrs;
            int khz = 0;
            HIPCHK(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, c->device));
            p.timeout = (uint64_t)(timeout_s * (khz > 0 ? khz : 100000) * 1e3);
            // the probe: kPeerProbeRounds full-slot exchanges checked bit for bit, which every rank runs now
            if (!c->d_probe) dalloc(c->d_probe, 2);
            HIPCHK(launch_peer_probe(p, c->d_probe, c->stream));
            double got[2] = {0, 0};
            HIPCHK(hipMemcpyAsync(got, c->d_probe, sizeof(got), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            if (got[0] != (double)kPeerProbeRounds || got[1] != 0.0)
                throw Fail{GICP_E_COMM, got[0] < 0.0 ? std::string("peer exchange probe failed (a rank did not arrive)")
                                                     : "peer exchange probe failed (" + std::to_string((int)got[1]) +
                                                           " of " + std::to_string(kPeerSlot * kPeerProbeRounds) +
                                                           " summed values wrong after " +
                                                           std::to_string((int)got[0]) + " rounds)"};
        } catch (...) {
            close_peers(c);
            throw;
        }
        // the peer exchange replaces any other exchange of this context
        if (c->comm) {
            ncclCommDestroy(c->comm);
            c->comm = nullptr;
        }
        c->hook = nullptr;
        c->peer = p;
        c->peer_timeout_s = timeout_s;
        c->nranks = nranks;
        c->rank = rank;
    });
}

int gicp_peer_close(gicp_ctx* c) {
    if (!c) return GICP_E_INVALID;
    return guard_impl(c, "gicp_peer_close", [&] { close_peers(c); });
}

const char* gicp_build_info(void) {
#ifndef GICP_SRC_HASH
#define GICP_SRC_HASH "unknown"
#endif
#ifndef GICP_GIT_REV
#define GICP_GIT_REV "unknown"
#endif
    return "src=" GICP_SRC_HASH ";git=" GICP_GIT_REV ";built=" __DATE__ " " __TIME__ ";arch=gfx950";
}

int gicp_rotated_covariances(gicp_ctx* c, int which, const double* R, double* out) {
    if (!c || !R || !out || (which != 0 && which != 1)) return GICP_E_INVALID;
    return guard_impl(c, "gicp_rotated_covariances", [&] {
        Cloud& cl = which == 0 ? c->tgt : c->src;
        if (!cl.n || !cl.cov_ready) throw Fail{GICP_E_STATE, "cloud not set"};
        const int d = cl.dim;
        for (int k = 0; k < d * d; ++k)
            if (!std::isfinite(R[k])) throw Fail{GICP_E_INVALID, "R contains non-finite values"};
        const size_t m = (size_t)cl.n * d * d;
        dreserve(c->d_rot, c->cap_rot, m);
        HIPCHK(launch_rotate_cov(cl.cov, cl.perm, cl.n, d, R, c->d_rot, c->stream));
        HIPCHK(hipMemcpyAsync(out, c->d_rot, sizeof(double) * m, hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
    });
}

}  // extern "C"
