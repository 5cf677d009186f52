// gicp_internal.h — device data layout shared by the HIP kernels and the host context.
//
// Every cloud (target and source) is stored Morton-sorted and cut into TILES of at most
// 64 consecutive points that never cross a grid cell of the chosen Morton level, so a
// tile is spatially compact (radius bounded by the cell).  64 consecutive tiles form a
// BLOCK.  Both carry an fp64 centre and fp32 half-extents; points are kept twice:
// fp64 (exact epilogue, fp64 fallback) and fp32 relative to their tile centre (the
// distance screen).  See DESIGN.md §3.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/gicp_hip.h"

namespace gicp {

constexpr int kWave = 64;          // CDNA wavefront
constexpr int kTile = 64;          // points per tile (= one wave of queries)
constexpr int kBlockTiles = 64;    // tiles per block (= one wave of tile tests)
constexpr int kWavesPerWG = 4;     // 256-thread workgroups, each wave independent
#ifndef GICP_CORR_WAVES
#define GICP_CORR_WAVES 4
#endif
constexpr int kCorrWaves = GICP_CORR_WAVES;       // waves per k_corr workgroup

constexpr int kListMax = 64;       // candidate target tiles kept per source tile
constexpr int kPoseRing = 64;      // passes a list stays usable for
#ifndef GICP_SUB_TILES
#define GICP_SUB_TILES 4
#endif
// sub-tiles per tile (finer culling of the row scan).  8 (8-row sub-tiles) screens 27-38 % fewer
// rows on the 1M bench but ran 2 % slower: twice the sub-box tests, and the tile metadata no longer
// fits k_corr's scalar registers (44 SGPRs spilled)
constexpr int kSub = GICP_SUB_TILES;
constexpr int kSubRows = 64 / kSub;    // rows per sub-tile (a multiple of 4: the scan's row group)
// target neighbour graph: each target point's kGraphK nearest other target points
constexpr int kGraphK = 20;
#ifndef GICP_GRAPH_HOPS
#define GICP_GRAPH_HOPS 4
#endif
constexpr int kGraphHops = GICP_GRAPH_HOPS;   // descent steps a k_corr lane may take before it walks
// error bound of the descent's fp32 distances, per metre of the coordinates involved (2^-19: the
// relative-to-node arithmetic errs by a few 2^-24 per operation)
constexpr float kGraphErr = 1.9073486328125e-06f;
// graph row layout (DevCloud::nbq / nbx): entries per 128-B line and per first half-line, and the index delta
// that marks an entry whose sorted-index delta does not fit 16 bits
constexpr int kGraphLineA = 15;
constexpr int kGraphHalf = 7;
constexpr int kGraphFar = -32768;
static_assert(2 + 2 * kGraphLineA == 32 && 2 + 2 * kGraphHalf == 16, "header + entries fill the line and its half");
static_assert(2 * (kGraphK - kGraphLineA) == 10, "the remaining entries fill 40 B of the 48-B record");

struct __attribute__((aligned(16))) TileInfo {
    double c[3];      // fp64 centre (midpoint of the fp64 AABB)
    float h[3];       // half-extents: max |rel32| over the tile's points, per axis
    int32_t start;    // first sorted point
    int32_t count;    // 1..64
    float radius;     // max |rel32| norm
    float sc[3][kSub];  // sub-tile box centres (rows kSubRows g ..) relative to c, fp32, axis-major
    float sh[3][kSub];  // sub-tile box half-extents (cover every rel32 of the sub-tile), axis-major
};

// The walk's view of a tile: what k_corr's candidate tests read for every tile of a candidate block (or
// list), 48 B so a wave's 64 records are three coalesced 16-B loads per lane (TileInfo is 144 B apart)
struct __attribute__((aligned(16))) TileBox {
    double c[3];      // = TileInfo::c
    float h[3];       // = TileInfo::h
    int32_t start;    // = TileInfo::start (any n < 2^31)
    int32_t count;    // = TileInfo::count
    int32_t pad;
};
static_assert(sizeof(TileBox) == 48, "TileBox is three 16-B words");

struct __attribute__((aligned(16))) BlockInfo {
    double c[3];
    float h[3];
    int32_t first;    // first tile
    int32_t ntiles;   // 1..64
    float pad;
};

// Device view of one indexed cloud (all pointers device memory, sorted order).
struct DevCloud {
    const double* xyz64;      // [n][4]  x y z 0
    const float4* rel32;      // [n]     x y z 0 relative to the tile centre
    const double4* cov;       // [n]     (a, m0, m1, m2): C = a I - m m^T
    const int32_t* perm;      // [n]     sorted -> original index
    const TileInfo* tiles;    // [ntiles]
    const BlockInfo* blocks;  // [nblocks] blocks of 64 tiles, then [ceil(nblocks / 64)] super-blocks of 64 blocks
    const uint32_t* tile_code;// [ntiles] Morton code of each tile's first point
    const TileBox* boxes;     // [ntiles] the walk's compact tile records
    // Morton seed lookup: seed_tab[p] = the last tile whose first code <= p << seed_shift (0 if none),
    // p < 2^seed_bits, seed_tab[2^seed_bits] = ntiles - 1: the tile of code c lies in
    // [seed_tab[c >> seed_shift], seed_tab[(c >> seed_shift) + 1]] (a few binary steps instead of log2 ntiles)
    const int32_t* seed_tab;
    int32_t seed_shift;
    // neighbour graph (target only; null when not built), DESIGN.md §3c.  Row i: dword 0 r(i) (fp32: every
    // target t != i with |x_t - x_i| < r is in the row), dword 1 the scale s, then kGraphK entries nearest-first,
    // two dwords each: (x_t - x_i) / s as 3 int16 rounded to nearest (|error| <= s / 2 per axis) and the
    // sorted-index delta t - i as a fourth int16 (kGraphFar when it does not fit: nbi holds it), so a descent
    // step needs no index read.  Entries 0 .. kGraphLineA - 1 fill the 128-B line nbq[i] (its first half holds
    // the header and entries 0 .. kGraphHalf - 1), the rest the 48-B record nbx[i].  An unused entry repeats
    // the last real one (offset and delta 0 in an empty row).  nbi[i][k] = sorted index of entry k (-1 unused).
    const uint4* nbq;         // [n][8]
    const uint4* nbx;         // [n][3]
    const int32_t* nbi;       // [n][kGraphK]
    int64_t n;
    int32_t ntiles;
    int32_t nblocks;
    double lo[3];             // Morton frame: code_a = (x_a - lo_a) * scale
    double scale;
    int32_t bits;             // bits per axis (10 for 3-D, 16 for 2-D)
    int32_t dim;
};

// Error bound of the fp32 distance screen: |d2_f32 - d2_f64| <= a sqrt(d2) + b + c d2.
struct Margin {
    float a, b, c;
};

struct GraphArgs {
    DevCloud cl;
    int32_t split;            // waves per query tile (1, or kSub: one wave per 16-row sub-tile), see CovArgs
    float search2;            // fp32 screen bound (d_n^2 + margins): the graph's neighbourhood cap
    Margin mg;
    float4* nb;               // [n][kGraphK] scratch: x_t - x_i fp32, t as the w bits
    float2* nbh;              // [n] scratch: (r, count)
    uint4* nbq;               // [n][8] out (packed rows: header and entries 0 .. kGraphLineA - 1)
    uint4* nbx;               // [n][3] out (entries kGraphLineA .. kGraphK - 1)
    int32_t* nbi;             // [n][kGraphK] out
};

struct CovArgs {
    DevCloud cl;
    int32_t q_begin, q_end;   // query tiles, counted within this rank's shard (all tiles when sh_n = 1)
    // source shards (the k_corr split, gicp_internal.h kShardChunk): this rank's query tile t is the cloud's
    // tile ((t / 64) sh_n + sh_r) 64 + t % 64 -- a rank computes the covariances of its own tiles only
    int32_t sh_n, sh_r;
    // waves per query tile: 1 (the tile's 64 points, one per lane), or kSub (one wave per 16-row sub-tile,
    // its box the sub-box: a small cloud -- a 100k stream frame is ~1.7k tiles, a third of one wave per
    // SIMD -- is bound by its longest neighbourhood walk, which the smaller box shortens)
    int32_t split;
    float search2;            // fp32 screen bound (d_n^2 + margins)
    double dn2;               // d_n^2, fp64, strict
    Margin mg;
    double eps_a;             // epsilon (a of C = a I - m m^T)
    double m_scale;           // sqrt(epsilon (1 - ratio))
    int32_t min_nb;           // minimum neighbours for a surface covariance
    double4* cov_out;         // [n] sorted
    int32_t* count_out;       // [n] sorted
    int32_t* amb_counter;     // diagnostics (may be null)
    float4* g_nb;             // k_knn_cov<D, K, true>: the graph rows (GraphArgs::nb), [n][kGraphK]
    float2* g_nbh;            // ... and (r, count) per point (GraphArgs::nbh)
};

// Device-resident state of the outer loop (gicp.py:106-110,155-167): the pose every pass reads,
// the convergence bookkeeping k_solve updates, and the last pass's statistics.
struct IterState {
    double T[16];             // current pose (d+1)^2 row-major (gicp.py:107,166)
    double loss;              // min_loss of the last inner solve (gicp.py:154)
    double last_loss;         // gicp.py:110,165
    double tol;               // gicp.py:78 tolerance
    int32_t converged;        // 1 once |last_loss - min_loss| < tolerance (gicp.py:160)
    int32_t converged_at;     // iteration index of that test, -1 if none
    int32_t iter;             // outer iterations executed
    int32_t fixed;            // 1: never stop on tolerance (benchmark mode)
    int32_t solve_fail;
    int32_t stop_reason;      // GICP_STOP_*
    // PCL-style criteria (include/gicp_hip.h gicp_params; <= 0 disables), checked after the update
    double trans_eps;         // |dt|^2 <= trans_eps and cos(angle) >= rot_cos of the increment
    double rot_cos;
    double fit_eps;           // |mse - prev_mse| < fit_eps
    double rel_eps;           // |mse - prev_mse| / prev_mse < rel_eps
    double prev_mse;          // +inf before the first pass
    double mse;               // mean squared correspondence distance of the last solved pass
    double pairs_total;       // distance pairs screened, summed over the passes k_solve consumed
    // peer exchange timing (diagnostic, wall-clock ticks of the final workgroup's exchange, this call): in the
    // header, so the host's one upload of the header at the start of a call also clears them
    double xchg_sum, xchg_min, xchg_n;
    double stats[80];         // statistics of the last pass (summed over ranks when a communicator is set)
    double stats_solved[80];  // copy of the statistics the last k_solve consumed (reporting)
};

constexpr int kGroupWG = 64;       // workgroups per first-level reduction group
// grids of at most this many units reduce in one level: the final workgroup sums every unit's partial itself
// (its loads cover 81 units per round trip, k_corr sum_rows), one ticket and one round trip of stores fewer;
// beyond it the one ticket's queue (every unit on one counter) and a third round trip of loads cost more
#ifndef GICP_FLAT_UNITS
#define GICP_FLAT_UNITS 128
#endif
constexpr int kFlatUnits = GICP_FLAT_UNITS;
// Source shards are interleaved in chunks of kShardChunk units (a unit = kCorrWaves source tiles,
// one k_corr workgroup): rank r of G reduces global chunks r, r + G, r + 2G, ...  Contiguous Morton
// ranges left the ranks unbalanced (the registration's far walls are the heavy tiles: one rank of 8
// took 1.7x another's k_corr time), and every rank waits for the slowest at the all-reduce.  A chunk
// of 64 tiles is still one compact region, so an XCD's L2 keeps its locality.
constexpr int kShardChunk = 16;
constexpr int kMaxGroups = 4096;   // ticket counters available
// one 128-B line per ticket counter: agent-scope atomics on one line serialise at the memory side, so tickets
// sharing a line made the groups' last arrivers queue behind each other (625 units: 2.8 us for the group ticket)
constexpr int kTicketStride = 32;

// In-kernel peer exchange of the statistics (include/gicp_hip.h gicp_peer_init).  Each rank
// owns an exchange area in fine-grained (uncached) device memory, mapped into every peer by IPC:
//   uint64 flag[2][kMaxPeers]              sequence number of the launch whose slot last arrived
//   double slot[2][kMaxPeers][kPeerSlot]   rank p's statistics of that launch
// indexed [parity of the exchange's sequence number][sending rank].  The sequence number counts the
// exchanges that actually happen (a launch that exits at once after convergence takes none): it is kept on
// the device (PeerArgs::ctr, the last number this rank wrote flags for) and advanced by the final workgroup
// as it exchanges, so consecutive exchanges always alternate parity.  Two parities then suffice: a rank
// writes exchange s + 1's slot only after its exchange s read every slot of s (stream order), and exchange
// s + 2's only after every rank wrote s + 1's flag, i.e. after every rank finished reading s.  gicp_peer_init
// starts every rank's counter at the maximum over the ranks (carried in the exported handles), so no flag
// left in any area by earlier exchanges (a timed-out one included) can pass for a new one.
constexpr int kMaxPeers = GICP_MAX_PEERS;
constexpr int kPeerSlot = 80;
constexpr int kPeerFlagWords = 2 * kMaxPeers;   // doubles before the slots
constexpr int kPeerProbeRounds = 8;             // full-slot exchanges gicp_peer_init's probe runs (both parities)
constexpr size_t kPeerAreaDoubles = kPeerFlagWords + (size_t)2 * kMaxPeers * kPeerSlot;
struct PeerArgs {
    double* const* area;       // device array [n]: rank p's area as mapped here (area[rank] = this rank's own)
    double* own;               // = area[rank]
    int32_t n;                 // ranks (0: no peer exchange)
    int32_t rank;
    uint64_t* ctr;             // device word: the sequence number of this rank's last exchange (flags written)
    uint64_t timeout;          // wall-clock ticks (wall_clock64) a rank waits for its peers
};

struct CorrArgs {
    DevCloud src, tgt;
    int32_t q_begin, q_end;   // k_corr: q_begin unused (0), q_end = the cloud's tile count
    // source shards (interleaved by kShardChunk units): this rank's unit u is the cloud's unit
    // u + (u / kShardChunk) sh_skip + sh_first, sh_skip = (G - 1) kShardChunk, sh_first = r kShardChunk
    int32_t sh_skip, sh_first;
    // workgroup -> unit map: 0 = XCD stripes (XCD x takes the contiguous eighth x), C > 0 = chunks of C
    // units dealt round-robin to the XCDs (1 = identity)
    int32_t unit_map;
    IterState* state;         // pose in, statistics out
    uint32_t* tickets;        // [(kMaxGroups + 1) kTicketStride] arrival counters (one per line), zero between
                              // launches (self-resetting)
    double* gpart;            // [kMaxGroups][nstat_ext] group partials
    int32_t single_pass;      // 1: run even if state->converged (gicp_iterate)
    float search2;            // fp32 screen bound (d_c^2 + margins)
    float gap_slack;          // rounding slack S of the box tests (search radius + 2 rho_t, x 2^-19)
    double dc;                // d_c, fp64, inclusive (distance > d_c rejects)
    double dc2_max;           // the largest double x with sqrt(x) <= d_c: "sqrt(d2) > d_c" <=> d2 > dc2_max
    Margin mg;
    int32_t* hint;            // [src.ntiles] best target tile of the previous pass
    double* partials;         // [gridDim.x][nstat_ext] workgroup partials
    int64_t* dbg_index;       // [N] original order (nullable)
    double* dbg_weight;       // [N][dim][dim] (nullable)
    double* dbg_dist;         // [N] (nullable)
    double* dbg_det;          // [N] det(W), 0 if rejected, sorted order (nullable; gicp_top_weights)
    int64_t* top_tgt;         // [N] with dbg_det, sorted order: original target index of the correspondence, -1 rejected
    int32_t cov_model;        // GICP_COV_* (include/gicp_hip.h)
    double pl_inv;            // 1 / (epsilon (1 - ratio)): n n^T = m m^T * pl_inv (point-to-plane)
    int32_t count_pairs;      // 1: accumulate evaluated pairs (diagnostic)
    // per-source-tile candidate lists (certified): built by a full walk with the
    // search radius inflated by `skin`, reused while the tile's displacement since the build pose
    // plus the wave's final search radius stays within the certified radius
    int32_t* list;            // [src.ntiles][kListMax] target tiles
    int32_t* list_len;        // [src.ntiles]
    float* list_rcert;        // [src.ntiles] certified radius (0: invalid)
    int32_t* list_pass;       // [src.ntiles] pass the list was built in
    double* poses;            // [kPoseRing][12] pose of each pass (R row-major, t)
    int32_t pass;             // this pass's id (monotonic per source cloud)
    int32_t use_lists;        // 0: always full walk (no lists)
    // a wave with 1 .. sparse_max walking lanes searches lane-parallel, one walking lane at a time (the candidate
    // tiles' rows kSparseGroup tiles per memory round trip) instead of one visit per tile; 0: never
    int32_t sparse_max;
    // a wave with 1 .. sparse_amb lanes the fp32 screen left ambiguous re-resolves them lane-parallel, one at a
    // time (its candidate tiles from the box hierarchy, a tile's rows one per lane, exact fp64), else wave-wide
    // with a walk (GICP_SPARSE_AMB; 0: always wave-wide)
    int32_t sparse_amb;
    float skin;
    // a tile rebuilding its list while the pose still moves uses skin' = min(max(skin, skin_gain x its
    // displacement over the last pass), skin_max): the list then outlasts a step of the same size
    float skin_gain, skin_max;
    // per-source-point nearest-neighbour certificates, sorted source order; null: off
    int32_t* cert_j;          // [src.n] sorted target index of the certified nearest, -1: none within R
    float* cert_gap;          // [src.n] runner-up gap (found) or empty radius R (none), relative to cert_pass
    int32_t* cert_pass;       // [src.ntiles] pass the tile's certificates refer to (-1: none)
    float kappa;              // runner-up gap the walk resolves (m); 0 without certificates
    float empty_r;            // d_c (fp32, rounded up): a lane with no target within R - delta > empty_r stays rejected
    unsigned long long* stamps;  // [waves][16] phase cycles + counters (STAMPS diagnostic build only; else null)
    // 1: the final workgroup also runs the inner solve + pose update (what k_solve does), when no exchange
    // of the statistics between ranks comes between them; `hist` = this iteration's gicp_trace row or null
    int32_t fuse_solve;
    double* hist;
    PeerArgs peer;            // n > 1: the final workgroup exchanges the statistics with its peers in-kernel
    // GICP_TAIL diagnostic build: this launch's tail record ([kTailWords] realtime stamps, 100 MHz), else null
    unsigned long long* tail;
};
// GICP_TAIL record of one k_corr launch: [0] workgroup 0's start, [1] the final workgroup's partial stored,
// then the final workgroup: [2] its group ticket won, [3] group sum stored, [4] final ticket won, [5] final
// sum in LDS, [6] peer exchange done, [7] statistics stored, [8] solve done; [9..15] how lanes' searches
// ended (counts over the launch): [9] lanes that descended the target graph, [10..13] lanes the descent proved
// at the start node's local minimum / at a row entry of the start node / after a hop / by an exactly resolved
// near tie, [14] walking lanes, [15] walking waves
constexpr int kTailWords = 16;

constexpr int nstat(int D) {
    return (D * (D + 1) / 2) * (D * (D + 1) / 2) + (D * (D + 1) / 2) * D + (D * (D + 1) / 2) + D * D + D + 2;
}
// partials carry extra diagnostics: ambiguous count, pairs evaluated, list rebuilds, sum |r|^2
// ... and lanes proved by the graph descent, waves that walked (GICP_PASS_INFO)
constexpr int nstat_ext(int D) { return nstat(D) + 6; }
static_assert(nstat_ext(3) <= 80, "IterState::stats holds the extended statistics");

}  // namespace gicp
