// gicp_kernels.hip — the MI355X (gfx950) hot path of GICP.
//
// Reference behaviour (python-implementation/gicp.py):
//   k_knn_cov   <- compute_covariance_matrix / _single_point, gicp.py:5-35
//                  (k nearest incl. self, distance strictly < d_n, np.cov, eig ->
//                  surface-aligned covariance; identity for isolated points)
//   k_corr      <- the per-iteration correspondence + weight loop, gicp.py:119-145
//                  (exact 1-NN in the target, accept d <= d_c, W = inv(C_s + C_t)),
//                  fused with the sufficient statistics of loss()/grad_loss()
//                  (gicp.py:52-76) so the inner minimisation needs no further pass
//   k_solve     <- the inner solve + convergence test on the device (gicp.py:148-167)
//
// Design: one wave = one query tile of <= 64 Morton-coherent points.
// Database tiles are culled with a three-level AABB hierarchy (super-blocks of 64 blocks of 64 tiles, tested
// one per lane, ballot), staged through LDS as fp32 SoA and scanned with a
// broadcast read; lanes keep packed (d2 | row) keys.  The fp32 screen carries an
// explicit error bound: a lane whose winner is within that bound of a rival (or of
// the d_n / d_c cut) is re-resolved exactly in fp64, so indices match an fp64
// KD-tree exactly.  No MFMA: there is no dense contraction in this path.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <utility>

#include "gicp_internal.h"
#include "gicp_solver.h"
#include "gicp_solve_dev.h"

namespace gicp {

// ---------------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ unsigned umed3(unsigned a, unsigned b, unsigned c) {
    return max(min(a, b), min(max(a, b), c));
}
__device__ __forceinline__ float key_d2(unsigned k) { return __uint_as_float(k & ~63u); }
// margin of the fp32 screen at d2 (raw v_sqrt_f32, inflated past its 1-ulp error: the bound stays conservative)
__device__ __forceinline__ float marg(const Margin& m, float d2) {
    return fmaf(m.a * 1.0001f, __builtin_amdgcn_sqrtf(d2), fmaf(m.c, d2, m.b));
}

// Wave-wide min / max of floats that are >= 0 or a negative "none" marker, result uniform
// (SGPR): signed-integer compares on the bit patterns (monotonic for such values, no NaN
// canonicalisation), each step one v_{min,max}_i32 with a DPP source: row_shr 1/2/4/8,
// row_bcast 15/31, then readlane 63.
#define GICP_WAVE_REDUCE(OP, ID, x)                                                      \
    x = OP(x, __builtin_amdgcn_update_dpp(ID, x, 0x111, 0xf, 0xf, false));               \
    x = OP(x, __builtin_amdgcn_update_dpp(ID, x, 0x112, 0xf, 0xf, false));               \
    x = OP(x, __builtin_amdgcn_update_dpp(ID, x, 0x114, 0xf, 0xf, false));               \
    x = OP(x, __builtin_amdgcn_update_dpp(ID, x, 0x118, 0xf, 0xf, false));               \
    x = OP(x, __builtin_amdgcn_update_dpp(ID, x, 0x142, 0xa, 0xf, false));               \
    x = OP(x, __builtin_amdgcn_update_dpp(ID, x, 0x143, 0xc, 0xf, false));
__device__ __forceinline__ float wave_minf(float v) {
    int x = __float_as_int(v);
    GICP_WAVE_REDUCE(min, 0x7fffffff, x)
    return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}
__device__ __forceinline__ float wave_maxf(float v) {
    int x = __float_as_int(v);
    GICP_WAVE_REDUCE(max, (int)0x80000000, x)
    return __int_as_float(__builtin_amdgcn_readlane(x, 63));
}
__device__ __forceinline__ float readlane_f(float v, int k) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
}
__device__ __forceinline__ double readlane_d(double v, int k) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), k);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// wave minimum of keys < 2^31 (screen keys: non-negative fp32 bits), uniform
__device__ __forceinline__ unsigned wave_min_key(unsigned v) {
    int x = (int)v;
    GICP_WAVE_REDUCE(min, 0x7fffffff, x)
    return (unsigned)__builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ double wave_mind(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wave_maxd(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ void wave_sync() { __builtin_amdgcn_wave_barrier(); }
// ascending bitonic sort of one (key, val) pair per lane across the wave; ties by val (deterministic)
__device__ __forceinline__ void wave_sort64(float& key, int& val) {
    const int l = __lane_id();
#pragma unroll
    for (int k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (int j = k >> 1; j > 0; j >>= 1) {
            const float pk = __shfl_xor(key, j);
            const int pv = __shfl_xor(val, j);
            const bool take_min = ((l & k) == 0) == ((l & j) == 0);
            const bool less = pk < key || (pk == key && pv < val);
            const bool greater = pk > key || (pk == key && pv > val);
            if (take_min ? less : greater) {
                key = pk;
                val = pv;
            }
        }
}
// any lane: the ballot's scalar result tested directly (no bool -> int -> compare round trip)
__device__ __forceinline__ bool wave_any(bool p) { return __builtin_amdgcn_ballot_w64(p) != 0; }

// Diagnostic-only phase timer (build with `make STAMPS=1`): s_memtime cycles per phase per wave.
// 0 setup, 1 traversal tests, 2 tile need-test + staging, 3 row scan, 4 fp64 fallback,
// 5 epilogue (W, statistics), 6 statistics reduction.  Compiles to nothing otherwise.
struct Stamps {
#ifdef GICP_STAMPS
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned long long last = 0, rt0 = 0;
    __device__ __forceinline__ void start() {
        last = __builtin_amdgcn_s_memtime();
        rt0 = __builtin_amdgcn_s_memrealtime();
    }
    __device__ __forceinline__ void mark(int c) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[c] += t - last;
        last = t;
    }
    // event counters: 0 tile visits, 1 tiles scanned, 2 chunks scanned, 3 list used, 4 list length,
    // 5 traversal block tests, 6 traversal candidate blocks, 7 fp64 fallback tiles
    unsigned cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    __device__ __forceinline__ void count(int k, unsigned v = 1) { cnt[k] += v; }
#elif defined(GICP_TIMELINE)   // `make VARIANT=tl VDEFS=-DGICP_TIMELINE`: wave start/end, phase ends, counters
    unsigned long long acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    unsigned cnt[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    // realtime (100 MHz) at the end of the certificate + descent phase and at the end of the walk; the walk's
    // kind (0 none, 1 candidate list, 2 list then full walk, 3 full walk, 4 sparse search); lanes that descended / walked
    unsigned long long tdesc = 0, twalk = 0, ta = 0, tb = 0, te = 0, tf = 0;
    unsigned kind = 0, ndesc = 0, nwalk = 0, nwalk_jp = 0;
    float wb0 = 0.f;
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void count(int k, unsigned v = 1) { cnt[k] += v; }
#else
    __device__ __forceinline__ void start() {}
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void count(int, unsigned = 1) {}
#endif
};

#ifdef GICP_TIMELINE
// realtime stamp taken once `a` and `b` are available (their loads complete): the asm's inputs make the
// compiler wait for them first, and volatile asms keep their order
template <class A, class B>
__device__ __forceinline__ unsigned long long tl_after(A a, B b) {
    unsigned long long t;
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : "v"(a), "v"(b) : "memory");
    return t;
}
#endif

// exact-rounding fp64 square distance, summed in axis order without FMA contraction
// (the order a KD-tree accumulates it in)
template <int D>
__device__ __forceinline__ double dist2_exact(const double* a, const double* b) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
        const double d = __dsub_rn(a[k], b[k]);
        s = __dadd_rn(s, __dmul_rn(d, d));
    }
    return s;
}

__device__ __forceinline__ uint32_t spread2(uint32_t x) {
    x &= 0xFFFFu;
    x = (x | (x << 8)) & 0x00FF00FFu;
    x = (x | (x << 4)) & 0x0F0F0F0Fu;
    x = (x | (x << 2)) & 0x33333333u;
    x = (x | (x << 1)) & 0x55555555u;
    return x;
}
__device__ __forceinline__ uint32_t spread3(uint32_t x) {
    x &= 0x3FFu;
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}
__device__ __forceinline__ uint32_t morton_code(const double* p, int dim, const double* lo, double scale, int bits) {
    const double maxc = (double)((1u << bits) - 1u);
    uint32_t q[3] = {0, 0, 0};
    for (int a = 0; a < dim; ++a) {
        double v = (p[a] - lo[a]) * scale;
        v = fmin(fmax(v, 0.0), maxc);
        q[a] = (uint32_t)v;
    }
    return dim == 3 ? (spread3(q[0]) | (spread3(q[1]) << 1) | (spread3(q[2]) << 2))
                    : (spread2(q[0]) | (spread2(q[1]) << 1));
}

// ---------------------------------------------------------------------------
// index build
// ---------------------------------------------------------------------------
__global__ void k_morton(const double* __restrict__ xyz, int64_t n, int dim, DevCloud fr, uint32_t* codes,
                         int32_t* idx) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double p[3] = {0, 0, 0};
    for (int a = 0; a < dim; ++a) p[a] = xyz[i * dim + a];
    codes[i] = morton_code(p, dim, fr.lo, fr.scale, fr.bits);
    idx[i] = (int32_t)i;
}

// One wave per tile: gather the tile's points (original order -> sorted), fp64 AABB,
// centre, fp32 relative coordinates, half-extents and radius.
// Order of the rows inside a tile: a recursive median split instead of the Morton order the tile
// was cut from.  Rows 0-31 / 32-63 are the halves along the tile's longest axis, each half is split
// along its own longest axis, and so on down to the sub-tile size, so the sub-tiles are compact
// boxes (a Morton run can straddle a cell boundary and span the whole tile).  Rows carry no meaning beyond the
// sub-tile boxes (ties are resolved on original indices), so only the culling changes.
__device__ __forceinline__ void split_order(double (&p)[3], int& o, int dim, bool v) {
    const int l = lane_id();
    const int cnt = __popcll(__ballot(v));   // valid rows are lanes 0 .. cnt-1, and stay there
    const bool vv = l < cnt;
    // each level halves every segment of `seg` rows along that segment's own longest axis
    for (int seg = kTile; seg > kSubRows; seg >>= 1) {
        double mn[3], mx[3];
        for (int a = 0; a < 3; ++a) {
            mn[a] = vv ? p[a] : 1e300;
            mx[a] = vv ? p[a] : -1e300;
            for (int s = 1; s < seg; s <<= 1) {   // xor offsets below seg stay inside the segment
                mn[a] = fmin(mn[a], __shfl_xor(mn[a], s));
                mx[a] = fmax(mx[a], __shfl_xor(mx[a], s));
            }
        }
        int ax = 0;
        for (int a = 1; a < dim; ++a)
            if (mx[a] - mn[a] > mx[ax] - mn[ax]) ax = a;
        const double span = mx[ax] - mn[ax];
        const float t = span > 0.0 ? (float)((p[ax] - mn[ax]) / span) : 0.f;
        float key = vv ? (float)(2 * (l / seg)) + t : 3e38f;   // segment s keeps keys in [2s, 2s + 1]
        int src = l;
        wave_sort64(key, src);
        for (int a = 0; a < 3; ++a) p[a] = __shfl(p[a], src);
        o = __shfl(o, src);
    }
}

__global__ void __launch_bounds__(256) k_build_tiles(const double* __restrict__ xyz_in, int dim,
                                                      int32_t* __restrict__ perm, TileInfo* tiles, TileBox* boxes,
                                                      int ntiles, double* xyz64, float4* rel32, int32_t* inv,
                                                      unsigned* rho_bits) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int T = blockIdx.x * kWavesPerWG + w;
    if (T >= ntiles) return;
    const int start = tiles[T].start, count = tiles[T].count;
    const bool v = l < count;
    const int i = start + l;
    double p[3] = {0, 0, 0};
    int o = 0;
    if (v) {
        o = perm[i];
        for (int a = 0; a < dim; ++a) p[a] = xyz_in[(int64_t)o * dim + a];
    }
    split_order(p, o, dim, v);   // valid rows stay in lanes 0 .. count-1
    if (v) {
        perm[i] = o;
        inv[o] = i;
        double4 q;
        q.x = p[0];
        q.y = p[1];
        q.z = p[2];
        q.w = 0.0;
        reinterpret_cast<double4*>(xyz64)[i] = q;
    }
    double c[3];
    for (int a = 0; a < 3; ++a) {
        const double mn = wave_mind(v ? p[a] : 1e300);
        const double mx = wave_maxd(v ? p[a] : -1e300);
        c[a] = a < dim ? 0.5 * (mn + mx) : 0.0;
    }
    float r[3];
    for (int a = 0; a < 3; ++a) r[a] = v ? (float)(p[a] - c[a]) : 0.0f;
    if (v) rel32[i] = make_float4(r[0], r[1], r[2], 0.0f);
    float h[3];
    for (int a = 0; a < 3; ++a) h[a] = wave_maxf(fabsf(r[a]));
    const float rad = wave_maxf(sqrtf(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]));
    // sub-tile boxes (min/max over each kSubRows-lane segment of the wave)
    float smn[3], smx[3];
    for (int a = 0; a < 3; ++a) {
        smn[a] = v ? r[a] : 3e38f;
        smx[a] = v ? r[a] : -3e38f;
        for (int o = 1; o < kSubRows; o <<= 1) {
            smn[a] = fminf(smn[a], __shfl_xor(smn[a], o));
            smx[a] = fmaxf(smx[a], __shfl_xor(smx[a], o));
        }
    }
    if (l % kSubRows == 0) {
        const int g = l / kSubRows;
        TileInfo& t = tiles[T];
        for (int a = 0; a < 3; ++a) {
            const bool empty = smn[a] > smx[a];
            const float cc = empty ? 0.f : 0.5f * (smn[a] + smx[a]);
            // half-extent rounded up so the box covers both extremes exactly
            const float hh = empty ? -1e30f : fmaxf(smx[a] - cc, cc - smn[a]) * (1.0f + 2.4e-7f);
            t.sc[a][g] = cc;
            t.sh[a][g] = hh;
        }
    }
    if (l == 0) {
        TileInfo& t = tiles[T];
        for (int a = 0; a < 3; ++a) {
            t.c[a] = c[a];
            t.h[a] = h[a];
        }
        t.radius = rad;
        TileBox& b = boxes[T];
        for (int a = 0; a < 3; ++a) {
            b.c[a] = c[a];
            b.h[a] = h[a];
        }
        b.start = start;
        b.count = count;
        b.pad = 0;
        atomicMax(rho_bits, __float_as_uint(rad));
    }
}

// One wave per block of 64 tiles: fp64 AABB over the tiles' boxes.
// One level of the box hierarchy: box B covers children [64 B, 64 B + 64) of the level below
// (tiles -> blocks; blocks -> super-blocks, stored after the blocks in the same array).
template <class Child>
__global__ void __launch_bounds__(256) k_build_blocks(const Child* __restrict__ kids, int nkids, BlockInfo* blocks,
                                                       int nblocks, int dim) {
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int B = blockIdx.x * kWavesPerWG + w;
    if (B >= nblocks) return;
    const int t = B * kBlockTiles + l;
    const bool v = t < nkids;
    double lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        lo[a] = v ? kids[t].c[a] - (double)kids[t].h[a] : 1e300;
        hi[a] = v ? kids[t].c[a] + (double)kids[t].h[a] : -1e300;
        lo[a] = wave_mind(lo[a]);
        hi[a] = wave_maxd(hi[a]);
    }
    if (l == 0) {
        BlockInfo& b = blocks[B];
        for (int a = 0; a < 3; ++a) {
            const double c = a < dim ? 0.5 * (lo[a] + hi[a]) : 0.0;
            const double hh = a < dim ? 0.5 * (hi[a] - lo[a]) : 0.0;
            b.c[a] = c;
            b.h[a] = __double2float_ru(hh) * (1.0f + 1e-6f);
        }
        b.first = B * kBlockTiles;
        b.ntiles = min(kBlockTiles, nkids - B * kBlockTiles);
        b.pad = 0.f;
    }
}

// ---------------------------------------------------------------------------
// traversal
// ---------------------------------------------------------------------------
template <int D>
struct Query {
    double ow[D];   // wave origin (query tile centre, transformed), uniform
    float ew[D];    // half-extents of the query tile around ow, uniform, conservative
    float pw[D];    // lane point relative to ow, fp32
    double p64[D];  // lane point, fp64 (transformed)
    bool valid;
};

// squared gap between the wave box (ow +- ew) and a box (c +- h); conservative in fp32
template <int D>
__device__ __forceinline__ float gap2_box(const Query<D>& q, const double* c, const float* h) {
    float g2 = 0.f;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        const float dl = fabsf((float)(q.ow[a] - c[a]));
        float g = dl - q.ew[a] - h[a];
        g -= (dl + q.ew[a] + h[a]) * 9.5367431640625e-7f;  // 2^-20 slack
        g = fmaxf(g, 0.f);
        g2 = fmaf(g, g, g2);
    }
    return g2;
}

// The query box of the lanes where `on` holds (the wave's lanes still searching): their fp32 offsets
// pw lie within ow' +- ew' (conservative: the centre is rounded, the half-extent padded).  A list
// walk or fallback tests candidate tiles against it instead of the whole source tile's box, so a
// wave with a few searching lanes visits only the tiles near them (the list, built for the whole
// box, covers any subset of its lanes).  Values are shifted by 2 ew (>= |pw|) to use the
// non-negative wave max; lanes with on = false pass the negative marker.
template <int D>
__device__ __forceinline__ Query<D> active_box(const Query<D>& q, bool on) {
    Query<D> qa = q;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        const float B = 2.f * q.ew[a] + 1e-30f;
        const float hi = wave_maxf(on ? q.pw[a] + B : -1.f) - B;
        const float lo = B - wave_maxf(on ? B - q.pw[a] : -1.f);
        const float mid = 0.5f * (lo + hi);
        qa.ow[a] = q.ow[a] + (double)mid;
        qa.ew[a] = 0.5f * (hi - lo) + 4.8e-7f * (fabsf(lo) + fabsf(hi) + B) + 1e-30f;
    }
    return qa;
}

// Two-level culled walk over the database tiles.  `visit(T)` returns true when it
// processed the tile (the wave's bound then shrinks); `wave_bound()` is the max over
// lanes of the squared search radius still needed.
// With skin > 0 every tile whose box lies within sqrt(wb) + skin of the wave box is also passed
// to collect(T) (wb as it stands when the tile is tested; wb only shrinks, so at the end the
// collected set holds every tile within sqrt(wb_final) + skin).
struct NoCount {
    __device__ __forceinline__ void count(int, unsigned = 1) {}
};
template <int D, class Visit, class WB, class Collect, class Cnt = NoCount>
__device__ __forceinline__ void traverse_c(const DevCloud& db, const Query<D>& q, int seed, Visit&& visit,
                                           WB&& wave_bound, float skin, Collect&& collect, Cnt* cnt = nullptr) {
    const int l = lane_id();
    auto infl = [&](float w) -> float {
        if (skin <= 0.f || w < 0.f) return w;
        const float r = __builtin_amdgcn_sqrtf(w) * 1.0001f + skin;
        return r * r;
    };
    float wb = wave_bound();
    float wbi = infl(wb);
    if (seed >= 0) {
        collect(seed);
        if (visit(seed)) {
            wb = wave_bound();
            wbi = infl(wb);
        }
    }
    // super-blocks (64 blocks each, stored after the blocks): a round of 64 block tests is one
    // super-block, skipped whole when its box (scalar loads, uniform test) is out of reach.  It contains
    // its blocks' boxes, so the visited tiles and their order are unchanged.
    typedef __attribute__((address_space(4))) const BlockInfo* ConstBlocks;
    const ConstBlocks cb0 = (ConstBlocks)(uintptr_t)db.blocks + db.nblocks;
    for (int b0 = 0; b0 < db.nblocks; b0 += kWave) {
        {
            const ConstBlocks sb = cb0 + (b0 / kWave);
            const double c[3] = {sb->c[0], sb->c[1], sb->c[2]};
            const float h[3] = {sb->h[0], sb->h[1], sb->h[2]};
            if (!__builtin_amdgcn_readfirstlane((int)(gap2_box<D>(q, c, h) <= wbi))) continue;   // uniform
        }
        if (cnt) cnt->count(5);
        const int b = b0 + l;
        bool cb = false;
        if (b < db.nblocks) cb = gap2_box<D>(q, db.blocks[b].c, db.blocks[b].h) <= wbi;
        uint64_t bm = __ballot(cb);
        while (bm) {
            const int bb = b0 + __ffsll((unsigned long long)bm) - 1;
            bm &= bm - 1;
            const int first = db.blocks[bb].first, nt = db.blocks[bb].ntiles;
            if (cnt) cnt->count(6);
            const int t = first + l;
            bool ct = false, cv = false;
            if (l < nt && t != seed) {
                const float g2 = gap2_box<D>(q, db.tiles[t].c, db.tiles[t].h);
                ct = g2 <= wbi;
                cv = g2 <= wb;
            }
            if (skin > 0.f) {
                uint64_t cm = __ballot(ct);
                while (cm) {
                    collect(first + __ffsll((unsigned long long)cm) - 1);
                    cm &= cm - 1;
                }
            }
            uint64_t tm = __ballot(cv);
            while (tm) {
                const int T = first + __ffsll((unsigned long long)tm) - 1;
                tm &= tm - 1;
                if (visit(T)) {
                    wb = wave_bound();
                    wbi = infl(wb);
                }
            }
        }
    }
}

template <int D, class Visit, class WB>
__device__ __forceinline__ void traverse(const DevCloud& db, const Query<D>& q, int seed, Visit&& visit,
                                         WB&& wave_bound) {
    traverse_c<D>(db, q, seed, visit, wave_bound, 0.f, [](int) {});
}

// per-wave LDS: tile staging during the walk, statistics transpose afterwards (same bytes)
struct WaveStage {
    float x[kTile], y[kTile], z[kTile];           // fp32 screen coordinates, SoA
    double x64[kTile], y64[kTile], z64[kTile];    // fp64 coordinates (covariance sums, fallback)
    int32_t perm[kTile];                          // original indices (fallback tie-break)
};
// statistics transpose image of 16 points: u[term][point] and v[term][point], rows padded to 17 doubles
// (a term's 16 points are written by 16 lanes to consecutive words; the MFMA operand reads of a row
// group spread over the banks)
// Only the rows of terms in use are stored (12 u and 10 v terms in 3-D): the MFMA lanes of the unused
// rows read a duplicate of the last row, whose products land in output rows / columns nobody reads.
// 22 x 17 doubles (2992 B) instead of 2 x 16 x 17: with the walk's staging (2560 B) in the same union
// and the wave's statistics written into it after the GEMM, a workgroup takes 12 KB of LDS, 13 per CU
// instead of 8 -- a CU whose resident workgroups each wait on one long-walking wave can start others.
constexpr int kStatRow = 17;
constexpr int kStatU = 12, kStatV = 10;
struct WaveStat {
    double u[kStatU * kStatRow];
    double v[kStatV * kStatRow];
};
union __attribute__((aligned(16))) WaveLds {
    WaveStage t;
    WaveStat st;
};

// Lane point relative to database tile T, and the per-lane squared gap to T's box.
template <int D>
__device__ __forceinline__ float lane_gap2(const Query<D>& q, const TileInfo& ti, float* pr) {
    float g2 = 0.f;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        pr[a] = q.pw[a] + (float)(q.ow[a] - ti.c[a]);
        const float ap = fabsf(pr[a]);
        float g = ap - ti.h[a] - (ap + ti.h[a]) * 9.5367431640625e-7f;
        g = fmaxf(g, 0.f);
        g2 = fmaf(g, g, g2);
    }
    return g2;
}

// uniform copy of a tile's metadata through the constant address space: scalar s_load_dwordx*
// into SGPRs (a generic pointer here compiles to ten vector loads + readfirstlane)
typedef __attribute__((address_space(4))) const TileInfo* ConstTiles;
__device__ __forceinline__ TileInfo tile_meta(const DevCloud& db, int T) {
    const ConstTiles ct = (ConstTiles)(uintptr_t)db.tiles + __builtin_amdgcn_readfirstlane(T);
    TileInfo t;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        t.c[a] = ct->c[a];
        t.h[a] = ct->h[a];
    }
    t.start = ct->start;
    t.count = ct->count;
    t.radius = ct->radius;
#pragma unroll
    for (int g = 0; g < kSub; ++g)
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            t.sc[a][g] = ct->sc[a][g];
            t.sh[a][g] = ct->sh[a][g];
        }
    return t;
}

// stage a tile's fp32 coordinates (padding rows at 1e30: their distance is +inf)
__device__ __forceinline__ void stage_f32(const DevCloud& db, const TileInfo& ti, WaveLds& L) {
    const int l = lane_id();
    float4 v = make_float4(1e30f, 1e30f, 1e30f, 0.f);
    if (l < ti.count) v = db.rel32[ti.start + l];
    L.t.x[l] = v.x;
    L.t.y[l] = v.y;
    L.t.z[l] = v.z;
    wave_sync();
}
__device__ __forceinline__ float4 load_rel(const DevCloud& db, int start, int count) {
    const int l = lane_id();
    float4 v = make_float4(1e30f, 1e30f, 1e30f, 0.f);
    if (l < count) v = db.rel32[start + l];
    return v;
}
__device__ __forceinline__ void stage_f32_from(const float4& v, WaveLds& L) {
    const int l = lane_id();
    L.t.x[l] = v.x;
    L.t.y[l] = v.y;
    L.t.z[l] = v.z;
    wave_sync();
}
// k_corr's full walk: traverse_c's order and culling, but each lane of a candidate block holds its
// tile's box gap and (start, count), so a candidate's coordinates are requested together with its
// metadata (visit_pre(T, &coords): one memory round trip per visited tile instead of two), and
// candidates the shrinking bound has put out of reach are dropped before they are visited (the test the
// block entry applied, repeated with the current bound; a tile it drops could not have been within
// any lane's bound).
template <int D, class VisitPre, class WB, class Collect, class Cnt = NoCount>
__device__ __forceinline__ void walk_c(const DevCloud& db, const Query<D>& q, int seed, VisitPre&& visit_pre,
                                       WB&& wave_bound, float skin, Collect&& collect, Cnt* cnt = nullptr) {
    const int l = lane_id();
    auto infl = [&](float w) -> float {
        if (skin <= 0.f || w < 0.f) return w;
        const float r = __builtin_amdgcn_sqrtf(w) * 1.0001f + skin;
        return r * r;
    };
    float wb = wave_bound();
    float wbi = infl(wb);
    if (seed >= 0) {
        collect(seed);
        if (visit_pre(seed, nullptr)) {
            wb = wave_bound();
            wbi = infl(wb);
        }
    }
    // super-blocks (64 blocks each, stored after the blocks): lane s tests super-block s0 + s, all of a
    // round of 64 requested at once (one memory round trip instead of one per super-block); a candidate
    // super-block's 64 blocks are tested by the lanes, a candidate block's 64 tiles likewise from the
    // compact TileBox records (block b's tiles are 64 b .. 64 b + 63).  Same tiles, same order as the
    // one-super-block-at-a-time walk.
    const int nsuper = (db.nblocks + kWave - 1) / kWave;
    for (int s0 = 0; s0 < nsuper; s0 += kWave) {
        float sg = 3e38f;
        if (s0 + l < nsuper) sg = gap2_box<D>(q, db.blocks[db.nblocks + s0 + l].c, db.blocks[db.nblocks + s0 + l].h);
        uint64_t sm = __ballot(sg <= wbi);
        while (sm) {
            const int sl = __ffsll((unsigned long long)sm) - 1;
            sm &= sm - 1;
            const int b0 = (s0 + sl) * kWave;
            if (cnt) cnt->count(5);
            const int b = b0 + l;
            bool cb = false;
            if (b < db.nblocks) cb = gap2_box<D>(q, db.blocks[b].c, db.blocks[b].h) <= wbi;
            uint64_t bm = __ballot(cb);
            while (bm) {
                const int bb = b0 + __ffsll((unsigned long long)bm) - 1;
                bm &= bm - 1;
                const int first = bb * kBlockTiles, nt = min(kBlockTiles, db.ntiles - first);
                if (cnt) cnt->count(6);
                const int t = first + l;
                bool ct = false;
                float g2 = 3e38f;
                int tst = 0, tcnt = 0;   // the tile's start, count
                if (l < nt && t != seed) {
                    const TileBox tb = db.boxes[t];
                    g2 = gap2_box<D>(q, tb.c, tb.h);
                    ct = g2 <= wbi;
                    tst = tb.start;
                    tcnt = tb.count;
                }
                if (skin > 0.f) {
                    uint64_t cm = __ballot(ct);
                    while (cm) {
                        collect(first + __ffsll((unsigned long long)cm) - 1);
                        cm &= cm - 1;
                    }
                }
                uint64_t tm = __ballot(g2 <= wb);
                auto pick = [&]() -> int { return tm ? __ffsll((unsigned long long)tm) - 1 : -1; };
                auto coords = [&](int kk) {
                    return load_rel(db, __builtin_amdgcn_readlane(tst, kk), __builtin_amdgcn_readlane(tcnt, kk));
                };
                for (int k = pick(); k >= 0; k = pick()) {
                    tm &= ~(1ull << k);
                    const float4 pv = coords(k);   // in flight with the tile's metadata load in visit_pre
                    if (visit_pre(first + k, &pv)) {
                        wb = wave_bound();
                        wbi = infl(wb);
                        tm &= __ballot(g2 <= wb);
                    }
                }
            }
        }
    }
}

__device__ __forceinline__ void stage_f64(const DevCloud& db, const TileInfo& ti, WaveLds& L) {
    const int l = lane_id();
    double4 v;
    v.x = v.y = v.z = 1e150;
    v.w = 0.0;
    if (l < ti.count) v = reinterpret_cast<const double4*>(db.xyz64)[ti.start + l];
    L.t.x64[l] = v.x;
    L.t.y64[l] = v.y;
    L.t.z64[l] = v.z;
    wave_sync();
}

typedef float f2v __attribute__((ext_vector_type(2)));

// squared screen distance of the lane point to two database rows at once (v_pk_* fp32);
// bit-identical to fmaf(dz, dz, fmaf(dy, dy, dx * dx)) per row
template <int D>
__device__ __forceinline__ f2v pair_d2(const float* pr, f2v qx, f2v qy, f2v qz) {
    const f2v dx = f2v{pr[0], pr[0]} - qx;
    const f2v dy = f2v{pr[1], pr[1]} - qy;
    f2v d2 = __builtin_elementwise_fma(dy, dy, dx * dx);
    if (D == 3) {
        const f2v dz = f2v{pr[2], pr[2]} - qz;
        d2 = __builtin_elementwise_fma(dz, dz, d2);
    }
    return d2;
}

// 0xFFFFFFC0 held in a VGPR so (d2 & mask) | row is one v_and_or_b32 (row stays an SGPR)
__device__ __forceinline__ unsigned key_mask() {
    unsigned m;
    asm volatile("v_mov_b32 %0, 0xffffffc0" : "=v"(m));
    return m;
}

// One group of 4 rows at compile-time offset J: 3 ds_read_b128 (SoA x/y/z), 2 packed pairs.
template <int J, int D, class Row>
__device__ __forceinline__ void scan_group(const WaveLds& L, const float* pr, unsigned M, Row& row) {
    const float4 X = *reinterpret_cast<const float4*>(L.t.x + J);
    const float4 Y = *reinterpret_cast<const float4*>(L.t.y + J);
    float4 Z = make_float4(0.f, 0.f, 0.f, 0.f);
    if (D == 3) Z = *reinterpret_cast<const float4*>(L.t.z + J);
    const f2v a = pair_d2<D>(pr, f2v{X.x, X.y}, f2v{Y.x, Y.y}, f2v{Z.x, Z.y});
    const f2v b = pair_d2<D>(pr, f2v{X.z, X.w}, f2v{Y.z, Y.w}, f2v{Z.z, Z.w});
    row((__float_as_uint(a.x) & M) | (unsigned)J, J);
    row((__float_as_uint(a.y) & M) | (unsigned)(J + 1), J + 1);
    row((__float_as_uint(b.x) & M) | (unsigned)(J + 2), J + 2);
    row((__float_as_uint(b.y) & M) | (unsigned)(J + 3), J + 3);
}

template <int D, class Row, int... G>
__device__ __forceinline__ void scan_groups(const WaveLds& L, int n4, unsigned sub, const float* pr, unsigned M,
                                            Row& row, std::integer_sequence<int, G...>) {
    // short-circuit fold: group G runs only while 4G < n4; skipped when its sub-tile is not needed
    (void)((4 * G < n4 ? (((sub >> (4 * G / kSubRows)) & 1u) ? scan_group<4 * G, D>(L, pr, M, row) : void(), true) : false) &&
           ...);
}

// Per-lane squared gap to each sub-box of the staged tile; bit g of the result is set when
// some lane within its bound needs sub-tile g.  Same conservative slack as lane_gap2.
template <int D>
__device__ __forceinline__ unsigned sub_mask(const TileInfo& ti, const float* pr, bool valid, float bound) {
    unsigned m = 0;
#pragma unroll
    for (int g = 0; g < kSub; ++g) {
        if (kSubRows * g >= ti.count) break;
        float g2 = 0.f;
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const float dl = fabsf(pr[a] - ti.sc[a][g]);
            float gg = dl - ti.sh[a][g] - (dl + ti.sh[a][g] + fabsf(pr[a])) * 9.5367431640625e-7f;
            gg = fmaxf(gg, 0.f);
            g2 = fmaf(gg, gg, g2);
        }
        if (__any(valid && g2 <= bound)) m |= 1u << g;
    }
    return m;
}

// k_corr's forms of lane_gap2 / sub_mask: no per-axis rounding slack; the caller compares against a
// bound inflated once by the launch-uniform slack S (CorrArgs::gap_slack: rounding of coordinates
// of magnitude <= sqrt(search2) + 2 rho_t, the only ones whose test can matter)
template <int D>
__device__ __forceinline__ float lane_gap2_ns(const Query<D>& q, const TileInfo& ti, float* pr) {
    float g2 = 0.f;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        pr[a] = q.pw[a] + (float)(q.ow[a] - ti.c[a]);
        const float g = fmaxf(fabsf(pr[a]) - ti.h[a], 0.f);
        g2 = fmaf(g, g, g2);
    }
    return g2;
}
template <int D>
__device__ __forceinline__ unsigned sub_mask_ns(const TileInfo& ti, const float* pr, float bound /* < 0: lane off */) {
    // two sub-boxes per packed op (sc/sh are axis-major, so boxes g and g+1 of an axis are adjacent):
    // g = max(max(d, -d) - sh, 0), g2 += g * g
    typedef float f2v __attribute__((ext_vector_type(2)));
    unsigned m = 0;
#pragma unroll
    for (int g = 0; g < kSub; g += 2) {
        if (kSubRows * g >= ti.count) break;
        f2v g2 = {0.f, 0.f};
#pragma unroll
        for (int a = 0; a < D; ++a) {
            const f2v d = f2v{pr[a], pr[a]} - f2v{ti.sc[a][g], ti.sc[a][g + 1]};
            const f2v ad = __builtin_elementwise_max(d, -d);
            const f2v gg = __builtin_elementwise_max(ad - f2v{ti.sh[a][g], ti.sh[a][g + 1]}, f2v{0.f, 0.f});
            g2 = __builtin_elementwise_fma(gg, gg, g2);
        }
        if (wave_any(g2.x <= bound)) m |= 1u << g;
        if (kSubRows * (g + 1) < ti.count && wave_any(g2.y <= bound)) m |= 2u << g;
    }
    return m;
}

__device__ __forceinline__ int rows_scanned(unsigned sub, int count) {
    int r = 0;
#pragma unroll
    for (int g = 0; g < kSub; ++g)
        if ((sub >> g) & 1u) r += min(kSubRows, max(0, ((count + 3) & ~3) - kSubRows * g));
    return r;
}

// Scan one staged tile: row(key, j) for every row of the sub-tiles in `sub`; key = (d2 bits & ~63) | row.
template <int D, class Row>
__device__ __forceinline__ void scan_tile(const WaveLds& L, int count, const float* pr, Row&& row,
                                          unsigned sub = 0xFFFFFFFFu) {
    const unsigned M = key_mask();
    scan_groups<D>(L, (count + 3) & ~3, sub, pr, M, row, std::make_integer_sequence<int, kTile / 4>{});
}

// ---------------------------------------------------------------------------
// surface covariance: k nearest (self included, < d_n), shifted sums, eigen
// ---------------------------------------------------------------------------
template <int D>
struct CovSums {
    double n;
    double s[D];
    double ss[D * (D + 1) / 2];
};

template <int D>
__device__ __forceinline__ void cov_add(CovSums<D>& A, const double* d) {
    A.n += 1.0;
    int k = 0;
#pragma unroll
    for (int a = 0; a < D; ++a) {
        A.s[a] += d[a];
#pragma unroll
        for (int b = a; b < D; ++b) A.ss[k++] += d[a] * d[b];
    }
}

// Symmetric 3x3 eigenvector of the smallest eigenvalue (cyclic Jacobi, fp64).
__device__ __forceinline__ void smallest_eigvec3(double A[3][3], double* n) {
    double V[3][3] = {{1, 0, 0}, {0, 1, 0}, {0, 0, 1}};
    for (int sweep = 0; sweep < 12; ++sweep) {
        const double off = fabs(A[0][1]) + fabs(A[0][2]) + fabs(A[1][2]);
        if (off == 0.0) break;
#pragma unroll
        for (int pq = 0; pq < 3; ++pq) {
            const int p = pq == 2 ? 1 : 0;
            const int qq = pq == 0 ? 1 : 2;
            const double apq = A[p][qq];
            if (apq == 0.0) continue;
            const double theta = (A[qq][qq] - A[p][p]) / (2.0 * apq);
            const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
            const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
            for (int k = 0; k < 3; ++k) {  // A <- J^T A J
                const double akp = A[k][p], akq = A[k][qq];
                A[k][p] = c * akp - s * akq;
                A[k][qq] = s * akp + c * akq;
            }
            for (int k = 0; k < 3; ++k) {
                const double apk = A[p][k], aqk = A[qq][k];
                A[p][k] = c * apk - s * aqk;
                A[qq][k] = s * apk + c * aqk;
            }
            for (int k = 0; k < 3; ++k) {
                const double vkp = V[k][p], vkq = V[k][qq];
                V[k][p] = c * vkp - s * vkq;
                V[k][qq] = s * vkp + c * vkq;
            }
        }
    }
    int m = 0;
    if (A[1][1] < A[m][m]) m = 1;
    if (A[2][2] < A[m][m]) m = 2;
    for (int k = 0; k < 3; ++k) n[k] = V[k][m];
}

// C = a I - m m^T from the neighbourhood sums (gicp.py:11-16 / SURVEY.md §8.A)
template <int D>
__device__ __forceinline__ double4 cov_descriptor(const CovSums<D>& A, int min_nb, double eps_a, double m_scale) {
    double4 out;
    out.x = 1.0;
    out.y = out.z = out.w = 0.0;  // identity (gicp.py:33-34)
    if (A.n < (double)min_nb) return out;
    const double n = A.n;
    double C[D][D];
    int k = 0;
    for (int a = 0; a < D; ++a)
        for (int b = a; b < D; ++b) {
            C[a][b] = C[b][a] = (A.ss[k] - A.s[a] * A.s[b] / n) / (n - 1.0);
            ++k;
        }
    out.x = eps_a;
    if (D == 2) {
        // principal eigenvector at 0.5 atan2(2 cxy, cxx - cyy); thin direction is its normal
        const double phi = 0.5 * atan2(2.0 * C[0][1], C[0][0] - C[1][1]);
        double sp, cp;
        sincos(phi, &sp, &cp);
        out.y = -sp * m_scale;
        out.z = cp * m_scale;
    } else {
        double M[3][3];
        for (int a = 0; a < 3; ++a)
            for (int b = 0; b < 3; ++b) M[a][b] = C[a % D][b % D];
        double nv[3];
        smallest_eigvec3(M, nv);
        out.y = nv[0] * m_scale;
        out.z = nv[1] * m_scale;
        out.w = nv[2] * m_scale;
    }
    return out;
}

// The wave's query for split build kernels: wave `wid` takes part g = wid % split of query tile
// T = first + wid / split.  Lanes keep their points relative to the tile centre (the screen's error model
// is unchanged); the culling box `qb` is the part's sub-box (centre c + sc, half-extents sh) when split.
// Returns the tile index, -1 if the wave has no rows.
template <int D>
__device__ __forceinline__ int split_query(const DevCloud& cl, int first, int last, int split, int sh_n, int sh_r,
                                          TileInfo& qt, Query<D>& q, Query<D>& qb, int& i) {
    const int wid = (int)blockIdx.x * kWavesPerWG + ((int)threadIdx.x >> 6), l = (int)threadIdx.x & 63;
    const int Tl = first + wid / split, g = wid % split;
    if (Tl >= last) return -1;
    constexpr int kChunkTiles = kShardChunk * kCorrWaves;   // tiles per shard chunk (k_corr's split)
    const int T = sh_n > 1 ? ((Tl / kChunkTiles) * sh_n + sh_r) * kChunkTiles + Tl % kChunkTiles : Tl;
    if (T >= cl.ntiles) return -1;
    qt = tile_meta(cl, T);
    const int rows = kTile / split, r0 = g * rows, r1 = min(qt.count, r0 + rows);
    if (r0 >= r1) return -1;
    q.valid = l < r1 - r0;
    i = qt.start + r0 + min(l, r1 - r0 - 1);
    const float4 rel = cl.rel32[i];
    const double4 p4 = reinterpret_cast<const double4*>(cl.xyz64)[i];
    const float relv[3] = {rel.x, rel.y, rel.z};
    const double p4v[3] = {p4.x, p4.y, p4.z};
#pragma unroll
    for (int a = 0; a < D; ++a) {
        q.ow[a] = qt.c[a];
        q.ew[a] = qt.h[a];
        q.pw[a] = relv[a];
        q.p64[a] = p4v[a];
    }
    qb = q;
    if (split > 1) {
#pragma unroll
        for (int a = 0; a < D; ++a) {
            qb.ow[a] = qt.c[a] + (double)qt.sc[a][g];
            qb.ew[a] = qt.sh[a][g] * (1.0f + 4.8e-7f) + 1e-30f;
        }
    }
    return T;
}

// G: the target's neighbour graph rows come out of the same two walks: phase 1 keeps the
// KL = max(K + 1, kGraphK + 2) smallest keys (the covariance uses the first K + 1, the graph all), phase 2
// visits every tile either needs and takes each row for the covariance sums (key <= tau) and / or the
// graph row (key <= tau_g).  Tiles are visited in the same order whatever the bound, so the sums and rows
// are those of separate walks, bit for bit.
template <int D, int K, bool G>
__global__ void __launch_bounds__(256) k_knn_cov(CovArgs A) {
    __shared__ WaveLds s_lds[kWavesPerWG];
    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    WaveLds& L = s_lds[w];
    const DevCloud& cl = A.cl;
    TileInfo qt;
    Query<D> q, qb;
    int i = 0;
    const int T = split_query<D>(cl, A.q_begin, A.q_end, A.split, A.sh_n, A.sh_r, qt, q, qb, i);
    if (T < 0) return;  // waves are independent (no workgroup barrier here)

    // ---- phase 1: fp32 screen for the K+1 smallest keys ------------------
    constexpr int K1 = K + 1, KG = kGraphK, KL = G ? (K1 > KG + 2 ? K1 : KG + 2) : K1;
    const unsigned init = __float_as_uint(A.search2) | 63u;
    unsigned lk[KL];
#pragma unroll
    for (int m = 0; m < KL; ++m) lk[m] = init;
    auto lane_bound = [&]() -> float {
        if (!q.valid) return -1.f;
        if (G) return key_d2(lk[KL - 1]);   // >= the covariance's own bound below
        const float kk = key_d2(lk[K1 - 1]), km = key_d2(lk[K1 - 2]);
        return fminf(kk, km + 2.f * marg(A.mg, km));
    };
    auto visit1 = [&](int Tt) -> bool {
        const TileInfo ti = tile_meta(cl, Tt);
        float pr[D];
        const bool need = lane_gap2<D>(q, ti, pr) <= lane_bound();
        if (!__any(need)) return false;
        // sub-tiles beyond the top of the truncation bucket of each lane's last list key hold no row the
        // list would take (a key below it screens at most at that bucket's top)
        const unsigned sub = sub_mask<D>(ti, pr, q.valid, __uint_as_float((lk[KL - 1] | 63u) + 1u));
        stage_f32(cl, ti, L);
        scan_tile<D>(L, ti.count, pr, [&](unsigned key, int) {
            if (__any(key < lk[KL - 1])) {
#pragma unroll
                for (int m = KL - 1; m > 0; --m) lk[m] = umed3(lk[m - 1], lk[m], key);
                lk[0] = min(lk[0], key);
            }
        }, sub);
        wave_sync();
        return true;
    };
    traverse<D>(cl, qb, T, visit1, [&]() { return wave_maxf(lane_bound()); });

    // graph: rows keyed <= tau_g (the (kGraphK + 1)-th key, self excluded from the row) and the radius the
    // row certifies (k_graph's rules: from the (kGraphK + 2)-th key, or the screen radius)
    unsigned tau_g = 0;
    float r2g = 0.f, tau_g_hi = -1.f;
    if constexpr (G) {
        tau_g = lk[KG];
        if (lk[KG + 1] >= init) {
            r2g = A.search2 - marg(A.mg, A.search2);
        } else {
            const float kd = key_d2(lk[KG + 1] > tau_g ? lk[KG + 1] : tau_g);
            r2g = kd - marg(A.mg, kd);
        }
        tau_g_hi = tau_g >= init ? A.search2 : __uint_as_float((tau_g | 63u) + 1u);
    }

    int c = 0;
#pragma unroll
    for (int m = 0; m < K1; ++m) c += lk[m] < init ? 1 : 0;
    const int nacc = min(c, K);
    unsigned tau = init;
#pragma unroll
    for (int m = 0; m < K; ++m)
        if (m == nacc - 1) tau = lk[m];
    const float tau_d2 = key_d2(tau);
    bool amb = false;
    if (c > K) {
        const float a1 = key_d2(lk[K - 1]), a2 = key_d2(lk[K]);
        amb = (a2 - a1) <= marg(A.mg, a1) + marg(A.mg, a2);
    }
    const float dn2_lo = (float)A.dn2 * (1.0f - 2.4e-7f);
    if (tau_d2 + marg(A.mg, tau_d2) >= dn2_lo) amb = true;
    amb = amb && q.valid;

    // ---- phase 2: fp64 shifted sums over the accepted keys ------------------
    CovSums<D> S;
    S.n = 0.0;
#pragma unroll
    for (int a = 0; a < D; ++a) S.s[a] = 0.0;
#pragma unroll
    for (int k = 0; k < D * (D + 1) / 2; ++k) S.ss[k] = 0.0;
    const bool take_lane = q.valid && !amb;
    // cull by the top of tau's truncation bucket: a point keyed <= tau may screen above key_d2(tau)
    const float tau_hi = __uint_as_float((tau | 63u) + 1u);
    // the lane's phase-2 bound: the covariance's, and the graph row's
    const float b2 = fmaxf(take_lane ? tau_hi : -1.f, (G && q.valid) ? tau_g_hi : -1.f);
    int gcnt = 0;
    bool gover = false;
    float4* row_out = G ? A.g_nb + (int64_t)i * KG : nullptr;
    auto visit2 = [&](int Tt) -> bool {
        const TileInfo ti = tile_meta(cl, Tt);
        float pr[D];
        const bool need = lane_gap2<D>(q, ti, pr) <= b2;
        if (!__any(need)) return false;
        const unsigned sub = sub_mask<D>(ti, pr, b2 >= 0.f, b2);
        stage_f32(cl, ti, L);
        stage_f64(cl, ti, L);
        scan_tile<D>(L, ti.count, pr, [&](unsigned key, int j) {
            const bool take = take_lane && key <= tau;
            if (__any(take)) {
                const double qq[3] = {L.t.x64[j], L.t.y64[j], L.t.z64[j]};
                double d[D];
#pragma unroll
                for (int a = 0; a < D; ++a) d[a] = qq[a] - q.p64[a];
                if (take) cov_add<D>(S, d);
            }
            if constexpr (G) {
                const int t = ti.start + j;
                if (q.valid && key <= tau_g && t != i) {
                    if (gcnt < KG) {
                        const double qq[3] = {L.t.x64[j], L.t.y64[j], L.t.z64[j]};
                        float v[3] = {0.f, 0.f, 0.f};
#pragma unroll
                        for (int a = 0; a < D; ++a) v[a] = (float)(qq[a] - q.p64[a]);
                        row_out[gcnt] = make_float4(v[0], v[1], v[2], __int_as_float(t));
                        ++gcnt;
                    } else {
                        gover = true;
                    }
                }
            }
        }, sub);
        wave_sync();
        return true;
    };
    traverse<D>(cl, qb, T, visit2, [&]() { return wave_maxf(b2); });
    if (G && q.valid) {
        // r rounded down; an overflowing row (ties at tau beyond kGraphK) certifies nothing
        const float r = gover ? 0.f : __builtin_amdgcn_sqrtf(fmaxf(r2g, 0.f)) * 0.99999f;
        A.g_nbh[i] = make_float2(r, __int_as_float(gcnt));
    }

    // ---- fp64 fallback for lanes the screen could not decide ----------------
    if (__any(amb)) {
        if (A.amb_counter && l == 0) atomicAdd(A.amb_counter, __popcll(__ballot(amb)));
        double lk64[K];
#pragma unroll
        for (int m = 0; m < K; ++m) lk64[m] = A.dn2;
        const float bound_f = A.search2;
        auto visit3 = [&](int Tt) -> bool {
            const TileInfo ti = tile_meta(cl, Tt);
            float pr[D];
            const float b64 = (float)lk64[K - 1];
            const bool need = amb && lane_gap2<D>(q, ti, pr) <= b64 + 2.f * marg(A.mg, b64);
            if (!__any(need)) return false;
            stage_f64(cl, ti, L);
            for (int j = 0; j < ti.count; ++j) {
                const double qq[3] = {L.t.x64[j], L.t.y64[j], L.t.z64[j]};
                const double d2 = dist2_exact<D>(qq, q.p64);
                if (__any(amb && d2 < lk64[K - 1])) {
                    if (amb) {
#pragma unroll
                        for (int m = K - 1; m > 0; --m) lk64[m] = fmin(lk64[m], fmax(lk64[m - 1], d2));
                        lk64[0] = fmin(lk64[0], d2);
                    }
                }
            }
            wave_sync();
            return true;
        };
        traverse<D>(cl, qb, T, visit3, [&]() { return wave_maxf(amb ? bound_f : -1.f); });
        int c64 = 0;
#pragma unroll
        for (int m = 0; m < K; ++m) c64 += lk64[m] < A.dn2 ? 1 : 0;
        double tau64 = A.dn2;
#pragma unroll
        for (int m = 0; m < K; ++m)
            if (m == c64 - 1) tau64 = lk64[m];
        int nless = 0;
#pragma unroll
        for (int m = 0; m < K; ++m) nless += lk64[m] < tau64 ? 1 : 0;
        int eq_left = c64 - nless;
        auto visit4 = [&](int Tt) -> bool {
            const TileInfo ti = tile_meta(cl, Tt);
            float pr[D];
            const float b64 = (float)tau64;
            const bool need = amb && lane_gap2<D>(q, ti, pr) <= b64 + 2.f * marg(A.mg, b64);
            if (!__any(need)) return false;
            stage_f64(cl, ti, L);
            for (int j = 0; j < ti.count; ++j) {
                const double qq[3] = {L.t.x64[j], L.t.y64[j], L.t.z64[j]};
                const double d2 = dist2_exact<D>(qq, q.p64);
                bool take = amb && c64 > 0 && (d2 < tau64 || (d2 == tau64 && eq_left > 0));
                if (take && d2 == tau64) --eq_left;
                if (__any(take)) {
                    double d[D];
#pragma unroll
                    for (int a = 0; a < D; ++a) d[a] = qq[a] - q.p64[a];
                    if (take) cov_add<D>(S, d);
                }
            }
            wave_sync();
            return true;
        };
        traverse<D>(cl, qb, T, visit4, [&]() {
            const float b64 = (float)tau64;
            return wave_maxf(amb ? b64 + 2.f * marg(A.mg, b64) : -1.f);
        });
    }

    if (q.valid) {
        A.cov_out[i] = cov_descriptor<D>(S, A.min_nb, A.eps_a, A.m_scale);
        A.count_out[i] = (int)S.n;
    }
}

// ---------------------------------------------------------------------------
// target neighbour graph: for every target point i its kGraphK nearest other target
// points (relative positions + sorted indices) and a radius r(i) such that EVERY target t != i with true
// |x_t - x_i| < r(i) is in the row.  Built once per target cloud by k_knn_cov<D, K, true> (the same walks
// as the covariances); k_corr's graph descent proves nearest neighbours with it.  Only conservativeness of
// r matters (no tie rules): phase 1 keeps the kGraphK + 2 smallest screened keys (self included); phase 2
// emits the rows keyed <= tau = the (kGraphK + 1)-th key, self excluded; a row not emitted has a screened
// key > tau, so its true d2 >= key_d2(lk[kGraphK + 1]) - margin when that key is above tau (else
// key_d2(tau) - margin); a lane that found fewer keys within the screen radius has every target within it:
// r2 = search2 - margin.
// Pack the graph rows (DevCloud::nbq / nbx): offsets quantised to int16 in units of s = max |offset| / 32767
// (error <= s / 2 per axis, which k_corr's bound adds), entries ordered nearest-first, each with its
// sorted-index delta (kGraphFar when it does not fit 16 bits), so a descent step finds the next node without
// reading nbi.
__global__ void __launch_bounds__(256) k_graph_pack(const float4* __restrict__ nb, const float2* __restrict__ nbh,
                                                    int64_t n, uint4* __restrict__ nbq, uint4* __restrict__ nbx,
                                                    int32_t* __restrict__ nbi) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float2 h = nbh[i];
    const int cnt = __float_as_int(h.y);
    float m = 0.f;
    for (int k = 0; k < cnt; ++k) {
        const float4 v = nb[i * kGraphK + k];
        m = fmaxf(m, fmaxf(fabsf(v.x), fmaxf(fabsf(v.y), fabsf(v.z))));
    }
    const float s = m > 0.f ? m / 32767.f : 1e-30f;
    const float inv = 1.f / s;
    // entries nearest-first (squared offset length, ties by sorted index): k_corr's descent reads the first
    // half-line and needs the rest only when an entry there could still be the nearest
    float key[kGraphK];
    int ord[kGraphK];
    for (int k = 0; k < cnt; ++k) {
        const float4 v = nb[i * kGraphK + k];
        const float kk = fmaf(v.z, v.z, fmaf(v.y, v.y, v.x * v.x));
        const int t = __float_as_int(v.w);
        int pos = k;
        while (pos > 0 && (key[pos - 1] > kk || (key[pos - 1] == kk && __float_as_int(nb[i * kGraphK + ord[pos - 1]].w) > t))) {
            key[pos] = key[pos - 1];
            ord[pos] = ord[pos - 1];
            --pos;
        }
        key[pos] = kk;
        ord[pos] = k;
    }
    uint32_t w[2 + 2 * kGraphK];
    w[0] = __float_as_uint(h.x);
    w[1] = __float_as_uint(s);
    // unused entries (k >= cnt) repeat the last real entry (or the node itself, offset and delta 0, in an
    // empty row), so the descent needs no per-entry validity test: a repeated entry never becomes the
    // strictly nearer candidate and at most makes the runner-up equal the winner, which the descent
    // treats as a near tie resolved exactly over the real entries (nbi = -1 marks the repeats)
    int q[4] = {0, 0, 0, 0};
    for (int k = 0; k < kGraphK; ++k) {
        int idx = -1;
        if (k < cnt) {
            const float4 v = nb[i * kGraphK + ord[k]];
            const float c[3] = {v.x, v.y, v.z};
            for (int a = 0; a < 3; ++a) q[a] = max(-32767, min(32767, __float2int_rn(c[a] * inv)));
            idx = __float_as_int(v.w);
            const int64_t d = (int64_t)idx - i;
            q[3] = d >= -32767 && d <= 32767 ? (int)d : kGraphFar;
        }
        w[2 + 2 * k] = ((uint32_t)q[0] & 0xFFFFu) | ((uint32_t)q[1] << 16);
        w[3 + 2 * k] = ((uint32_t)q[2] & 0xFFFFu) | ((uint32_t)q[3] << 16);
        nbi[i * kGraphK + k] = idx;
    }
    for (int c = 0; c < 8; ++c) nbq[i * 8 + c] = make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
    uint32_t x[12] = {};
    for (int k = 0; k < 2 * (kGraphK - kGraphLineA); ++k) x[k] = w[2 + 2 * kGraphLineA + k];
    for (int c = 0; c < 3; ++c) nbx[i * 3 + c] = make_uint4(x[4 * c], x[4 * c + 1], x[4 * c + 2], x[4 * c + 3]);
}

// ---------------------------------------------------------------------------
// per-iteration correspondences + weights + statistics
// ---------------------------------------------------------------------------
// Register budget of k_corr: on gfx950 a wave with next_free_sgpr >= 94 leaves 6 waves per SIMD,
// <= 90 leaves 7 and <= 72 (with <= 64 VGPRs) 8 (scripts/probes/occupancy.hip measures it; the
// compiler's own occupancy estimate does not model it).  6 waves per SIMD: 75 VGPRs, no VGPR spill;
// held to 7 (72 VGPRs, 88 SGPRs) the allocator spills 6 VGPRs and ~30 SGPRs, and the 1M/1M bench ran
// 0.7-1.3 % slower (interleaved A/B, scripts/variants.sh) once the per-lane search cap and the adaptive
// list skin were in (it was the faster setting before them).
#ifndef GICP_CORR_ATTR
#if defined(GICP_CORR_WAVES_PER_EU)
#define GICP_CORR_ATTR __attribute__((amdgpu_num_sgpr(GICP_CORR_SGPR), amdgpu_waves_per_eu(GICP_CORR_WAVES_PER_EU, GICP_CORR_WAVES_PER_EU)))
#else
#define GICP_CORR_ATTR __attribute__((amdgpu_num_sgpr(GICP_CORR_SGPR), amdgpu_waves_per_eu(6, 6)))
#endif
#endif
#ifndef GICP_CORR_SGPR
#define GICP_CORR_SGPR 100
#endif

template <int D>
struct StatIdx {
    static constexpr int NS = D * (D + 1) / 2;
    static constexpr int pa(int p) { return D == 3 ? (p < 3 ? 0 : (p < 5 ? 1 : 2)) : (p < 2 ? 0 : 1); }
    static constexpr int pb(int p) {
        return D == 3 ? (p == 0 ? 0 : p == 1 ? 1 : p == 2 ? 2 : p == 3 ? 1 : 2) : (p == 0 ? 0 : 1);
    }
};

// statistic k of one point: A[ab][ij], B[ab][i], C[ab], gR[a][i], gt[a], c0, count
template <int D>
__device__ __forceinline__ double stat_value(int k, const double (&W)[D][D], const double (&s)[D],
                                             const double (&wr)[D], double rwr) {
    using SI = StatIdx<D>;
    constexpr int NS = SI::NS;
    if (k < NS * NS) {
        const int p = k / NS, qd = k % NS;
        return W[SI::pa(p)][SI::pb(p)] * (s[SI::pa(qd)] * s[SI::pb(qd)]);
    }
    k -= NS * NS;
    if (k < NS * D) return W[SI::pa(k / D)][SI::pb(k / D)] * s[k % D];
    k -= NS * D;
    if (k < NS) return W[SI::pa(k)][SI::pb(k)];
    k -= NS;
    if (k < D * D) return wr[k / D] * s[k % D];
    k -= D * D;
    if (k < D) return wr[k];
    k -= D;
    if (k == 0) return rwr;
    return 1.0;
}

#ifndef GICP_SPARSE_GROUP
#define GICP_SPARSE_GROUP 4
#endif
constexpr int kSparseGroup = GICP_SPARSE_GROUP;   // candidate tiles per round trip of a sparse wave's search

// In-kernel exchange of a workgroup's NV values with every peer rank (PeerArgs, gicp_internal.h), called by
// all threads of one workgroup: `vals` (LDS) goes into this rank's slot of every rank's area, then the
// launch's sequence number into the flags; the workgroup waits until every rank's flag of this launch has
// arrived in its own area (at most P.timeout wall-clock ticks: a missing peer fails the exchange, it never
// hangs the launch) and replaces `vals` by the sum over ranks in rank order -- the same bits on every
// rank.  Returns false on a timeout (uniform over the workgroup).  System-scope stores and a system
// release before the flags; acquire loads on the flags; the areas are uncached device memory.
template <int NV>
__device__ bool peer_exchange(const PeerArgs P, uint64_t seq, double* vals) {   // (P by value: a reference into
                                                                             // the kernel arguments made a scratch copy)
    static_assert(NV <= kPeerSlot, "an exchange slot holds the values");
    __shared__ int s_fail;
    const int R = P.n, me = P.rank, tid = (int)threadIdx.x, nt = (int)blockDim.x;
    const int par = (int)(seq & 1u);
    for (int p = 0; p < R; ++p) {   // (p uniform: one scalar load of each peer's pointer)
        double* const dst = P.area[p] + kPeerFlagWords + (size_t)(par * kMaxPeers + me) * kPeerSlot;
        for (int k = tid; k < NV; k += nt) __hip_atomic_store(dst + k, vals[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    __threadfence_system();   // this thread's slot stores complete and visible system-wide
    if (tid == 0) s_fail = 0;
    __syncthreads();          // ... every thread's, before any flag
    if (tid < R) {
        uint64_t* f = reinterpret_cast<uint64_t*>(P.area[tid]) + par * kMaxPeers + me;
        __hip_atomic_store(f, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (tid == 0) *P.ctr = seq;   // flags of `seq` are out (also when the wait below times out)
        const uint64_t* g = reinterpret_cast<const uint64_t*>(P.own) + par * kMaxPeers + tid;
        const uint64_t t0 = (uint64_t)wall_clock64();
        while (__hip_atomic_load(g, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != seq) {
            if ((uint64_t)wall_clock64() - t0 > P.timeout) {
                s_fail = 1;
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __syncthreads();
    if (s_fail) return false;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");   // every thread: the peers' slots after their flags
    for (int k = tid; k < NV; k += nt) {
        double s = 0.0;
        for (int p = 0; p < R; ++p)
            s += __hip_atomic_load(P.own + kPeerFlagWords + (size_t)(par * kMaxPeers + p) * kPeerSlot + k,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        vals[k] = s;
    }
    __syncthreads();
    return true;
}

// gicp_peer_init's probe: `rounds` back-to-back exchanges of a full slot (kPeerSlot values, both parities), each
// value a pattern of (rank, value index, round) whose sum over the ranks is exact in fp64, so every summed
// value must come back bit-exact: a mapping, store ordering or flag protocol that misbehaves across the
// devices shows up here before the first registration.  out = (rounds completed, or -1 on a timeout; values
// that came back wrong).
__device__ __forceinline__ double probe_value(int rank, int k, int r) {
    return ldexp((double)((rank + 1) * 1000003 + k * 97 + r * 7919), -7);
}
__global__ void __launch_bounds__(64) k_peer_probe(PeerArgs P, int rounds, double* out) {
    __shared__ double v[kPeerSlot];
    __shared__ uint64_t s_seq;
    __shared__ int s_bad;
    if (threadIdx.x == 0) {
        s_seq = *P.ctr;
        s_bad = 0;
    }
    int done = 0;
    for (int r = 0; r < rounds; ++r) {
        for (int k = threadIdx.x; k < kPeerSlot; k += blockDim.x) v[k] = probe_value(P.rank, k, r);
        __syncthreads();
        if (threadIdx.x == 0) ++s_seq;
        __syncthreads();
        if (!peer_exchange<kPeerSlot>(P, s_seq, v)) {
            done = -1;
            break;
        }
        int bad = 0;
        for (int k = threadIdx.x; k < kPeerSlot; k += blockDim.x) {
            double want = 0.0;
            for (int p = 0; p < P.n; ++p) want += probe_value(p, k, r);
            bad += v[k] != want;
        }
        if (bad) atomicAdd(&s_bad, bad);
        __syncthreads();
        done = r + 1;
    }
    if (threadIdx.x == 0) {
        out[0] = (double)done;
        out[1] = (double)s_bad;
    }
}

template <int D>
__global__ void __launch_bounds__(64 * kCorrWaves) GICP_CORR_ATTR k_corr(CorrArgs A) {
    constexpr int NSX = nstat_ext(D);
    constexpr int NSS = nstat(D);
    __shared__ WaveLds s_lds[kCorrWaves];
    // per-wave statistics: written into the wave's own LDS once its statistics GEMM has read it
    static_assert(sizeof(double) * NSX <= sizeof(WaveLds), "a wave's statistics fit its LDS");
    auto wstat = [&](int u) -> double* { return reinterpret_cast<double*>(&s_lds[u]); };

    const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
    WaveLds& L = s_lds[w];
    const DevCloud& sc = A.src;
    const DevCloud& tg = A.tgt;

    // workgroup -> unit (kCorrWaves consecutive source tiles).  Workgroup b runs on XCD b % 8: the
    // first 8 q8 workgroups are striped so that XCD x walks the contiguous unit range [x q8, x q8 + q8)
    // in index order (its L2 then holds that region of the target); the remaining units run in index
    // order.  (Orders that start the previous pass's long units first were measured slower: the
    // walking set changes from pass to pass)
    const int nunits = (int)gridDim.x, q8 = nunits / 8;
    int unit = (int)blockIdx.x;
    if (A.unit_map == 0) {
        if (unit < 8 * q8) unit = (unit & 7) * q8 + (unit >> 3);
    } else {   // the k-th workgroup of XCD x takes unit k % C of the XCD's (k / C)-th chunk of C units
        const int C = A.unit_map, full = nunits / (8 * C) * (8 * C);
        if (unit < full) unit = (((unit >> 3) / C) * 8 + (unit & 7)) * C + (unit >> 3) % C;
    }
    unit = __builtin_amdgcn_readfirstlane(unit);
    // this rank's unit -> the cloud's unit (shards interleaved by chunks, gicp_internal.h)
    int T = (unit + (unit / kShardChunk) * A.sh_skip + A.sh_first) * kCorrWaves + w;
    if (T >= A.q_end) T = -1;
    T = __builtin_amdgcn_readfirstlane(T);

    // Everything the wave needs before its first decision, requested in ONE batch of scalar loads (one
    // memory round trip; a scalar wait covers every load in flight, so a use between them would split
    // the batch): the pass's pose and convergence flag (device state), the source tile's metadata, the
    // pass its certificates refer to and last pass's best target tile.  Requested for tile 0 when the
    // wave has none.  (cert_pass / hint are written only by this wave, at its end; the scalar cache
    // starts each launch invalidated.)
    const int Tq = T < 0 ? 0 : T;
    typedef __attribute__((address_space(4))) const IterState* ConstState;
    typedef __attribute__((address_space(4))) const int32_t* ConstI32;
    {   // the four array pointers (kernel arguments) in SGPRs first: their loads would otherwise be
        // interleaved with the batch and each wait for one would wait for the data loads issued before it
        const void* p0 = A.state;
        const void* p1 = sc.tiles;
        const void* p2 = A.cert_pass;
        const void* p3 = A.hint;
        asm volatile("" ::"s"(p0), "s"(p1), "s"(p2), "s"(p3));
    }
    const ConstState cs0 = (ConstState)(uintptr_t)A.state;
    const TileInfo st = tile_meta(sc, Tq);
    const int cpass0 = ((ConstI32)(uintptr_t)A.cert_pass)[Tq];
    const int hint0 = ((ConstI32)(uintptr_t)A.hint)[Tq];
    const bool done = cs0->converged && !A.single_pass;
    struct {
        double R[9], t[3];
        float R32[9];
    } P;
#pragma unroll
    for (int a = 0; a < D; ++a) {
#pragma unroll
        for (int b = 0; b < D; ++b) {
            P.R[a * D + b] = cs0->T[a * (D + 1) + b];
            P.R32[a * D + b] = (float)P.R[a * D + b];
        }
        P.t[a] = cs0->T[a * (D + 1) + D];
    }

#ifdef GICP_TAIL
    unsigned long long tl[kTailWords] = {};
    __shared__ unsigned s_walk[8];
    if (threadIdx.x < 8) s_walk[threadIdx.x] = 0;
    __syncthreads();
    if (A.tail && blockIdx.x == 0 && threadIdx.x == 0) A.tail[0] = __builtin_amdgcn_s_memrealtime();   // (first dispatched)
#define GICP_TAIL_MARK(k) do { if (A.tail) tl[k] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define GICP_TAIL_MARK(k) do {} while (0)
#endif
    Stamps S;
    S.start();
#ifdef GICP_TIMELINE
    if (A.stamps && l == 0)   // stored at once: no register held across the wave
        A.stamps[((int64_t)blockIdx.x * kCorrWaves + w) * 20 + 16] = __builtin_amdgcn_s_memrealtime();
    S.ta = tl_after(P.R[0] + st.c[0], cpass0 + hint0 + st.count);   // the prologue's scalar batch is in
#endif
    if ((A.use_lists || A.cert_j) && blockIdx.x == 0 && threadIdx.x == 0 && !done) {   // this pass's pose into the ring
        double* ring = A.poses + (A.pass % kPoseRing) * 12;
        for (int a = 0; a < 3; ++a) {
            for (int b = 0; b < 3; ++b) ring[a * 3 + b] = (a < D && b < D) ? P.R[a * D + b] : 0.0;
            ring[9 + a] = a < D ? P.t[a] : 0.0;
        }
    }
    int pairs = 0, list_rebuilds = 0, namb_total = 0, ngproved = 0, nwalked = 0;
    if (T < 0 && done) return;
    if (T >= 0) {
    bool on = false;          // accepted correspondence
    double W[D][D] = {}, sv[D] = {}, wr[D] = {}, rwr = 0.0, r2 = 0.0;
    bool amb = false;
    {
        if (done) return;
        Query<D> q;
        q.valid = l < st.count;
        int i = st.start + min(l, st.count - 1);
        // the point's index again where the epilogue needs it: recomputed from the tile's scalars (an empty
        // asm keeps the compiler from carrying the first copy, and its 64-bit address, through the search's
        // register peak, where it was spilled to scratch)
        auto refresh_i = [&]() {
            i = st.start + min(lane_id(), st.count - 1);
            asm volatile("" : "+v"(i));
        };
        const float4 rel = sc.rel32[i];
        const float relv[3] = {rel.x, rel.y, rel.z};
#pragma unroll
        for (int a = 0; a < D; ++a) {
            double o = P.t[a];
            float pw = 0.f, ew = 0.f;
#pragma unroll
            for (int b = 0; b < D; ++b) {
                o += P.R[a * D + b] * st.c[b];
                pw = fmaf(P.R32[a * D + b], relv[b], pw);
                ew = fmaf(fabsf(P.R32[a * D + b]), st.h[b], ew);
            }
            q.ow[a] = o;
            q.pw[a] = pw;
            q.ew[a] = ew * (1.0f + 4.8e-7f) + 1e-30f;
        }
        const bool lists = A.use_lists != 0;

        // seed: last pass's best target tile for this source tile, else the Morton neighbour
        int seed = hint0;
        if (seed < 0 || seed >= tg.ntiles) {
            const uint32_t code = morton_code(q.ow, D, tg.lo, tg.scale, tg.bits);
            int lo = 0, hi = tg.ntiles - 1;
            if (tg.seed_tab) {   // the bucket's range: both ends in one round trip
                const uint32_t b = code >> tg.seed_shift;
                lo = tg.seed_tab[b];
                hi = tg.seed_tab[b + 1];
            }
            while (lo < hi) {  // last tile whose first code <= code
                const int mid = (lo + hi + 1) >> 1;
                if (tg.tile_code[mid] <= code) lo = mid;
                else hi = mid - 1;
            }
            seed = lo;
        }

        // displacement bound of any point of this source tile between the pose of pass `bp` (pose ring)
        // and this pass: |dR c + dt| + ||dR||_F rho; < 0 if that pose has left the ring
        auto disp_since = [&](int bp) -> float {
            if (bp < 0 || A.pass - bp <= 0 || A.pass - bp >= kPoseRing) return -1.f;
            const double* Pb = A.poses + (bp % kPoseRing) * 12;
            double dc2 = 0.0, dr2 = 0.0;
#pragma unroll
            for (int a = 0; a < D; ++a) {
                double m = P.t[a] - Pb[9 + a];
#pragma unroll
                for (int b = 0; b < D; ++b) {
                    const double dr = P.R[a * D + b] - Pb[a * 3 + b];
                    m += dr * st.c[b];
                    dr2 += dr * dr;
                }
                dc2 += m * m;
            }
            // an upper bound: fp32 square roots of the rounded sums, covered by the 1.0001 factor
            return (__builtin_amdgcn_sqrtf((float)dc2) + __builtin_amdgcn_sqrtf((float)dr2) * st.radius) * 1.0001f + 1e-30f;
        };

        // ---- per-point nearest-neighbour certificates ------------------------
        // A lane whose last scan proved "target j is nearest and every other target is >= gap farther"
        // (or "no target within R") keeps that answer while its displacement since then, delta, obeys
        // 2 delta < gap (R - delta > d_c: still rejected, gicp.py:136): d(p', j) <= d1 + delta < d2 - delta <= d(p', k).
        // Certified lanes take no part in the walk; a wave whose lanes are all certified skips it.
        bool cert = false;
        int cj = -1;
        float cgap = 0.f, cdelta = -1.f;
        int jp = -1;   // the point's last match (loaded unconditionally: in flight with cert_pass)
        if (A.cert_j) {
            jp = A.cert_j[i];
            const float g0 = A.cert_gap[i];
            cdelta = disp_since(cpass0);
            // (wave-uniform: in 3-D held in a scalar register through the descent and walk -- a vector one was
            // spilled there; the 2-D kernel allocates better without)
            if constexpr (D == 3) cdelta = __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(cdelta)));
            if (cdelta >= 0.f && q.valid) {
                cj = jp;
                cgap = g0;
                cert = cj >= 0 ? 2.f * cdelta < cgap : cgap - cdelta > A.empty_r;
            }
        }
#ifdef GICP_TIMELINE
        S.tb = tl_after(rel.x + cgap, jp);   // the certificates and the point's offset are in
#endif
        // the point relative to its last match jp, fp32 (error well inside the screen margin): the
        // search cap below and the graph descent start from it
        bool have_jp = false;
        float qr[3] = {0.f, 0.f, 0.f}, d2jp = 0.f;
        uint32_t w0[16];   // the first half of jp's graph row (the descent's first step), requested with jp
        if (A.cert_j && q.valid && !cert && jp >= 0 && jp < tg.n) {
            const double4 t4 = reinterpret_cast<const double4*>(tg.xyz64)[jp];
            if (tg.nbq) {
                const uint4* row = tg.nbq + (int64_t)jp * 8;
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    const uint4 v = row[c];
                    w0[4 * c] = v.x;
                    w0[4 * c + 1] = v.y;
                    w0[4 * c + 2] = v.z;
                    w0[4 * c + 3] = v.w;
                }
            }
            const double tv[3] = {t4.x, t4.y, t4.z};
#pragma unroll
            for (int a = 0; a < D; ++a) {
                qr[a] = (float)(q.ow[a] - tv[a]) + q.pw[a];
                d2jp = fmaf(qr[a], qr[a], d2jp);
            }
            have_jp = true;
        }
        // ---- graph descent: nearest neighbour proved from the target graph --------
        // From node j = jp, candidates {j} + row(j).  With b the nearest candidate: any target t nearer
        // to p' than b lies within d(p', j) + d(p', b) of j (triangle inequality), so if that is < r(j)
        // t is a candidate and b is the exact nearest; at a local minimum (b = j) the test is
        // 2 d(p', j) < r(j).  Otherwise hop to b (at most kGraphHops steps) or leave the lane to the
        // walk.  Distances are fp32 on coordinates relative to the node; e bounds their error.  A near
        // tie among candidates (gap <= 2e) is left to the walk (its fp64 tie rules).  The lane's new
        // certificate: every other target is >= min(runner-up, r(j) - d(p', j)) - e away.
        bool gcert = false;
        float ggap = 0.f;
#ifdef GICP_TAIL
        int gwhy = 0;   // diagnostic: how the descent ended for a lane it did not prove
        int gout = 0;   // ... and for one it proved: 1 at the start node's local minimum, 2 at a row entry of
                        // the start node, 3 after a hop, 4 a near tie resolved exactly
#define GICP_WHY(k) (gwhy = (k))
#define GICP_OUT(k) (gout = (k))
#else
#define GICP_WHY(k) ((void)0)
#define GICP_OUT(k) ((void)0)
#endif
        if (tg.nbq && wave_any(have_jp)) {
            bool act = have_jp;
            int node = jp;
            bool tie = false;       // a near tie the row covers: resolved in fp64 below
            int tnode = 0;
            float tfar = 0.f;
            // error of qr so far (absolute, m): its fp32 formation, then each hop's offset and subtraction
            float eq = kGraphErr * (st.radius + __builtin_amdgcn_sqrtf(d2jp));
            for (int h = 0; h < kGraphHops; ++h) {
                if (!wave_any(act)) break;
                if (act) {
                    uint32_t w[32];
                    const uint4* row = tg.nbq + (int64_t)node * 8;
                    // the line in two halves (header + entries 0 .. kGraphHalf - 1, then the rest of line A):
                    // half the registers live
                    auto load_half = [&](int c0) {
#pragma unroll
                        for (int c = c0; c < c0 + 4; ++c) {
                            const uint4 v = row[c];
                            w[4 * c] = v.x;
                            w[4 * c + 1] = v.y;
                            w[4 * c + 2] = v.z;
                            w[4 * c + 3] = v.w;
                        }
                    };
                    if (h == 0) {
#pragma unroll
                        for (int k = 0; k < 16; ++k) w[k] = w0[k];
                    } else {
                        load_half(0);
                    }
                    const float r = __uint_as_float(w[0]), sc = __uint_as_float(w[1]);
                    const float d0s = fmaf(qr[0], qr[0], fmaf(qr[1], qr[1], qr[2] * qr[2]));
                    float b1 = d0s, b2 = 3e38f;
                    int bk = -1;               // the winner's entry (-1: the node itself) ...
                    uint32_t wa = 0u, wb = 0u; // ... and its two dwords (offset and index delta)
                    uint32_t xb[10];           // entries kGraphLineA .. (nbx), read last
                    // entry k's two dwords: 3 int16 offsets, then the int16 index delta
                    auto dwords = [&](int k, uint32_t& a, uint32_t& b) {
                        if (k < kGraphLineA) {
                            a = w[2 + 2 * k];
                            b = w[3 + 2 * k];
                        } else {
                            a = xb[2 * (k - kGraphLineA)];
                            b = xb[2 * (k - kGraphLineA) + 1];
                        }
                    };
                    auto coords = [&](int k, float* c) {
                        uint32_t a, b;
                        dwords(k, a, b);
                        c[0] = (float)(((int)(a << 16)) >> 16);
                        c[1] = (float)((int)a >> 16);
                        c[2] = (float)(((int)(b << 16)) >> 16);
                    };
                    // the winner so far and the runner-up (non-negative floats order like their bits: the
                    // runner-up is the median of {winner, runner-up, new}, one v_med3_u32, no NaN canonicalisation)
                    auto upd = [&](float dd, int k) {
                        const unsigned ud = __float_as_uint(dd), u1 = __float_as_uint(b1);
                        const bool lt = ud < u1;
                        b2 = __uint_as_float(umed3(u1, __float_as_uint(b2), ud));
                        b1 = __uint_as_float(min(u1, ud));
                        if (lt) {
                            bk = k;
                            dwords(k, wa, wb);
                        }
                    };
                    // (an unused entry repeats a real one, k_graph_pack: no validity test here)
                    auto entry = [&](int k) {
                        float c[3];
                        coords(k, c);
                        const float dx = fmaf(-sc, c[0], qr[0]);
                        const float dy = fmaf(-sc, c[1], qr[1]);
                        const float dz = fmaf(-sc, c[2], qr[2]);
                        upd(fmaf(dx, dx, fmaf(dy, dy, dz * dz)), k);
                    };
                    // entries k and k + 1 on packed fp32 (v_pk_fma_f32 / v_pk_mul_f32: half the distance VALU)
                    auto entry2 = [&](int k) {
                        float ca[3], cb[3];
                        coords(k, ca);
                        coords(k + 1, cb);
                        const f2v ms = {-sc, -sc};
                        const f2v dx = __builtin_elementwise_fma(ms, f2v{ca[0], cb[0]}, f2v{qr[0], qr[0]});
                        const f2v dy = __builtin_elementwise_fma(ms, f2v{ca[1], cb[1]}, f2v{qr[1], qr[1]});
                        const f2v dz = __builtin_elementwise_fma(ms, f2v{ca[2], cb[2]}, f2v{qr[2], qr[2]});
                        const f2v dd = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, dz * dz));
                        upd(dd.x, k);
                        upd(dd.y, k + 1);
                    };
                    auto entries = [&](int k0, int k1) {   // entries k0 .. k1 - 1
#pragma unroll
                        for (int k = k0; k + 1 < k1; k += 2) entry2(k);
                        if ((k1 - k0) & 1) entry(k1 - 1);
                    };
                    // |offset| of entry k (quantised): every later entry lies at >= it - s from the node
                    auto reach = [&](int k) -> float {
                        float c[3];
                        coords(k, c);
                        const float ox = sc * c[0], oy = sc * c[1], oz = sc * c[2];
                        return __builtin_amdgcn_sqrtf(fmaf(ox, ox, fmaf(oy, oy, oz * oz)));
                    };
                    entries(0, kGraphHalf);
                    const float d0 = __builtin_amdgcn_sqrtf(d0s);
                    // distance error: qr's, an entry's quantisation (<= s/2 per axis), the arithmetic
                    const float e = eq + 0.87f * sc + kGraphErr * (d0 + r);
                    // The row is sorted nearest-first (k_graph_pack): every entry after entry k lies at
                    // >= reach(k) - s from the node (quantisation), so at >= reach(k) - s - d0 - e from p' and
                    // screens >= lc.  The rest of the row is read only by lanes where such an entry could
                    // still be the nearest or within the tie band of it; elsewhere lc bounds the runner-up
                    // (sound for the gap).
                    float lc = reach(kGraphHalf - 1) - sc - d0 - 2.f * e;
                    bool need = lc <= __builtin_amdgcn_sqrtf(b1) + 2.f * e;
                    if (wave_any(need)) {
                        if (need) {
                            load_half(4);
                            entries(kGraphHalf, kGraphLineA);
                            lc = reach(kGraphLineA - 1) - sc - d0 - 2.f * e;
                            need = lc <= __builtin_amdgcn_sqrtf(b1) + 2.f * e;
                        }
                        if (wave_any(need)) {
                            if (need) {
                                const uint4* rx = tg.nbx + (int64_t)node * 3;
#pragma unroll
                                for (int c = 0; c < 2; ++c) {
                                    const uint4 v = rx[c];
                                    xb[4 * c] = v.x;
                                    xb[4 * c + 1] = v.y;
                                    xb[4 * c + 2] = v.z;
                                    xb[4 * c + 3] = v.w;
                                }
                                const uint2 v2 = *reinterpret_cast<const uint2*>(rx + 2);
                                xb[8] = v2.x;
                                xb[9] = v2.y;
                                entries(kGraphLineA, kGraphK);
                            }
                        }
                    }
                    if (!need) b2 = fminf(b2, lc * lc);
                    // the winner's sorted index without reading nbi, unless its delta did not fit 16 bits
                    auto next_index = [&]() -> int {
                        const int bd = (int)wb >> 16;
                        return bd != kGraphFar ? node + bd : tg.nbi[(int64_t)node * kGraphK + bk];
                    };
                    const float e1 = __builtin_amdgcn_sqrtf(b1), e2 = __builtin_amdgcn_sqrtf(b2);
                    if (e2 - e1 <= 2.f * e) {
                        // near tie: if the row covers it (same test as below), the nearest is one of the
                        // candidates within e1 + 2e, resolved exactly after the loop
                        tie = d0 + e1 + 2.f * e < r;
                        tfar = r - d0 - e;   // every target outside the row is at least this far
                        tnode = node;
                        act = false;                              // else the walk decides
                        if (!tie) GICP_WHY(2);
                    } else if (d0 + e1 + 2.f * e < r) {           // proof (e1 = d0 at a local minimum)
                        gcert = true;
                        GICP_OUT(h > 0 ? 3 : bk < 0 ? 1 : 2);
                        cj = bk < 0 ? node : next_index();
                        ggap = fminf(e2, r - d0) - e1 - 2.f * e;
                        act = false;
                    } else if (bk < 0) {
                        act = false;                              // local minimum without proof
                        GICP_WHY(1);
                    } else {                                      // hop: p' relative to the nearer candidate
                        // (the winner's offset again from its dwords: the same fused multiply-adds as its
                        // distance above)
                        const float c0 = (float)(((int)(wa << 16)) >> 16), c1 = (float)((int)wa >> 16);
                        const float c2 = (float)(((int)(wb << 16)) >> 16);
                        qr[0] = fmaf(-sc, c0, qr[0]);
                        qr[1] = fmaf(-sc, c1, qr[1]);
                        qr[2] = fmaf(-sc, c2, qr[2]);
                        eq = e;
                        node = next_index();
                    }
                }
            }
            if (act) GICP_WHY(3);   // hops exhausted
            // near ties: every candidate of the tie node's row (and the node) exactly in fp64, the nearest
            // by the KD-tree's tie rule (smaller original index); the lane's certificate gap is the exact
            // runner-up among them, or the row's reach when that is nearer
            if (wave_any(tie)) {
                if (tie) {
                    double p64[D];
                    {
                        const double4 s4 = reinterpret_cast<const double4*>(A.src.xyz64)[i];
                        const double s4v[3] = {s4.x, s4.y, s4.z};
#pragma unroll
                        for (int a = 0; a < D; ++a) {
                            double p = P.t[a];
#pragma unroll
                            for (int b = 0; b < D; ++b) p += P.R[a * D + b] * s4v[b];
                            p64[a] = p;
                        }
                    }
                    double bd2 = 1e300, sd2 = 1e300;
                    int bj = -1, bo = 0x7fffffff;
                    auto consider = [&](int t) {
                        const double4 t4 = reinterpret_cast<const double4*>(tg.xyz64)[t];
                        const double tv[3] = {t4.x, t4.y, t4.z};
                        const double d2 = dist2_exact<D>(tv, p64);
                        const int og = tg.perm[t];
                        if (d2 < bd2 || (d2 == bd2 && og < bo)) {
                            sd2 = bd2;
                            bd2 = d2;
                            bj = t;
                            bo = og;
                        } else {
                            sd2 = fmin(sd2, d2);
                        }
                    };
                    consider(tnode);
                    const int32_t* ri = tg.nbi + (int64_t)tnode * kGraphK;
                    for (int k = 0; k < kGraphK; ++k) {
                        const int t = ri[k];
                        if (t >= 0) consider(t);
                    }
                    gcert = bj >= 0;
                    if (gcert) GICP_OUT(4);
                    cj = bj;
                    const double g = (fmin(sqrt(sd2), (double)tfar) - sqrt(bd2)) * (1.0 - 1e-6) - 1e-12;
                    ggap = g > 0.0 ? (float)g * (1.0f - 1e-6f) : 0.f;
                }
            }
            if (gcert) {
                cert = true;
                cgap = ggap;
            }
        }
        const bool any_gcert = wave_any(gcert);
        const bool skip_walk = !wave_any(q.valid && !cert);
#ifdef GICP_TAIL
        if (A.tail) {   // how searches ended (per-wave counts into the workgroup's LDS, one global add per
                        // workgroup at its end): [9] lanes that descended, [10..13] proved by gout 1..4,
                        // [14] walking lanes, [15] walking waves
            const bool wl = q.valid && !cert;
            const uint64_t wm = __ballot(wl);
            const int cd = __popcll(__ballot(have_jp));
            if (l == 0 && cd) atomicAdd(&s_walk[0], (unsigned)cd);
            for (int k = 1; k <= 4; ++k) {
                const int c = __popcll(__ballot(gout == k));
                if (l == 0 && c) atomicAdd(&s_walk[k], (unsigned)c);
            }
            if (l == 0 && wm) {
                atomicAdd(&s_walk[5], (unsigned)__popcll(wm));
                atomicAdd(&s_walk[6], 1u);
            }
            (void)gwhy;
        }
#endif
        ngproved = __popcll(__ballot(gcert));
        nwalked = skip_walk ? 0 : 1;
#ifdef GICP_TIMELINE
        S.tdesc = tl_after(ngproved, (int)skip_walk);
        S.ndesc = (unsigned)__popcll(__ballot(have_jp));
        S.nwalk = (unsigned)__popcll(__ballot(q.valid && !cert));
        S.nwalk_jp = (unsigned)__popcll(__ballot(q.valid && !cert && have_jp));
#endif
        // the widening pays only if the next pass moves the tile by less than kappa / 2: a tile that moved
        // farther than kappa since its last pass (the pose is still converging) walks without it
        const float kap = cdelta > A.kappa ? 0.f : A.kappa;

        // ---- fp32 screen: best and runner-up keys -------------------------
        const unsigned init = __float_as_uint(A.search2) | 63u;
        unsigned best = init, sec = init;
        int best_tile = -1;
        // the bound as a function of the winner's screened d2 b: the winner plus the screen's ambiguity
        // band, widened to (sqrt(b) + kappa)^2 when certificates are kept (runner-up gap known up to kappa)
        auto bound_of = [&](float b) -> float {
            const float w = b + 2.f * marg(A.mg, b);
            const float r = __builtin_amdgcn_sqrtf(b) + kap;
            return fmaxf(w, r * r);
        };
        // Search cap from the last pass's match jp of this point (any target bounds the nearest's
        // distance): d2 to jp estimated in fp32 (error within the screen margin, like the screen's own),
        // so the screened winner's d2 is <= b0 = d2 + 2 margin and the bound the walk would end with is
        // <= bound_of(b0).  Lanes start the walk at that radius instead of the screen radius; every row
        // within the final bound is still scanned, so the result is unchanged (bit-identical, tested).
        float cap = 3e38f;
        if (have_jp && !cert && !skip_walk) cap = bound_of(d2jp + 2.f * marg(A.mg, d2jp)) * 1.0001f;
        // lane search bound: the runner-up, or bound_of(winner), within the cap
        auto lane_bound = [&]() -> float {
            if (!q.valid || cert) return -1.f;
            return fminf(cap, fminf(key_d2(sec), bound_of(key_d2(best))));
        };
        float lb = lane_bound();   // refreshed after every merge
#ifdef GICP_TIMELINE
        S.wb0 = __builtin_amdgcn_sqrtf(fmaxf(wave_maxf(lb), 0.f));
#endif
        // lb inflated by the rounding slack, for the slack-free box tests
        auto inflate = [&](float w) -> float {
            if (w < 0.f) return w;
            const float r = __builtin_amdgcn_sqrtf(w) * 1.0001f + 2.f * A.gap_slack;
            return r * r;
        };
        float lbx = inflate(lb);
        // lane k: list entry k once the list walk has visited it; a full walk that continues a list walk
        // whose certificate failed skips those tiles (their rows are already in every lane's best and
        // runner-up; -1 elsewhere, so no other walk skips anything)
        int lvis = -1;
        // visit target tile Tt; `pre` = its coordinates already loaded (prefetch) or null
        auto visit_pre = [&](int Tt, const float4* pre) -> bool {
            if (wave_any(lvis == Tt)) return false;
            S.mark(1);
            S.count(0);
            const TileInfo ti = tile_meta(tg, Tt);
            float pr[D];
            // lbx < 0 on lanes without a query: one compare per test
            if (!wave_any(lane_gap2_ns<D>(q, ti, pr) <= lbx)) {
                S.mark(2);
                return false;
            }
            const unsigned sub = sub_mask_ns<D>(ti, pr, lbx);
            if (pre) stage_f32_from(*pre, L);
            else stage_f32(tg, ti, L);
            S.mark(2);
            unsigned tb = 0xFFFFFFFFu, ts = 0xFFFFFFFFu;
            scan_tile<D>(L, ti.count, pr, [&](unsigned key, int) {
                ts = umed3(tb, ts, key);
                tb = min(tb, key);
            }, sub);
            pairs += rows_scanned(sub, ti.count);
            S.count(1);
            S.count(2, __popc(sub));
            if (tb < best) {
                sec = min(best, ts);
                best = tb;
                best_tile = Tt;
            } else {
                sec = min(sec, tb);
            }
            lb = lane_bound();
            lbx = inflate(lb);
            wave_sync();
            S.mark(3);
            return true;
        };
        S.mark(0);
        // candidate list of this source tile: usable if built within the pose ring and the tile's
        // displacement since then is inside the certified radius
        bool use = false;
        float delta = 0.f, rc = 0.f;
        int nl = 0;
        if (lists && !skip_walk) {
            nl = A.list_len[T];
            rc = A.list_rcert[T];
            if (nl > 0 && rc > 0.f) {
                delta = disp_since(A.list_pass[T]);
                use = delta >= 0.f && delta < rc;
            }
        }
        int ent = 0;   // lane k: list entry k (when the list is used)

        // ---- sparse waves: a lane-parallel search per walking lane ----------------
        // A wave with a few walking lanes (most of passes 4-19's walking waves have one) walked one visit
        // per tile, one dependent memory round trip each, its lanes all screening rows for one or two
        // points.  Here, for one walking lane at a time: its candidate tiles (the source tile's certified
        // list when that covers the lane, else the super-block / block / tile boxes) are screened
        // kSparseGroup tiles per round trip with lane r holding row r of each tile (coalesced, no LDS),
        // every row keyed exactly as scan_tile keys it, the per-lane best and runner-up merged over the
        // wave after each group (whose new bound prunes the remaining candidates).  Exact: every tile whose
        // box is within the lane's bound is screened in full and the bound only shrinks; the list is
        // neither used past its certificate nor rebuilt (it stays valid for its own pose).
        const uint64_t walkers = skip_walk ? 0ull : __ballot(lb >= 0.f);
        const bool sparse = walkers != 0ull && __popcll(walkers) <= A.sparse_max;
        auto sparse_search = [&](int wl) {
            float pw[D];
#pragma unroll
            for (int a = 0; a < D; ++a) pw[a] = readlane_f(q.pw[a], wl);
            // the walking lane's point as a box: what active_box<D>(q, l == wl) gives for one lane (centre ow + pw,
            // half-extent its padding for pw's rounding, 4.8e-7 (|lo| + |hi| + 2 ew)), without its wave reductions
            Query<D> qp = q;
#pragma unroll
            for (int a = 0; a < D; ++a) {
                const float B = 2.f * q.ew[a] + 1e-30f;
                qp.ow[a] = q.ow[a] + (double)pw[a];
                qp.ew[a] = 4.8e-7f * (2.f * fabsf(pw[a]) + B) + 1e-30f;
            }
            const float capw = readlane_f(cap, wl);
            float wb = readlane_f(lb, wl);
            unsigned tb = init, ts = init;   // lane r: the best and runner-up key of row r over the tiles screened
            int tt = -1;                      // ... and the tile of its best
            unsigned wbest = init, wsec = init;
            int wtile = -1;
            const unsigned M = key_mask();
            auto reduce = [&]() {
                wbest = wave_min_key(tb);
                const int win = __ffsll((unsigned long long)__ballot(tb == wbest)) - 1;
                wsec = wave_min_key(l == win ? ts : tb);
                wtile = __builtin_amdgcn_readlane(tt, win);
                wb = fminf(capw, fminf(key_d2(wsec), bound_of(key_d2(wbest))));
            };
            // the candidates held by the lanes of `cm` (lane k: tile ct, rows cst .. cst + ccnt, co = the fp32 offset
            // (float)(ow - c) of the tile's centre c -- the term lane_gap2_ns adds to a lane's pw --, box gap cg)
            auto screen = [&](uint64_t cm, int ct, int cst, int ccnt, const float* co, float cg) {
                cm &= __ballot(cg <= wb);
                while (cm) {
                    int ks[kSparseGroup];
                    float rx[kSparseGroup], ry[kSparseGroup], rz[kSparseGroup];
#pragma unroll
                    for (int u = 0; u < kSparseGroup; ++u) {   // the group's rows, all requested before any is used
                        const int k = cm ? __ffsll((unsigned long long)cm) - 1 : -1;
                        ks[u] = k;
                        rx[u] = ry[u] = rz[u] = 1e30f;
                        if (k >= 0) {
                            cm &= cm - 1;
                            const int st0 = __builtin_amdgcn_readlane(cst, k), cn = __builtin_amdgcn_readlane(ccnt, k);
                            if (l < cn) {
                                const float* rp = reinterpret_cast<const float*>(tg.rel32 + st0 + l);
                                rx[u] = rp[0];
                                ry[u] = rp[1];
                                if (D == 3) rz[u] = rp[2];
                            }
                            pairs += cn;
                            S.count(0);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < kSparseGroup; ++u) {
                        const int k = ks[u];
                        if (k < 0) break;
                        float pr[3] = {0.f, 0.f, 0.f};
#pragma unroll
                        for (int a = 0; a < D; ++a) pr[a] = pw[a] + readlane_f(co[a], k);
                        const float dx = pr[0] - rx[u], dy = pr[1] - ry[u];
                        float d2 = fmaf(dy, dy, dx * dx);
                        if (D == 3) {
                            const float dz = pr[2] - rz[u];
                            d2 = fmaf(dz, dz, d2);
                        }
                        const unsigned key = (__float_as_uint(d2) & M) | (unsigned)l;
                        ts = umed3(tb, ts, key);
                        if (key < tb) tt = __builtin_amdgcn_readlane(ct, k);
                        tb = min(tb, key);
                    }
                    reduce();
                    cm &= __ballot(cg <= wb);
                }
            };
            bool covered = false;
            if (use) {   // the list's entries near this lane, then whether the list covers its final bound
                int lt = 0, lst = 0, lcn = 0;
                float lc[3] = {0.f, 0.f, 0.f};
                float lg = 3e38f;
                if (l < nl) {
                    lt = A.list[(int64_t)T * kListMax + l];
                    const TileBox tbx = tg.boxes[lt];
                    lg = gap2_box<D>(qp, tbx.c, tbx.h);
#pragma unroll
                    for (int a = 0; a < D; ++a) lc[a] = (float)(q.ow[a] - tbx.c[a]);
                    lst = tbx.start;
                    lcn = tbx.count;
                }
                screen(__ballot(l < nl), lt, lst, lcn, lc, lg);
                covered = __builtin_amdgcn_sqrtf(fmaxf(wb, 0.f)) * 1.0001f + delta <= rc;
                if (covered) S.count(3);
                if (!covered) {   // start over with the bound the list gave (every tile within it is rescreened)
                    tb = ts = init;
                    tt = -1;
                }
            }
            if (!covered) {   // super-blocks -> blocks -> tiles against the lane's box, as walk_c
                const int nsuper = (tg.nblocks + kWave - 1) / kWave;
                for (int s0 = 0; s0 < nsuper; s0 += kWave) {
                    float sg = 3e38f;
                    if (s0 + l < nsuper) sg = gap2_box<D>(qp, tg.blocks[tg.nblocks + s0 + l].c, tg.blocks[tg.nblocks + s0 + l].h);
                    uint64_t sm = __ballot(sg <= wb);
                    while (sm) {
                        const int sl = __ffsll((unsigned long long)sm) - 1;
                        sm &= sm - 1;
                        if (!(readlane_f(sg, sl) <= wb)) continue;
                        S.count(5);
                        const int b0 = (s0 + sl) * kWave, b = b0 + l;
                        float bg = 3e38f;
                        if (b < tg.nblocks) bg = gap2_box<D>(qp, tg.blocks[b].c, tg.blocks[b].h);
                        uint64_t bm = __ballot(bg <= wb);
                        while (bm) {
                            const int bl = __ffsll((unsigned long long)bm) - 1;
                            bm &= bm - 1;
                            if (!(readlane_f(bg, bl) <= wb)) continue;
                            S.count(6);
                            const int first = (b0 + bl) * kBlockTiles, nt = min(kBlockTiles, tg.ntiles - first);
                            int ht = first + l, hst = 0, hcn = 0;
                            float hc[3] = {0.f, 0.f, 0.f};
                            float hg = 3e38f;
                            if (l < nt) {
                                const TileBox tbx = tg.boxes[ht];
                                hg = gap2_box<D>(qp, tbx.c, tbx.h);
#pragma unroll
                                for (int a = 0; a < D; ++a) hc[a] = (float)(q.ow[a] - tbx.c[a]);
                                hst = tbx.start;
                                hcn = tbx.count;
                            }
                            screen(__ballot(l < nt), ht, hst, hcn, hc, hg);
                        }
                    }
                }
            }
            if (l == wl) {
                best = wbest;
                sec = wsec;
                best_tile = wtile;
            }
        };
        if (sparse) {
            uint64_t wm = walkers;
            while (wm) {
                const int wl = __ffsll((unsigned long long)wm) - 1;
                wm &= wm - 1;
                sparse_search(wl);
            }
            lb = lane_bound();
            lbx = inflate(lb);
        }
        const bool use_sparse = sparse;   // (the walk's kind, diagnostics)
        if (sparse) use = false;
        if (use) {
            S.count(3);
            S.count(4, nl);
            // lane k holds list entry k: its box gap to the wave box, start and count
            int est = 0, ecnt = 0;
            float eg2 = 3e38f;
            const Query<D> qa = active_box<D>(q, lb >= 0.f);   // the searching lanes' box
            if (l < nl) {
                ent = A.list[(int64_t)T * kListMax + l];
                const TileBox eb = tg.boxes[ent];   // the 48-B record (TileInfo's fields are 144 B apart)
                eg2 = gap2_box<D>(qa, eb.c, eb.h);
                est = eb.start;
                ecnt = eb.count;
            }
            float wb = wave_maxf(lb);
            uint64_t rem = __ballot(l < nl && eg2 <= wb);
            // nearest remaining entry (wave-uniform lane index), -1 if none
            // lists are stored nearest-first (sorted when built): the next entry is the lowest set bit
            auto pick = [&]() -> int { return rem ? __ffsll((unsigned long long)rem) - 1 : -1; };
            int k = pick();
            float4 pv = make_float4(0.f, 0.f, 0.f, 0.f);
            if (k >= 0) pv = load_rel(tg, __builtin_amdgcn_readlane(est, k), __builtin_amdgcn_readlane(ecnt, k));
            while (k >= 0) {
                rem &= ~(1ull << k);
                const int kn = pick();   // prefetch the next-nearest while this one is scanned
                float4 pvn = make_float4(0.f, 0.f, 0.f, 0.f);
                if (kn >= 0) pvn = load_rel(tg, __builtin_amdgcn_readlane(est, kn), __builtin_amdgcn_readlane(ecnt, kn));
                if (visit_pre(__builtin_amdgcn_readlane(ent, k), &pv)) {
                    wb = wave_maxf(lb);
                    rem &= __ballot(eg2 <= wb);
                }
                if (l == k) lvis = ent;
                if (kn >= 0 && ((rem >> kn) & 1ull)) {
                    k = kn;
                    pv = pvn;
                } else {
                    k = pick();
                    if (k >= 0) pv = load_rel(tg, __builtin_amdgcn_readlane(est, k), __builtin_amdgcn_readlane(ecnt, k));
                }
            }
            const float wbf = wave_maxf(lb);
            if (__builtin_amdgcn_sqrtf(fmaxf(wbf, 0.f)) * 1.0001f + delta > rc) {
                // not certified: the full walk (which rebuilds the list) continues from the list walk's
                // best, runner-up and bounds and skips the tiles the list walk visited: each lane's result
                // is still the minimum over every row within its final bound, and a row never scanned
                // lies beyond the bound its tile or sub-tile was tested against, which only shrank
                use = false;
                ++list_rebuilds;
            }
        }
        if (!use && !skip_walk && !sparse) {
            float skin = A.skin;   // adaptive: a moving tile's list covers a step like its last one
            if (lists && A.skin_gain > 0.f) {
                const float dl = disp_since(A.pass - 1);
                if (dl > 0.f) skin = fminf(fmaxf(skin, A.skin_gain * dl), A.skin_max);
            }
            int ncol = 0;
            int cent = 0x7fffffff;   // lane k: collected entry k
            auto collect = [&](int Tt) {
                if (l == ncol) cent = Tt;
                ++ncol;
            };
            walk_c<D>(tg, q, seed, visit_pre, [&]() { return wave_maxf(lb); }, lists ? skin : 0.f,
                      collect, &S);
            if (lists) {
                const float wbf = wave_maxf(lb);
                const float r = ncol <= kListMax ? __builtin_amdgcn_sqrtf(fmaxf(wbf, 0.f)) * 0.9999f + skin : 0.f;
                if (ncol <= kListMax) {   // store nearest-first: by centre distance to the wave box
                    float key = 3e38f;
                    if (l < ncol) {
                        key = 0.f;
#pragma unroll
                        for (int a = 0; a < D; ++a) {
                            const float d = (float)(tg.boxes[cent].c[a] - q.ow[a]);
                            key = fmaf(d, d, key);
                        }
                    }
                    wave_sort64(key, cent);
                    if (l < ncol) A.list[(int64_t)T * kListMax + l] = cent;
                }
                if (l == 0) {
                    A.list_len[T] = min(ncol, kListMax);
                    A.list_rcert[T] = r;
                    A.list_pass[T] = A.pass;
                }
            }
        }
        S.mark(1);
#ifdef GICP_TIMELINE
        S.twalk = tl_after(best, best_tile);
        S.kind = skip_walk ? 0u : use_sparse ? 4u : use ? 1u : list_rebuilds > 0 ? 2u : 3u;
#endif

        // the fp64 source point is needed only from here on (kept out of the walk's registers).  A wave
        // that walked needs it now (fp64 fallback); one that skipped the walk requests it with its
        // matches and covariances in the epilogue: one memory round trip instead of two
        // the transformed point q.p64 (the untransformed one, sv, a statistics term, is set from the epilogue's
        // own request of the point: held from here it was spilled through the fp64 re-resolution)
        auto source_point = [&](const double4& s4) {
            const double s4v[3] = {s4.x, s4.y, s4.z};
#pragma unroll
            for (int a = 0; a < D; ++a) {
                double p = P.t[a];
#pragma unroll
                for (int b = 0; b < D; ++b) p += P.R[a * D + b] * s4v[b];
                q.p64[a] = p;
            }
        };
        refresh_i();
        if (!skip_walk) source_point(reinterpret_cast<const double4*>(sc.xyz64)[i]);
        const bool found = cert ? cj >= 0 : (q.valid && best < init);
        int j = -1;
        double d2e = 0.0;
        if (cert) {
            j = cj;
        } else if (found) {
            const float b = key_d2(best), s2 = key_d2(sec);
            amb = (s2 - b) <= marg(A.mg, b) + marg(A.mg, s2);
            j = tg.boxes[best_tile].start + (int)(best & 63u);
        }
        // Every lane's certificate is restated relative to this pass's pose where the wave walked; a wave
        // that skipped the walk leaves its certificates (and cert_pass) as they are: they stay relative to
        // the older pose, whose direct displacement to later poses is no larger than the summed steps,
        // and the pass writes nothing for it -- until that pose is half the pose ring old.
        if (A.cert_j && (!skip_walk || any_gcert || A.pass - cpass0 >= kPoseRing / 2)) {
            if (q.valid) {
                float g = 0.f;
                if (gcert) {
                    g = cgap;   // proved at this pass's pose
                } else if (cert) {
                    g = cj >= 0 ? cgap - 2.f * cdelta : cgap - cdelta;
                } else if (found) {
                    if (!amb) {   // other targets: scanned >= sec - margin, unscanned > the final bound
                        const float b = key_d2(best), s2 = key_d2(sec);
                        const float lo2 = fminf(s2 - marg(A.mg, s2), lane_bound());
                        const float hi2 = b + marg(A.mg, b);
                        g = (__builtin_amdgcn_sqrtf(fmaxf(lo2, 0.f)) - __builtin_amdgcn_sqrtf(hi2)) * 0.999f;
                    }
                } else {   // nothing within the screen radius: every target's d^2 >= search2 - margin
                    g = __builtin_amdgcn_sqrtf(A.search2 - marg(A.mg, A.search2)) * 0.9999f;
                }
                A.cert_j[i] = cert ? cj : (found && !amb ? j : -1);
                A.cert_gap[i] = (found && amb) ? 0.f : g;
            }
            if (l == 0) A.cert_pass[T] = A.pass;
        }
        // hint for the next pass: the first lane's winning tile
        const uint64_t fm = __ballot(found && !cert);
        if (fm && A.hint) {
            const int src_lane = __ffsll((unsigned long long)fm) - 1;
            const int bt = __shfl(best_tile, src_lane);
            if (l == 0) A.hint[T] = bt;
        }

        // ---- fp64 re-resolution of the lanes the screen could not decide ----
        if (!skip_walk && __any(amb)) {
            double bd2 = 1e300;   // exact best d^2 among the rows scanned
            float sd2 = 3e38f;    // runner-up d^2, rounded down (a lower bound is all a certificate needs)
            int bj = -1;   // its sorted index; the original index (tie-break) is read only on exact ties
            const float lim = key_d2(best) + 2.f * marg(A.mg, key_d2(best));
            auto visit64 = [&](int Tt) -> bool {
                const TileInfo ti = tile_meta(tg, Tt);
                float pr[D];
                const bool need = amb && lane_gap2<D>(q, ti, pr) <= lim;
                if (!__any(need)) return false;
                S.count(7);
                const unsigned sub = sub_mask<D>(ti, pr, amb, lim);
                stage_f64(tg, ti, L);
                if (l < ti.count) L.t.perm[l] = tg.perm[ti.start + l];
                wave_sync();
                for (int g = 0; g < kSub; ++g) {
                    if (!((sub >> g) & 1u)) continue;
                    const int je = min(kSubRows * g + kSubRows, ti.count);
#pragma unroll 4
                    for (int jj = kSubRows * g; jj < je; ++jj) {
                        const double qq[3] = {L.t.x64[jj], L.t.y64[jj], L.t.z64[jj]};
                        const double d2 = dist2_exact<D>(qq, q.p64);
                        const int og = L.t.perm[jj];
                        if (amb) {
                            if (d2 < bd2 || (d2 == bd2 && bj >= 0 && og < tg.perm[bj])) {
                                sd2 = (float)bd2 * 0.99999976f;
                                bd2 = d2;
                                bj = ti.start + jj;
                            } else {
                                sd2 = fminf(sd2, (float)d2 * 0.99999976f);
                            }
                        }
                    }
                }
                wave_sync();
                return true;
            };
            const uint64_t am = __ballot(amb);
            if (__popcll(am) <= A.sparse_amb) {
                // few re-resolved lanes (the usual case): for one at a time, its candidate tiles -- every tile
                // whose box lies within lim of the lane's point, from the super-block / block / tile boxes as the
                // sparse search finds them -- are screened exactly with lane r holding row r of a tile (one
                // memory round trip per tile, no staging, no row loop), the tile's nearest by the tie
                // rule and its runner-up taken over the wave.  Same nearest as visit64 (the exact minimum over
                // a superset of the rows within lim, ties to the smaller original index); the runner-up may
                // also count rows beyond lim, which only the (sound) certificate gap sees.
                uint64_t wm = am;
                while (wm) {
                    const int wl = __ffsll((unsigned long long)wm) - 1;
                    wm &= wm - 1;
                    double pa[3] = {0.0, 0.0, 0.0};
                    Query<D> qp = q;
#pragma unroll
                    for (int a = 0; a < D; ++a) {
                        pa[a] = readlane_d(q.p64[a], wl);
                        const float pw = readlane_f(q.pw[a], wl);
                        const float B = 2.f * q.ew[a] + 1e-30f;
                        qp.ow[a] = q.ow[a] + (double)pw;
                        qp.ew[a] = 4.8e-7f * (2.f * fabsf(pw) + B) + 1e-30f;
                    }
                    const float limw = readlane_f(lim, wl);
                    double ub = 1e300;            // the lane's exact best d^2 so far (uniform) ...
                    int uo = 0x7fffffff, uj = -1; // ... its original and sorted index
                    float us = 3e38f;             // ... and the runner-up, rounded down as visit64 rounds it
                    // the tiles of the lanes in cm (lane k: start ts, count tc), one per round trip
                    auto screen64 = [&](uint64_t cm, int ts, int tc) {
                        while (cm) {
                            const int k = __ffsll((unsigned long long)cm) - 1;
                            cm &= cm - 1;
                            const int s0 = __builtin_amdgcn_readlane(ts, k), c0 = __builtin_amdgcn_readlane(tc, k);
                            S.count(7);
                            double d2 = 1e300;
                            int og = 0x7fffffff;
                            if (l < c0) {
                                const double4 x = reinterpret_cast<const double4*>(tg.xyz64)[s0 + l];
                                og = tg.perm[s0 + l];
                                const double xv[3] = {x.x, x.y, x.z};
                                d2 = dist2_exact<D>(xv, pa);
                            }
                            const double m = wave_mind(d2);
                            const uint64_t eq = __ballot(d2 == m);
                            const int om = (int)wave_min_key(d2 == m ? (unsigned)og : 0x7fffffffu);
                            const int wn = __ffsll((unsigned long long)__ballot(d2 == m && og == om)) - 1;
                            const double st = __popcll(eq) >= 2 ? m : wave_mind(l == wn ? 1e300 : d2);
                            if (m < ub || (m == ub && om < uo)) {
                                us = fminf(us, fminf((float)ub * 0.99999976f, (float)st * 0.99999976f));
                                ub = m;
                                uo = om;
                                uj = s0 + wn;
                            } else {
                                us = fminf(us, (float)m * 0.99999976f);
                            }
                        }
                    };
                    const int nsuper = (tg.nblocks + kWave - 1) / kWave;
                    for (int s0 = 0; s0 < nsuper; s0 += kWave) {
                        float sg = 3e38f;
                        if (s0 + l < nsuper) sg = gap2_box<D>(qp, tg.blocks[tg.nblocks + s0 + l].c, tg.blocks[tg.nblocks + s0 + l].h);
                        uint64_t sm = __ballot(sg <= limw);
                        while (sm) {
                            const int sl = __ffsll((unsigned long long)sm) - 1;
                            sm &= sm - 1;
                            const int b0 = (s0 + sl) * kWave, b = b0 + l;
                            float bg = 3e38f;
                            if (b < tg.nblocks) bg = gap2_box<D>(qp, tg.blocks[b].c, tg.blocks[b].h);
                            uint64_t bm = __ballot(bg <= limw);
                            while (bm) {
                                const int bl = __ffsll((unsigned long long)bm) - 1;
                                bm &= bm - 1;
                                const int first = (b0 + bl) * kBlockTiles, nt = min(kBlockTiles, tg.ntiles - first);
                                int hst = 0, hcn = 0;
                                float hg = 3e38f;
                                if (l < nt) {
                                    const TileBox tbx = tg.boxes[first + l];
                                    hg = gap2_box<D>(qp, tbx.c, tbx.h);
                                    hst = tbx.start;
                                    hcn = tbx.count;
                                }
                                screen64(__ballot(l < nt && hg <= limw), hst, hcn);
                            }
                        }
                    }
                    if (l == wl) {
                        bd2 = ub;
                        sd2 = us;
                        bj = uj;
                    }
                }
            } else if (use) {   // the certified candidate list covers every tile within lb >= lim
                const Query<D> qb = active_box<D>(q, amb);   // entries near the re-resolved lanes only
                bool near = false;
                const float limw = wave_maxf(amb ? lim : -1.f);
                if (l < nl) near = gap2_box<D>(qb, tg.boxes[ent].c, tg.boxes[ent].h) <= limw;
                uint64_t em = __ballot(near);
                while (em) {
                    const int k = __ffsll((unsigned long long)em) - 1;
                    em &= em - 1;
                    visit64(__builtin_amdgcn_readlane(ent, k));
                }
            } else {
                // candidate tiles against the box of the re-resolved lanes only (not the whole source
                // tile's), found as the full walk finds them (TileBox records, one round trip per level);
                // visit64's per-lane test decides what is scanned, so the result does not depend on it
                const Query<D> qb = active_box<D>(q, amb);
                walk_c<D>(tg, qb, seed, [&](int Tt, const float4*) { return visit64(Tt); },
                          [&]() { return wave_maxf(amb ? lim : -1.f); }, 0.f, [](int) {});
            }
            if (amb) j = bj;
            // exact certificate of a re-resolved lane: every row within lim was scanned in fp64, so
            // each other target lies at d^2 >= min(runner-up, lim); a near tie certifies only while
            // the pose moves by less than half its (tiny, possibly zero) gap
            if (A.cert_j && amb) {
                const double g = (sqrt((double)fminf(sd2, lim)) - sqrt(bd2)) * (1.0 - 1e-6) - 1e-12;
                A.cert_j[i] = bj;
                A.cert_gap[i] = g > 0.0 ? (float)g * (1.0f - 1e-6f) : 0.f;
            }
        }

        S.mark(4);
        // ---- epilogue: distance check, W = inv(R C_s R^T + C_t), statistics --
        const double4 s4e = reinterpret_cast<const double4*>(sc.xyz64)[i];
        sv[0] = s4e.x;
        sv[1] = s4e.y;
        if (D == 3) sv[D - 1] = s4e.z;
        if (found && j >= 0) {
            // match position and both covariances requested together (one memory round trip)
            const double4 q4 = reinterpret_cast<const double4*>(tg.xyz64)[j];
            const double4 ct = tg.cov[j];
            const double4 cs = sc.cov[i];
            if (skip_walk) source_point(s4e);
            const double qv[3] = {q4.x, q4.y, q4.z};
            d2e = dist2_exact<D>(qv, q.p64);
#ifdef GICP_TIMELINE
            S.te = tl_after(d2e, ct.x + cs.x);   // the epilogue's gathers are in
#endif
            if (A.dbg_dist) A.dbg_dist[sc.perm[i]] = sqrt(d2e);
            // gicp.py:136: reject only if distance > d_c; sqrt(d2) > d_c <=> d2 > dc2_max (host-computed,
            // sqrt is correctly rounded and monotone), so no square root here
            if (d2e <= A.dc2_max) {
                on = true;
                const double mt[3] = {ct.y, ct.z, ct.w};
                if (A.cov_model == GICP_COV_POINT_TO_POINT) {          // C_s = 0, C_t = I: W = I
#pragma unroll
                    for (int a = 0; a < D; ++a)
#pragma unroll
                        for (int b = 0; b < D; ++b) W[a][b] = a == b ? 1.0 : 0.0;
                } else if (A.cov_model == GICP_COV_POINT_TO_PLANE) {   // W = n_t n_t^T, n = m / |m|_model
#pragma unroll
                    for (int a = 0; a < D; ++a)
#pragma unroll
                        for (int b = 0; b < D; ++b) W[a][b] = mt[a] * mt[b] * A.pl_inv;
                } else {
                const double ms[3] = {cs.y, cs.z, cs.w};
                double mr[D];
#pragma unroll
                for (int a = 0; a < D; ++a) {
                    mr[a] = 0.0;
#pragma unroll
                    for (int b = 0; b < D; ++b) mr[a] += P.R[a * D + b] * ms[b];
                }
                double S[D][D];
#pragma unroll
                for (int a = 0; a < D; ++a)
#pragma unroll
                    for (int b = 0; b < D; ++b)
                        S[a][b] = (a == b ? cs.x + ct.x : 0.0) - mr[a] * mr[b] - mt[a] * mt[b];
                if constexpr (D == 2) {
                    const double det = S[0][0] * S[1][1] - S[0][1] * S[1][0];
                    const double id = solver_detail::recip(det);
                    W[0][0] = S[1][1] * id;
                    W[1][1] = S[0][0] * id;
                    W[0][1] = W[1][0] = -S[0][1] * id;
                } else {
                    const double c00 = S[1][1] * S[2][2] - S[1][2] * S[2][1];
                    const double c01 = S[0][2] * S[2][1] - S[0][1] * S[2][2];
                    const double c02 = S[0][1] * S[1][2] - S[0][2] * S[1][1];
                    const double c11 = S[0][0] * S[2][2] - S[0][2] * S[2][0];
                    const double c12 = S[0][2] * S[1][0] - S[0][0] * S[1][2];
                    const double c22 = S[0][0] * S[1][1] - S[0][1] * S[1][0];
                    const double det = S[0][0] * c00 + S[0][1] * c01 + S[0][2] * c02;
                    const double id = solver_detail::recip(det);   // (refined v_rcp_f64, within ~1 ulp)
                    W[0][0] = c00 * id;
                    W[0][1] = W[1][0] = c01 * id;
                    W[0][2] = W[2][0] = c02 * id;
                    W[1][1] = c11 * id;
                    W[1][2] = W[2][1] = c12 * id;
                    W[2][2] = c22 * id;
                }
                }   // plane-to-plane
                double r[D];
#pragma unroll
                for (int a = 0; a < D; ++a) r[a] = qv[a] - q.p64[a];
                r2 = 0.0;
#pragma unroll
                for (int a = 0; a < D; ++a) r2 += r[a] * r[a];
                rwr = 0.0;
#pragma unroll
                for (int a = 0; a < D; ++a) {
                    wr[a] = 0.0;
#pragma unroll
                    for (int b = 0; b < D; ++b) wr[a] += W[a][b] * r[b];
                    rwr += r[a] * wr[a];
                }
            }
            if (A.dbg_index) A.dbg_index[sc.perm[i]] = on ? (int64_t)tg.perm[j] : -1;
        } else if (q.valid) {
            if (skip_walk) source_point(s4e);
            if (A.dbg_index) A.dbg_index[sc.perm[i]] = -1;
            if (A.dbg_dist) A.dbg_dist[sc.perm[i]] = 1.0 / 0.0;
        }
        if (A.dbg_det && q.valid) {   // det(W) for gicp_top_weights (gicp.py:170), 0 if rejected
            double dt = 0.0;
            if (on) {
                if constexpr (D == 2) dt = W[0][0] * W[1][1] - W[0][1] * W[1][0];
                else
                    dt = W[0][0] * (W[1][1] * W[2][2] - W[1][2] * W[2][1]) -
                         W[0][1] * (W[1][0] * W[2][2] - W[1][2] * W[2][0]) +
                         W[0][2] * (W[1][0] * W[2][1] - W[1][1] * W[2][0]);
            }
            A.dbg_det[i] = dt;   // sorted order (coalesced); the top-k maps its winners through perm
            A.top_tgt[i] = on ? (int64_t)tg.perm[j] : -1;
        }
        if (A.dbg_weight && q.valid) {
            double* o = A.dbg_weight + (int64_t)sc.perm[i] * D * D;
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int b = 0; b < D; ++b) o[a * D + b] = on ? W[a][b] : 0.0;
        }
        amb = amb && q.valid;
    }

    S.mark(5);
    // ---- wave reduction of the statistics: a 16x16x64 fp64 GEMM on MFMA ---------------------
    // stats[p][q] = sum over lanes of u_p v_q with u = (W sym, W r, r^T W r, 1, |r|^2), v = (s s sym, s,
    // 1).  Points are transposed through LDS 16 at a time as u[term][point] /
    // v[term][point]: lane = point writes its terms to one column (every address a constant offset of
    // one base, no per-write address arithmetic), lane l reads A[p = l&15][k = l>>4] /
    // B[k][q = l&15] of v_mfma_f64_16x16x4_f64 from row l&15 at a constant offset per MFMA.
    {
        constexpr int NS = D * (D + 1) / 2;
        constexpr int NU = NS + D + 3;   // u terms in use (the rest of the 16 rows stay zero)
        constexpr int NV = NS + D + 1;   // v terms in use
        // u_k / v_k of this lane's point, formed at the write (k is a compile-time constant there)
        // W, W r and r^T W r are exact zeros unless `on` (never written otherwise), so only the count
        // entry of u needs the mask: a rejected or padding lane's u is 0 and its finite v adds nothing
        auto uel = [&](int k) -> double {
            if (k < NS) return W[StatIdx<D>::pa(k)][StatIdx<D>::pb(k)];
            if (k < NS + D) return wr[k - NS];
            if (k == NS + D) return rwr;
            if (k == NS + D + 1) return on ? 1.0 : 0.0;
            return r2;   // |r|^2 (0 unless on): PCL's MSE numerator, extended slot NSS + 3
        };
        auto vel = [&](int k) -> double {
            if (k < NS) return sv[StatIdx<D>::pa(k)] * sv[StatIdx<D>::pb(k)];
            if (k < NS + D) return sv[k - NS];
            return 1.0;
        };
        typedef double d4v __attribute__((ext_vector_type(4)));
        d4v acc = {0.0, 0.0, 0.0, 0.0};
        WaveStat& X = s_lds[w].st;
        // points that contribute nothing (rejected, or the tile's padding lanes) have u = 0: a group
        // of 16 or an MFMA's 4 points with none accepted adds exact zeros and is skipped (uniform test)
        static_assert(NU <= kStatU && NV <= kStatV, "statistics terms fit the transpose image");
        const uint64_t onm = __ballot(on);
        wave_sync();
        double* const wu = &X.u[l & 15];
        double* const wv = &X.v[l & 15];
        const double* const ru = &X.u[min(l & 15, NU - 1) * kStatRow + (l >> 4)];
        const double* const rv = &X.v[min(l & 15, NV - 1) * kStatRow + (l >> 4)];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            if (((onm >> (16 * g)) & 0xFFFFull) == 0) continue;
            if ((l >> 4) == g) {
#pragma unroll
                for (int k = 0; k < NU; ++k) wu[k * kStatRow] = uel(k);
#pragma unroll
                for (int k = 0; k < NV; ++k) wv[k * kStatRow] = vel(k);
            }
            wave_sync();
#pragma unroll
            for (int cc = 0; cc < 4; ++cc) {
                if (((onm >> (16 * g + 4 * cc)) & 0xFull) == 0) continue;
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(ru[4 * cc], rv[4 * cc], acc, 0, 0, 0);
            }
            wave_sync();
        }
        // lane l holds stats[p = (l>>4) + 4j][q = l&15], j = 0..3; the GEMM's operands are read, so the
        // wave's statistics now overwrite its LDS: zeros, then each statistic from its owner lane
        double* const wst = wstat(w);
        for (int k = l; k < NSX; k += 64) wst[k] = 0.0;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int p = (l >> 4) + 4 * j, qq = l & 15;
            int idx = -1;
            if (p < NS) {
                if (qq < NS) idx = p * NS + qq;
                else if (qq < NS + D) idx = NS * NS + p * D + (qq - NS);
                else if (qq == NS + D) idx = NS * NS + NS * D + p;
            } else if (p < NS + D) {
                if (qq >= NS && qq < NS + D) idx = NS * NS + NS * D + NS + (p - NS) * D + (qq - NS);
                else if (qq == NS + D) idx = NS * NS + NS * D + NS + D * D + (p - NS);
            } else if (qq == NS + D && p <= NS + D + 1) {
                idx = NS * NS + NS * D + NS + D * D + D + (p - NS - D);   // c0, count
            } else if (qq == NS + D && p == NS + D + 2) {
                idx = NSS + 3;                                            // sum |r|^2
            }
            if (idx >= 0) wst[idx] = acc[j];   // each (p,q) has one owner lane: no race
        }
        namb_total += (int)__popcll(__ballot(amb));
    }
    } else {   // no tile: zeros
        for (int k = l; k < NSX; k += 64) wstat(w)[k] = 0.0;
    }
    if (l == 0) {
        double* const wst = wstat(w);
        wst[NSS] = (double)namb_total;
        wst[NSS + 1] = (double)pairs * 64.0;
        wst[NSS + 2] = (double)list_rebuilds;
        wst[NSS + 4] = (double)ngproved;
        wst[NSS + 5] = (double)nwalked;
    }
    S.mark(6);
#if defined(GICP_STAMPS) || defined(GICP_TIMELINE)
#ifndef GICP_TIMELINE
    S.acc[7] = (unsigned long long)pairs;
#endif   // slot 7: rows scanned (not cycles)
    if (A.stamps && l == 0) {
        unsigned long long* o = A.stamps + ((int64_t)blockIdx.x * kCorrWaves + w) * 20;
#ifndef GICP_TIMELINE
        for (int c = 0; c < 8; ++c) o[c] = S.acc[c];
        for (int c = 0; c < 8; ++c) o[8 + c] = S.cnt[c];
#endif
#ifndef GICP_TIMELINE
        o[16] = S.rt0;                                   // 100 MHz realtime: wave start / end
#else
        o[0] = (unsigned)T;                              // the wave's source tile, its radius and size
        o[1] = __float_as_uint(st.radius);
        o[2] = (unsigned)st.count;
        o[3] = S.tdesc;                                  // certificates + descent done (0: the wave had no tile)
        o[4] = S.twalk;                                  // walk done
        o[5] = S.kind | (S.ndesc << 8) | (S.nwalk << 16) | (S.nwalk_jp << 24);
        o[6] = S.ta;                                     // the prologue's scalar batch in
        o[7] = S.tb;                                     // certificates in
        for (int c = 0; c < 8; ++c) o[8 + c] = S.cnt[c];
        o[10] = S.te;                                    // the epilogue's gathers in (0: no accepted lane... none found)
        o[12] = tl_after(pairs, namb_total);             // statistics GEMM done, before the partials
        o[14] = __float_as_uint(S.wb0);                  // the walk's starting radius (max over walking lanes)
#endif
        o[17] = __builtin_amdgcn_s_memrealtime();
        o[18] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
        o[19] = (unsigned)__builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
    }
#endif
    __syncthreads();
    // ---- deterministic two-level reduction inside the launch ----------------
    // Workgroup partials are stored write-through (sc1) and drained before one lane's agent-scope
    // ticket add; the last arriver of each group of kGroupWG workgroups (told by the value its add
    // returned) takes an agent acquire and sums the group in index order; the last group does the
    // same over the groups and writes the statistics into the device state.  Tickets self-reset.
    __shared__ int s_last;
    for (int t = threadIdx.x; t < NSX; t += 64 * kCorrWaves) {
        double s = 0.0;
#pragma unroll
        for (int u = 0; u < kCorrWaves; ++u) s += wstat(u)[t];
        __hip_atomic_store(&A.partials[(int64_t)unit * NSX + t], s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    GICP_TAIL_MARK(1);
#ifdef GICP_TAIL
    if (A.tail && threadIdx.x < 7 && s_walk[threadIdx.x]) atomicAdd(A.tail + 9 + threadIdx.x, (unsigned long long)s_walk[threadIdx.x]);
#endif
    __syncthreads();
    // one level when a few round trips of the final workgroup's loads cover every unit (kFlatUnits), else
    // groups of kGroupWG units first
    const bool flat = nunits <= kFlatUnits;
    const int ng = flat ? 1 : (nunits + kGroupWG - 1) / kGroupWG;
    const int g = flat ? 0 : unit / kGroupWG;   // the reduction follows the unit, not the launch order
    if (threadIdx.x == 0) {
        const int gn = flat ? nunits : min(kGroupWG, nunits - g * kGroupWG);
        uint32_t* const tk = flat ? &A.tickets[kMaxGroups * kTicketStride] : &A.tickets[g * kTicketStride];
        s_last = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(gn - 1);
        if (s_last) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        GICP_TAIL_MARK(2);
    }
    __syncthreads();
    if (!s_last) return;
    // rows [b0, b1) of `src` ([row][NSX]) summed per statistic in row order: 3 threads per statistic,
    // each with its loads all in flight before the first add, combined in fixed order through LDS
    // reduction scratch aliases the waves' staging LDS (every wave is past its walk here)
    static_assert(sizeof(double) * 4 * NSX <= sizeof(WaveLds) * kCorrWaves, "reduction scratch fits the staging LDS");
    double (*s_red)[NSX] = reinterpret_cast<double (*)[NSX]>(&s_lds[0]);
    double* s_sum = reinterpret_cast<double*>(&s_lds[0]) + 3 * NSX;
    auto sum_rows = [&](const double* src, int b0, int b1, double* dst_stat) {
        constexpr int PART = 27;   // rows per thread per chunk: 3 x 27 = 81 covers a 64-unit group and the 79 groups of 1M in one round trip
        constexpr int NP = (64 * kCorrWaves) / NSX >= 3 ? 3 : 1;  // threads per statistic
        constexpr int NT = 64 * kCorrWaves;
        const int tid = threadIdx.x;
        for (int s0 = 0; s0 < NSX; s0 += NT / NP) {   // statistics handled in this sweep
            const int st = s0 + tid % (NT / NP), part = tid / (NT / NP);
            const bool act = part < NP && st < NSX && tid % (NT / NP) < NSX;
            double acc = 0.0;
            for (int c0 = b0; c0 < b1; c0 += NP * PART) {
                if (act) {
                    double v[PART];
#pragma unroll
                    for (int k = 0; k < PART; ++k) {
                        const int b = c0 + part * PART + k;
                        v[k] = b < b1 ? __hip_atomic_load(&src[(int64_t)b * NSX + st], __ATOMIC_RELAXED,
                                                          __HIP_MEMORY_SCOPE_AGENT)
                                      : 0.0;
                    }
                    double sp = 0.0;
#pragma unroll
                    for (int k = 0; k < PART; ++k) sp += v[k];
                    s_red[part][st] = sp;
                }
                __syncthreads();
                if (act && part == 0) {
                    double t = s_red[0][st];
#pragma unroll
                    for (int k = 1; k < NP; ++k) t += s_red[k][st];
                    acc += t;
                }
                __syncthreads();
            }
            if (act && part == 0) dst_stat[st] = acc;
        }
        __syncthreads();
    };
    const bool fuse = A.fuse_solve != 0;
    const bool xchg = A.peer.n > 1;
    double hv = 0.0;
    __shared__ uint64_t s_seq;
    uint64_t seq0 = 0;
    if (!flat) {
        {
            const int b0 = g * kGroupWG, b1 = min(nunits, b0 + kGroupWG);
            sum_rows(A.partials, b0, b1, s_sum);
            for (int t = threadIdx.x; t < NSX; t += 64 * kCorrWaves)
                __hip_atomic_store(&A.gpart[(int64_t)g * NSX + t], s_sum[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        GICP_TAIL_MARK(3);
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(&A.tickets[g * kTicketStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = __hip_atomic_fetch_add(&A.tickets[kMaxGroups * kTicketStride], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                     (unsigned)(ng - 1);
            if (s_last) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            GICP_TAIL_MARK(4);
        }
        __syncthreads();
        if (!s_last) return;
    }
    // the final workgroup.  With no exchange between ranks it also runs the solve and the pose update
    // (gicp_solve_dev.h, one wave) -- the state header is requested now, in flight with the reduction's loads,
    // and so is this rank's exchange counter
    if (fuse && threadIdx.x < kStateHeader) hv = reinterpret_cast<const double*>(A.state)[threadIdx.x];
    if (xchg && threadIdx.x == 0) seq0 = *A.peer.ctr;
    if (flat) sum_rows(A.partials, 0, nunits, s_sum);   // every unit's partial, in unit order
    else sum_rows(A.gpart, 0, ng, s_sum);
    GICP_TAIL_MARK(5);
    if (xchg) {   // the sum over ranks, in-kernel
        if (threadIdx.x == 0) s_seq = seq0 + 1;
        __syncthreads();
        const uint64_t x0 = (uint64_t)wall_clock64();
        if (!peer_exchange<NSX>(A.peer, s_seq, s_sum)) {
            if (threadIdx.x == 0) {   // a peer never arrived: fail the call, later launches exit at once
                A.state->solve_fail = 2;
                A.state->converged = 1;
                __hip_atomic_store(&A.tickets[kMaxGroups * kTicketStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            return;
        }
        if (threadIdx.x == 0) {   // how long this rank's exchange took (its stores to every rank's flags arriving)
            const double dt = (double)((uint64_t)wall_clock64() - x0);
            const double m = A.state->xchg_min;
            A.state->xchg_sum += dt;
            A.state->xchg_min = m > 0.0 ? fmin(m, dt) : dt;
            A.state->xchg_n += 1.0;
        }
    }
    GICP_TAIL_MARK(6);
    for (int t = threadIdx.x; t < NSX; t += 64 * kCorrWaves) A.state->stats[t] = s_sum[t];
    if (threadIdx.x == 0) __hip_atomic_store(&A.tickets[kMaxGroups * kTicketStride], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    GICP_TAIL_MARK(7);
#ifdef GICP_TAIL
    auto tail_out = [&]() {
        if (A.tail && threadIdx.x == 0)
            for (int k = 1; k < 9; ++k) A.tail[k] = tl[k];
    };
    if (!fuse) tail_out();
#endif
    if (!fuse || threadIdx.x >= 64) return;
    // LDS after the reduction scratch: the header image (its `stats` field unused: the statistics are s_sum)
    // and the solve's exchange area
    static_assert(sizeof(double) * 4 * NSX + sizeof(IterState) + sizeof(SolveLds<D>) <= sizeof(WaveLds) * kCorrWaves,
                  "solve LDS fits the staging LDS");
    IterState* s_hdr = reinterpret_cast<IterState*>(s_sum + NSX);
    SolveLds<D>* s_sl = reinterpret_cast<SolveLds<D>*>(s_sum + NSX + sizeof(IterState) / sizeof(double));
    if (threadIdx.x < kStateHeader) reinterpret_cast<double*>(s_hdr)[threadIdx.x] = hv;
    wave_sync();
    solve_update<D>(A.state, s_hdr, s_sum, *s_sl, A.hist);
    GICP_TAIL_MARK(8);
#ifdef GICP_TAIL
    tail_out();
#endif
}

// One wave: solve_update on the statistics in the device state (after the multi-GPU all-reduce).
// The state (header + statistics, ~110 doubles) comes into LDS with one load per lane in a single
// round trip -- the statistics were just written by k_corr's last workgroup, likely on another XCD, so
// each dependent global read costs a full memory latency; every later read is an LDS read.
template <int D>
__global__ void __launch_bounds__(64) k_solve(IterState* S, double* hist) {
    constexpr int NLOAD = (int)(offsetof(IterState, stats) / sizeof(double)) + nstat_ext(D);
    static_assert(NLOAD <= 128, "state header + statistics: two loads per lane");
    __shared__ IterState s_state;
    __shared__ SolveLds<D> s_sl;
    GICP_SOLVE_STAMP(0);
    const int l = threadIdx.x;
    const double* g = reinterpret_cast<const double*>(S);
    double* sd = reinterpret_cast<double*>(&s_state);
    const double v0 = g[l];
    double v1 = 0.0;
    if (l + 64 < NLOAD) v1 = g[l + 64];
    sd[l] = v0;
    if (l + 64 < NLOAD) sd[l + 64] = v1;
    __syncthreads();
    GICP_SOLVE_STAMP(1);
    if (s_state.converged) return;
    solve_update<D>(S, &s_state, s_state.stats, s_sl, hist);
    GICP_SOLVE_STAMP(13);
}

// ---------------------------------------------------------------------------
// top-k of det(W) for the drop-in's visualisation extras (gicp.py:169-172)
// ---------------------------------------------------------------------------
// Order: larger det first, equal dets -> larger original index first, i.e. the last k positions of a
// stable ascending argsort.  NaN (rows of other ranks' shards, memset 0xFF) never enters a list.
constexpr int kTopMax = 16;

__device__ __forceinline__ bool top_gt(double va, int64_t ia, double vb, int64_t ib) {
    return va > vb || (va == vb && ia > ib);
}

// Each thread keeps its k best in registers (descending, unrolled so nothing spills), then the block
// pops its k best with k rounds of a block-wide argmax over the threads' heads.
struct TopList {
    double v[kTopMax];
    int64_t i[kTopMax];   // (original index << 32) | sorted position: ties order by the original index
    __device__ void init() {
#pragma unroll
        for (int p = 0; p < kTopMax; ++p) {
            v[p] = -INFINITY;
            i[p] = -1;
        }
    }
    __device__ void insert(double cv, int64_t ci, int k) {
        if (!top_gt(cv, ci, -INFINITY, -1)) return;   // NaN / sentinel
#pragma unroll
        for (int p = 0; p < kTopMax; ++p) {
            if (p < k && top_gt(cv, ci, v[p], i[p])) {
                const double tv = v[p];
                const int64_t ti = i[p];
                v[p] = cv;
                i[p] = ci;
                cv = tv;
                ci = ti;
            }
        }
    }
};

__device__ void top_block_emit(TopList& L, int k, double* out_v, int64_t* out_i) {
    __shared__ double s_v[4];
    __shared__ int64_t s_i[4];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (int r = 0; r < k; ++r) {
        double bv = L.v[0];
        int64_t bi = L.i[0];
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) {
            const double ov = __shfl_xor(bv, off);
            const int64_t oi = __shfl_xor(bi, off);
            if (top_gt(ov, oi, bv, bi)) {
                bv = ov;
                bi = oi;
            }
        }
        if (lane == 0) {
            s_v[w] = bv;
            s_i[w] = bi;
        }
        __syncthreads();
        bv = s_v[0];
        bi = s_i[0];
        for (int u = 1; u < (int)(blockDim.x >> 6); ++u)
            if (top_gt(s_v[u], s_i[u], bv, bi)) {
                bv = s_v[u];
                bi = s_i[u];
            }
        __syncthreads();
        if (threadIdx.x == 0) {
            out_v[r] = bv;
            out_i[r] = bi;
        }
        if (bi >= 0 && L.i[0] == bi && L.v[0] == bv) {   // indices are unique: exactly one owner pops
#pragma unroll
            for (int p = 0; p + 1 < kTopMax; ++p) {
                L.v[p] = L.v[p + 1];
                L.i[p] = L.i[p + 1];
            }
            L.v[kTopMax - 1] = -INFINITY;
            L.i[kTopMax - 1] = -1;
        }
    }
}

// stage 1: block b reduces its contiguous chunk of det[0, n) to k candidates
__global__ void __launch_bounds__(256) k_top1(const double* __restrict__ det, const int32_t* __restrict__ perm,
                                              int64_t n, int k, double* pv, int64_t* pi) {
    const int64_t chunk = (n + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = (int64_t)blockIdx.x * chunk, b1 = min(n, b0 + chunk);
    TopList L;
    L.init();
    for (int64_t x = b0 + threadIdx.x; x < b1; x += blockDim.x)
        L.insert(det[x], ((int64_t)perm[x] << 32) | (int64_t)x, k);
    top_block_emit(L, k, pv + (int64_t)blockIdx.x * k, pi + (int64_t)blockIdx.x * k);
}

// stage 2: one block merges the m = blocks x k candidates; ascending output (np.argsort(...)[-k:]),
// plus the matched target index of each winner
// stage 2: one block reduces the stage-1 candidates; outputs ascending (np.argsort(det)[-k:] order), the
// source as its original index, the target from the pass's sorted-order record (tgt_sorted)
__global__ void __launch_bounds__(256) k_top2(const double* pv, const int64_t* pi, int m, int k,
                                              const int64_t* __restrict__ tgt_sorted, double* ov, int64_t* osrc,
                                              int64_t* otgt) {
    __shared__ double s_ov[kTopMax];
    __shared__ int64_t s_oi[kTopMax];
    TopList L;
    L.init();
    for (int x = threadIdx.x; x < m; x += blockDim.x) L.insert(pv[x], pi[x], k);
    top_block_emit(L, k, s_ov, s_oi);
    __syncthreads();
    if ((int)threadIdx.x < k) {
        const int r = k - 1 - (int)threadIdx.x;   // descending -> ascending
        const int64_t si = s_oi[r];
        ov[threadIdx.x] = si >= 0 ? s_ov[r] : 0.0;
        osrc[threadIdx.x] = si >= 0 ? (si >> 32) : -1;
        otgt[threadIdx.x] = si >= 0 ? tgt_sorted[si & 0xFFFFFFFFll] : -1;
    }
}

// Each launcher reports hipGetLastError() after its launches.  HIP's last error is per thread and shared
// with every other HIP user on it (torch, RCCL, the caller): one such user's failed call left there must not
// fail this library's launch check, so each launcher clears it first.
static inline void clear_foreign_error() { (void)hipGetLastError(); }

hipError_t launch_top_weights(const double* det, const int64_t* tgt_sorted, const int32_t* perm, int64_t n, int k,
                              double* scratch_v, int64_t* scratch_i, int blocks, double* ov, int64_t* osrc,
                              int64_t* otgt, hipStream_t st) {
    clear_foreign_error();
    if (k < 1 || k > kTopMax || blocks < 1) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_top1, dim3(blocks), dim3(256), 0, st, det, perm, n, k, scratch_v, scratch_i);
    hipLaunchKernelGGL(k_top2, dim3(1), dim3(256), 0, st, scratch_v, scratch_i, blocks * k, k, tgt_sorted, ov, osrc,
                       otgt);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// rotated covariances (gicp.py:120-121 all_source_cov_matrices): R C Rᵀ = a I − (R m)(R m)ᵀ per
// point, written in original order.  HBM-bound: 36 B read, D² × 8 B written per point.
// ---------------------------------------------------------------------------
struct Rot {
    double r[9];
};

template <int D>
__global__ void __launch_bounds__(256) k_rotate_cov(const double4* __restrict__ cov, const int32_t* __restrict__ perm,
                                                    int64_t n, Rot R, double* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double4 c = cov[i];
    const double m[3] = {c.y, c.z, c.w};
    double rm[D];
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double v = 0.0;
#pragma unroll
        for (int b = 0; b < D; ++b) v = fma(R.r[a * D + b], m[b], v);
        rm[a] = v;
    }
    double* o = out + (int64_t)perm[i] * D * D;
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
        for (int b = 0; b < D; ++b) o[a * D + b] = (a == b ? c.x : 0.0) - __dmul_rn(rm[a], rm[b]);   // no fma: the
}                                                                                                 // host formula's rounding

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
hipError_t launch_rotate_cov(const double4* cov, const int32_t* perm, int64_t n, int dim, const double* R, double* out,
                             hipStream_t st) {
    clear_foreign_error();
    if (n <= 0) return hipSuccess;
    Rot r{};
    for (int k = 0; k < dim * dim; ++k) r.r[k] = R[k];
    const unsigned g = (unsigned)((n + 255) / 256);
    if (dim == 2) hipLaunchKernelGGL(k_rotate_cov<2>, dim3(g), dim3(256), 0, st, cov, perm, n, r, out);
    else hipLaunchKernelGGL(k_rotate_cov<3>, dim3(g), dim3(256), 0, st, cov, perm, n, r, out);
    return hipGetLastError();
}

hipError_t launch_morton(const double* xyz, int64_t n, int dim, const DevCloud& fr, uint32_t* codes, int32_t* idx,
                         hipStream_t st) {
    clear_foreign_error();
    const int bs = 256;
    const unsigned g = (unsigned)((n + bs - 1) / bs);
    hipLaunchKernelGGL(k_morton, dim3(g), dim3(bs), 0, st, xyz, n, dim, fr, codes, idx);
    return hipGetLastError();
}

hipError_t launch_build_tiles(const double* xyz_in, int dim, int32_t* perm, TileInfo* tiles, TileBox* boxes,
                              int ntiles, double* xyz64, float4* rel32, int32_t* inv, unsigned* rho_bits,
                              hipStream_t st) {
    clear_foreign_error();
    const unsigned g = (unsigned)((ntiles + kWavesPerWG - 1) / kWavesPerWG);
    hipLaunchKernelGGL(k_build_tiles, dim3(g), dim3(256), 0, st, xyz_in, dim, perm, tiles, boxes, ntiles, xyz64,
                       rel32, inv, rho_bits);
    return hipGetLastError();
}

hipError_t launch_build_blocks(const TileInfo* tiles, int ntiles, BlockInfo* blocks, int nblocks, int dim,
                               hipStream_t st) {
    clear_foreign_error();
    const unsigned g = (unsigned)((nblocks + kWavesPerWG - 1) / kWavesPerWG);
    hipLaunchKernelGGL(k_build_blocks<TileInfo>, dim3(g), dim3(256), 0, st, tiles, ntiles, blocks, nblocks, dim);
    const int nsuper = (nblocks + kBlockTiles - 1) / kBlockTiles;   // super-blocks at blocks[nblocks..]
    const unsigned g2 = (unsigned)((nsuper + kWavesPerWG - 1) / kWavesPerWG);
    hipLaunchKernelGGL(k_build_blocks<BlockInfo>, dim3(g2), dim3(256), 0, st, (const BlockInfo*)blocks, nblocks,
                       blocks + nblocks, nsuper, dim);
    return hipGetLastError();
}

hipError_t launch_knn_cov(const CovArgs& a, int dim, int k, bool graph, hipStream_t st) {
    clear_foreign_error();
    const int nq = a.q_end - a.q_begin;
    if (nq <= 0) return hipSuccess;
    if (a.split != 1 && a.split != kSub) return hipErrorInvalidValue;
    const unsigned g = (unsigned)(((int64_t)nq * a.split + kWavesPerWG - 1) / kWavesPerWG);
#define GICP_KNN(DD, KK)                                                                              \
    if (dim == DD && k == KK) {                                                                        \
        if (graph) hipLaunchKernelGGL((k_knn_cov<DD, KK, true>), dim3(g), dim3(256), 0, st, a);        \
        else hipLaunchKernelGGL((k_knn_cov<DD, KK, false>), dim3(g), dim3(256), 0, st, a);             \
        return hipGetLastError();                                                                      \
    }
    GICP_KNN(2, 6)
    GICP_KNN(3, 20)
    GICP_KNN(3, 10)
    GICP_KNN(2, 10)
#undef GICP_KNN
    return hipErrorInvalidValue;
}

hipError_t launch_graph_pack(const GraphArgs& a, hipStream_t st) {
    clear_foreign_error();
    if (a.cl.n <= 0) return hipSuccess;
    const unsigned gp = (unsigned)((a.cl.n + 255) / 256);
    hipLaunchKernelGGL(k_graph_pack, dim3(gp), dim3(256), 0, st, a.nb, a.nbh, a.cl.n, a.nbq, a.nbx, a.nbi);
    return hipGetLastError();
}

// Workgroups (units) of a k_corr launch: kCorrWaves source tiles each; with shards, the units of
// the global chunks shard, shard + nshards, ... (kShardChunk units each, the last one possibly partial).
int corr_grid(int q_tiles, int shard, int nshards) {
    if (q_tiles <= 0) return 0;
    const int units = (q_tiles + kCorrWaves - 1) / kCorrWaves;
    if (nshards <= 1) return units;
    const int nchunks = (units + kShardChunk - 1) / kShardChunk;
    int mine = 0;
    for (int c = shard; c < nchunks; c += nshards) mine += std::min(kShardChunk, units - c * kShardChunk);
    return mine;
}

hipError_t launch_corr(const CorrArgs& a, int dim, int grid, hipStream_t st) {
    clear_foreign_error();
    if (grid <= 0) return hipSuccess;
    if (dim == 2) hipLaunchKernelGGL(k_corr<2>, dim3(grid), dim3(64 * kCorrWaves), 0, st, a);
    else hipLaunchKernelGGL(k_corr<3>, dim3(grid), dim3(64 * kCorrWaves), 0, st, a);
    return hipGetLastError();
}

// reset_tile_state's per-source-tile and per-point resets in one launch
__global__ void __launch_bounds__(256) k_reset_tiles(int32_t* hint, int32_t* list_len, float* list_rcert,
                                                     int32_t* cert_pass, int nt, int32_t* cert_j, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nt) {
        hint[i] = -1;
        list_len[i] = 0;
        list_rcert[i] = 0.f;
        if (cert_pass) cert_pass[i] = -1;
    }
    if (i < n) cert_j[i] = -1;
}

hipError_t launch_reset_tiles(int32_t* hint, int32_t* list_len, float* list_rcert, int32_t* cert_pass, int nt,
                              int32_t* cert_j, int64_t n, hipStream_t st) {
    clear_foreign_error();
    const int64_t m = std::max<int64_t>(nt, n);
    if (m <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_reset_tiles, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, hint, list_len, list_rcert,
                       cert_pass, nt, cert_j, n);
    return hipGetLastError();
}

hipError_t launch_peer_probe(const PeerArgs& p, double* out, hipStream_t st) {
    clear_foreign_error();
    hipLaunchKernelGGL(k_peer_probe, dim3(1), dim3(64), 0, st, p, kPeerProbeRounds, out);
    return hipGetLastError();
}

hipError_t launch_solve(IterState* st, int dim, hipStream_t stream, double* hist) {
    clear_foreign_error();
    if (dim == 2) hipLaunchKernelGGL(k_solve<2>, dim3(1), dim3(64), 0, stream, st, hist);
    else hipLaunchKernelGGL(k_solve<3>, dim3(1), dim3(64), 0, stream, st, hist);
    return hipGetLastError();
}

}  // namespace gicp
