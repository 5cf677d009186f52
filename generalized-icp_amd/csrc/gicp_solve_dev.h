// gicp_solve_dev.h — the inner solve of one outer iteration (gicp.py:148-154) and the convergence test and
// pose update after it (gicp.py:155-167), run by ONE wave on the device.  k_solve<D> runs it as its own
// launch (after the multi-GPU exchange of the statistics); with no exchange, k_corr<D>'s last workgroup runs
// it right after the statistics reduction (one launch and one kernel boundary fewer per
// iteration).
//
// solve_pose_t (gicp_solver.h) restated for one wave inside k_corr's register budget (80 VGPRs at 6 waves
// per SIMD, no scratch frame).  The set-up (K = Htt^-1 Htr, the reduced Hessian H', g', c0') is lane-parallel
// through LDS; the Newton iterations hold row i of H' in lane i's registers and every uniform value (R,
// dr = R - R_k, the gradient, the M x M system) in scalar registers, and meet through cross-lane reads (DPP
// row sums, readlane) rather than LDS barriers; the M x M system runs redundantly in every lane (uniform
// control flow).  Same iterates as the serial solver up to summation order.
#pragma once
#include <hip/hip_runtime.h>

#include "gicp_internal.h"
#include "gicp_solver.h"

namespace gicp {

// Diagnostic hook of the solve's stages (a probe build defines it; nothing otherwise)
#ifndef GICP_SOLVE_STAMP
#define GICP_SOLVE_STAMP(k) ((void)0)
#endif

// Orders the solving wave's LDS traffic between lanes: a wave executes its LDS instructions in order, so
// only the compiler must not move loads or stores across (the memory clobbers; the wave barrier alone
// is not a memory operation to it) -- which also keeps it from hoisting LDS reads out of the loops and
// holding them in registers.
__device__ __forceinline__ void solve_sync() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
}

// Cross-lane helpers of the Newton iterations (uniform results are scalar registers)
__device__ __forceinline__ double readlane_dbl(double v, int k) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), k);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), k);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double wave_uniform(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readfirstlane((int)(b & 0xffffffffll));
    const int hi = __builtin_amdgcn_readfirstlane((int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL>
__device__ __forceinline__ double dpp_dbl(double x) {   // lanes outside the row read 0 (old value)
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xf, 0xf, false);
    const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// sum of lanes 0..15 (row_shr 1, 2, 4, 8: lane 15 ends with the row's sum), uniform
__device__ __forceinline__ double row_sum16(double x) {
    x += dpp_dbl<0x111>(x);
    x += dpp_dbl<0x112>(x);
    x += dpp_dbl<0x114>(x);
    x += dpp_dbl<0x118>(x);
    return readlane_dbl(x, 15);
}
__device__ __forceinline__ double sel3(int b, double x0, double x1, double x2) { return b == 0 ? x0 : b == 1 ? x1 : x2; }
__device__ __forceinline__ double sel4(int i, double x0, double x1, double x2, double x3) {
    return i == 0 ? x0 : i == 1 ? x1 : i == 2 ? x2 : x3;
}
template <int N>
__device__ __forceinline__ double sel_arr(int i, const double (&a)[N]) {
    double v = a[0];
#pragma unroll
    for (int j = 1; j < N; ++j) v = i == j ? a[j] : v;
    return v;
}
// entry (a, b) of exp([w]) R from column b of R (c0, c1, c2 = R_0b, R_1b, R_2b): exp_mul_entry's formula with
// the row a a per-lane value
__device__ __forceinline__ double exp_mul_entry_col(const double* w, double s1, double s2, double c, double c0,
                                                    double c1, double c2, int a) {
    const double wa = a == 0 ? w[0] : a == 1 ? w[1] : w[2];
    const double x0 = a == 0 ? 0.0 : a == 1 ? w[2] : -w[1];
    const double x1 = a == 0 ? -w[2] : a == 1 ? 0.0 : w[0];
    const double x2 = a == 0 ? w[1] : a == 1 ? -w[0] : 0.0;
    const double e0 = (a == 0 ? c : 0.0) + s2 * wa * w[0] + s1 * x0;
    const double e1 = (a == 1 ? c : 0.0) + s2 * wa * w[1] + s1 * x1;
    const double e2 = (a == 2 ? c : 0.0) + s2 * wa * w[2] + s1 * x2;
    return e0 * c0 + e1 * c1 + e2 * c2;
}

// LDS of the one-wave solve
template <int D>
struct SolveLds {
    static constexpr int NR = D * D, M = D == 2 ? 1 : 3, N1 = D + 1;
    double kc[D][NR];           // K = Htt^-1 Htr, column i from lane i
    double kt[D];               // Htt^-1 gt
    double hrow[NR][NR];        // row i of H' (written and read by lane i)
    double R[NR], Rk[NR];       // the solved and the starting rotation (row-major)
    double T[N1 * N1];          // the result pose
};

// Minimise the quadratic of `st` over SE(D) from Tk (both readable by every lane: LDS).
// Leaves the pose in sl.T (visible to the wave on return) and its loss in `loss`; false when the
// translation block is not positive definite (pose unchanged, loss 0, as solve_pose_t's ok = 0).
template <int D>
__device__ __forceinline__ bool solve_pose_wave(const double* st, const double* Tk, SolveLds<D>& sl, double& loss) {
    using namespace solver_detail;
    constexpr int NS = D * (D + 1) / 2, NR = D * D, N1 = D + 1, M = D == 2 ? 1 : 3;
    const int lane = threadIdx.x & 63;
    const int i = lane < NR ? lane : 0;   // lanes >= NR shadow row 0 and never store
    const double* A = st;
    const double* B = A + NS * NS;
    const double* C = B + NS * D;
    const double* gR = C + NS;
    const double* gt = gR + D * D;
    if (lane < N1 * N1) sl.T[lane] = Tk[lane];
    loss = 0.0;
    if (!(gt[D + 1] > 0.5)) {   // no correspondences: loss identically 0, pose unchanged
        solve_sync();
        return true;
    }
    {
        double Ht[D][D], Hti[D][D];
#pragma unroll
        for (int a = 0; a < D; ++a)
#pragma unroll
            for (int b = 0; b < D; ++b) Ht[a][b] = C[sym<D>(a, b)];
        if (!spd_inv<D>(Ht, Hti)) {
            solve_sync();
            return false;
        }
        double rhs[D], x[D], kt[D];
#pragma unroll
        for (int a = 0; a < D; ++a) rhs[a] = gt[a];
        sym_mul<D>(Hti, rhs, kt);
        // column i of K = Htt^-1 Htr on lane i
        const int ci = i / D, cj = i % D;
#pragma unroll
        for (int b = 0; b < D; ++b) rhs[b] = B[sym<D>(ci, b) * D + cj];
        sym_mul<D>(Hti, rhs, x);
        if (lane < NR) {
#pragma unroll
            for (int a = 0; a < D; ++a) sl.kc[a][lane] = x[a];
            sl.R[lane] = sl.Rk[lane] = Tk[(lane / D) * N1 + lane % D];
        }
        if (lane == 0)
#pragma unroll
            for (int a = 0; a < D; ++a) sl.kt[a] = kt[a];
    }
    solve_sync();
    // row i of H' (LDS, lane i's) and g'_i; c0' (uniform)
    double gpi, c0p;
    {
        const int ia = i / D, ii = i % D;
        double bi[D];
#pragma unroll
        for (int a = 0; a < D; ++a) bi[a] = B[sym<D>(ia, a) * D + ii];
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            double s = A[sym<D>(ia, j / D) * NS + sym<D>(ii, j % D)];
#pragma unroll
            for (int a = 0; a < D; ++a) s -= bi[a] * sl.kc[a][j];
            if (lane < NR) sl.hrow[lane][j] = s;
        }
        gpi = gR[i];
#pragma unroll
        for (int a = 0; a < D; ++a) gpi -= bi[a] * sl.kt[a];
        c0p = gt[D];
#pragma unroll
        for (int a = 0; a < D; ++a) c0p -= gt[a] * sl.kt[a];
    }

    // The Newton iterations keep every uniform value in scalar registers and exchange lane values through
    // cross-lane reads instead of LDS round trips (round 6: the LDS form's five barrier phases per step were
    // most of its ~1.5 us): lane i < NR holds row i of H' in registers; R and dr = R - R_k are uniform; the
    // gradient and the reduced Hessian are sums over the NR lanes (DPP row sums); the trial rotation's
    // entries are computed one per lane and read back by every lane; the loss at the trial rotation is
    // summed in lane order, the serial solver's order.
    const double gpl = lane < NR ? gpi : 0.0;
    const double* const Hr = sl.hrow[lane < NR ? lane : 0];   // lanes >= NR read row 0 and weigh it by 0
    double R[NR];
#pragma unroll
    for (int j = 0; j < NR; ++j) R[j] = wave_uniform(sl.Rk[j]);
    double hdr = 0.0;   // (H' dr)_i at the current R (dr = R - R_k = 0 at the start)
    const double Rkl = lane < NR ? sl.Rk[lane] : 0.0;   // this lane's entry of R_k
    const int la = (lane < NR ? lane : 0) / D, lb = (lane < NR ? lane : 0) % D;
    // column b of R for this lane's entry i = (a, b): cl[c] = R_cb (3-D); 2-D cl = (R_0b, R_1b)
    double cl[D];
    auto load_col = [&]() {
        if constexpr (D == 2) {
            cl[0] = (lb == 0) ? R[0] : R[1];
            cl[1] = (lb == 0) ? R[2] : R[3];
        } else {
            cl[0] = sel3(lb, R[0], R[1], R[2]);
            cl[1] = sel3(lb, R[3], R[4], R[5]);
            cl[2] = sel3(lb, R[6], R[7], R[8]);
        }
    };
    // vec(G_k R)_i (3-D: rows of G_k R are +-rows of R or 0; 2-D: G R = (-R[2], -R[3], R[0], R[1]))
    auto gen_entry = [&](int k) -> double {
        if constexpr (D == 2) {
            return la == 0 ? -cl[1] : cl[0];
        } else {
            if (k == 0) return la == 0 ? 0.0 : la == 1 ? -cl[2] : cl[1];
            if (k == 1) return la == 0 ? cl[2] : la == 1 ? 0.0 : -cl[0];
            return la == 0 ? -cl[1] : la == 1 ? cl[0] : 0.0;
        }
    };
    // vec(1/2 (G_k G_l + G_l G_k) R)_i: 3-D 1/2 ([a == l] R_kb + [a == k] R_lb) - delta_kl R_ab; 2-D -R_i
    auto sym2_entry = [&](int k, int l) -> double {
        if constexpr (D == 2) {
            return -(la == 0 ? cl[0] : cl[1]);
        } else {
            const double rab = la == 0 ? cl[0] : la == 1 ? cl[1] : cl[2];
            return 0.5 * ((la == l ? cl[k] : 0.0) + (la == k ? cl[l] : 0.0)) - (k == l ? rab : 0.0);
        }
    };
    // the loss at rotation Rn (one entry per lane: rn = Rn_i) -- phi of the serial solver: f = c0' + sum_i
    // (dr_i (H' dr)_i - 2 g'_i dr_i), summed in lane order; leaves (H' dr_n)_i in hi
    auto eval = [&](double rn, double& hi) -> double {
        const double dl = lane < NR ? rn - Rkl : 0.0;
        hi = 0.0;
#pragma unroll
        for (int j = 0; j < NR; ++j) hi += Hr[j] * readlane_dbl(dl, j);
        const double term = dl * hi - 2.0 * gpl * dl;
        double f = c0p;
#pragma unroll
        for (int j = 0; j < NR; ++j) f += readlane_dbl(term, j);
        return f;
    };

    double f = c0p;   // at R = R_k: dr = 0, the loss is c0' exactly
    double lam = 0.0;
    GICP_SOLVE_STAMP(3);
    for (int it = 0; it < 100; ++it) {
        GICP_SOLVE_STAMP(4 + min(it, 3));
        constexpr int NH = M * (M + 1) / 2;
        double grad[M], Hs[M][M];
        {
            const double u = hdr - gpl;   // (H' dr - g')_i
            load_col();
            double gk[M], hd[M];
#pragma unroll
            for (int k = 0; k < M; ++k) {
                gk[k] = lane < NR ? gen_entry(k) : 0.0;
                hd[k] = gdot<D>(k, R, Hr);   // (H' vec(G_k R))_i
            }
            GICP_SOLVE_STAMP(8);
#pragma unroll
            for (int k = 0; k < M; ++k) grad[k] = 2.0 * row_sum16(u * gk[k]);
            int q = 0;
#pragma unroll
            for (int k = 0; k < M; ++k)
#pragma unroll
                for (int l = k; l < M; ++l, ++q) {
                    const double c = lane < NR ? gk[k] * hd[l] + u * sym2_entry(k, l) : 0.0;
                    Hs[k][l] = Hs[l][k] = 2.0 * row_sum16(c);
                }
            (void)NH;
        }
        GICP_SOLVE_STAMP(9);
        double gmax = 0.0, hscale = 0.0;
#pragma unroll
        for (int k = 0; k < M; ++k) {
            gmax = fmax(gmax, fabs(grad[k]));
            hscale = fmax(hscale, fabs(Hs[k][k]));
        }
        if (gmax == 0.0) break;
        bool stepped = false, flat = false, quad = false;
        double wmax = 0.0;
        for (int tries = 0; tries < 60; ++tries) {
            // (all initialised: an array left undefined on one path becomes a value carried across the
            // loops, i.e. registers held through the whole solve)
            double Hd[M][M], Hdi[M][M] = {}, ng[M], w[M] = {};
#pragma unroll
            for (int k = 0; k < M; ++k) {
#pragma unroll
                for (int l = 0; l < M; ++l) Hd[k][l] = Hs[k][l] + (k == l ? lam * (hscale + kc(1e-300)) : 0.0);
                ng[k] = -grad[k];
            }
            double dd = 0.0;
            bool ok = spd_inv<M>(Hd, Hdi);
            if (ok) {
                sym_mul<M>(Hdi, ng, w);
#pragma unroll
                for (int k = 0; k < M; ++k) dd += w[k] * grad[k];
                ok = dd < 0.0;
            }
            GICP_SOLVE_STAMP(10);
            if (ok) {
                double rn;   // this lane's entry of exp([w]) R
                if constexpr (D == 2) {
                    double c, s;
                    sincos_lean(w[0], s, c);
                    rn = la == 0 ? c * cl[0] - s * cl[1] : s * cl[0] + c * cl[1];
                } else {
                    double s1, s2, c;
                    exp_coeffs(w, s1, s2, c);
                    rn = exp_mul_entry_col(w, s1, s2, c, cl[0], cl[1], cl[2], la);
                }
                GICP_SOLVE_STAMP(11);
                double hn;
                const double fn = eval(rn, hn);
                wmax = 0.0;
#pragma unroll
                for (int k = 0; k < M; ++k) wmax = fmax(wmax, fabs(w[k]));
                // the model decrease -dd/2 is below the rounding of f: no step can be resolved, stop
                // instead of damping towards |w| < 1e-15 (the tries would only chase rounding noise)
                if (fn > f && -dd <= kc(kFlatEps) * fabs(f)) {
                    flat = true;
                    break;
                }
                if (fn <= f || wmax < kc(1e-15)) {
                    if (fn <= f) {
#pragma unroll
                        for (int j = 0; j < NR; ++j) R[j] = readlane_dbl(rn, j);
                        hdr = hn;
                        f = fn;
                    }
                    stepped = true;
                    quad = fn <= f && lam == 0.0 && wmax < kc(kQuadStop);   // (f = fn when accepted)
                    lam = lam > 0.0 ? lam * kc(0.1) : 0.0;
                    if (lam < kc(1e-12)) lam = 0.0;
                    break;
                }
            }
            lam = lam == 0.0 ? kc(1e-9) : lam * kc(10.0);
        }
        if (!stepped || flat || quad || wmax < kc(1e-15)) break;
    }
    if (lane < NR) sl.R[lane] = sel_arr<NR>(lane, R);
    solve_sync();
    GICP_SOLVE_STAMP(12);
    // t from the eliminated block
    if (lane == 0) {
#pragma unroll
        for (int a = 0; a < D; ++a) {
            double s = sl.kt[a];
#pragma unroll
            for (int c = 0; c < NR; ++c) s -= sl.kc[a][c] * (sl.R[c] - sl.Rk[c]);
            sl.T[a * N1 + D] = Tk[a * N1 + D] + s;
#pragma unroll
            for (int b = 0; b < D; ++b) sl.T[a * N1 + b] = sl.R[a * D + b];
        }
#pragma unroll
        for (int b = 0; b < D; ++b) sl.T[D * N1 + b] = 0.0;
        sl.T[D * N1 + D] = 1.0;
    }
    loss = f;
    solve_sync();
    return true;
}

// The inner solve (gicp.py:148-154) from a pass's statistics `st`, then the convergence test and pose
// update of gicp.py:155-167, on the device so iterations need no host sync.  Run by one wave.  `Ls` is
// an LDS copy of the device state S's header and `st` the statistics in LDS: everything is read from
// them, only the results go to S.
template <int D>
__device__ __forceinline__ void solve_update(IterState* S, const IterState* Ls, const double* st, SolveLds<D>& sl,
                                             double* hist) {
    const int lane = threadIdx.x & 63;
    constexpr int NSX = nstat_ext(D);
    if (lane < NSX) S->stats_solved[lane] = st[lane];
    if (lane + 64 < NSX) S->stats_solved[lane + 64] = st[lane + 64];
    double loss;
    const bool ok = solve_pose_wave<D>(st, Ls->T, sl, loss);
    if (lane != 0) return;
    const IterState* SR = Ls;   // the state as this launch found it
    const double* rT = sl.T;    // the solve's pose
    const int it = SR->iter;
    if (hist) {   // gicp_trace row of this iteration: the pose its pass ran at, then min_loss
        constexpr int NT = (D + 1) * (D + 1);
#pragma unroll
        for (int k = 0; k < NT; ++k) hist[k] = SR->T[k];
        hist[NT] = loss;
    }
    S->iter = it + 1;
    if (!ok) S->solve_fail = 1;
    S->loss = loss;
    constexpr int NSS = nstat(D);
    S->pairs_total = SR->pairs_total + st[NSS + 1];
    const double cnt = st[NSS - 1];
    const double mse = cnt > 0.0 ? st[NSS + 3] * solver_detail::recip(cnt) : 0.0;
    S->mse = mse;
    if (!SR->fixed && fabs(SR->last_loss - loss) < SR->tol) {   // gicp.py:160: stop before the update
        S->converged = 1;
        S->converged_at = it;
        S->stop_reason = GICP_STOP_LOSS;
        return;
    }
    S->last_loss = loss;
    // PCL-style criteria on the increment dT = T_new T_old^-1 and the pass's MSE; PCL applies the
    // update and then tests, so these stop AFTER the update (include/gicp_hip.h GICP_STOP_*)
    int reason = GICP_STOP_NONE;
    if (!SR->fixed) {
        constexpr int N1 = D + 1;
        double tr = 0.0, tsq = 0.0;
#pragma unroll
        for (int a = 0; a < D; ++a) {
            double dta = rT[a * N1 + D];
#pragma unroll
            for (int b = 0; b < D; ++b) {
                double dr = 0.0;   // (R_new R_old^T)[a][b]
#pragma unroll
                for (int c = 0; c < D; ++c) dr += rT[a * N1 + c] * SR->T[b * N1 + c];
                if (a == b) tr += dr;
                dta -= dr * SR->T[b * N1 + D];
            }
            tsq += dta * dta;
        }
        const double cosang = D == 3 ? 0.5 * (tr - 1.0) : 0.5 * tr;
        const double dm = fabs(mse - SR->prev_mse);
        if (SR->trans_eps > 0.0 && cosang >= SR->rot_cos && tsq <= SR->trans_eps) reason = GICP_STOP_TRANSFORM;
        else if (SR->fit_eps > 0.0 && dm < SR->fit_eps) reason = GICP_STOP_ABS_MSE;
        else if (SR->rel_eps > 0.0 && dm / SR->prev_mse < SR->rel_eps) reason = GICP_STOP_REL_MSE;
        S->prev_mse = mse;
    }
#pragma unroll
    for (int k = 0; k < (D + 1) * (D + 1); ++k) S->T[k] = rT[k];
    if (reason != GICP_STOP_NONE) {
        S->converged = 1;
        S->converged_at = it;
        S->stop_reason = reason;
    }
}

// LDS image of the state header (IterState up to `stats`): loaded with one load per lane
constexpr int kStateHeader = (int)(offsetof(IterState, stats) / sizeof(double));

}  // namespace gicp
