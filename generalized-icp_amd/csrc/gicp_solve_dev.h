// gicp_solve_dev.h — the inner solve of one outer iteration (gicp.py:148-154) and the convergence test and
// pose update after it (gicp.py:155-167), run by ONE wave on the device.  k_solve<D> runs it as its own
// launch (after the multi-GPU exchange of the statistics); with no exchange, k_corr<D>'s last workgroup runs
// it right after the statistics reduction (one launch and one kernel boundary fewer per
// iteration).
//
// Register-lean: solve_pose_t (gicp_solver.h) restated so that only lane-distributed values live in
// registers across its phases.  The reduced NR x NR Hessian H' is held one row per lane (lane i < NR) in
// LDS, the uniform rotation iterates (R, the trial Rn, R_k), K = Htt^-1 Htr and the result pose in LDS too;
// each phase reads what it needs and writes what the next one needs, so the solve fits k_corr's register
// budget (80 VGPRs at 6 waves per SIMD) without a scratch frame.  The matrix-vector products (H' dr,
// H' vec(G_l R), the loss) are lane-parallel and meet through LDS; the M x M Newton system and the rotation
// update run redundantly in every lane (uniform control flow).  Same iterates as the serial solver up to
// summation order.
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

// LDS of the one-wave solve
template <int D>
struct SolveLds {
    static constexpr int NR = D * D, M = D == 2 ? 1 : 3, N1 = D + 1;
    double hrow[NR][NR];        // row i of H' (written and read by lane i)
    double kc[D][NR];           // K = Htt^-1 Htr, column i from lane i
    double kt[D];               // Htt^-1 gt
    double R[NR], Rn[NR], Rk[NR];   // current, trial and starting rotation (row-major)
    double dr[NR];              // Rn - Rk
    double u[NR], hd[M][NR];    // u = H' dr - g' and H' vec(G_l R), lane-distributed
    double pq[NR + M * (M + 1) / 2];   // P = R U^T, then vec(G_k R).(H' vec(G_l R)) for l >= k
    double f[2][NR];            // loss partials, double-buffered: one barrier per evaluation
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
    // row i of H' and g'_i; c0' (uniform)
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

    // loss at Rn (phi of the serial solver) and, on lane i, u_i = (H' dr - g')_i
    int fbuf = 0;
    auto eval = [&](double& ui) -> double {
        double hi = 0.0;
#pragma unroll
        for (int j = 0; j < NR; ++j) hi += sl.hrow[i][j] * sl.dr[j];
        const double dri = sl.dr[i];
        ui = hi - gpi;
        // alternate buffers: a buffer is rewritten two evaluations later, and every path between
        // passes a barrier after its reads (this eval's or the next iteration's), so no second one here
        double* const fb = sl.f[fbuf];
        fbuf ^= 1;
        if (lane < NR) fb[lane] = dri * hi - 2.0 * gpi * dri;
        solve_sync();
        double f = c0p;
#pragma unroll
        for (int j = 0; j < NR; ++j) f += fb[j];
        return f;
    };

    // at R = R_k: dr = 0, so u_i = -g'_i and the loss is c0' exactly (what eval(R_k) would return)
    double ui = -gpi;
    double f = c0p;
    double lam = 0.0;
    GICP_SOLVE_STAMP(3);
    for (int it = 0; it < 100; ++it) {
        GICP_SOLVE_STAMP(4 + min(it, 3));
        if (lane < NR) {
            sl.u[lane] = ui;
            double Rr[NR], Hr[NR];
#pragma unroll
            for (int k = 0; k < NR; ++k) {
                Rr[k] = sl.R[k];
                Hr[k] = sl.hrow[lane][k];
            }
#pragma unroll
            for (int l = 0; l < M; ++l) sl.hd[l][lane] = gdot<D>(l, Rr, Hr);   // (H' vec(G_l R))_i
        }
        solve_sync();
        GICP_SOLVE_STAMP(8);
        // grad_k = 2 u.vec(G_k R) and the second-order term u.vec(1/2 (G_k G_l + G_l G_k) R) of the
        // serial solver, through P = R U^T (U = u as a D x D matrix): u.vec(X R) = tr(X P),
        // G_k G_l = e_l e_k^T - delta_kl I in 3-D and G^2 = -I in 2-D.  The entries of P and the M(M+1)/2
        // products vec(G_k R).(H' vec(G_l R)) come one per lane.
        constexpr int NH = M * (M + 1) / 2;
        if (lane < NR) {
            const int a = lane / D, b = lane % D;
            double p = 0.0;
#pragma unroll
            for (int c = 0; c < D; ++c) p += sl.R[a * D + c] * sl.u[b * D + c];
            sl.pq[lane] = p;
        } else if (lane < NR + NH) {
            const int q = lane - NR;   // (k, l), l >= k, in row order
            const int k = M == 1 ? 0 : (q < 3 ? 0 : q < 5 ? 1 : 2);
            const int l = M == 1 ? 0 : (q < 3 ? q : q < 5 ? q - 2 : 2);
            double Rr[NR], hv[NR];
#pragma unroll
            for (int c = 0; c < NR; ++c) {
                Rr[c] = sl.R[c];
                hv[c] = sl.hd[l][c];
            }
            sl.pq[lane] = gdot<D>(k, Rr, hv);
        }
        solve_sync();
        double grad[M], Hs[M][M];
        {
            double P[D][D];
#pragma unroll
            for (int a = 0; a < D; ++a)
#pragma unroll
                for (int b = 0; b < D; ++b) P[a][b] = sl.pq[a * D + b];
            if constexpr (D == 2) {
                grad[0] = 2.0 * (P[0][1] - P[1][0]);
            } else {
                grad[0] = 2.0 * (P[1][2] - P[2][1]);
                grad[1] = 2.0 * (P[2][0] - P[0][2]);
                grad[2] = 2.0 * (P[0][1] - P[1][0]);
            }
            double trP = 0.0;
#pragma unroll
            for (int a = 0; a < D; ++a) trP += P[a][a];
            int q = NR;
#pragma unroll
            for (int k = 0; k < M; ++k)
#pragma unroll
                for (int l = k; l < M; ++l) {
                    const double t2 = D == 2 ? -trP : 0.5 * (P[k][l] + P[l][k]) - (k == l ? trP : 0.0);
                    Hs[k][l] = Hs[l][k] = 2.0 * sl.pq[q++] + 2.0 * t2;
                }
        }
        GICP_SOLVE_STAMP(9);
        // (no barrier here: u / hd are rewritten only after the eval below, whose barriers order these
        // reads; every path to the next iteration runs it)
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
                if (lane < NR) {   // one entry per lane
                    const double rn = rot_update_entry<D>(w, sl.R, lane);
                    sl.Rn[lane] = rn;
                    sl.dr[lane] = rn - sl.Rk[lane];
                }
                solve_sync();
                GICP_SOLVE_STAMP(11);
                double un;
                const double fn = eval(un);
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
                        if (lane < NR) sl.R[lane] = sl.Rn[lane];
                        f = fn;
                        ui = un;
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
        solve_sync();   // the accepted R before the next iteration's reads
    }
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
