// gicp_solver.h — the inner solve of GICP from the reduced statistics, host AND device.
//
// Reference: gicp.py:148-154 minimises sum_i r_i^T W_i r_i, r_i = q_i - R s_i - t, with the
// correspondences and weights of the iteration held fixed, starting at the previous optimum.
// For fixed (q, W) that loss is exactly  f(z) = c0 - 2 g^T (z - z_k) + (z - z_k)^T H (z - z_k)
// in z = (vec R row-major, t).  t is eliminated in closed form (Schur
// complement) and the rotation is found by damped Newton on SO(d) from R_k.
//
// Written with fixed sizes and fully unrolled loops (no data-dependent indexing, Cholesky
// instead of pivoting) so the same code runs on the host (gicp_solve_pose) and in one GPU
// lane (the device-side loop of gicp_align) with every array in registers.
#pragma once
#include <hip/hip_runtime.h>

namespace gicp {

#define GICP_HD __host__ __device__ __forceinline__
// probes for solver experiments (a host harness defines them; no-ops in the library)
#ifndef GICP_SOLVER_PROBE_ITER
#define GICP_SOLVER_PROBE_ITER() ((void)0)
#define GICP_SOLVER_PROBE_TRY() ((void)0)
#endif

// Newton stops when a rejected step's model decrease -dd/2 is within 4 ulps of the loss
#ifndef GICP_FLAT_EPS
#define GICP_FLAT_EPS 8.0
#endif
constexpr double kFlatEps = GICP_FLAT_EPS * 2.220446049250313e-16;
// After an accepted undamped Newton step of size |w| < kQuadStop the next step would be ~|w|^2
// (quadratic convergence; the rotation's third derivative is O(1) relative to the Hessian), below
// fp64 resolution of a rotation: stop instead of spending one more iteration to measure it
#ifndef GICP_QUAD_STOP
#define GICP_QUAD_STOP 1e-8
#endif
constexpr double kQuadStop = GICP_QUAD_STOP;

template <int D>
struct SolveOut {
    double T[(D + 1) * (D + 1)];
    double loss;
    int ok;
};

namespace solver_detail {

// A floating-point constant materialised where it is used (device).  fp64 VALU operands cannot be
// literals on gfx9, so every such constant lives in a register pair, and the compiler hoists them all out
// of the solve's loops -- ~20 pairs held through the solve, which inside k_corr's 80-VGPR budget spill.
// The empty volatile asm keeps each one at its use (two s_mov_b32 there).  Identity on the host.
GICP_HD double kc(double v) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+s"(v));
#endif
    return v;
}

template <int D>
GICP_HD constexpr int sym(int a, int b) {
    return a <= b ? a * D - a * (a - 1) / 2 + (b - a) : b * D - b * (b - 1) / 2 + (a - b);
}

// 1/x.  On the device v_rcp_f64 refined by two Newton-Raphson steps (within an ulp or two of the
// quotient; a correctly rounded fp64 division is a ~10-instruction dependent chain with its own
// scaling and fix-up, ~0.4 us of a one-wave solve); on the host the division itself.
GICP_HD double recip(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r = __builtin_amdgcn_rcp(x);
    r = fma(r, fma(-x, r, 1.0), r);
    r = fma(r, fma(-x, r, 1.0), r);
    return r;
#else
    return 1.0 / x;
#endif
}

// Inverse of a symmetric N x N matrix (N <= 3, only the upper triangle is read) by its adjugate,
// with the positive-definiteness test of the leading principal minors (Sylvester); false if not
// SPD.  One reciprocal in all (a Cholesky factor costs N square roots and N(N+1)/2 + N^2 divisions,
// which dominated the device solve: one wave, fp64 div/sqrt are ~10-instruction dependent chains).
// The matrices here (the translation block of the Hessian, the damped 3 x 3 Newton system) are
// small and well conditioned.
template <int N>
GICP_HD bool spd_inv(const double (&M)[N][N], double (&Mi)[N][N]) {
    static_assert(N >= 1 && N <= 3, "spd_inv: N <= 3");
    if constexpr (N == 1) {
        if (!(M[0][0] > 0.0)) return false;
        Mi[0][0] = recip(M[0][0]);
    } else if constexpr (N == 2) {
        const double det = M[0][0] * M[1][1] - M[0][1] * M[0][1];
        if (!(M[0][0] > 0.0 && det > 0.0)) return false;
        const double id = recip(det);
        Mi[0][0] = M[1][1] * id;
        Mi[1][1] = M[0][0] * id;
        Mi[0][1] = Mi[1][0] = -M[0][1] * id;
    } else {
        const double c00 = M[1][1] * M[2][2] - M[1][2] * M[1][2];
        const double c01 = M[0][2] * M[1][2] - M[0][1] * M[2][2];
        const double c02 = M[0][1] * M[1][2] - M[0][2] * M[1][1];
        const double c11 = M[0][0] * M[2][2] - M[0][2] * M[0][2];
        const double c12 = M[0][2] * M[0][1] - M[0][0] * M[1][2];
        const double c22 = M[0][0] * M[1][1] - M[0][1] * M[0][1];
        const double det = M[0][0] * c00 + M[0][1] * c01 + M[0][2] * c02;
        if (!(M[0][0] > 0.0 && c22 > 0.0 && det > 0.0)) return false;
        const double id = recip(det);
        Mi[0][0] = c00 * id;
        Mi[0][1] = Mi[1][0] = c01 * id;
        Mi[0][2] = Mi[2][0] = c02 * id;
        Mi[1][1] = c11 * id;
        Mi[1][2] = Mi[2][1] = c12 * id;
        Mi[2][2] = c22 * id;
    }
    return true;
}
template <int N>
GICP_HD void sym_mul(const double (&Mi)[N][N], const double (&b)[N], double (&x)[N]) {
#pragma unroll
    for (int i = 0; i < N; ++i) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < N; ++k) s += Mi[i][k] * b[k];
        x[i] = s;
    }
}

// sin and cos of th.  On the device without libm's argument reduction, whose path for huge arguments
// (Payne-Hanek) needs more registers than the whole one-wave solve may use inside k_corr: th is reduced
// modulo 2 pi in two parts (Cody-Waite; a huge th only loses accuracy in the angle, never in
// s^2 + c^2 = 1), halved to below 1/32 (at most 7 times), the series evaluated there (truncation
// < 3e-18, the same coefficients as rot_update's small-angle branch: every fp64 constant is a register
// pair in the loop) and the double-angle formulas applied back.  On the host the libm functions.
GICP_HD void sincos_lean(double th, double& s, double& c) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double n = rint(th * 0.15915494309189535);             // th / (2 pi)
    double x = fma(-n, kc(6.28318530717958623e+00), th);        // 2 pi = C1 + C2, C1 = fl(2 pi)
    x = fma(-n, kc(2.44929359829470641e-16), x);
    int k = 0;
    while (!(fabs(x) < 0.03125) && k < 7) {
        x *= 0.5;
        ++k;
    }
    const double x2 = x * x;
    s = x * (1.0 + x2 * (kc(-1.0 / 6) + x2 * (kc(1.0 / 120) + x2 * kc(-1.0 / 5040))));
    c = 1.0 - x2 * (0.5 + x2 * (kc(-1.0 / 24) + x2 * (kc(1.0 / 720) + x2 * kc(-1.0 / 40320))));
    for (; k > 0; --k) {
        const double s2 = 2.0 * s * c;
        c = (c - s) * (c + s);
        s = s2;
    }
#else
    s = sin(th);
    c = cos(th);
#endif
}

// exp([w]) = c I + s1 [w]x + s2 w w^T (3-D): s1 = sin(th)/th, s2 = (1 - cos th)/th^2, c = cos th = 1 - s2 th^2
GICP_HD void exp_coeffs(const double* w, double& s1, double& s2, double& c) {
    const double th2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
    if (th2 < kc(9.765625e-4)) {
        // by their series in th^2 (th < 1/32): truncation < th^8/362880 < 3e-18 here, and neither sin/cos
        // nor a square root on the device's single-wave solve (the Newton steps are small)
        s1 = 1.0 + th2 * (kc(-1.0 / 6) + th2 * (kc(1.0 / 120) + th2 * kc(-1.0 / 5040)));
        s2 = 0.5 + th2 * (kc(-1.0 / 24) + th2 * (kc(1.0 / 720) + th2 * kc(-1.0 / 40320)));
    } else {
        const double th = sqrt(th2);
        double sn, cs;
        sincos_lean(th, sn, cs);
        s1 = sn / th;
        s2 = (1.0 - cs) / th2;
    }
    c = 1.0 - s2 * th2;   // ([w]x^2 = w w^T - th^2 I)
}

// entry (a, b) of exp([w]) R, 3-D, from exp_coeffs
GICP_HD double exp_mul_entry(const double* w, double s1, double s2, double c, const double* R, int a, int b) {
    const double wa = a == 0 ? w[0] : a == 1 ? w[1] : w[2];
    // row a of [w]x: (0, -w2, w1), (w2, 0, -w0), (-w1, w0, 0)
    const double x0 = a == 0 ? 0.0 : a == 1 ? w[2] : -w[1];
    const double x1 = a == 0 ? -w[2] : a == 1 ? 0.0 : w[0];
    const double x2 = a == 0 ? w[1] : a == 1 ? -w[0] : 0.0;
    const double e0 = (a == 0 ? c : 0.0) + s2 * wa * w[0] + s1 * x0;
    const double e1 = (a == 1 ? c : 0.0) + s2 * wa * w[1] + s1 * x1;
    const double e2 = (a == 2 ? c : 0.0) + s2 * wa * w[2] + s1 * x2;
    return e0 * R[b] + e1 * R[3 + b] + e2 * R[6 + b];
}

// R <- exp([w]) R (left perturbation)
template <int D>
GICP_HD void rot_update(const double* w, const double (&R)[D * D], double (&Rn)[D * D]) {
    if constexpr (D == 2) {
        double c, s;
        sincos_lean(w[0], s, c);
#pragma unroll
        for (int b = 0; b < 2; ++b) {
            Rn[b] = c * R[b] - s * R[2 + b];
            Rn[2 + b] = s * R[b] + c * R[2 + b];
        }
    } else {
        double s1, s2, c;
        exp_coeffs(w, s1, s2, c);
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
            for (int b = 0; b < 3; ++b) Rn[a * 3 + b] = exp_mul_entry(w, s1, s2, c, R, a, b);
    }
}

// entry j of rot_update's result, R in memory (LDS): the device solve computes one entry per lane
template <int D>
GICP_HD double rot_update_entry(const double* w, const double* R, int j) {
    if constexpr (D == 2) {
        double c, s;
        sincos_lean(w[0], s, c);
        const int b = j & 1;
        return j < 2 ? c * R[b] - s * R[2 + b] : s * R[b] + c * R[2 + b];
    } else {
        double s1, s2, c;
        exp_coeffs(w, s1, s2, c);
        return exp_mul_entry(w, s1, s2, c, R, j / 3, j % 3);
    }
}

// generator k of so(d) applied from the left: out = G_k R
template <int D>
GICP_HD void gen_mul(int k, const double (&R)[D * D], double (&out)[D * D]) {
    if constexpr (D == 2) {
        out[0] = -R[2];
        out[1] = -R[3];
        out[2] = R[0];
        out[3] = R[1];
    } else {
        // G_k = [e_k]x ; rows: (G R)_a = sum_b G_ab R_b
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            const double r0 = R[b], r1 = R[3 + b], r2 = R[6 + b];
            if (k == 0) {
                out[b] = 0.0;
                out[3 + b] = -r2;
                out[6 + b] = r1;
            } else if (k == 1) {
                out[b] = r2;
                out[3 + b] = 0.0;
                out[6 + b] = -r0;
            } else {
                out[b] = -r1;
                out[3 + b] = r0;
                out[6 + b] = 0.0;
            }
        }
    }
}

// sum_j vec(G_k R)_j v_j with only the six nonzero entries of G_k R (3-D; the zeros would still cost
// an FMA each: 0 * x is not foldable without fast-math)
template <int D>
GICP_HD double gdot(int k, const double (&R)[D * D], const double* v) {
    double s = 0.0;
    if constexpr (D == 2) {
        s = -R[2] * v[0] - R[3] * v[1] + R[0] * v[2] + R[1] * v[3];
    } else {
#pragma unroll
        for (int b = 0; b < 3; ++b) {
            if (k == 0) s += R[3 + b] * v[6 + b] - R[6 + b] * v[3 + b];
            else if (k == 1) s += R[6 + b] * v[b] - R[b] * v[6 + b];
            else s += R[b] * v[3 + b] - R[3 + b] * v[b];
        }
    }
    return s;
}

}  // namespace solver_detail

// Minimise the quadratic of `st` (layout DESIGN.md §4) over SE(D) from Tk.
template <int D>
GICP_HD SolveOut<D> solve_pose_t(const double* st, const double* Tk) {
    using namespace solver_detail;
    constexpr int NS = D * (D + 1) / 2, NR = D * D, N1 = D + 1, M = D == 2 ? 1 : 3;
    SolveOut<D> out;
    out.ok = 1;
#pragma unroll
    for (int k = 0; k < N1 * N1; ++k) out.T[k] = Tk[k];
    out.loss = 0.0;
    const double* A = st;
    const double* B = A + NS * NS;
    const double* C = B + NS * D;
    const double* gR = C + NS;
    const double* gt = gR + D * D;
    const double c0 = gt[D];
    const double cnt = gt[D + 1];
    if (!(cnt > 0.5)) return out;   // no correspondences: loss identically 0, pose unchanged

    double Rk[NR], tk[D];
#pragma unroll
    for (int a = 0; a < D; ++a) {
#pragma unroll
        for (int b = 0; b < D; ++b) Rk[a * D + b] = Tk[a * N1 + b];
        tk[a] = Tk[a * N1 + D];
    }
    // Htt^-1, K = Htt^-1 Htr, kt = Htt^-1 gt
    double Ht[D][D], Hti[D][D];
#pragma unroll
    for (int a = 0; a < D; ++a)
#pragma unroll
        for (int b = 0; b < D; ++b) Ht[a][b] = C[sym<D>(a, b)];
    if (!spd_inv<D>(Ht, Hti)) {
        out.ok = 0;
        return out;
    }
    double kt[D], Kc[D][NR];
    {
        double rhs[D], x[D];
#pragma unroll
        for (int a = 0; a < D; ++a) rhs[a] = gt[a];
        sym_mul<D>(Hti, rhs, x);
#pragma unroll
        for (int a = 0; a < D; ++a) kt[a] = x[a];
#pragma unroll
        for (int c = 0; c < NR; ++c) {
            const int ci = c / D, cj = c % D;   // column (ci, cj) of Htr: H[t_b][(ci,cj)] = B[sym(ci,b)][cj]
#pragma unroll
            for (int b = 0; b < D; ++b) rhs[b] = B[sym<D>(ci, b) * D + cj];
            sym_mul<D>(Hti, rhs, x);
#pragma unroll
            for (int a = 0; a < D; ++a) Kc[a][c] = x[a];
        }
    }
    // reduced quadratic in dr: c0' - 2 g'^T dr + dr^T H' dr
    double Hp[NR][NR], gp[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        const int ia = i / D, ii = i % D;
#pragma unroll
        for (int j = 0; j < NR; ++j) {
            const int jb = j / D, jj = j % D;
            double s = A[sym<D>(ia, jb) * NS + sym<D>(ii, jj)];
#pragma unroll
            for (int a = 0; a < D; ++a) s -= B[sym<D>(ia, a) * D + ii] * Kc[a][j];
            Hp[i][j] = s;
        }
        double s = gR[i];
#pragma unroll
        for (int a = 0; a < D; ++a) s -= B[sym<D>(ia, a) * D + ii] * kt[a];
        gp[i] = s;
    }
    double c0p = c0;
#pragma unroll
    for (int a = 0; a < D; ++a) c0p -= gt[a] * kt[a];

    auto phi = [&](const double (&R)[NR]) {
        double dr[NR], f = c0p;
#pragma unroll
        for (int i = 0; i < NR; ++i) dr[i] = R[i] - Rk[i];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            double hi = 0.0;
#pragma unroll
            for (int j = 0; j < NR; ++j) hi += Hp[i][j] * dr[j];
            f += dr[i] * hi - 2.0 * gp[i] * dr[i];
        }
        return f;
    };

    double R[NR];
#pragma unroll
    for (int i = 0; i < NR; ++i) R[i] = Rk[i];
    double f = phi(R);
    double lam = 0.0;
    for (int it = 0; it < 100; ++it) {
        GICP_SOLVER_PROBE_ITER();
        double u[NR];
#pragma unroll
        for (int i = 0; i < NR; ++i) {
            double s = -gp[i];
#pragma unroll
            for (int j = 0; j < NR; ++j) s += Hp[i][j] * (R[j] - Rk[j]);
            u[i] = s;   // H' dr - g'
        }
        double Dk[M][NR], grad[M], Hs[M][M];
#pragma unroll
        for (int k = 0; k < M; ++k) {
            gen_mul<D>(k, R, Dk[k]);
            double s = 0.0;
#pragma unroll
            for (int i = 0; i < NR; ++i) s += u[i] * Dk[k][i];
            grad[k] = 2.0 * s;
        }
#pragma unroll
        for (int l = 0; l < M; ++l) {
            double HD[NR];
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                double s = 0.0;
#pragma unroll
                for (int j = 0; j < NR; ++j) s += Hp[i][j] * Dk[l][j];
                HD[i] = s;
            }
#pragma unroll
            for (int k = 0; k < M; ++k) {
                double s = 0.0;
#pragma unroll
                for (int i = 0; i < NR; ++i) s += Dk[k][i] * HD[i];
                // second-order term: u . vec(1/2 (G_k G_l + G_l G_k) R)
                double GkDl[NR], GlDk[NR];
                gen_mul<D>(k, Dk[l], GkDl);
                gen_mul<D>(l, Dk[k], GlDk);
                double t2 = 0.0;
#pragma unroll
                for (int i = 0; i < NR; ++i) t2 += u[i] * 0.5 * (GkDl[i] + GlDk[i]);
                Hs[k][l] = 2.0 * s + 2.0 * t2;
            }
        }
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
            GICP_SOLVER_PROBE_TRY();
            double Hd[M][M], Hdi[M][M], ng[M], w[M];
#pragma unroll
            for (int k = 0; k < M; ++k) {
#pragma unroll
                for (int l = 0; l < M; ++l) Hd[k][l] = Hs[k][l] + (k == l ? lam * (hscale + 1e-300) : 0.0);
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
            if (ok) {
                double Rn[NR];
                rot_update<D>(w, R, Rn);
                const double fn = phi(Rn);
                wmax = 0.0;
#pragma unroll
                for (int k = 0; k < M; ++k) wmax = fmax(wmax, fabs(w[k]));
                // the model decrease -dd/2 is below the rounding of f: no step can be resolved, stop
                // instead of damping towards |w| < 1e-15 (the tries would only chase rounding noise)
                if (fn > f && -dd <= kFlatEps * fabs(f)) {
                    flat = true;
                    break;
                }
                if (fn <= f || wmax < 1e-15) {
                    if (fn <= f) {
#pragma unroll
                        for (int i = 0; i < NR; ++i) R[i] = Rn[i];
                        f = fn;
                    }
                    stepped = true;
                    quad = fn <= f && lam == 0.0 && wmax < kQuadStop;   // (f = fn when accepted)
                    lam = lam > 0.0 ? lam * 0.1 : 0.0;
                    if (lam < 1e-12) lam = 0.0;
                    break;
                }
            }
            lam = lam == 0.0 ? 1e-9 : lam * 10.0;
        }
        if (!stepped || flat || quad || wmax < 1e-15) break;
    }
    // t from the eliminated block
#pragma unroll
    for (int a = 0; a < D; ++a) {
        double s = kt[a];
#pragma unroll
        for (int c = 0; c < NR; ++c) s -= Kc[a][c] * (R[c] - Rk[c]);
        out.T[a * N1 + D] = tk[a] + s;
#pragma unroll
        for (int b = 0; b < D; ++b) out.T[a * N1 + b] = R[a * D + b];
    }
#pragma unroll
    for (int b = 0; b < D; ++b) out.T[D * N1 + b] = 0.0;
    out.T[D * N1 + D] = 1.0;
    out.loss = f;
    return out;
}

}  // namespace gicp
