// gicp_cg.cpp — the 2-D inner solve of gicp.py:148-154 on the host, natively.
//
// The reference minimises its loss over the offset (tx, ty, theta) with scipy.optimize.fmin_cg
// (gicp.py:152; SciPy is not vendored by the reference, SciPy 1.15.3 is the version its golden vectors were
// captured with).  Its inexact stopping is part of the reference's behaviour (SURVEY.md
// §0.4), so the inner solve here is not a better minimiser but the same algorithm, restated from SciPy
// 1.15.3's published sources, step for step and rounding for rounding:
//   _optimize.py     _minimize_cg: Polak-Ribiere+ CG, gtol 1e-5 (inf-norm), maxiter 200 n, the
//                    sufficient-descent extra condition (sigma_3 = 0.01), c1 = 1e-4, c2 = 0.4
//                    _line_search_wolfe12: line_search_wolfe1 (MINPACK-2 dcsrch), then line_search_wolfe2
//   _linesearch.py   scalar_search_wolfe1 / scalar_search_wolfe2 / _zoom / _cubicmin / _quadmin
//   _dcsrch.py       DCSRCH._iterate, dcstep (More & Thuente)
//   _differentiable_functions.py  ScalarFunction's one-point memo (what nfev / ngev count)
// The objective is the closed form of the loss on the pass's 26 statistics: per evaluation
// O(1) instead of the reference's O(N) (gicp.py:52-76).  np.dot of SciPy's small vectors is an FMA chain
// (OpenBLAS ddot; checked against numpy in tests/test_cg_native.py), so dot() below is one too; every
// other operation is the elementwise IEEE operation NumPy performs.  tests/test_cg_native.py pins the result
// bit for bit against scipy's fmin_cg run on the same closed form.
//
// The algorithm, control flow and constants below are derived from SciPy, whose licence follows:
//
//   Copyright (c) 2001-2002 Enthought, Inc. 2003, SciPy Developers.
//   All rights reserved.
//
//   Redistribution and use in source and binary forms, with or without modification, are permitted provided
//   that the following conditions are met:
//
//   1. Redistributions of source code must retain the above copyright notice, this list of conditions and the
//      following disclaimer.
//   2. Redistributions in binary form must reproduce the above copyright notice, this list of conditions and
//      the following disclaimer in the documentation and/or other materials provided with the distribution.
//   3. Neither the name of the copyright holder nor the names of its contributors may be used to endorse or
//      promote products derived from this software without specific prior written permission.
//
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS IS" AND ANY EXPRESS OR IMPLIED
//   WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A
//   PARTICULAR PURPOSE ARE DISCLAIMED. IN NO EVENT SHALL THE COPYRIGHT HOLDER OR CONTRIBUTORS BE LIABLE FOR ANY
//   DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL DAMAGES (INCLUDING, BUT NOT LIMITED TO,
//   PROCUREMENT OF SUBSTITUTE GOODS OR SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION)
//   HOWEVER CAUSED AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY, OR TORT (INCLUDING
//   NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE OF THIS SOFTWARE, EVEN IF ADVISED OF THE
//   POSSIBILITY OF SUCH DAMAGE.
//
// The line search follows SciPy's _dcsrch.py, SciPy's translation of MINPACK-2's dcsrch / dcstep
// (J. J. Moré and D. J. Thuente, Argonne National Laboratory and University of Minnesota).
#pragma clang fp contract(off)

#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/gicp_hip.h"

namespace {

constexpr int N = 3;   // (tx, ty, theta)

// np.dot of two float64 vectors (OpenBLAS ddot: fused multiply-adds from the first element)
double dot(const double* a, const double* b, int n = N) {
    double s = 0.0;
    for (int i = 0; i < n; ++i) s = std::fma(a[i], b[i], s);
    return s;
}
double maxabs(const double* a) {   // vecnorm(x, inf) = np.amax(np.abs(x)) (NaN propagates)
    double m = std::fabs(a[0]);
    for (int i = 1; i < N; ++i) {
        const double v = std::fabs(a[i]);
        if (std::isnan(v) || v > m) m = std::isnan(m) ? m : v;
    }
    return m;
}
// Python's max(a, b) / min(a, b): the first argument unless the second compares greater / smaller
double pymax(double a, double b) { return b > a ? b : a; }
double pymin(double a, double b) { return b < a ? b : a; }
double npclip(double x, double lo, double hi) {   // np.clip: minimum(maximum(x, lo), hi), NaN propagates
    if (std::isnan(x)) return x;
    return x < lo ? lo : (x > hi ? hi : x);
}
double npsign(double x) { return std::isnan(x) ? x : (x > 0 ? 1.0 : (x < 0 ? -1.0 : 0.0)); }
double sq(double x) { return std::pow(x, 2.0); }   // Python / NumPy scalar x ** 2

// The loss of gicp.py:52-58 on one pass's statistics, as a function of the offset x = (tx, ty, theta):
// f = c0 - 2 g4.dz + dz.H4.dz with dz = (tx, ty, cos theta, sin theta) - z_k
struct Closed2D {
    double H4[4][4], g4[4], c0, zk[4];

    void init(const double* st, const double* Tk) {
        // 2-D layout (gicp_internal.h nstat<2>): A[3][3], B[3][2], C[3], gR[2][2], gt[2], c0, count;
        // symmetric pairs (0,0) (0,1) (1,1); z6 = (R00, R01, R10, R11, tx, ty) = L (tx, ty, cos, sin)
        auto pos = [](int a, int b) { return a == b ? (a == 0 ? 0 : 2) : 1; };
        const double* A = st;
        const double* B = st + 9;
        const double* Cc = st + 15;
        const double* gR = st + 18;
        const double* gt = st + 22;
        double H[6][6];
        for (int a = 0; a < 2; ++a)
            for (int i = 0; i < 2; ++i) {
                for (int b = 0; b < 2; ++b) {
                    for (int j = 0; j < 2; ++j) H[a * 2 + i][b * 2 + j] = A[pos(a, b) * 3 + pos(i, j)];
                    H[a * 2 + i][4 + b] = H[4 + b][a * 2 + i] = B[pos(a, b) * 2 + i];
                }
            }
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) H[4 + a][4 + b] = Cc[pos(a, b)];
        const double g6[6] = {gR[0], gR[1], gR[2], gR[3], gt[0], gt[1]};
        static const double L[6][4] = {{0, 0, 1, 0}, {0, 0, 0, -1}, {0, 0, 0, 1}, {0, 0, 1, 0}, {1, 0, 0, 0}, {0, 1, 0, 0}};
        for (int p = 0; p < 4; ++p) {   // H4 = L^T H L, g4 = L^T g: sums in index order
            double gs = 0.0;
            for (int i = 0; i < 6; ++i) gs += L[i][p] * g6[i];
            g4[p] = gs;
            for (int q = 0; q < 4; ++q) {
                double s = 0.0;
                for (int i = 0; i < 6; ++i)
                    for (int j = 0; j < 6; ++j) s += L[i][p] * H[i][j] * L[j][q];
                H4[p][q] = s;
            }
        }
        c0 = st[24];
        zk[0] = Tk[2];
        zk[1] = Tk[5];
        zk[2] = Tk[0];
        zk[3] = Tk[3];
    }
    void terms(const double* x, double* dz, double* Hd, double& c, double& s) const {
        c = std::cos(x[2]);
        s = std::sin(x[2]);
        dz[0] = x[0] - zk[0];
        dz[1] = x[1] - zk[1];
        dz[2] = c - zk[2];
        dz[3] = s - zk[3];
        for (int p = 0; p < 4; ++p) {
            double h = 0.0;
            for (int q = 0; q < 4; ++q) h += H4[p][q] * dz[q];
            Hd[p] = h;
        }
    }
    double f(const double* x) const {
        double dz[4], Hd[4], c, s;
        terms(x, dz, Hd, c, s);
        double gz = 0.0, q = 0.0;
        for (int p = 0; p < 4; ++p) gz += g4[p] * dz[p];
        for (int p = 0; p < 4; ++p) q += dz[p] * Hd[p];
        return (c0 - 2.0 * gz) + q;
    }
    void g(const double* x, double* out) const {
        double dz[4], Hd[4], c, s;
        terms(x, dz, Hd, c, s);
        double v[4];
        for (int p = 0; p < 4; ++p) v[p] = -2.0 * g4[p] + 2.0 * Hd[p];
        out[0] = v[0];
        out[1] = v[1];
        out[2] = -s * v[2] + c * v[3];
    }
};

// ScalarFunction's memo: one point, its value and gradient evaluated at most once each (nfev / ngev)
struct Fn {
    const Closed2D& o;
    double x[N];
    double fx = 0.0, gx[N] = {0, 0, 0};
    bool fu = false, gu = false;
    int nfev = 0, ngev = 0;
    Fn(const Closed2D& ob, const double* x0) : o(ob) {
        std::memcpy(x, x0, sizeof(x));
        fun(x0);    // ScalarFunction.__init__: _update_fun, then _update_grad
        grad(x0);
    }
    void at(const double* xn) {
        bool eq = true;
        for (int i = 0; i < N; ++i) eq = eq && xn[i] == x[i];   // np.array_equal
        if (!eq) {
            std::memcpy(x, xn, sizeof(x));
            fu = gu = false;
        }
    }
    double fun(const double* xn) {
        at(xn);
        if (!fu) {
            fx = o.f(x);
            ++nfev;
            fu = true;
        }
        return fx;
    }
    const double* grad(const double* xn) {
        at(xn);
        if (!gu) {
            o.g(x, gx);
            ++ngev;
            gu = true;
        }
        return gx;
    }
};

// _minimize_cg's state shared with its line-search callbacks
struct CG {
    Fn& F;
    double xk[N], pk[N], gfk[N], deltak = 0.0;
    static constexpr double gtol = 1e-5, c1 = 1e-4, c2 = 0.4, sigma3 = 0.01;
    // polak_ribiere_powell_step's cached result
    bool cached = false;
    double c_alpha = 0.0, c_x[N], c_p[N], c_g[N], c_gnorm = 0.0;

    explicit CG(Fn& f) : F(f) {}

    void xat(double s, double* out) const {   // xk + s * pk
        for (int i = 0; i < N; ++i) out[i] = xk[i] + s * pk[i];
    }
    double phi(double s) {
        double x[N];
        xat(s, x);
        return F.fun(x);
    }
    // derphi: gradient at xk + s pk into gval, returns gval . pk
    double derphi(double s, double* gval) {
        double x[N];
        xat(s, x);
        std::memcpy(gval, F.grad(x), sizeof(double) * N);
        return dot(gval, pk);
    }
    void prp_step(double alpha, const double* gk1_in, double* x1, double* p1, double* g1, double& gnorm) {
        xat(alpha, x1);
        if (gk1_in) std::memcpy(g1, gk1_in, sizeof(double) * N);
        else std::memcpy(g1, F.grad(x1), sizeof(double) * N);
        double yk[N];
        for (int i = 0; i < N; ++i) yk[i] = g1[i] - gfk[i];
        const double beta = pymax(0.0, dot(yk, g1) / deltak);
        for (int i = 0; i < N; ++i) p1[i] = -g1[i] + beta * pk[i];
        gnorm = maxabs(g1);
    }
    bool descent_condition(double alpha, const double* gk1) {
        prp_step(alpha, gk1, c_x, c_p, c_g, c_gnorm);
        cached = true;
        c_alpha = alpha;
        if (c_gnorm <= gtol) return true;
        return dot(c_p, c_g) <= -sigma3 * dot(c_g, c_g);
    }

    // ---- line_search_wolfe1: scalar_search_wolfe1 + DCSRCH (MINPACK-2) ----
    struct Dcsrch {
        double ftol, gtol, xtol, stpmin, stpmax;
        bool brackt = false;
        int stage = 1;
        double ginit = 0, gtest = 0, gx = 0, gy = 0, finit = 0, fx = 0, fy = 0, stx = 0, sty = 0, stmin = 0, stmax = 0,
               width = 0, width1 = 0;
    };
    enum Task { FG, START, CONV, WARN, ERR };

    static void dcstep(double& stx, double& fx, double& dx, double& sty, double& fy, double& dy, double& stp, double fp,
                       double dp, bool& brackt, double stpmin, double stpmax) {
        const double sgnd = npsign(dp) * npsign(dx);
        auto m3 = [](double a, double b, double c) { return pymax(pymax(a, b), c); };   // Python max(a, b, c)
        double stpf;
        if (fp > fx) {
            const double theta = 3.0 * (fx - fp) / (stp - stx) + dx + dp;
            const double s = m3(std::fabs(theta), std::fabs(dx), std::fabs(dp));
            double gamma = s * std::sqrt(sq(theta / s) - (dx / s) * (dp / s));
            if (stp < stx) gamma = -gamma;
            const double p = (gamma - dx) + theta;
            const double q = ((gamma - dx) + gamma) + dp;
            const double r = p / q;
            const double stpc = stx + r * (stp - stx);
            const double stpq = stx + ((dx / ((fx - fp) / (stp - stx) + dx)) / 2.0) * (stp - stx);
            if (std::fabs(stpc - stx) <= std::fabs(stpq - stx)) stpf = stpc;
            else stpf = stpc + (stpq - stpc) / 2.0;
            brackt = true;
        } else if (sgnd < 0.0) {
            const double theta = 3 * (fx - fp) / (stp - stx) + dx + dp;
            const double s = m3(std::fabs(theta), std::fabs(dx), std::fabs(dp));
            double gamma = s * std::sqrt(sq(theta / s) - (dx / s) * (dp / s));
            if (stp > stx) gamma = -gamma;
            const double p = (gamma - dp) + theta;
            const double q = ((gamma - dp) + gamma) + dx;
            const double r = p / q;
            const double stpc = stp + r * (stx - stp);
            const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
            stpf = std::fabs(stpc - stp) > std::fabs(stpq - stp) ? stpc : stpq;
            brackt = true;
        } else if (std::fabs(dp) < std::fabs(dx)) {
            const double theta = 3 * (fx - fp) / (stp - stx) + dx + dp;
            const double s = m3(std::fabs(theta), std::fabs(dx), std::fabs(dp));
            double gamma = s * std::sqrt(pymax(0.0, sq(theta / s) - (dx / s) * (dp / s)));
            if (stp > stx) gamma = -gamma;
            const double p = (gamma - dp) + theta;
            const double q = (gamma + (dx - dp)) + gamma;
            const double r = p / q;
            double stpc;
            if (r < 0 && gamma != 0) stpc = stp + r * (stx - stp);
            else if (stp > stx) stpc = stpmax;
            else stpc = stpmin;
            const double stpq = stp + (dp / (dp - dx)) * (stx - stp);
            if (brackt) {
                stpf = std::fabs(stpc - stp) < std::fabs(stpq - stp) ? stpc : stpq;
                if (stp > stx) stpf = pymin(stp + 0.66 * (sty - stp), stpf);
                else stpf = pymax(stp + 0.66 * (sty - stp), stpf);
            } else {
                stpf = std::fabs(stpc - stp) > std::fabs(stpq - stp) ? stpc : stpq;
                stpf = npclip(stpf, stpmin, stpmax);
            }
        } else {
            if (brackt) {
                const double theta = 3.0 * (fp - fy) / (sty - stp) + dy + dp;
                const double s = m3(std::fabs(theta), std::fabs(dy), std::fabs(dp));
                double gamma = s * std::sqrt(sq(theta / s) - (dy / s) * (dp / s));
                if (stp > sty) gamma = -gamma;
                const double p = (gamma - dp) + theta;
                const double q = ((gamma - dp) + gamma) + dy;
                const double r = p / q;
                stpf = stp + r * (sty - stp);
            } else if (stp > stx) {
                stpf = stpmax;
            } else {
                stpf = stpmin;
            }
        }
        if (fp > fx) {
            sty = stp;
            fy = fp;
            dy = dp;
        } else {
            if (sgnd < 0) {
                sty = stx;
                fy = fx;
                dy = dx;
            }
            stx = stp;
            fx = fp;
            dx = dp;
        }
        stp = stpf;
    }

    static Task dcsrch_iterate(Dcsrch& D, double& stp, double f, double g, Task task) {
        constexpr double p5 = 0.5, p66 = 0.66, xtrapl = 1.1, xtrapu = 4.0;
        if (task == START) {
            if (stp < D.stpmin || stp > D.stpmax || g >= 0 || D.ftol < 0 || D.gtol < 0 || D.xtol < 0 || D.stpmin < 0 ||
                D.stpmax < D.stpmin)
                return ERR;
            D.brackt = false;
            D.stage = 1;
            D.finit = f;
            D.ginit = g;
            D.gtest = D.ftol * D.ginit;
            D.width = D.stpmax - D.stpmin;
            D.width1 = D.width / p5;
            D.stx = 0.0;
            D.fx = D.finit;
            D.gx = D.ginit;
            D.sty = 0.0;
            D.fy = D.finit;
            D.gy = D.ginit;
            D.stmin = 0;
            D.stmax = stp + xtrapu * stp;
            return FG;
        }
        const double ftest = D.finit + stp * D.gtest;
        if (D.stage == 1 && f <= ftest && g >= 0) D.stage = 2;
        Task t = FG;
        if (D.brackt && (stp <= D.stmin || stp >= D.stmax)) t = WARN;
        if (D.brackt && D.stmax - D.stmin <= D.xtol * D.stmax) t = WARN;
        if (stp == D.stpmax && f <= ftest && g <= D.gtest) t = WARN;
        if (stp == D.stpmin && (f > ftest || g >= D.gtest)) t = WARN;
        if (f <= ftest && std::fabs(g) <= D.gtol * -D.ginit) t = CONV;
        if (t == WARN || t == CONV) return t;
        if (D.stage == 1 && f <= D.fx && f > ftest) {
            const double fm = f - stp * D.gtest;
            double fxm = D.fx - D.stx * D.gtest;
            double fym = D.fy - D.sty * D.gtest;
            const double gm = g - D.gtest;
            double gxm = D.gx - D.gtest;
            double gym = D.gy - D.gtest;
            dcstep(D.stx, fxm, gxm, D.sty, fym, gym, stp, fm, gm, D.brackt, D.stmin, D.stmax);
            D.fx = fxm + D.stx * D.gtest;
            D.fy = fym + D.sty * D.gtest;
            D.gx = gxm + D.gtest;
            D.gy = gym + D.gtest;
        } else {
            dcstep(D.stx, D.fx, D.gx, D.sty, D.fy, D.gy, stp, f, g, D.brackt, D.stmin, D.stmax);
        }
        if (D.brackt) {
            if (std::fabs(D.sty - D.stx) >= p66 * D.width1) stp = D.stx + p5 * (D.sty - D.stx);
            D.width1 = D.width;
            D.width = std::fabs(D.sty - D.stx);
        }
        if (D.brackt) {
            D.stmin = pymin(D.stx, D.sty);
            D.stmax = pymax(D.stx, D.sty);
        } else {
            D.stmin = stp + xtrapl * (stp - D.stx);
            D.stmax = stp + xtrapu * (stp - D.stx);
        }
        stp = npclip(stp, D.stpmin, D.stpmax);
        if ((D.brackt && (stp <= D.stmin || stp >= D.stmax)) || (D.brackt && D.stmax - D.stmin <= D.xtol * D.stmax))
            stp = D.stx;
        return FG;
    }

    // line_search_wolfe1 -> (ok, stp, phi1 = f at stp, phi0, gval = gradient at stp)
    bool wolfe1(double old_fval, double old_old_fval, double& stp_out, double& phi1, double& phi0_out, double* gval) {
        std::memcpy(gval, gfk, sizeof(double) * N);
        const double derphi0 = dot(gfk, pk);
        const double phi0 = old_fval;
        double alpha1;
        if (derphi0 != 0) {   // (old_phi0 is never None here)
            alpha1 = pymin(1.0, 1.01 * 2 * (phi0 - old_old_fval) / derphi0);
            if (alpha1 < 0) alpha1 = 1.0;
        } else {
            alpha1 = 1.0;
        }
        Dcsrch D{c1, c2, 1e-14, 1e-100, 1e100};
        double stp = alpha1, f1 = phi0, g1 = derphi0;
        Task task = START;
        bool ok = false;
        int i = 0;
        for (; i < 100; ++i) {
            task = dcsrch_iterate(D, stp, f1, g1, task);
            if (!std::isfinite(stp)) {
                task = WARN;
                break;
            }
            if (task == FG) {
                f1 = phi(stp);
                g1 = derphi(stp, gval);
            } else {
                break;
            }
        }
        ok = i < 100 && task != ERR && task != WARN;
        stp_out = stp;
        phi1 = f1;
        phi0_out = phi0;
        return ok;
    }

    // ---- line_search_wolfe2: scalar_search_wolfe2 + _zoom ----
    struct W2 {
        CG& cg;
        double gval[N];
        bool have_ga = false;
        double gval_alpha = 0.0;
        double derphi(double a) {
            const double d = cg.derphi(a, gval);
            have_ga = true;
            gval_alpha = a;
            return d;
        }
        bool extra(double a) {   // extra_condition2
            if (!have_ga || gval_alpha != a) derphi(a);
            return cg.descent_condition(a, gval);
        }
    };

    static bool cubicmin(double a, double fa, double fpa, double b, double fb, double c, double fc, double& xmin) {
        // np.errstate(divide/over/invalid='raise'): any division by zero or non-finite intermediate -> None
        const double C = fpa, db = b - a, dc = c - a;
        const double denom = sq(db * dc) * (db - dc);
        const double d00 = sq(dc), d01 = -sq(db), d10 = -std::pow(dc, 3.0), d11 = std::pow(db, 3.0);
        const double v0 = fb - fa - C * db, v1 = fc - fa - C * dc;
        double A = std::fma(d00, v0, d01 * v1);   // np.dot(2x2, 2): fma(M[i][0], v0, M[i][1] v1)
        double B = std::fma(d10, v0, d11 * v1);
        const double pre[] = {db, dc, db * dc, denom, d00, d01, d10, d11, v0, v1, A, B};
        for (double v : pre)
            if (!std::isfinite(v)) return false;
        if (denom == 0.0) return false;
        A /= denom;
        B /= denom;
        const double radical = B * B - 3 * A * C;
        if (!std::isfinite(A) || !std::isfinite(B) || !std::isfinite(radical) || radical < 0 || 3 * A == 0.0) return false;
        xmin = a + (-B + std::sqrt(radical)) / (3 * A);
        return std::isfinite(xmin);
    }
    static bool quadmin(double a, double fa, double fpa, double b, double fb, double& xmin) {
        const double D = fa, C = fpa, db = b - a * 1.0;
        const double dd = db * db;
        if (!std::isfinite(dd) || dd == 0.0) return false;
        const double num = fb - D - C * db;
        const double B = num / dd;
        if (!std::isfinite(num) || !std::isfinite(B) || 2.0 * B == 0.0) return false;
        xmin = a - C / (2.0 * B);
        return std::isfinite(xmin);
    }

    bool zoom(W2& w, double a_lo, double a_hi, double phi_lo, double phi_hi, double derphi_lo, double phi0,
              double derphi0, double& a_star, double& val_star, bool& have_dstar) {
        constexpr int maxiter = 10;
        constexpr double delta1 = 0.2, delta2 = 0.1;
        double phi_rec = phi0, a_rec = 0;
        int i = 0;
        double a_j = 0.0, cchk = 0.0;
        for (;;) {
            const double dalpha = a_hi - a_lo;
            double a, b;
            if (dalpha < 0) {
                a = a_hi;
                b = a_lo;
            } else {
                a = a_lo;
                b = a_hi;
            }
            bool none = true;
            if (i > 0) {
                cchk = delta1 * dalpha;
                none = !cubicmin(a_lo, phi_lo, derphi_lo, a_hi, phi_hi, a_rec, phi_rec, a_j);
            }
            if (i == 0 || none || a_j > b - cchk || a_j < a + cchk) {
                const double qchk = delta2 * dalpha;
                const bool qnone = !quadmin(a_lo, phi_lo, derphi_lo, a_hi, phi_hi, a_j);
                if (qnone || a_j > b - qchk || a_j < a + qchk) a_j = a_lo + 0.5 * dalpha;
            }
            const double phi_aj = phi(a_j);
            if (phi_aj > phi0 + c1 * a_j * derphi0 || phi_aj >= phi_lo) {
                phi_rec = phi_hi;
                a_rec = a_hi;
                a_hi = a_j;
                phi_hi = phi_aj;
            } else {
                const double derphi_aj = w.derphi(a_j);
                if (std::fabs(derphi_aj) <= -c2 * derphi0 && w.extra(a_j)) {
                    a_star = a_j;
                    val_star = phi_aj;
                    have_dstar = true;
                    return true;
                }
                if (derphi_aj * (a_hi - a_lo) >= 0) {
                    phi_rec = phi_hi;
                    a_rec = a_hi;
                    a_hi = a_lo;
                    phi_hi = phi_lo;
                } else {
                    phi_rec = phi_lo;
                    a_rec = a_lo;
                }
                a_lo = a_j;
                phi_lo = phi_aj;
                derphi_lo = derphi_aj;
            }
            ++i;
            if (i > maxiter) return false;
        }
    }

    // line_search_wolfe2 -> (ok, alpha, phi_star, old_fval (phi0 or old_phi0), gval or none)
    bool wolfe2(double old_fval, double old_old_fval, double& alpha_out, double& phi_star, double& phi0_out,
                double* gval_out, bool& have_g) {
        constexpr double amax = 1e100;
        constexpr int maxiter = 10;
        W2 w{*this, {0, 0, 0}};
        const double derphi0 = dot(gfk, pk);
        double phi0 = old_fval;
        double alpha0 = 0;
        double alpha1 = derphi0 != 0 ? pymin(1.0, 1.01 * 2 * (phi0 - old_old_fval) / derphi0) : 1.0;
        if (alpha1 < 0) alpha1 = 1.0;
        alpha1 = pymin(alpha1, amax);
        double phi_a1 = phi(alpha1);
        double phi_a0 = phi0, derphi_a0 = derphi0;
        bool found = false, have_d = false;
        double alpha_star = 0.0;
        int i = 0;
        for (; i < maxiter; ++i) {
            if (alpha1 == 0 || alpha0 > amax) {   // rounding errors / beyond amax: no step
                phi_star = phi0;
                phi0 = old_old_fval;
                found = false;
                have_d = false;
                break;
            }
            const bool not_first = i > 0;
            if (phi_a1 > phi0 + c1 * alpha1 * derphi0 || (phi_a1 >= phi_a0 && not_first)) {
                found = zoom(w, alpha0, alpha1, phi_a0, phi_a1, derphi_a0, phi0, derphi0, alpha_star, phi_star, have_d);
                break;
            }
            const double derphi_a1 = w.derphi(alpha1);
            if (std::fabs(derphi_a1) <= -c2 * derphi0 && w.extra(alpha1)) {
                alpha_star = alpha1;
                phi_star = phi_a1;
                have_d = found = true;
                break;
            }
            if (derphi_a1 >= 0) {
                found = zoom(w, alpha1, alpha0, phi_a1, phi_a0, derphi_a1, phi0, derphi0, alpha_star, phi_star, have_d);
                break;
            }
            const double alpha2 = pymin(2 * alpha1, amax);
            alpha0 = alpha1;
            alpha1 = alpha2;
            phi_a0 = phi_a1;
            phi_a1 = phi(alpha1);
            derphi_a0 = derphi_a1;
        }
        if (i == maxiter) {   // for-else: not converged, the last trial step is returned without a gradient
            alpha_star = alpha1;
            phi_star = phi_a1;
            have_d = false;
            found = true;
        }
        alpha_out = alpha_star;
        phi0_out = phi0;
        have_g = have_d;
        if (have_d) std::memcpy(gval_out, w.gval, sizeof(double) * N);
        return found;
    }
};

}  // namespace

extern "C" int gicp_cg_inner_2d(const double* stats, const double* T_k, const double* x0, double* xopt, double* fopt,
                                int32_t* counts) {
    if (!stats || !T_k || !x0 || !xopt) return GICP_E_INVALID;
    Closed2D ob;
    ob.init(stats, T_k);
    Fn F(ob, x0);
    CG cg(F);
    std::memcpy(cg.xk, x0, sizeof(double) * N);
    const int maxiter = 200 * N;
    double old_fval = F.fun(cg.xk);
    std::memcpy(cg.gfk, F.grad(cg.xk), sizeof(double) * N);
    int k = 0;
    double old_old_fval = old_fval + std::sqrt(dot(cg.gfk, cg.gfk)) / 2;   // np.linalg.norm: sqrt(x.dot(x))
    int warnflag = 0;
    for (int i = 0; i < N; ++i) cg.pk[i] = -cg.gfk[i];
    double gnorm = maxabs(cg.gfk);
    while (gnorm > CG::gtol && k < maxiter) {
        cg.deltak = dot(cg.gfk, cg.gfk);
        cg.cached = false;
        double alpha = 0.0, f1 = 0.0, f0 = 0.0, g1[N] = {0, 0, 0};
        bool have_g = true;
        bool ok = cg.wolfe1(old_fval, old_old_fval, alpha, f1, f0, g1);
        if (ok && !cg.descent_condition(alpha, g1)) ok = false;   // extra_condition rejects the step
        if (!ok) ok = cg.wolfe2(old_fval, old_old_fval, alpha, f1, f0, g1, have_g);
        if (!ok) {   // _LineSearchError
            warnflag = 2;
            break;
        }
        old_fval = f1;
        old_old_fval = f0;
        double x1[N], p1[N], gk1[N], gn1;
        if (cg.cached && alpha == cg.c_alpha) {
            std::memcpy(x1, cg.c_x, sizeof(x1));
            std::memcpy(p1, cg.c_p, sizeof(p1));
            std::memcpy(gk1, cg.c_g, sizeof(gk1));
            gn1 = cg.c_gnorm;
        } else {
            cg.prp_step(alpha, have_g ? g1 : nullptr, x1, p1, gk1, gn1);
        }
        std::memcpy(cg.xk, x1, sizeof(x1));
        std::memcpy(cg.pk, p1, sizeof(p1));
        std::memcpy(cg.gfk, gk1, sizeof(gk1));
        gnorm = gn1;
        ++k;
    }
    if (warnflag != 2) {
        bool nan = std::isnan(gnorm) || std::isnan(old_fval);
        for (int i = 0; i < N; ++i) nan = nan || std::isnan(cg.xk[i]);
        if (k >= maxiter) warnflag = 1;
        else if (nan) warnflag = 3;
    }
    std::memcpy(xopt, cg.xk, sizeof(double) * N);
    if (fopt) *fopt = old_fval;
    if (counts) {
        counts[0] = F.nfev;
        counts[1] = F.ngev;
        counts[2] = warnflag;
        counts[3] = k;
    }
    return GICP_OK;
}
