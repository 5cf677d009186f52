// gicp_solver.cpp — host solve of the GICP inner problem from the reduced statistics.
//
// Reference: gicp.py:148-154 minimises sum_i r_i^T W_i r_i, r_i = q_i - R s_i - t, over
// (tx, ty, theta) with scipy's fmin_cg, starting at the previous optimum, with the
// correspondences and weights of the current iteration held fixed.  For fixed
// (q, W) that loss is exactly a quadratic form in z = (vec R, t):
//     f(z) = c0 - 2 g^T (z - z_k) + (z - z_k)^T H (z - z_k)
// whose coefficients the GPU reduces in one pass.  Here t is eliminated
// in closed form (Schur complement) and the rotation is found by damped Newton on
// SO(d) from R_k.  Everything is O(1) in the number of points.
#include <cmath>
#include <cstring>

#include "gicp_internal.h"

namespace gicp {

namespace {

constexpr int kMaxZ = 12;

struct Quad {
    int d = 3, nr = 9;
    double H[kMaxZ][kMaxZ];
    double g[kMaxZ];
    double c0 = 0.0, count = 0.0;
};

int sym_index(int d, int a, int b) {
    if (a > b) {
        const int t = a;
        a = b;
        b = t;
    }
    // row-major upper triangle: (0,0)(0,1)..(0,d-1)(1,1)..
    return a * d - a * (a - 1) / 2 + (b - a);
}

void expand(int d, const double* st, Quad& Q) {
    const int ns = d * (d + 1) / 2;
    Q.d = d;
    Q.nr = d * d;
    std::memset(Q.H, 0, sizeof(Q.H));
    std::memset(Q.g, 0, sizeof(Q.g));
    const double* A = st;
    const double* B = A + ns * ns;
    const double* C = B + ns * d;
    const double* gR = C + ns;
    const double* gt = gR + d * d;
    Q.c0 = gt[d];
    Q.count = gt[d + 1];
    const int nr = d * d;
    for (int a = 0; a < d; ++a)
        for (int i = 0; i < d; ++i) {
            for (int b = 0; b < d; ++b) {
                for (int j = 0; j < d; ++j) Q.H[a * d + i][b * d + j] = A[sym_index(d, a, b) * ns + sym_index(d, i, j)];
                const double v = B[sym_index(d, a, b) * d + i];
                Q.H[a * d + i][nr + b] = v;
                Q.H[nr + b][a * d + i] = v;
            }
            Q.g[a * d + i] = gR[a * d + i];
        }
    for (int a = 0; a < d; ++a) {
        for (int b = 0; b < d; ++b) Q.H[nr + a][nr + b] = C[sym_index(d, a, b)];
        Q.g[nr + a] = gt[a];
    }
}

// Solve M x = b (n <= 9) by Gaussian elimination with partial pivoting; false if singular.
bool lin_solve(int n, const double* Min, const double* b, double* x) {
    double M[kMaxZ][kMaxZ + 1];
    for (int i = 0; i < n; ++i) {
        for (int j = 0; j < n; ++j) M[i][j] = Min[i * n + j];
        M[i][n] = b[i];
    }
    for (int c = 0; c < n; ++c) {
        int p = c;
        for (int r = c + 1; r < n; ++r)
            if (std::fabs(M[r][c]) > std::fabs(M[p][c])) p = r;
        if (!(std::fabs(M[p][c]) > 0.0)) return false;
        if (p != c)
            for (int j = 0; j <= n; ++j) {
                const double t = M[c][j];
                M[c][j] = M[p][j];
                M[p][j] = t;
            }
        for (int r = c + 1; r < n; ++r) {
            const double f = M[r][c] / M[c][c];
            if (f == 0.0) continue;
            for (int j = c; j <= n; ++j) M[r][j] -= f * M[c][j];
        }
    }
    for (int i = n - 1; i >= 0; --i) {
        double s = M[i][n];
        for (int j = i + 1; j < n; ++j) s -= M[i][j] * x[j];
        x[i] = s / M[i][i];
    }
    for (int i = 0; i < n; ++i)
        if (!std::isfinite(x[i])) return false;
    return true;
}

// rotation by the exponential map, left-multiplied: R <- exp([w]) R
void apply_rot(int d, const double* w, const double* R, double* Rn) {
    double E[9];
    if (d == 2) {
        const double c = std::cos(w[0]), s = std::sin(w[0]);
        E[0] = c;
        E[1] = -s;
        E[2] = s;
        E[3] = c;
        for (int a = 0; a < 2; ++a)
            for (int b = 0; b < 2; ++b) Rn[a * 2 + b] = E[a * 2] * R[b] + E[a * 2 + 1] * R[2 + b];
        return;
    }
    const double th = std::sqrt(w[0] * w[0] + w[1] * w[1] + w[2] * w[2]);
    const double K[9] = {0, -w[2], w[1], w[2], 0, -w[0], -w[1], w[0], 0};
    double K2[9];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) K2[a * 3 + b] = K[a * 3] * K[b] + K[a * 3 + 1] * K[3 + b] + K[a * 3 + 2] * K[6 + b];
    double s1, s2;
    if (th < 1e-8) {
        s1 = 1.0 - th * th / 6.0;
        s2 = 0.5 - th * th / 24.0;
    } else {
        s1 = std::sin(th) / th;
        s2 = (1.0 - std::cos(th)) / (th * th);
    }
    for (int k = 0; k < 9; ++k) E[k] = (k % 4 == 0 ? 1.0 : 0.0) + s1 * K[k] + s2 * K2[k];
    for (int a = 0; a < 3; ++a)
        for (int b = 0; b < 3; ++b) Rn[a * 3 + b] = E[a * 3] * R[b] + E[a * 3 + 1] * R[3 + b] + E[a * 3 + 2] * R[6 + b];
}

// generator matrices of so(d): d=2 one, d=3 three (e_k x .)
void generator(int d, int k, double* G) {
    if (d == 2) {
        G[0] = 0;
        G[1] = -1;
        G[2] = 1;
        G[3] = 0;
        return;
    }
    const double e[3] = {k == 0 ? 1.0 : 0.0, k == 1 ? 1.0 : 0.0, k == 2 ? 1.0 : 0.0};
    const double K[9] = {0, -e[2], e[1], e[2], 0, -e[0], -e[1], e[0], 0};
    std::memcpy(G, K, sizeof(K));
}

void matmul(int d, const double* A, const double* B, double* C) {
    for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b) {
            double s = 0.0;
            for (int k = 0; k < d; ++k) s += A[a * d + k] * B[k * d + b];
            C[a * d + b] = s;
        }
}

}  // namespace

// Minimise the quadratic over SE(d) from T_k; returns 0 on success.
int solve_pose(int d, const double* st, const double* Tk, double* Tout, double* loss_out) {
    if (d != 2 && d != 3) return -1;
    const int n1 = d + 1;
    Quad Q;
    expand(d, st, Q);
    const int nr = d * d;
    double Rk[9], tk[3];
    for (int a = 0; a < d; ++a) {
        for (int b = 0; b < d; ++b) Rk[a * d + b] = Tk[a * n1 + b];
        tk[a] = Tk[a * n1 + d];
    }
    for (int k = 0; k < n1 * n1; ++k) Tout[k] = Tk[k];
    if (!(Q.count > 0.5)) {  // no correspondences: the loss is identically 0 (gicp.py:148 on all-zero W)
        if (loss_out) *loss_out = 0.0;
        return 0;
    }
    // eliminate t: Htt dt = gt - Htr dr
    double Htt[9], Ki[3 * 9], kt[3];
    for (int a = 0; a < d; ++a)
        for (int b = 0; b < d; ++b) Htt[a * d + b] = Q.H[nr + a][nr + b];
    if (!lin_solve(d, Htt, Q.g + nr, kt)) return -2;
    for (int c = 0; c < nr; ++c) {
        double col[3], x[3];
        for (int a = 0; a < d; ++a) col[a] = Q.H[nr + a][c];
        if (!lin_solve(d, Htt, col, x)) return -2;
        for (int a = 0; a < d; ++a) Ki[a * nr + c] = x[a];
    }
    // reduced quadratic in dr: c0' - 2 g'^T dr + dr^T H' dr
    double Hp[9][9], gp[9];
    for (int i = 0; i < nr; ++i) {
        for (int j = 0; j < nr; ++j) {
            double s = Q.H[i][j];
            for (int a = 0; a < d; ++a) s -= Q.H[i][nr + a] * Ki[a * nr + j];
            Hp[i][j] = s;
        }
        double s = Q.g[i];
        for (int a = 0; a < d; ++a) s -= Q.H[i][nr + a] * kt[a];
        gp[i] = s;
    }
    double c0p = Q.c0;
    for (int a = 0; a < d; ++a) c0p -= Q.g[nr + a] * kt[a];

    auto phi = [&](const double* R) {
        double dr[9], f = c0p;
        for (int i = 0; i < nr; ++i) dr[i] = R[i] - Rk[i];
        for (int i = 0; i < nr; ++i) {
            double hi = 0.0;
            for (int j = 0; j < nr; ++j) hi += Hp[i][j] * dr[j];
            f += dr[i] * hi - 2.0 * gp[i] * dr[i];
        }
        return f;
    };

    const int m = d == 2 ? 1 : 3;
    double R[9];
    std::memcpy(R, Rk, sizeof(double) * nr);
    double f = phi(R);
    double lam = 0.0;
    for (int it = 0; it < 200; ++it) {
        double dr[9], u[9];
        for (int i = 0; i < nr; ++i) dr[i] = R[i] - Rk[i];
        for (int i = 0; i < nr; ++i) {
            double s = -gp[i];
            for (int j = 0; j < nr; ++j) s += Hp[i][j] * dr[j];
            u[i] = s;  // (H' dr - g')
        }
        double Dk[3][9], grad[3], Hs[9];
        for (int k = 0; k < m; ++k) {
            double G[9];
            generator(d, k, G);
            matmul(d, G, R, Dk[k]);
            double s = 0.0;
            for (int i = 0; i < nr; ++i) s += u[i] * Dk[k][i];
            grad[k] = 2.0 * s;
        }
        for (int k = 0; k < m; ++k)
            for (int l = 0; l < m; ++l) {
                double s = 0.0;
                for (int i = 0; i < nr; ++i) {
                    double hi = 0.0;
                    for (int j = 0; j < nr; ++j) hi += Hp[i][j] * Dk[l][j];
                    s += Dk[k][i] * hi;
                }
                double Gk[9], Gl[9], GG[9], GG2[9], S2[9];
                generator(d, k, Gk);
                generator(d, l, Gl);
                matmul(d, Gk, Gl, GG);
                matmul(d, Gl, Gk, GG2);
                for (int i = 0; i < nr; ++i) GG[i] = 0.5 * (GG[i] + GG2[i]);
                matmul(d, GG, R, S2);
                double t2 = 0.0;
                for (int i = 0; i < nr; ++i) t2 += u[i] * S2[i];
                Hs[k * m + l] = 2.0 * s + 2.0 * t2;
            }
        double gmax = 0.0, hscale = 0.0;
        for (int k = 0; k < m; ++k) {
            gmax = std::fmax(gmax, std::fabs(grad[k]));
            hscale = std::fmax(hscale, std::fabs(Hs[k * m + k]));
        }
        if (gmax == 0.0) break;
        bool stepped = false;
        double wmax = 0.0;
        for (int tries = 0; tries < 60; ++tries) {
            double Hd[9], w[3], ng[3];
            for (int k = 0; k < m * m; ++k) Hd[k] = Hs[k];
            for (int k = 0; k < m; ++k) {
                Hd[k * m + k] += lam * (hscale + 1e-300);
                ng[k] = -grad[k];
            }
            bool ok = lin_solve(m, Hd, ng, w);
            // a Newton step must be a descent direction
            double dd = 0.0;
            for (int k = 0; k < m; ++k) dd += w[k] * grad[k];
            if (ok && dd < 0.0) {
                double Rn[9];
                apply_rot(d, w, R, Rn);
                const double fn = phi(Rn);
                wmax = 0.0;
                for (int k = 0; k < m; ++k) wmax = std::fmax(wmax, std::fabs(w[k]));
                if (fn <= f || wmax < 1e-15) {
                    if (fn <= f) {
                        std::memcpy(R, Rn, sizeof(double) * nr);
                        f = fn;
                    }
                    stepped = true;
                    lam = lam > 0.0 ? lam * 0.1 : 0.0;
                    if (lam < 1e-12) lam = 0.0;
                    break;
                }
            }
            lam = lam == 0.0 ? 1e-9 : lam * 10.0;
        }
        if (!stepped || wmax < 1e-15) break;
    }
    // t from the eliminated block
    double dr[9];
    for (int i = 0; i < nr; ++i) dr[i] = R[i] - Rk[i];
    for (int a = 0; a < d; ++a) {
        double s = kt[a];
        for (int c = 0; c < nr; ++c) s -= Ki[a * nr + c] * dr[c];
        Tout[a * n1 + d] = tk[a] + s;
        for (int b = 0; b < d; ++b) Tout[a * n1 + b] = R[a * d + b];
    }
    for (int b = 0; b < d; ++b) Tout[d * n1 + b] = 0.0;
    Tout[d * n1 + d] = 1.0;
    if (loss_out) *loss_out = f;
    return 0;
}

}  // namespace gicp
