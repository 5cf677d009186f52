// gicp_solver.cpp — host entry of the inner solve (the algorithm lives in gicp_solver.h, which
// the device-side iteration loop runs too, so host and GPU solves are the same code).
#include "gicp_solver.h"

namespace gicp {

int solve_pose(int d, const double* st, const double* Tk, double* Tout, double* loss_out) {
    if (d == 2) {
        const SolveOut<2> r = solve_pose_t<2>(st, Tk);
        for (int k = 0; k < 9; ++k) Tout[k] = r.T[k];
        if (loss_out) *loss_out = r.loss;
        return r.ok ? 0 : -2;
    }
    if (d == 3) {
        const SolveOut<3> r = solve_pose_t<3>(st, Tk);
        for (int k = 0; k < 16; ++k) Tout[k] = r.T[k];
        if (loss_out) *loss_out = r.loss;
        return r.ok ? 0 : -2;
    }
    return -1;
}

}  // namespace gicp
