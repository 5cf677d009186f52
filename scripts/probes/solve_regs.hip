// Register probe of the one-wave solve (diagnostic, not shipped): the solve compiled alone under k_corr's
// occupancy target, so its VGPR need is seen in seconds instead of a full kernels build.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -I generalized-icp_amd/csrc -I include \
//         scripts/probes/solve_regs.hip -o /tmp/solve_regs.s -Rpass-analysis=kernel-resource-usage
#include "gicp_solve_dev.h"
namespace gicp {
template <int D>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(6, 6))) k_probe(IterState* S, double* hist) {
    __shared__ IterState s_hdr;
    __shared__ double s_st[80];
    __shared__ SolveLds<D> s_sl;
    const double* g = reinterpret_cast<const double*>(S);
    if (threadIdx.x < 110) reinterpret_cast<double*>(&s_hdr)[threadIdx.x] = g[threadIdx.x];
    if (threadIdx.x < 80) s_st[threadIdx.x] = g[threadIdx.x + 40];
    __syncthreads();
    if (threadIdx.x >= 64) return;
    solve_update<D>(S, &s_hdr, s_st, s_sl, hist);
}
template __global__ void k_probe<3>(IterState*, double*);
template __global__ void k_probe<2>(IterState*, double*);
}
