// k_solve micro-benchmark and stage timer (diagnostic, not shipped).
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -mllvm -amdgpu-mfma-vgpr-form -I generalized-icp_amd/csrc \
//         -I include scripts/probes/solve_bench.hip -o scripts/probes/solve_bench
//   ./solve_bench STATS.bin POSES.bin   (scripts/capture_stats.py output, raw little-endian fp64)
// Runs the library's k_solve<3> on every captured pass (state = that pass's pose + statistics, fixed
// iterations), timed back to back with HIP events, then once per pass with s_memtime stage stamps.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>
#ifndef NO_STAMPS
__shared__ unsigned long long g_sst[16];
__device__ unsigned long long* g_stamp_out;
#define GICP_SOLVE_STAMP(k)                                                                  \
    do {                                                                                     \
        if (threadIdx.x == 0) {                                                              \
            if ((k) == 0)                                                                    \
                for (int q_ = 1; q_ < 14; ++q_) g_sst[q_] = 0;                               \
            g_sst[k] = __builtin_amdgcn_s_memtime();                                         \
            if ((k) == 0) g_sst[14] = __builtin_amdgcn_s_memrealtime();                      \
            if ((k) == 13) {                                                                 \
                g_sst[15] = __builtin_amdgcn_s_memrealtime();                                \
                unsigned long long* o = g_stamp_out;                                         \
                if (o)                                                                       \
                    for (int q_ = 0; q_ < 16; ++q_) o[q_] = g_sst[q_];                       \
            }                                                                                \
        }                                                                                    \
    } while (0)
#endif
#include "gicp_kernels.hip"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

int main(int argc, char** argv) {
    using gicp::IterState;
    FILE* fs = fopen(argv[1], "rb");
    FILE* fp = fopen(argv[2], "rb");
    if (!fs || !fp) { printf("usage: solve_bench STATS.bin POSES.bin\n"); return 1; }
    std::vector<IterState> H;
    double st[74], T[16];
    while (fread(st, 8, 74, fs) == 74 && fread(T, 8, 16, fp) == 16) {
        IterState s;
        memset(&s, 0, sizeof s);
        memcpy(s.T, T, sizeof T);
        memcpy(s.stats, st, sizeof st);
        s.tol = 1e-6;
        s.fixed = 1;
        s.converged_at = -1;
        s.prev_mse = 1.0 / 0.0;
        s.last_loss = 1.0 / 0.0;
        H.push_back(s);
    }
    const int P = (int)H.size();
    IterState* d;
    CK(hipMalloc(&d, sizeof(IterState) * P));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    float tot = 0.f;
    for (int r = 0; r < reps; ++r) {
        CK(hipMemcpy(d, H.data(), sizeof(IterState) * P, hipMemcpyHostToDevice));
        CK(hipEventRecord(e0));
        for (int p = 0; p < P; ++p) hipLaunchKernelGGL(gicp::k_solve<3>, dim3(1), dim3(64), 0, 0, d + p, (double*)nullptr);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (r > 0) tot += ms;
    }
    printf("k_solve<3> back to back: %.2f us per launch (events over %d launches)\n", tot * 1e3 / ((reps - 1) * P), P);
#ifdef NO_STAMPS
    return 0;
#endif
    unsigned long long* dst;
    CK(hipMalloc(&dst, 16 * 8 * P));
    CK(hipMemset(dst, 0, 16 * 8 * P));
    CK(hipMemset(d, 0, sizeof(IterState) * P));
    for (int p = 0; p < P; ++p) {
        unsigned long long* o = dst + 16 * p;
#ifndef NO_STAMPS
        CK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_out), &o, sizeof o));
#endif
        CK(hipMemcpy(d + p, &H[p], sizeof(IterState), hipMemcpyHostToDevice));
        hipLaunchKernelGGL(gicp::k_solve<3>, dim3(1), dim3(64), 0, 0, d + p, (double*)nullptr);
        CK(hipDeviceSynchronize());
    }
    std::vector<unsigned long long> hs(16 * P);
    CK(hipMemcpy(hs.data(), dst, 16 * 8 * P, hipMemcpyDeviceToHost));
    printf("stage stamps (s_memtime ticks from kernel start): load | setup | eval0 | newton starts (4) | last iteration: matvec, Hs, inv, rot | solved | end ; realtime us\n");
    for (int p = 0; p < P; ++p) {
        const unsigned long long* h = &hs[16 * p];
        printf("pass %2d:", p);
        const int order[] = {1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13};
        for (int k : order) printf(" %6lld", h[k] ? (long long)(h[k] - h[0]) : -1LL);
        printf("  rt %.2f us\n", (h[15] - h[14]) / 100.0);
    }
    return 0;
}
