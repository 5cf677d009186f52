// Back-to-back launch period of small kernels on one stream (diagnostic, not shipped): what the per-iteration
// kernel boundary costs k_corr's small grids.  hipcc -O3 --offload-arch=gfx950 launch_gap.hip -o launch_gap
//   ./launch_gap   -> period per launch (us) for: empty 1 WG; 79 / 527 / 1536 WGs x 256 threads; a 700-B
//                     kernel argument; 79 WGs writing 1 KB each; 79 WGs with an agent-scope ticket
#include <hip/hip_runtime.h>
#include <cstdio>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct Big {
    double v[87];   // ~700 B, like CorrArgs
    int* out;
};

__global__ void k_empty(int* out) {
    if (out && threadIdx.x == 1000000) out[0] = 1;
}
__global__ void k_big(Big b) {
    if (b.out && threadIdx.x == 1000000) b.out[0] = (int)b.v[3];
}
__global__ void k_write(double* buf) {   // each workgroup writes 1 KB (dirty lines at the kernel end)
    if (threadIdx.x < 128) buf[blockIdx.x * 128 + threadIdx.x] = (double)threadIdx.x;
}
__global__ void k_ticket(unsigned* t, double* out) {   // last arriver of all workgroups does one more round trip
    __shared__ int last;
    if (threadIdx.x == 0) last = __hip_atomic_fetch_add(t, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
    __syncthreads();
    if (last && threadIdx.x == 0) {
        *t = 0;
        out[0] += 1.0;
    }
}

template <class F>
float period(F launch, int n) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (int i = 0; i < 50; ++i) launch();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a, 0);
    for (int i = 0; i < n; ++i) launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms * 1e3f / n;
}

int main() {
    int* d_out;
    double* d_buf;
    unsigned* d_t;
    CK(hipMalloc(&d_out, 64));
    CK(hipMalloc(&d_buf, 2048 * 1024));
    CK(hipMalloc(&d_t, 64));
    CK(hipMemset(d_t, 0, 64));
    Big b{};
    b.out = d_out;
    const int n = 2000;
    printf("empty 1 WG x 64        : %.2f us\n", period([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, 0, d_out); }, n));
    for (int g : {79, 527, 625, 1536, 5000})
        printf("empty %4d WG x 256     : %.2f us\n", g, period([&] { hipLaunchKernelGGL(k_empty, dim3(g), dim3(256), 0, 0, d_out); }, n));
    printf("700-B arg, 79 WG x 256 : %.2f us\n", period([&] { hipLaunchKernelGGL(k_big, dim3(79), dim3(256), 0, 0, b); }, n));
    printf("1 KB write, 79 WG      : %.2f us\n", period([&] { hipLaunchKernelGGL(k_write, dim3(79), dim3(256), 0, 0, d_buf); }, n));
    printf("1 KB write, 1536 WG    : %.2f us\n", period([&] { hipLaunchKernelGGL(k_write, dim3(1536), dim3(256), 0, 0, d_buf); }, n));
    printf("ticket, 79 WG          : %.2f us\n", period([&] { hipLaunchKernelGGL(k_ticket, dim3(79), dim3(256), 0, 0, d_t, (double*)d_buf); }, n));
    printf("ticket, 625 WG         : %.2f us\n", period([&] { hipLaunchKernelGGL(k_ticket, dim3(625), dim3(256), 0, 0, d_t, (double*)d_buf); }, n));
    return 0;
}
