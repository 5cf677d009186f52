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
template <int N>
struct Arg {
    double v[N];
    int* out;
};
template <int N>
__global__ void k_arg(Arg<N> b) {
    if (b.out && threadIdx.x == 1000000) b.out[0] = (int)b.v[N - 1];
}

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

// in-kernel latency (100 MHz realtime ticks) of a kernel-argument load and of a device-memory load that the
// previous launch wrote: where does k_corr's first round trip go
__global__ void k_lat(Big b, double* dev, unsigned long long* out) {
    if (threadIdx.x != 0) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    double v = b.v[80];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    asm volatile("" ::"s"(v));
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const double w = __hip_atomic_load(dev + 8 * blockIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
    const double x = dev[4096 + 8 * blockIdx.x];   // plain load
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned long long t3 = __builtin_amdgcn_s_memrealtime();
    dev[8 * blockIdx.x] = v + w + x;   // the next launch reads what this one wrote
    out[blockIdx.x * 4 + 0] = t1 - t0;
    out[blockIdx.x * 4 + 1] = t2 - t1;
    out[blockIdx.x * 4 + 2] = t3 - t2;
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
    {
        Arg<7> a8{};   a8.out = d_out;
        Arg<15> a16{}; a16.out = d_out;
        Arg<31> a32{}; a32.out = d_out;
        Arg<47> a48{}; a48.out = d_out;
        Arg<63> a64{}; a64.out = d_out;
        printf("64-B arg, 79 WG        : %.2f us\n", period([&] { hipLaunchKernelGGL(k_arg<7>, dim3(79), dim3(256), 0, 0, a8); }, n));
        printf("128-B arg, 79 WG       : %.2f us\n", period([&] { hipLaunchKernelGGL(k_arg<15>, dim3(79), dim3(256), 0, 0, a16); }, n));
        printf("256-B arg, 79 WG       : %.2f us\n", period([&] { hipLaunchKernelGGL(k_arg<31>, dim3(79), dim3(256), 0, 0, a32); }, n));
        printf("384-B arg, 79 WG       : %.2f us\n", period([&] { hipLaunchKernelGGL(k_arg<47>, dim3(79), dim3(256), 0, 0, a48); }, n));
        printf("512-B arg, 79 WG       : %.2f us\n", period([&] { hipLaunchKernelGGL(k_arg<63>, dim3(79), dim3(256), 0, 0, a64); }, n));
    }
    printf("1 KB write, 79 WG      : %.2f us\n", period([&] { hipLaunchKernelGGL(k_write, dim3(79), dim3(256), 0, 0, d_buf); }, n));
    printf("1 KB write, 1536 WG    : %.2f us\n", period([&] { hipLaunchKernelGGL(k_write, dim3(1536), dim3(256), 0, 0, d_buf); }, n));
    printf("ticket, 79 WG          : %.2f us\n", period([&] { hipLaunchKernelGGL(k_ticket, dim3(79), dim3(256), 0, 0, d_t, (double*)d_buf); }, n));
    printf("ticket, 625 WG         : %.2f us\n", period([&] { hipLaunchKernelGGL(k_ticket, dim3(625), dim3(256), 0, 0, d_t, (double*)d_buf); }, n));
    unsigned long long* d_lat;
    CK(hipMalloc(&d_lat, 64 * 4 * 8));
    double acc[3] = {0, 0, 0};
    const int reps = 200;
    for (int r = 0; r < reps; ++r) {
        hipLaunchKernelGGL(k_lat, dim3(64), dim3(64), 0, 0, b, (double*)d_buf, d_lat);
        unsigned long long h[64 * 4];
        CK(hipMemcpy(h, d_lat, sizeof h, hipMemcpyDeviceToHost));
        for (int w = 0; w < 64; ++w)
            for (int k = 0; k < 3; ++k) acc[k] += h[w * 4 + k] / 100.0 / 64 / reps;
    }
    printf("in-kernel latency (us): kernarg load %.2f, agent-scope load of data the previous launch wrote %.2f, plain load %.2f\n",
           acc[0], acc[1], acc[2]);
    return 0;
}
