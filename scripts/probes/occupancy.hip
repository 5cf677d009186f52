// Probe: how many 256-thread workgroups are resident per CU for a given LDS size and register
// footprint (k_corr-like: 70 VGPRs, 100 SGPRs).  Each wave spins ~30 us and records its realtime
// start/end; the max overlap count is printed.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>
template <int LDS, int REGS>
__global__ void __launch_bounds__(256) k(unsigned long long* t, int* sink) {
    __shared__ char buf[LDS];
    if (REGS == 1) asm volatile("" ::: "s55");
    if (REGS == 2) asm volatile("" ::: "s63");
    if (REGS == 3) asm volatile("" ::: "s71");
    if (REGS == 4) asm volatile("" ::: "s93");
    if (REGS == 5) asm volatile("" ::: "s95");
    if (REGS == 6) asm volatile("" ::: "s97");
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    buf[threadIdx.x % LDS] = (char)threadIdx.x;
    __syncthreads();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 3000) __builtin_amdgcn_s_sleep(2);
    if ((threadIdx.x & 63) == 0) {
        const int w = blockIdx.x * 4 + (threadIdx.x >> 6);
        t[2 * w] = t0;
        t[2 * w + 1] = __builtin_amdgcn_s_memrealtime();
    }
    if (buf[(threadIdx.x * 7) % LDS] == 127 && threadIdx.x == 999) *sink = 1;
}
template <int LDS, int REGS>
void run(const char* name) {
    const int nb = 256 * 16;
    unsigned long long* d;
    int* s;
    (void)hipMalloc(&d, sizeof(unsigned long long) * 2 * nb * 4);
    (void)hipMalloc(&s, 4);
    hipLaunchKernelGGL((k<LDS, REGS>), dim3(nb), dim3(256), 0, 0, d, s);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(2 * nb * 4);
    (void)hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost);
    std::vector<std::pair<unsigned long long, int>> ev;
    for (int w = 0; w < nb * 4; ++w) {
        ev.push_back({h[2 * w], 1});
        ev.push_back({h[2 * w + 1], -1});
    }
    std::sort(ev.begin(), ev.end());
    int cur = 0, mx = 0;
    for (auto& e : ev) mx = std::max(mx, cur += e.second);
    std::printf("%-28s max resident waves %d (%.2f per CU)\n", name, mx, mx / 256.0);
    (void)hipFree(d);
    (void)hipFree(s);
}
int main() {
    run<16, 1>("56 sgpr");
    run<16, 2>("64 sgpr");
    run<16, 3>("72 sgpr");
    run<16, 4>("94 sgpr");
    run<16, 5>("96 sgpr");
    run<16, 6>("98 sgpr");
    return 0;
}
