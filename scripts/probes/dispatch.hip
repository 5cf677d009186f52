// Probe: what a k_corr-shaped workgroup costs to dispatch, and what a persistent, queue-fed grid
// saves.  Each "unit" = one 256-thread workgroup's work in k_corr: every wave
// waits W cycles (s_sleep: a latency-bound wave that issues nothing), then the unit stores an 80-double
// partial and takes an agent-scope ticket (k_corr's reduction step).  Two forms over U units:
//   plain:      grid = U, one unit per workgroup (k_corr today)
//   persistent: grid = R, workgroups pull units from 8 per-XCD heads (atomicAdd), next unit requested
//               while the current one runs
// LDS is padded to k_corr's 20 KB per workgroup so residency matches (6 workgroups per CU).
//   hipcc -O3 --offload-arch=gfx950 dispatch.hip -o dispatch && ./dispatch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int NSX = 80;

__device__ __forceinline__ void work(long long cycles) {
    if (cycles <= 0) return;
    const long long t0 = __builtin_amdgcn_s_memtime();
    while (__builtin_amdgcn_s_memtime() - t0 < cycles) __builtin_amdgcn_s_sleep(2);
}

__device__ __forceinline__ void unit_reduce(int unit, double* partials, unsigned* tickets, double v) {
    if (threadIdx.x < NSX)
        __hip_atomic_store(&partials[(long long)unit * NSX + threadIdx.x], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_fetch_add(&tickets[unit / 64], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(256) k_plain(int units, long long cycles, double* partials, unsigned* tickets) {
    __shared__ double pad[2500];   // ~20 KB: k_corr's LDS footprint
    const int unit = blockIdx.x;
    if (threadIdx.x == 0) pad[0] = unit;
    work(cycles);
    unit_reduce(unit, partials, tickets, pad[0] * 0.0 + 1.0);
}

// static: workgroup b runs units [b k, b k + k) one after another (no queue, no atomics to dequeue)
__global__ void __launch_bounds__(256) k_static(int units, int k, long long cycles, double* partials, unsigned* tickets) {
    __shared__ double pad[2500];
    for (int u = blockIdx.x * k; u < min(units, blockIdx.x * k + k); ++u) {
        if (threadIdx.x == 0) pad[0] = u;
        work(cycles);
        unit_reduce(u, partials, tickets, pad[0] * 0.0 + 1.0);
        __syncthreads();
    }
}

__global__ void __launch_bounds__(256) k_persist(int units, long long cycles, double* partials, unsigned* tickets,
                                                 unsigned* heads) {
    __shared__ double pad[2500];
    __shared__ int s_next;
    const int x = blockIdx.x & 7;                       // this workgroup's XCD (placement: speed only)
    const int per = (units + 7) / 8, lo = x * per, hi = min(units, lo + per);
    int cur = -1;
    if (threadIdx.x == 0) {
        const unsigned k = __hip_atomic_fetch_add(&heads[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        s_next = lo + (int)k < hi ? lo + (int)k : -1;
    }
    __syncthreads();
    cur = s_next;
    while (cur >= 0) {
        __syncthreads();
        if (threadIdx.x == 0) {   // the next unit, requested while this one runs
            const unsigned k = __hip_atomic_fetch_add(&heads[x], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_next = lo + (int)k < hi ? lo + (int)k : -1;
        }
        if (threadIdx.x == 0) pad[0] = cur;
        work(cycles);
        unit_reduce(cur, partials, tickets, pad[0] * 0.0 + 1.0);
        __syncthreads();
        cur = s_next;
    }
}

int main() {
    int dev = 0, ncu = 0;
    CHK(hipSetDevice(dev));
    CHK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    int per_cu = 0;
    CHK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_persist, 256, 0));
    const int R = per_cu * ncu;
    printf("CUs %d, resident workgroups per CU %d -> persistent grid %d\n", ncu, per_cu, R);
    const int U = 5025;
    double* partials;
    unsigned *tickets, *heads;
    CHK(hipMalloc(&partials, sizeof(double) * U * NSX));
    CHK(hipMalloc(&tickets, sizeof(unsigned) * 4096));
    CHK(hipMalloc(&heads, sizeof(unsigned) * 8));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    for (int units : {5025, 630}) {
        for (long long cyc : {0LL, 12000LL, 24000LL}) {
            printf("units %5d  wave wait %6lld cyc:", units, cyc);
            for (int form = 0; form < 6; ++form) {   // plain, static k = 2, 3, 4, 8, persistent
                const int ks[6] = {1, 2, 3, 4, 8, 0};
                const int k = ks[form];
                const int reps = 50;
                float ms;
                for (int r = -5; r < reps; ++r) {
                    if (r == 0) CHK(hipEventRecord(e0));
                    if (form == 5) {
                        CHK(hipMemsetAsync(heads, 0, 32));
                        hipLaunchKernelGGL(k_persist, dim3(std::min(R, units)), dim3(256), 0, 0, units, cyc, partials,
                                           tickets, heads);
                    } else if (k == 1) {
                        hipLaunchKernelGGL(k_plain, dim3(units), dim3(256), 0, 0, units, cyc, partials, tickets);
                    } else {
                        hipLaunchKernelGGL(k_static, dim3((units + k - 1) / k), dim3(256), 0, 0, units, k, cyc,
                                           partials, tickets);
                    }
                }
                CHK(hipEventRecord(e1));
                CHK(hipEventSynchronize(e1));
                CHK(hipEventElapsedTime(&ms, e0, e1));
                const char* nm[6] = {"plain", "k2", "k3", "k4", "k8", "persist(+memset)"};
                printf("  %s %6.2f", nm[form], ms / reps * 1e3);
            }
            printf(" us\n");
        }
    }
    {   // an empty launch (1 workgroup, nothing) back to back: the launch floor
        float ms;
        CHK(hipEventRecord(e0));
        for (int r = 0; r < 100; ++r) hipLaunchKernelGGL(k_plain, dim3(1), dim3(256), 0, 0, 1, 0LL, partials, tickets);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("one-workgroup launch back to back: %.2f us\n", ms / 100 * 1e3);
    }
    return 0;
}
