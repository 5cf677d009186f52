// Probe: semantics of v_permlane{16,32}_swap and the v_mfma_f32_16x16x4_f32 operand/result maps
// as k_corr's MFMA screen uses them. Prints PASS/FAIL lines.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
typedef float f4v __attribute__((ext_vector_type(4)));
__global__ void k(unsigned* xo, float* mo) {
    const int l = threadIdx.x;
    unsigned x[4];
    for (int m = 0; m < 4; ++m) x[m] = (unsigned)(m * 1000 + l);   // X_m, lane l (block g = l>>4)
    auto r02 = __builtin_amdgcn_permlane32_swap(x[0], x[2], false, false);
    x[0] = r02[0]; x[2] = r02[1];
    auto r13 = __builtin_amdgcn_permlane32_swap(x[1], x[3], false, false);
    x[1] = r13[0]; x[3] = r13[1];
    auto r01 = __builtin_amdgcn_permlane16_swap(x[0], x[1], false, false);
    x[0] = r01[0]; x[1] = r01[1];
    auto r23 = __builtin_amdgcn_permlane16_swap(x[2], x[3], false, false);
    x[2] = r23[0]; x[3] = r23[1];
    for (int g = 0; g < 4; ++g) xo[g * 64 + l] = x[g];
    // MFMA: A[i][k] = 10 i + k (lane supplies A[l&15][l>>4]); B[k][j] = 100 j + k*k (lane supplies B[l>>4][l&15])
    const float a = 10.f * (l & 15) + (l >> 4);
    const float b = 100.f * (l & 15) + (l >> 4) * (l >> 4);
    f4v c = {0.5f, 0.5f, 0.5f, 0.5f};
    f4v d = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    for (int v = 0; v < 4; ++v) mo[v * 64 + l] = d[v];
}
int main() {
    unsigned* xo; float* mo;
    hipMalloc(&xo, 256 * 4); hipMalloc(&mo, 256 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, xo, mo);
    unsigned hx[256]; float hm[256];
    hipMemcpy(hx, xo, 1024, hipMemcpyDeviceToHost); hipMemcpy(hm, mo, 1024, hipMemcpyDeviceToHost);
    int bad = 0;
    // expected: Y_g at lane l (block b = l>>4) = X_b at lane (l&15) + 16 g
    for (int g = 0; g < 4; ++g) for (int l = 0; l < 64; ++l) {
        const unsigned e = (unsigned)((l >> 4) * 1000 + (l & 15) + 16 * g);
        if (hx[g * 64 + l] != e) { if (bad < 5) printf("xpose g=%d l=%d got %u want %u\n", g, l, hx[g*64+l], e); ++bad; }
    }
    printf("%s transpose4\n", bad ? "FAIL" : "PASS");
    int badm = 0;
    for (int v = 0; v < 4; ++v) for (int l = 0; l < 64; ++l) {
        const int i = 4 * (l >> 4) + v, j = l & 15;   // row i, col j
        double s = 0.5;
        for (int kk = 0; kk < 4; ++kk) s += (10.0 * i + kk) * (100.0 * j + kk * kk);
        if (std::fabs(hm[v * 64 + l] - s) > 1e-3 * std::fabs(s)) { if (badm < 5) printf("mfma v=%d l=%d got %g want %g\n", v, l, hm[v*64+l], s); ++badm; }
    }
    printf("%s mfma_f32_16x16x4 map (D row = 4*(l>>4)+v, col = l&15)\n", badm ? "FAIL" : "PASS");
    return bad || badm;
}
