// Exhaustive check (all 2^32 fp32 bit patterns) of a cheap reciprocal against the IEEE division
// 1.0f / x that the kernels and the oracle use: y0 = v_rcp_f32(x), one FMA Newton step
// y1 = fma(fma(-x, y0, 1), y0, y0).  Reports the mismatches per binade of |x|.
//   hipcc --offload-arch=gfx950 -O3 tools/rcp_exhaustive.hip -o tools/rcp_exhaustive && tools/rcp_exhaustive
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void k_check(unsigned long long* bad, unsigned int* first_bad, unsigned long long base) {
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const unsigned int bits = (unsigned int)i;
    const float x = __uint_as_float(bits);
    const unsigned int e = (bits >> 23) & 0xff;
    if (e == 0xff) return;  // inf / nan
    const float ref = 1.0f / x;
    const float y0 = __builtin_amdgcn_rcpf(x);
    const float y1 = __fmaf_rn(__fmaf_rn(-x, y0, 1.0f), y0, y0);
    if (__float_as_uint(y1) != __float_as_uint(ref)) {
        atomicAdd(&bad[e], 1ull);
        atomicMin(&first_bad[e], bits & 0x7fffffffu);
    }
}

int main() {
    unsigned long long* bad;
    unsigned int* first;
    hipMalloc(&bad, 256 * sizeof(unsigned long long));
    hipMalloc(&first, 256 * sizeof(unsigned int));
    hipMemset(bad, 0, 256 * sizeof(unsigned long long));
    hipMemset(first, 0xff, 256 * sizeof(unsigned int));
    const unsigned long long chunk = 1ull << 30;
    for (unsigned long long base = 0; base < (1ull << 32); base += chunk)
        hipLaunchKernelGGL(k_check, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, bad, first, base);
    unsigned long long h[256];
    unsigned int f[256];
    hipMemcpy(h, bad, sizeof h, hipMemcpyDeviceToHost);
    hipMemcpy(f, first, sizeof f, hipMemcpyDeviceToHost);
    unsigned long long tot = 0;
    for (int e = 0; e < 256; ++e) {
        tot += h[e];
        if (h[e]) printf("exponent field %3d (|x| ~ 2^%d): %llu mismatches, first |x| bits 0x%08x\n", e, e - 127, h[e], f[e]);
    }
    printf("total mismatches: %llu\n", tot);
    return 0;
}
