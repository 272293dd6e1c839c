// Exhaustive proofs for the shorter correctly rounded fp32 sequences of pt_math.h (pt_div,
// pt_rcp, pt_sqrt) against the compiler's IEEE expansions that the oracle's arithmetic equals
// (a / b, 1.0f / x, sqrtf with -fhip-fp32-correctly-rounded-divide-sqrt, the HIP default).
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off tools/divsqrt_exhaustive.hip -o tools/divsqrt_exhaustive
//   tools/divsqrt_exhaustive rcp          all 2^32 x: pt_rcp's fast path and its guard
//   tools/divsqrt_exhaustive sqrt         all 2^32 x: pt_sqrt's fast path and its guard
//   tools/divsqrt_exhaustive sqrtnb       all 2^32 x: pt_sqrt_nb (branchless)
//   tools/divsqrt_exhaustive div EA EB    all 2^23 x 2^23 significand pairs of a in [2^EA, 2^EA+1),
//                                         b in [2^EB, 2^EB+1) (EA / EB = -127: the denormal binade)
//   tools/divsqrt_exhaustive divrand N    N * 2^30 random bit patterns (a, b), specials included
// Every mode prints mismatches (fast path taken but bits differ; NaN == NaN) and the fraction of
// inputs the guard sends to the IEEE fallback.  A proof run must print "mismatches: 0".
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../optixpathtracer_amd/csrc/pt_fastdiv.h"

__device__ __forceinline__ bool same_bits(float a, float b) {
    return __float_as_uint(a) == __float_as_uint(b) || (a != a && b != b);
}

struct Counters {
    unsigned long long bad, slow, tot;
    unsigned int first_a, first_b;
};

__global__ void k_rcp(Counters* c, unsigned long long base) {
    const unsigned int bits = (unsigned int)(base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x);
    const float x = __uint_as_float(bits);
    const float ref = 1.0f / x;
    float y;
    const bool fast = pt::rcp_fast(x, y);
    const bool bad = (fast && !same_bits(y, ref)) || !same_bits(pt::pt_rcp(x), ref);
    const unsigned long long nb = __ballot(bad), ns = __ballot(!fast);
    if ((threadIdx.x & 63) == 0) {
        if (nb) atomicAdd(&c->bad, (unsigned long long)__popcll(nb));
        if (ns) atomicAdd(&c->slow, (unsigned long long)__popcll(ns));
    }
    if (bad) atomicMin(&c->first_a, bits);
}

__global__ void k_sqrtnb(Counters* c, unsigned long long base) {  // the branchless variant, every input
    const unsigned int bits = (unsigned int)(base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x);
    const float x = __uint_as_float(bits);
    const bool bad = !same_bits(pt::pt_sqrt_nb(x), sqrtf(x));
    const unsigned long long nb = __ballot(bad);
    if ((threadIdx.x & 63) == 0 && nb) atomicAdd(&c->bad, (unsigned long long)__popcll(nb));
    if (bad) atomicMin(&c->first_a, bits);
}

__global__ void k_sqrt(Counters* c, unsigned long long base) {
    const unsigned int bits = (unsigned int)(base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x);
    const float x = __uint_as_float(bits);
    const float ref = sqrtf(x);
    float y;
    const bool fast = pt::sqrt_fast(x, y);
    const bool bad = (fast && !same_bits(y, ref)) || !same_bits(pt::pt_sqrt(x), ref);
    const unsigned long long nb = __ballot(bad), ns = __ballot(!fast);
    if ((threadIdx.x & 63) == 0) {
        if (nb) atomicAdd(&c->bad, (unsigned long long)__popcll(nb));
        if (ns) atomicAdd(&c->slow, (unsigned long long)__popcll(ns));
    }
    if (bad) atomicMin(&c->first_a, bits);
}

// one thread per b significand, a loop over `na` a significands starting at a0
__global__ void k_div(Counters* c, unsigned int ea_field, unsigned int eb_field, unsigned int a0, unsigned int na) {
    const unsigned int mb = blockIdx.x * blockDim.x + threadIdx.x;  // < 2^23
    const float b = __uint_as_float((eb_field << 23) | mb);
    unsigned int nbad = 0, first = 0xffffffffu;
    for (unsigned int i = 0; i < na; ++i) {
        const unsigned int abits = (ea_field << 23) | (a0 + i);
        const float a = __uint_as_float(abits);
        const float ref = a / b;
        const float q = pt::pt_div(a, b);
        if (!same_bits(q, ref)) {
            ++nbad;
            first = min(first, abits);
        }
    }
    if (nbad) {
        atomicAdd(&c->bad, (unsigned long long)nbad);
        atomicMin(&c->first_a, first);
        atomicMin(&c->first_b, __float_as_uint(b));
    }
}

__device__ __forceinline__ unsigned int mix32(unsigned long long z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return (unsigned int)(z ^ (z >> 31));
}
__device__ __forceinline__ float pick(unsigned int r, unsigned int r2) {
    // one in 16 operands special or from an extreme binade
    const unsigned int kind = r2 & 15;
    const unsigned int sign = r2 & 0x80000000u;
    if (kind == 0) {
        const unsigned int sp[8] = {0u, 0x7f800000u, 0x7fc00000u, 1u, 0x007fffffu, 0x00800000u, 0x7f7fffffu, 0x3f800000u};
        return __uint_as_float(sp[(r2 >> 4) & 7] | sign);
    }
    if (kind == 1) return __uint_as_float((r & 0x807fffffu) | (((r2 >> 8) % 24u) << 23));           // tiny binades
    if (kind == 2) return __uint_as_float((r & 0x807fffffu) | ((230u + (r2 >> 8) % 25u) << 23));    // huge binades
    return __uint_as_float(r);
}
__global__ void k_divrand(Counters* c, unsigned long long base) {
    const unsigned long long i = base + blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    const float a = pick(mix32(4 * i), mix32(4 * i + 1));
    const float b = pick(mix32(4 * i + 2), mix32(4 * i + 3));
    const float ref = a / b;
    const float q = pt::pt_div(a, b);
    const bool bad = !same_bits(q, ref);
    if (bad) {
        atomicAdd(&c->bad, 1ull);
        atomicMin(&c->first_a, __float_as_uint(a));
        atomicMin(&c->first_b, __float_as_uint(b));
    }
}

static void report(const char* what, const Counters& h, double total) {
    printf("%s: mismatches: %llu  fallback: %llu (%.3g of %.4g inputs)", what, h.bad, h.slow, h.slow / total, total);
    if (h.bad) printf("  first bad a 0x%08x b 0x%08x", h.first_a, h.first_b);
    printf("\n");
    fflush(stdout);
}

int main(int argc, char** argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s rcp|sqrt|div EA EB|divrand N\n", argv[0]);
        return 2;
    }
    Counters* d;
    hipMalloc(&d, sizeof(Counters));
    Counters init{0, 0, 0, 0xffffffffu, 0xffffffffu};
    hipMemcpy(d, &init, sizeof init, hipMemcpyHostToDevice);
    Counters h;
    const char* mode = argv[1];
    if (!strcmp(mode, "rcp") || !strcmp(mode, "sqrt") || !strcmp(mode, "sqrtnb")) {
        const unsigned long long chunk = 1ull << 30;
        for (unsigned long long base = 0; base < (1ull << 32); base += chunk) {
            if (!strcmp(mode, "rcp"))
                hipLaunchKernelGGL(k_rcp, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, d, base);
            else if (!strcmp(mode, "sqrt"))
                hipLaunchKernelGGL(k_sqrt, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, d, base);
            else
                hipLaunchKernelGGL(k_sqrtnb, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, d, base);
        }
        hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
        report(mode, h, 4294967296.0);
    } else if (!strcmp(mode, "div") && argc >= 4) {
        const int ea = atoi(argv[2]), eb = atoi(argv[3]);
        const unsigned int fa = (unsigned int)(ea + 127), fb = (unsigned int)(eb + 127);
        const unsigned int na = 2048;
        for (unsigned int a0 = 0; a0 < (1u << 23); a0 += na) {
            hipLaunchKernelGGL(k_div, dim3((1u << 23) / 256), dim3(256), 0, 0, d, fa, fb, a0, na);
            if ((a0 & ((1u << 20) - 1)) == 0) {
                hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
                printf("  div 2^%d / 2^%d: a significands %u/8388608, mismatches so far %llu\n", ea, eb, a0, h.bad);
                fflush(stdout);
            }
        }
        hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
        char w[64];
        snprintf(w, sizeof w, "div 2^%d / 2^%d (all 2^46 significand pairs)", ea, eb);
        report(w, h, 70368744177664.0);
    } else if (!strcmp(mode, "divrand") && argc >= 3) {
        const int n = atoi(argv[2]);
        const unsigned long long chunk = 1ull << 30;
        for (int k = 0; k < n; ++k) hipLaunchKernelGGL(k_divrand, dim3((unsigned)(chunk / 256)), dim3(256), 0, 0, d, k * chunk);
        hipMemcpy(&h, d, sizeof h, hipMemcpyDeviceToHost);
        report("divrand", h, (double)n * chunk);
    } else {
        fprintf(stderr, "bad mode\n");
        return 2;
    }
    return h.bad ? 1 : 0;
}
