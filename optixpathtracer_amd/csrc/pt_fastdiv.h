// pt_fastdiv.h — correctly rounded fp32 division, reciprocal and square root in fewer gfx950
// instructions than the compiler's expansions, with results identical bit for bit.
//
// The reference builds its BSDFs without fast math (PTX div.rn / sqrt.rn, SURVEY §7 "Hard
// parts"), and the oracle divides with IEEE `/` and `sqrtf`.  The compiler's correctly rounded
// expansions on gfx950 are 11 VALU instructions per division (two v_div_scale, v_rcp, five FMAs
// or multiplies, v_div_fmas, v_div_fixup) and 16 per square root (input scaling below 2^-96,
// v_sqrt, a +-1 ulp correction by two residuals, output unscaling, a zero/inf class fix-up).
// Division and square root are 27 % of the layered NEE kernel's VALU instructions (DESIGN §5,
// round-4 census).  The sequences here are shorter and exact:
//
// * div_short / pt_div: the compiler's sequence minus its second residual correction (9
//   instructions).  After v_div_scale the scaled denominator d has 1/d normal, and v_rcp + one
//   Newton step gives y = RN(1/d) exactly there (tools/rcp_exhaustive.hip, all 2^32 inputs).
//   With y = RN(1/d) and q0 = RN(n*y) within an ulp of n/d, the remainder r = n - d*q0 is exact
//   and RN(q0 + r*y) = RN(n/d) (Markstein's theorem); v_div_fixup still applies the special
//   cases.  When v_div_scale flags a result v_div_fmas must rescale (a denormal or near-overflow
//   quotient) the lane takes the compiler's last step in a branch that waves skip.
// * sqrt_fast / pt_sqrt_nb: v_sqrt and the +-1 ulp residual correction with the compiler's input
//   scaling below 2^-96, without its zero / infinity class fix-up: 14 instructions, branchless.
// * rcp_fast / pt_rcp, pt_sqrt: guarded fast paths with an IEEE fallback branch; exact, but
//   measured slower in the kernels (register pressure) and not the defaults.
// Proofs: tools/divsqrt_exhaustive.hip -- every fp32 input for the reciprocal and both square
// roots; for the division every pair of significands (2^46) in 16 exponent regimes covering
// each v_div_scale case, plus 9 * 2^34 random pairs with specials; 0 mismatches
// (profiles/r05_dsx_*.log).

#pragma once
#include <hip/hip_runtime.h>

namespace pt {

__device__ __forceinline__ float div_short(float a, float b) {
    bool unused, scale;
    const float d = __builtin_amdgcn_div_scalef(a, b, false, &unused);  // scaled denominator
    const float n = __builtin_amdgcn_div_scalef(a, b, true, &scale);    // scaled numerator
    const float y0 = __builtin_amdgcn_rcpf(d);
    const float y = __builtin_fmaf(__builtin_fmaf(-d, y0, 1.0f), y0, y0);  // RN(1/d)
    const float q0 = n * y;
    const float r = __builtin_fmaf(-d, q0, n);  // exact
    float q = __builtin_fmaf(r, y, q0);         // RN(n/d)
    // v_div_scale flags a quotient that v_div_fmas must rescale (near overflow, or a denormal
    // result, whose coarser rounding grid the one-correction quotient does not respect: one
    // mismatch in 2^34 random pairs without this).  Those lanes take the compiler's last step.
    // (Expected false, so the compiler keeps it a branch instead of computing both steps on
    // every lane; no asm barrier, which would also stop it from merging equal divisions.)
#ifndef PT_DIV_PROBE_NOBRANCH
#define PT_DIV_PROBE_NOBRANCH 0  // timing probe only (wrong on rescaled quotients): the branch's cost
#endif
    if (!PT_DIV_PROBE_NOBRANCH && __builtin_expect(scale, 0))
        q = __builtin_amdgcn_div_fmasf(__builtin_fmaf(-d, q, n), y, q, true);
    return __builtin_amdgcn_div_fixupf(q, b, a);
}

// class masks of __builtin_amdgcn_classf: bit 3 negative normal, bit 8 positive normal
constexpr int kClassNormal = (1 << 3) | (1 << 8);

__device__ __forceinline__ bool rcp_fast(float x, float& y) {
    const float y0 = __builtin_amdgcn_rcpf(x);
    y = __builtin_fmaf(__builtin_fmaf(-x, y0, 1.0f), y0, y0);
    return __builtin_amdgcn_classf(y, kClassNormal) && __builtin_amdgcn_classf(x, kClassNormal);
}

__device__ __forceinline__ bool sqrt_fast(float x, float& y) {
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u);
    const float su = __uint_as_float(__float_as_uint(s) + 1u);
    const float rd = __builtin_fmaf(-sd, s, x);
    const float ru = __builtin_fmaf(-su, s, x);
    float t = rd <= 0.0f ? sd : s;
    y = ru > 0.0f ? su : t;
    return !(x < 0x1.0p-96f);
}

// The production entry points: fast path, and the IEEE operation on the lanes outside its
// proven domain (a wave skips the branch when it has none).
__device__ __forceinline__ float pt_div(float a, float b) { return div_short(a, b); }
__device__ __forceinline__ float pt_rcp(float x) {
    float y;
    if (!rcp_fast(x, y)) {
        asm volatile("");
        y = 1.0f / x;
    }
    return y;
}
__device__ __forceinline__ float pt_sqrt(float x) {
    float y;
    if (!sqrt_fast(x, y)) {
        asm volatile("");
        y = __builtin_sqrtf(x);
    }
    return y;
}

// Branchless square root: the compiler's input scaling below 2^-96 (x * 2^32, result * 2^-16)
// around sqrt_fast's correction, without its zero / infinity class fix-up (sqrt_fast returns +-0
// and +inf unchanged; all 2^32 inputs checked).
__device__ __forceinline__ float pt_sqrt_nb(float x) {
    const bool tiny = x < 0x1.0p-96f;
    const float xs = tiny ? x * 0x1.0p+32f : x;
    float y;
    (void)sqrt_fast(xs, y);
    return tiny ? y * 0x1.0p-16f : y;
}

}  // namespace pt
