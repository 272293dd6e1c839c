// pt_math.h — float3 arithmetic with glm 0.9.9.8 rounding order, for the gfx950 kernels.
//
// The reference's device code is written against glm (3rdParty/glm, used by
// Renderer/OptiX/devicePrograms.cu and PBRT/*.h).  These helpers reproduce exactly the
// association order of the glm functions the hot path calls (dot = (x*x'+y*y')+z*z',
// normalize = v * (1/sqrt(dot)), cross per compute_cross, mat3*vec3 column sums), so the
// kernels round identically to the CPU oracle (built -ffp-contract=off; the HIP sources
// are built -ffp-contract=off as well, see Makefile).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PT_HD __host__ __device__ __forceinline__

#include "pt_fastdiv.h"

// Correctly rounded division, reciprocal and square root.  On the device the division and the
// square root take the shorter exact sequences of pt_fastdiv.h; on the host they are the IEEE
// operations.  Both give the same bits.  Measured per operation (interleaved A/B, DESIGN.md §5,
// profiles/r05d_ab_*.log): PT_FAST_DIV 1 and PT_FAST_SQRT 2 (branchless) took the Default /
// Layered / Sponza-class configs +9.8 / +11.6 / +6.7 % with Dielectric unchanged; the guarded
// reciprocal (PT_FAST_RCP 1) raised the Conductor kernels' registers 80 -> 108 VGPRs and lost,
// so 1 / x stays the compiler's.  PT_FAST_DIVSQRT 0 selects the compiler's expansions throughout.
#ifndef PT_FAST_DIVSQRT
#define PT_FAST_DIVSQRT 1
#endif
#ifndef PT_FAST_DIV
#define PT_FAST_DIV PT_FAST_DIVSQRT
#endif
#ifndef PT_FAST_RCP
#define PT_FAST_RCP 0
#endif
#ifndef PT_FAST_SQRT
#define PT_FAST_SQRT (PT_FAST_DIVSQRT ? 2 : 0)
#endif

namespace pt {

#if defined(__HIP_DEVICE_COMPILE__)
PT_HD float fdiv(float a, float b) { return PT_FAST_DIV ? pt_div(a, b) : a / b; }
PT_HD float frcp(float x) { return PT_FAST_RCP == 1 ? pt_rcp(x) : PT_FAST_RCP == 2 ? pt_div(1.0f, x) : 1.0f / x; }
PT_HD float fsqrt(float x) { return PT_FAST_SQRT == 1 ? pt_sqrt(x) : PT_FAST_SQRT == 2 ? pt_sqrt_nb(x) : sqrtf(x); }
#else
PT_HD float fdiv(float a, float b) { return a / b; }
PT_HD float frcp(float x) { return 1.0f / x; }
PT_HD float fsqrt(float x) { return sqrtf(x); }
#endif

struct f3 {
    float x, y, z;
};

PT_HD f3 mk(float x, float y, float z) { return f3{x, y, z}; }
// PT_PK_F3 = 1: on the device the x and y channels of the f3 products and sums go through
// two-wide vectors, which gfx950 executes as v_pk_mul_f32 / v_pk_add_f32 (IEEE per element, so
// every result is the same bits as the scalar operations).
#ifndef PT_PK_F3
#define PT_PK_F3 0
#endif
#if PT_PK_F3 && defined(__HIP_DEVICE_COMPILE__)
typedef float pk2 __attribute__((ext_vector_type(2)));
PT_HD pk2 lo2(f3 a) { return pk2{a.x, a.y}; }
PT_HD f3 operator+(f3 a, f3 b) { const pk2 v = lo2(a) + lo2(b); return mk(v.x, v.y, a.z + b.z); }
PT_HD f3 operator-(f3 a, f3 b) { const pk2 v = lo2(a) - lo2(b); return mk(v.x, v.y, a.z - b.z); }
PT_HD f3 operator*(f3 a, f3 b) { const pk2 v = lo2(a) * lo2(b); return mk(v.x, v.y, a.z * b.z); }
PT_HD f3 operator*(f3 a, float s) { const pk2 v = lo2(a) * pk2{s, s}; return mk(v.x, v.y, a.z * s); }
PT_HD f3 operator*(float s, f3 a) { const pk2 v = pk2{s, s} * lo2(a); return mk(v.x, v.y, s * a.z); }
#else
PT_HD f3 operator+(f3 a, f3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
PT_HD f3 operator-(f3 a, f3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
PT_HD f3 operator*(f3 a, f3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
PT_HD f3 operator*(f3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
PT_HD f3 operator*(float s, f3 a) { return mk(s * a.x, s * a.y, s * a.z); }
#endif
PT_HD f3 operator/(f3 a, float s) { return mk(fdiv(a.x, s), fdiv(a.y, s), fdiv(a.z, s)); }
PT_HD f3 operator-(f3 a) { return mk(-a.x, -a.y, -a.z); }
PT_HD bool is_zero(f3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }

PT_HD float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
PT_HD f3 cross(f3 a, f3 b) {
    return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
PT_HD f3 normalize(f3 a) {
    float i = frcp(fsqrt(dot(a, a)));
    return a * i;
}
PT_HD float length(f3 a) { return fsqrt(dot(a, a)); }
PT_HD float sqr(float x) { return x * x; }
// glm::max/min/clamp on scalars (func_common.inl:17-30,505-509)
PT_HD float gmax(float x, float y) { return (x < y) ? y : x; }
PT_HD float gmin(float x, float y) { return (y < x) ? y : x; }
PT_HD float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
PT_HD float gabs(float x) { return x >= 0.0f ? x : -x; }
PT_HD float save_max(f3 a) { return gmax(gmax(a.x, a.y), a.z); }   // glmCUDA.h:99-101
PT_HD float abs_dot(f3 a, f3 b) { return fabsf(dot(a, b)); }       // glmCUDA.h:119-121
PT_HD float length_sqr(f3 a) { return sqr(a.x) + sqr(a.y) + sqr(a.z); }

// Shading frame: columns T, B, N (devicePrograms.cu:168-212).
struct Frame {
    f3 t, b, n;
};
// WorldToShading * v  (transpose(mat3(T,B,N)) * v)
PT_HD f3 to_local(const Frame& f, f3 v) { return mk(dot(f.t, v), dot(f.b, v), dot(f.n, v)); }
// ShadingToWorld * v  (glm mat3*vec3: m[0]*x + m[1]*y + m[2]*z, per row)
PT_HD f3 to_world(const Frame& f, f3 v) {
    return mk(f.t.x * v.x + f.b.x * v.y + f.n.x * v.z, f.t.y * v.x + f.b.y * v.y + f.n.y * v.z,
              f.t.z * v.x + f.b.z * v.y + f.n.z * v.z);
}

// glm mat4 (column-major) * vec4: (m0*v0 + m1*v1) + (m2*v2 + m3*v3)  (type_mat4x4.inl:561-575)
PT_HD void mat4_mul_vec4(const float* m, const float v[4], float out[4]) {
    for (int r = 0; r < 4; ++r) {
        float a0 = m[0 * 4 + r] * v[0];
        float a1 = m[1 * 4 + r] * v[1];
        float a2 = m[2 * 4 + r] * v[2];
        float a3 = m[3 * 4 + r] * v[3];
        out[r] = (a0 + a1) + (a2 + a3);
    }
}

// ---- RNG: random.h:34-84 -------------------------------------------------------------
PT_HD uint32_t tea16(uint32_t val0, uint32_t val1) {
    uint32_t v0 = val0, v1 = val1, s0 = 0;
#pragma unroll
    for (int n = 0; n < 16; n++) {
        s0 += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}
PT_HD float rnd(uint32_t& prev) {
    prev = 1664525u * prev + 1013904223u;
    return (float)(prev & 0x00FFFFFFu) / (float)0x01000000;
}
// ---- transcendentals of the hot path, identical bit for bit to the oracle's -------------
// The reference calls CUDA libdevice sinf/cosf (random.h:76-84, LambertDiffuse.h:35-55), expf
// (GlossyDiffuse.h:97-105) and powf (devicePrograms.cu:62-73), whose ulp-level results neither
// ocml nor glibc reproduce.  The kernels and the CPU oracle (oracle/pt_oracle.c) therefore both
// evaluate these fixed, explicitly fused single-precision polynomials (Cody-Waite reduction +
// Cephes minimax coefficients: sin/cos/exp <= ~1 ulp) on the bounded domains the path uses, so GPU and
// oracle images agree bit for bit instead of diverging on a flipped random decision.
// sin/cos for |x| <= 2^15 (the path passes |x| <= 2 pi): quadrant k = rint(x * 2/pi), r = x - k pi/2
// in three fma steps, then sin(r) / cos(r) on [-pi/4, pi/4].
PT_HD void pt_sincosf(float x, float& s, float& c) {
    const float k = rintf(x * 0x1.45f306p-1f);
    float r = fmaf(-k, 0x1.921fb6p+0f, x);
    r = fmaf(-k, -0x1.777a5cp-25f, r);
    r = fmaf(-k, -0x1.ee59dap-50f, r);
    const float z = r * r;
    const float sp = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), z * r, r);
    const float cp = fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f),
                          z * z, fmaf(-0.5f, z, 1.0f));
    const int q = (int)k & 3;
    s = q == 0 ? sp : q == 1 ? cp : q == 2 ? -sp : -cp;
    c = q == 0 ? cp : q == 1 ? -sp : q == 2 ? -cp : sp;
}
// exp(x) for x <= 0 (transmittance): 0 below -86 (keeps every result a normal float); NaN stays NaN.
PT_HD float pt_expf_neg(float x) {
    if (!(x > -86.0f)) return x != x ? x : 0.0f;
    const float k = floorf(fmaf(x, 0x1.715476p+0f, 0.5f));
    float r = fmaf(-k, 0.693359375f, x);
    r = fmaf(-k, -2.12194440e-4f, r);
    float p = fmaf(fmaf(fmaf(fmaf(fmaf(1.9875691500e-4f, r, 1.3981999507e-3f), r, 8.3334519073e-3f), r,
                             4.1665795894e-2f), r, 1.6666665459e-1f), r, 5.0000001201e-1f);
    p = fmaf(p, r * r, r) + 1.0f;
    return ldexpf(p, (int)k);
}
// ln(x) for normal x in (0, 1]: x = m 2^e with m in [sqrt(1/2), sqrt(2)), Cephes logf polynomial.
PT_HD float pt_logf_unit(float x) {
    int e;
    float m = frexpf(x, &e);
    if (m < 0.70710678118654752f) {
        m = m + m;
        e -= 1;
    }
    const float f = m - 1.0f, z = f * f;
    float y = 7.0376836292e-2f;
    y = fmaf(y, f, -1.1514610310e-1f);
    y = fmaf(y, f, 1.1676998740e-1f);
    y = fmaf(y, f, -1.2420140846e-1f);
    y = fmaf(y, f, 1.4249322787e-1f);
    y = fmaf(y, f, -1.6668057665e-1f);
    y = fmaf(y, f, 2.0000714765e-1f);
    y = fmaf(y, f, -2.4999993993e-1f);
    y = fmaf(y, f, 3.3333331174e-1f);
    y = (y * f) * z;
    const float fe = (float)e;
    y = fmaf(fe, -2.12194440e-4f, y);
    y = fmaf(-0.5f, z, y);
    return (f + y) + fe * 0.693359375f;
}
// x^e for x in (0, 1] and e > 0 (the sRGB decode: x >= 0.052, e = 2.4); single-precision
// exp(e ln x) amplifies the rounding of ln x by e: <= ~7 ulp, immaterial for 8-bit texels
PT_HD float pt_powf_unit(float x, float e) { return pt_expf_neg(e * pt_logf_unit(x)); }

// PTX cvt.rzi.u32.f32 semantics (saturate, NaN -> 0) for PBRT/GlossyDiffuse.h:215-218,417-418.
PT_HD uint32_t f2u_sat(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}

}  // namespace pt
