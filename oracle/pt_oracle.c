/*
 * pt_oracle.c — CPU ORACLE (test infrastructure only; see pt_oracle.h header comment).
 *
 * A literal, scalar, plain-C restatement of the reference hot path.  Every function cites
 * the reference file:line it follows (paths relative to
 * OptixPathtracer/source/Renderer/OptiX/ unless stated).  Floating-point expressions keep
 * the reference's (glm 0.9.9.8) association order so that the HIP product, which follows
 * the same order, agrees up to libm-vs-ocml transcendental ulps.  Build with
 * -ffp-contract=off (oracle/Makefile).
 *
 * Choices the reference leaves to closed code (OptiX 7.3 traversal) are documented where
 * made: Moller-Trumbore triangle test with OptiX barycentric convention (u weights v1,
 * v weights v2), closed-interval [tmin,tmax], closest hit ordered by (t, global primitive
 * index) so the result is independent of the acceleration structure.  "parity unpinned".
 */
#include "pt_oracle.h"

#include <float.h>
#include <math.h>
#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------------------ */
/* vector helpers — glm 0.9.9.8 semantics                                                */
/* ------------------------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mulv(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 muls(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 smul(float s, v3 a) { return mk(s * a.x, s * a.y, s * a.z); }
static inline v3 divs(v3 a, float s) { return mk(a.x / s, a.y / s, a.z / s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline int iszero3(v3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
/* glm compute_dot<vec3>: tmp = a*b; tmp.x + tmp.y + tmp.z */
static inline float dot3(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* glm compute_cross */
static inline v3 cross3(v3 a, v3 b) {
    return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y);
}
/* glm normalize = v * inversesqrt(dot(v,v)), inversesqrt = 1/sqrt */
static inline v3 normalize3(v3 a) { float i = 1.0f / sqrtf(dot3(a, a)); return muls(a, i); }
static inline float length3(v3 a) { return sqrtf(dot3(a, a)); }
/* glm max(x,y) = (x < y) ? y : x ; min(x,y) = (y < x) ? y : x ; clamp = min(max(x,lo),hi) */
static inline float gmax(float x, float y) { return (x < y) ? y : x; }
static inline float gmin(float x, float y) { return (y < x) ? y : x; }
static inline float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
/* glm::abs(float): x >= 0 ? x : -x */
static inline float gabs(float x) { return x >= 0.0f ? x : -x; }
static inline float sqr(float x) { return x * x; }
/* glmCUDA.h:99-101 SaveMax(vec3) */
static inline float savemax3(v3 a) { return gmax(gmax(a.x, a.y), a.z); }
/* glmCUDA.h:119-121 */
static inline float absdot(v3 a, v3 b) { return fabsf(dot3(a, b)); }
/* glmCUDA.h:123-125 */
static inline float lensqr3(v3 a) { return sqr(a.x) + sqr(a.y) + sqr(a.z); }
static const v3 ZAXIS = {0.0f, 0.0f, 1.0f};

/* glm mat4 (column-major m[c*4+r]) * vec4 — type_mat4x4.inl:561-575:
 * (m0*v0 + m1*v1) + (m2*v2 + m3*v3) */
static void mat4_mul_vec4(const float* m, const float v[4], float out[4]) {
    for (int r = 0; r < 4; ++r) {
        float a0 = m[0 * 4 + r] * v[0];
        float a1 = m[1 * 4 + r] * v[1];
        float a2 = m[2 * 4 + r] * v[2];
        float a3 = m[3 * 4 + r] * v[3];
        out[r] = (a0 + a1) + (a2 + a3);
    }
}

/* ------------------------------------------------------------------------------------ */
/* RNG — random.h:34-84                                                                  */
/* ------------------------------------------------------------------------------------ */
uint32_t orc_tea16(uint32_t val0, uint32_t val1) {  /* random.h:34-48 */
    uint32_t v0 = val0, v1 = val1, s0 = 0;
    for (unsigned n = 0; n < 16; n++) {
        s0 += 0x9e3779b9u;
        v0 += ((v1 << 4) + 0xa341316cu) ^ (v1 + s0) ^ ((v1 >> 5) + 0xc8013ea4u);
        v1 += ((v0 << 4) + 0xad90777du) ^ (v0 + s0) ^ ((v0 >> 5) + 0x7e95761eu);
    }
    return v0;
}
static inline uint32_t lcg(uint32_t* prev) {  /* random.h:51-57 */
    *prev = 1664525u * *prev + 1013904223u;
    return *prev & 0x00FFFFFFu;
}
static inline float rnd(uint32_t* prev) {  /* random.h:66-69 */
    return (float)lcg(prev) / (float)0x01000000;
}
void orc_rnd_seq(uint32_t seed, int32_t n, float* out, uint32_t* seed_out) {
    for (int32_t i = 0; i < n; ++i) out[i] = rnd(&seed);
    if (seed_out) *seed_out = seed;
}
/* float -> unsigned as PTX cvt.rzi.u32.f32 (saturating, NaN -> 0); the reference relies on
 * it at PBRT/GlossyDiffuse.h:215-218,417-418 (devicePrograms.cu.ptx uses cvt.rzi.u32.f32). */
uint32_t orc_f2u_sat(float f) {
    if (!(f > 0.0f)) return 0u;
    if (f >= 4294967296.0f) return 0xFFFFFFFFu;
    return (uint32_t)f;
}
/* Transcendentals.  The reference calls CUDA libdevice sinf/cosf/expf/powf, whose ulp-level
 * results glibc does not reproduce (nor does the GPU build's ocml).  The oracle and the HIP
 * kernels (optixpathtracer_amd/csrc/pt_math.h) both evaluate these fixed, explicitly fused
 * single-precision polynomials on the bounded domains the path uses (Cody-Waite reduction +
 * Cephes minimax coefficients: sin/cos/exp within ~1 ulp, x^2.4 within ~7), restated independently so
 * GPU and oracle agree bit for bit.  fmaf is correctly rounded on both sides. */
static void orc_sincosf(float x, float* s, float* c) {  /* |x| <= 2^15 */
    const float k = rintf(x * 0x1.45f306p-1f);
    float r = fmaf(-k, 0x1.921fb6p+0f, x);
    r = fmaf(-k, -0x1.777a5cp-25f, r);
    r = fmaf(-k, -0x1.ee59dap-50f, r);
    const float z = r * r;
    const float sp = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), z * r, r);
    const float cp = fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f),
                          z * z, fmaf(-0.5f, z, 1.0f));
    const int q = (int)k & 3;
    *s = q == 0 ? sp : q == 1 ? cp : q == 2 ? -sp : -cp;
    *c = q == 0 ? cp : q == 1 ? -sp : q == 2 ? -cp : sp;
}
static float orc_expf_neg(float x) {  /* x <= 0; 0 below -86, NaN stays NaN */
    if (!(x > -86.0f)) return x != x ? x : 0.0f;
    const float k = floorf(fmaf(x, 0x1.715476p+0f, 0.5f));
    float r = fmaf(-k, 0.693359375f, x);
    r = fmaf(-k, -2.12194440e-4f, r);
    float p = fmaf(fmaf(fmaf(fmaf(fmaf(1.9875691500e-4f, r, 1.3981999507e-3f), r, 8.3334519073e-3f), r,
                             4.1665795894e-2f), r, 1.6666665459e-1f), r, 5.0000001201e-1f);
    p = fmaf(p, r * r, r) + 1.0f;
    return ldexpf(p, (int)k);
}
static float orc_logf_unit(float x) {  /* normal x in (0, 1] */
    int e;
    float m = frexpf(x, &e);
    if (m < 0.70710678118654752f) { m = m + m; e -= 1; }
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
static float orc_powf_unit(float x, float e) { return orc_expf_neg(e * orc_logf_unit(x)); }
/* exported for the tests (accuracy against numpy float64) */
void orc_math_eval(int32_t fn, const float* x, float* out, int32_t n) {
    for (int32_t i = 0; i < n; ++i) {
        float s, c;
        switch (fn) {
            case 0: orc_sincosf(x[i], &s, &c); out[i] = s; break;
            case 1: orc_sincosf(x[i], &s, &c); out[i] = c; break;
            case 2: out[i] = orc_expf_neg(x[i]); break;
            default: out[i] = orc_powf_unit(x[i], 2.4f); break;
        }
    }
}

/* random.h:76-84; argument evaluation left-to-right (confirmed in devicePrograms.cu.ptx) */
static void disk_polar(uint32_t* seed, float* px, float* py) {
    const float pi = (float)3.14159265359;
    float u0 = rnd(seed);
    float u1 = rnd(seed);
    float r = sqrtf(u0);
    float theta = 2.0f * pi * u1;
    float st, ct;
    orc_sincosf(theta, &st, &ct);
    *px = r * ct;
    *py = r * st;
}

/* ------------------------------------------------------------------------------------ */
/* Spherical geometry — PBRT/SphericalGeometry.h:8-29                                    */
/* ------------------------------------------------------------------------------------ */
static inline float cos2t(v3 w) { return sqr(w.z); }
static inline float abscost(v3 w) { return gabs(w.z); }
static inline float sin2t(v3 w) { return gmax(0.0f, 1.0f - cos2t(w)); }
static inline float sint(v3 w) { return sqrtf(sin2t(w)); }
static inline float tan2t(v3 w) { return sin2t(w) / cos2t(w); }
static inline float cosphi(v3 w) {
    float s = sint(w);
    return (s == 0.0f) ? 1.0f : gclamp(w.x / s, -1.0f, 1.0f);
}
static inline float sinphi(v3 w) {
    float s = sint(w);
    return (s == 0.0f) ? 0.0f : gclamp(w.y / s, -1.0f, 1.0f);
}
static inline int samehemi(v3 w, v3 wp) { return w.z * wp.z > 0.0f; }

/* ------------------------------------------------------------------------------------ */
/* Trowbridge-Reitz microfacet — PBRT/Microfacet.h:9-119 (isotropic alpha)               */
/* ------------------------------------------------------------------------------------ */
static float mf_D(v3 wm, float alpha) {  /* Microfacet.h:9-20 */
    const float pi = 3.14159265359f;
    float t2 = tan2t(wm);
    if (isinf(t2)) return 0.0f;
    float cos4 = sqr(cos2t(wm));
    if (cos4 < 1e-16f) return 0.0f;
    float e = t2 * (sqr(cosphi(wm) / alpha) + sqr(sinphi(wm) / alpha));
    return 1.0f / (pi * alpha * alpha * cos4 * sqr(1.0f + e));
}
static float mf_lambda(v3 w, float alpha) {  /* Microfacet.h:46-52 */
    float t2 = tan2t(w);
    if (isinf(t2)) return 0.0f;
    float a2 = sqr(cosphi(w) * alpha) + sqr(sinphi(w) * alpha);
    return (sqrtf(1.0f + a2 * t2) - 1.0f) / 2.0f;
}
static float mf_G(v3 wo, v3 wi, float alpha) {  /* Microfacet.h:62-64 */
    return 1.0f / (1.0f + mf_lambda(wo, alpha) + mf_lambda(wi, alpha));
}
static float mf_G1(v3 w, float alpha) { return 1.0f / (1.0f + mf_lambda(w, alpha)); }
static float mf_Dw(v3 w, v3 wm, float alpha) {  /* Microfacet.h:81-84 */
    return mf_G1(w, alpha) / abscost(w) * mf_D(wm, alpha) * absdot(w, wm);
}
static float mf_pdf(v3 w, v3 wm, float alpha) { return mf_Dw(w, wm, alpha); }
static v3 mf_sample_wm(uint32_t* seed, v3 w, float alpha) {  /* Microfacet.h:90-119 */
    v3 wh = normalize3(mk(alpha * w.x, alpha * w.y, w.z));
    if (wh.z < 0.0f) wh = neg(wh);
    v3 T1 = (wh.z < 0.99999f) ? normalize3(cross3(ZAXIS, wh)) : mk(1.0f, 0.0f, 0.0f);
    v3 T2 = cross3(wh, T1);
    float px, py;
    disk_polar(seed, &px, &py);
    float h = sqrtf(1.0f - sqr(px));
    float x = (1.0f + wh.z) / 2.0f;
    py = (1.0f - x) * h + x * py;
    float pz = sqrtf(gmax(0.0f, 1.0f - (sqr(px) + sqr(py))));
    v3 nh = mk(px * T1.x + py * T2.x + pz * wh.x, px * T1.y + py * T2.y + pz * wh.y,
               px * T1.z + py * T2.z + pz * wh.z);
    return normalize3(mk(alpha * nh.x, alpha * nh.y, gmax(1e-6f, nh.z)));
}

/* ------------------------------------------------------------------------------------ */
/* BSDF sample record — PBRT/BSDFSample.h:5-14                                          */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    v3 color;
    float pdf;
    v3 dir;
    int refl, trans, spec, glossy;
} bsample;

/* ------------------------------------------------------------------------------------ */
/* Conductor — PBRT/Conductor.h:42-190, Complex.h:5-63                                   */
/* ------------------------------------------------------------------------------------ */
typedef struct { float re, im; } cplx;
static inline cplx cx(float re, float im) { cplx c = {re, im}; return c; }
static inline cplx cadd(cplx a, cplx b) { return cx(a.re + b.re, a.im + b.im); }
static inline cplx csub(cplx a, cplx b) { return cx(a.re - b.re, a.im - b.im); }
static inline cplx cmul(cplx a, cplx b) {
    return cx(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re);
}
static inline cplx cdiv(cplx a, cplx z) {
    float scale = 1.0f / (z.re * z.re + z.im * z.im);
    return cx(scale * (a.re * z.re + a.im * z.im), scale * (a.im * z.re - a.re * z.im));
}
static inline float cnorm(cplx z) { return z.re * z.re + z.im * z.im; }
static cplx csqrt_(cplx z) {  /* Complex.h:52-63 */
    float n = sqrtf(cnorm(z));
    float t1 = sqrtf(0.5f * (n + gabs(z.re)));
    float t2 = 0.5f * z.im / t1;
    if (n == 0.0f) return cx(0.0f, 0.0f);
    if (z.re >= 0.0f) return cx(t1, t2);
    return cx(gabs(t2), copysignf(t1, z.im));
}
static float fr_complex(float cos_i, cplx eta) {  /* Conductor.h:42-52 */
    cos_i = gclamp(cos_i, 0.0f, 1.0f);
    float sin2i = 1.0f - sqr(cos_i);
    cplx sin2t_ = cdiv(cx(sin2i, 0.0f), cmul(eta, eta));
    cplx cost = csqrt_(csub(cx(1.0f, 0.0f), sin2t_));
    cplx ec = cmul(eta, cx(cos_i, 0.0f));
    cplx r_parl = cdiv(csub(ec, cost), cadd(ec, cost));
    cplx ect = cmul(eta, cost);
    cplx r_perp = cdiv(csub(cx(cos_i, 0.0f), ect), cadd(cx(cos_i, 0.0f), ect));
    return (cnorm(r_parl) + cnorm(r_perp)) / 2.0f;
}
static v3 fresnel_complex(float cos_i, v3 refl) {  /* Conductor.h:54-92 */
    float r[3] = {gclamp(refl.x, 0.0f, 0.9999f), gclamp(refl.y, 0.0f, 0.9999f),
                  gclamp(refl.z, 0.0f, 0.9999f)};
    float out[3];
    for (int c = 0; c < 3; ++c) {
        float om = 1.0f - r[c];
        om = om > 0.0f ? om : 0.0f;  /* SaveMax(v, 0) glmCUDA.h:90-97 */
        float k = 2.0f * sqrtf(r[c]) / sqrtf(om);
        out[c] = fr_complex(cos_i, cx(1.0f, k));
    }
    return mk(out[0], out[1], out[2]);
}
static v3 conductor_f(v3 albedo, float roughness, v3 wo, v3 wi) {  /* Conductor.h:97-120 */
    float alpha = sqr(roughness);
    if (!samehemi(wo, wi)) return mk(0, 0, 0);
    if (alpha < 1e-3f) return mk(0, 0, 0);
    float co = abscost(wo), ci = abscost(wi);
    if (ci == 0.0f || co == 0.0f) return mk(0, 0, 0);
    v3 wm = add(wi, wo);
    if (lensqr3(wm) == 0.0f) return mk(0, 0, 0);
    wm = normalize3(wm);
    v3 F = fresnel_complex(absdot(wo, wm), albedo);
    float D = mf_D(wm, alpha), G = mf_G(wo, wi, alpha);
    float den = 4.0f * ci * co;
    return mk(D * F.x * G / den, D * F.y * G / den, D * F.z * G / den);
}
static int conductor_sample(uint32_t* seed, v3 albedo, float roughness, v3 wo, bsample* s) {
    /* Conductor.h:122-190 */
    float alpha = sqr(roughness);
    if (alpha < 1e-3f) {
        v3 wi = mk(-wo.x, -wo.y, wo.z);
        float ac = abscost(wi);
        s->color = divs(fresnel_complex(ac, albedo), ac);
        s->dir = wi;
        s->pdf = 1.0f;
        s->refl = 1; s->trans = 0; s->spec = 1; s->glossy = 0;
        return 1;
    }
    if (wo.z == 0.0f) return 0;
    v3 wm = mf_sample_wm(seed, wo, alpha);
    float d2 = 2.0f * dot3(wo, wm);
    v3 wi = add(neg(wo), smul(d2, wm));  /* Reflect lambda, Conductor.h:154-156 */
    if (!samehemi(wo, wi)) return 0;
    float pdf = mf_pdf(wo, wm, alpha) / (4.0f * absdot(wo, wm));
    float co = abscost(wo), ci = abscost(wi);
    if (ci == 0.0f || co == 0.0f) return 0;
    v3 F = fresnel_complex(absdot(wo, wm), albedo);
    float D = mf_D(wm, alpha), G = mf_G(wo, wi, alpha);
    float den = 4.0f * ci * co;
    s->color = mk(D * F.x * G / den, D * F.y * G / den, D * F.z * G / den);
    s->dir = wi;
    s->pdf = pdf;
    s->refl = 1; s->trans = 0; s->spec = 0; s->glossy = 1;
    return 1;
}

/* ------------------------------------------------------------------------------------ */
/* Lambert — PBRT/LambertDiffuse.h:35-140                                                */
/* ------------------------------------------------------------------------------------ */
static const float INV_PI = 0.31830988618379067154f;
static void disk_concentric(uint32_t* seed, float* dx, float* dy) {  /* :35-55 */
    const float PiOver4 = 0.78539816339744830961f;
    const float PiOver2 = 1.57079632679489661923f;
    float u0 = rnd(seed);
    float u1 = rnd(seed);
    float ox = 2.0f * u0 - 1.0f, oy = 2.0f * u1 - 1.0f;
    if (ox == 0.0f && oy == 0.0f) { *dx = 0.0f; *dy = 0.0f; return; }
    float theta, r;
    if (gabs(ox) > gabs(oy)) { r = ox; theta = PiOver4 * (oy / ox); }
    else { r = oy; theta = PiOver2 - PiOver4 * (ox / oy); }
    float st, ct;
    orc_sincosf(theta, &st, &ct);
    *dx = r * ct;
    *dy = r * st;
}
static v3 lambert_f(v3 albedo, v3 wo, v3 wi) {  /* :86-92 */
    if (!samehemi(wo, wi)) return mk(0, 0, 0);
    return muls(albedo, INV_PI);
}
static int lambert_sample(uint32_t* seed, v3 albedo, v3 wo, bsample* s, int reflection) {
    /* :110-132 — note: z is forced >= 0 regardless of wo's hemisphere (quirk 9) */
    (void)wo;
    if (!reflection) return 0;
    float dx, dy;
    disk_concentric(seed, &dx, &dy);
    float z = sqrtf(gmax(0.0f, 1.0f - sqr(dx) - sqr(dy)));
    v3 d = mk(dx, dy, z);
    if (d.z < 0.0f) d.z *= -1.0f;
    d = normalize3(d);
    s->dir = d;
    s->pdf = abscost(d) * INV_PI;
    s->color = muls(albedo, INV_PI);
    s->refl = 1; s->trans = 0; s->glossy = 0; s->spec = 0;
    return 1;
}
static float lambert_pdf(v3 wo, v3 wi, int reflection) {  /* :134-140 */
    if (!reflection || !samehemi(wi, wo)) return 0.0f;
    return abscost(wi) * INV_PI;
}

/* ------------------------------------------------------------------------------------ */
/* Dielectric (eta = 1.5) — PBRT/Dielectric.h:20-343                                     */
/* ------------------------------------------------------------------------------------ */
enum { RADIANCE = 0, IMPORTANCE = 1 };
static float fresnel_dielectric(float cos_i, float ior) {  /* :20-42 */
    cos_i = gclamp(cos_i, -1.0f, 1.0f);
    if (cos_i < 0.0f) { ior = 1.0f / ior; cos_i = -cos_i; }
    float sin2i = 1.0f - sqr(cos_i);
    float sin2t_ = sin2i / sqr(ior);
    if (sin2t_ >= 1.0f) return 1.0f;
    float cost = sqrtf(1.0f - sin2t_);
    float r_parl = (ior * cos_i - cost) / (ior * cos_i + cost);
    float r_perp = (cos_i - ior * cost) / (cos_i + ior * cost);
    return (sqr(r_parl) + sqr(r_perp)) / 2.0f;
}
static int refract_(v3 wi, v3 n, float eta, float* etap, v3* wt) {  /* :68-92 */
    float cos_i = dot3(n, wi);
    if (cos_i < 0.0f) { eta = 1.0f / eta; cos_i = -cos_i; n = neg(n); }
    float sin2i = gmax(0.0f, 1.0f - sqr(cos_i));
    float sin2t_ = sin2i / sqr(eta);
    if (sin2t_ >= 1.0f) return 0;
    float cost = sqrtf(1.0f - sin2t_);
    float k = cos_i / eta - cost;
    *wt = add(divs(neg(wi), eta), smul(k, n));
    if (etap) *etap = eta;
    return 1;
}
/* glm::faceforward(-normalize(wm), (0,0,1), normalize(wm)) */
static v3 ff_z(v3 wm) {
    v3 n = normalize3(wm);
    return (dot3(n, ZAXIS) < 0.0f) ? neg(n) : n;
}
static v3 dielectric_f(float roughness, v3 wo, v3 wi, int mode) {  /* :96-139 */
    const float eta = 1.5f;
    float alpha = sqr(roughness);
    if (alpha < 1e-3f) return mk(0, 0, 0);
    float co = wo.z, ci = wi.z;
    int reflect = ci * co > 0.0f;
    float etap = 1.0f;
    if (!reflect) etap = co > 0.0f ? eta : (1.0f / eta);
    v3 wm = add(muls(wi, etap), wo);
    if (ci == 0.0f || co == 0.0f || sqr(length3(wm)) == 0.0f) return mk(0, 0, 0);
    wm = ff_z(wm);
    if (dot3(wm, wi) * ci < 0.0f || dot3(wm, wo) * co < 0.0f) return mk(0, 0, 0);
    float F = fresnel_dielectric(dot3(wo, wm), eta);
    if (reflect) {
        float v = mf_D(wm, alpha) * mf_G(wo, wi, alpha) * F / fabsf(4.0f * ci * co);
        return mk(v, v, v);
    }
    float denom = sqr(dot3(wi, wm) + dot3(wo, wm) / etap) * ci * co;
    float ft = mf_D(wm, alpha) * (1.0f - F) * mf_G(wo, wi, alpha) *
               fabsf(dot3(wi, wm) * dot3(wo, wm) / denom);
    if (mode == RADIANCE) ft /= sqr(etap);
    return mk(ft, ft, ft);
}
static int dielectric_sample(uint32_t* seed, float roughness, v3 wo, bsample* s, int mode,
                             int reflection, int transmission) {  /* :146-288 */
    const float eta = 1.5f;
    float alpha = sqr(roughness);
    float uc = rnd(seed);  /* always drawn first (:149) */
    if (alpha < 1e-3f) {
        float R = fresnel_dielectric(wo.z, eta);
        float T = 1.0f - R;
        float pr = R, pt = T;
        if (!reflection) pr = 0.0f;
        if (!transmission) pt = 0.0f;
        if (pr == 0.0f && pt == 0.0f) return 0;
        if (uc < pr / (pr + pt)) {
            v3 wi = mk(-wo.x, -wo.y, wo.z);
            float fr = R / abscost(wi);
            s->color = mk(fr, fr, fr);
            s->dir = wi;
            s->pdf = pr / (pr + pt);
            s->refl = 1; s->trans = 0; s->glossy = 0; s->spec = 1;
            return 1;
        }
        v3 wi;
        float etap;
        if (!refract_(wo, ZAXIS, eta, &etap, &wi)) return 0;
        float ft = T / abscost(wi);
        if (mode == RADIANCE) ft /= sqr(etap);
        s->color = mk(ft, ft, ft);
        s->dir = wi;
        s->pdf = pt / (pr + pt);
        s->refl = 0; s->trans = 1; s->glossy = 0; s->spec = 1;
        return 1;
    }
    v3 wm = mf_sample_wm(seed, wo, alpha);
    float R = fresnel_dielectric(dot3(wo, wm), eta);
    float T = 1.0f - R;
    float pr = R, pt = T;
    if (!reflection) pr = 0.0f;
    if (!transmission) pt = 0.0f;
    if (pr == 0.0f && pt == 0.0f) return 0;
    if (uc < pr / (pr + pt)) {
        /* glm::reflect(-wo, wm) = I - N*dot(N,I)*2 */
        v3 I = neg(wo);
        float d = dot3(wm, I);
        v3 wi = mk(I.x - wm.x * d * 2.0f, I.y - wm.y * d * 2.0f, I.z - wm.z * d * 2.0f);
        if (!samehemi(wo, wi)) return 0;
        float pdf = mf_pdf(wo, wm, alpha) / (4.0f * absdot(wo, wm)) * pr / (pr + pt);
        float f = mf_D(wm, alpha) * mf_G(wo, wi, alpha) * R / (4.0f * wi.z * wo.z);
        s->color = mk(f, f, f);
        s->dir = wi;
        s->pdf = pdf;
        s->refl = 1; s->trans = 0; s->glossy = 1; s->spec = 0;
        return 1;
    }
    float etap;
    v3 wi = mk(0, 0, 0);
    int tir = !refract_(wo, wm, eta, &etap, &wi);
    if (tir || samehemi(wo, wi) || wi.z == 0.0f) return 0;
    float denom = sqr(dot3(wi, wm) + dot3(wo, wm) / etap);
    float dwm_dwi = absdot(wi, wm) / denom;
    float pdf = mf_pdf(wo, wm, alpha) * dwm_dwi * pt / (pr + pt);
    float ft = T * mf_D(wm, alpha) * mf_G(wo, wi, alpha) *
               fabsf(dot3(wi, wm) * dot3(wo, wm) / (wi.z * wo.z * denom));
    if (mode == RADIANCE) ft /= sqr(etap);
    s->color = mk(ft, ft, ft);
    s->dir = wi;
    s->pdf = pdf;
    s->refl = 0; s->trans = 1; s->glossy = 1; s->spec = 0;
    return 1;
}
static float dielectric_pdf(float roughness, v3 wo, v3 wi, int reflection, int transmission) {
    /* :290-343 */
    const float eta = 1.5f;
    float alpha = sqr(roughness);
    if (alpha < 1e-3f) return 0.0f;
    float co = wo.z, ci = wi.z;
    int reflect = ci * co > 0.0f;
    float etap = 1.0f;
    if (!reflect) etap = co > 0.0f ? eta : (1.0f / eta);
    v3 wm = add(muls(wi, etap), wo);
    if (ci == 0.0f || co == 0.0f || lensqr3(wm) == 0.0f) return 0.0f;
    wm = ff_z(wm);
    if (dot3(wm, wi) * ci < 0.0f || dot3(wm, wo) * co < 0.0f) return 0.0f;
    float R = fresnel_dielectric(dot3(wo, wm), eta);
    float T = 1.0f - R;
    float pr = R, pt = T;
    if (!reflection) pr = 0.0f;
    if (!transmission) pt = 0.0f;
    if (pr == 0.0f && pt == 0.0f) return 0.0f;
    if (reflect) return mf_pdf(wo, wm, alpha) / (4.0f * absdot(wo, wm)) * pr / (pr + pt);
    float denom = sqr(dot3(wi, wm) + dot3(wo, wm) / etap);
    float dwm_dwi = absdot(wi, wm) / denom;
    return mf_pdf(wo, wm, alpha) * dwm_dwi * pt / (pr + pt);
}

/* ------------------------------------------------------------------------------------ */
/* Layered "GlossyDiffuse": dielectric over Lambert — PBRT/GlossyDiffuse.h:91-524         */
/* ------------------------------------------------------------------------------------ */
static float power_heuristic(float fpdf, float gpdf) {  /* :91-95 with nf = ng = 1 */
    float f = 1.0f * fpdf, g = 1.0f * gpdf;
    return sqr(f) / (sqr(f) + sqr(g));
}
static float transmittance(float dz, v3 w) {  /* :97-105 */
    if (gabs(dz) <= FLT_MIN) return 1.0f;
    return orc_expf_neg(-gabs(dz / w.z));
}
static v3 layer_f(int top, v3 albedo, float roughness, v3 wo, v3 wi, int mode) {
    return top ? dielectric_f(roughness, wo, wi, mode) : lambert_f(albedo, wo, wi);
}
static int layer_sample(int top, uint32_t* seed, v3 albedo, float roughness, v3 wo, bsample* s,
                        int mode, int refl, int trans) {
    return top ? dielectric_sample(seed, roughness, wo, s, mode, refl, trans)
               : lambert_sample(seed, albedo, wo, s, refl);
}
static float layer_pdf(int top, float roughness, v3 wo, v3 wi, int refl, int trans) {
    return top ? dielectric_pdf(roughness, wo, wi, refl, trans) : lambert_pdf(wo, wi, refl);
}
static int bs_bad(int ok, const bsample* b) {
    return !ok || iszero3(b->color) || b->pdf == 0.0f || b->dir.z == 0.0f;
}

static v3 layered_f(uint32_t* seed, v3 albedo, float roughness, v3 wo, v3 wi) {  /* :141-367 */
    const int mode = RADIANCE;
    const int nSamples = 5;
    const float thickness = 0.01f;
    const int maxDepth = 10;
    int topSpec = sqr(roughness) < 1e-3f;
    const int botSpec = 0;
    v3 f = mk(0, 0, 0);
    if (wo.z < 0.0f) { wo = neg(wo); wi = neg(wi); }
    const int enteredTop = 1;
    int same = samehemi(wo, wi);
    int exitTop, nonExitTop, exitSpec, nonExitSpec;
    if (same ^ enteredTop) { exitSpec = botSpec; nonExitSpec = topSpec; exitTop = 0; nonExitTop = 1; }
    else { exitSpec = topSpec; nonExitSpec = botSpec; exitTop = 1; nonExitTop = 0; }
    float exitZ = (same ^ enteredTop) ? 0.0f : thickness;
    if (same) f = mulv(mk(5.0f, 5.0f, 5.0f), layer_f(enteredTop, albedo, roughness, wo, wi, mode));

    uint32_t ns = orc_tea16(orc_f2u_sat(wo.x * 1000.0f), orc_f2u_sat(wo.y * 1000.0f));
    ns = orc_tea16(ns, orc_f2u_sat(wi.x * 1000.0f));
    ns = orc_tea16(ns, orc_f2u_sat(wi.y * 1000.0f));
    ns = orc_tea16(ns, *seed);

    for (int s = 0; s < nSamples; ++s) {
        bsample wos, wis, bs;
        int ok = layer_sample(enteredTop, seed, albedo, roughness, wo, &wos, mode, 0, 1);
        if (bs_bad(ok, &wos)) continue;
        ok = layer_sample(exitTop, seed, albedo, roughness, wi, &wis, IMPORTANCE, 0, 1);
        if (bs_bad(ok, &wis)) continue;
        float a = abscost(wos.dir);
        v3 beta = mk(wos.color.x * a / wos.pdf, wos.color.y * a / wos.pdf, wos.color.z * a / wos.pdf);
        float z = enteredTop ? thickness : 0.0f;
        v3 w = wos.dir;
        for (int depth = 0; depth < maxDepth; ++depth) {
            if (depth > 3 && savemax3(beta) < 0.25f) {
                float q = gmax(0.0f, 1.0f - savemax3(beta));
                if (rnd(&ns) < q) break;
                beta = divs(beta, 1.0f - q);
            }
            /* mediaAlbedo == 0: advance to the other interface (:263-268) */
            z = (z == thickness) ? 0.0f : thickness;
            beta = muls(beta, transmittance(thickness, w));
            if (z == exitZ) {
                ok = layer_sample(exitTop, seed, albedo, roughness, neg(w), &bs, mode, 1, 0);
                if (bs_bad(ok, &bs)) break;
                float c = abscost(bs.dir);
                beta = mulv(beta, mk(bs.color.x * c / bs.pdf, bs.color.y * c / bs.pdf, bs.color.z * c / bs.pdf));
                w = bs.dir;
            } else {
                if (!nonExitSpec) {
                    float wt = 1.0f;
                    if (!exitSpec)
                        wt = power_heuristic(wis.pdf, layer_pdf(nonExitTop, roughness, neg(w), neg(wis.dir), 1, 1));
                    v3 lf = layer_f(nonExitTop, albedo, roughness, neg(w), neg(wis.dir), mode);
                    float ac = abscost(wis.dir);
                    float tr = transmittance(thickness, wis.dir);
                    v3 t1 = mulv(beta, lf);
                    t1 = muls(t1, ac);
                    t1 = muls(t1, wt);
                    t1 = muls(t1, tr);
                    t1 = mulv(t1, wis.color);
                    t1 = divs(t1, wis.pdf);
                    f = add(f, t1);
                }
                ok = layer_sample(nonExitTop, seed, albedo, roughness, neg(w), &bs, mode, 1, 0);
                if (bs_bad(ok, &bs)) break;
                float c = abscost(bs.dir);
                beta = mulv(beta, mk(bs.color.x * c / bs.pdf, bs.color.y * c / bs.pdf, bs.color.z * c / bs.pdf));
                w = bs.dir;
                if (!exitSpec) {
                    v3 fExit = layer_f(exitTop, albedo, roughness, neg(w), wi, mode);
                    if (!iszero3(fExit)) {
                        float wt = 1.0f;
                        if (!nonExitSpec) {
                            float exitPDF = layer_pdf(exitTop, roughness, neg(w), wi, 0, 1);
                            wt = power_heuristic(bs.pdf, exitPDF);
                        }
                        float tr = transmittance(thickness, bs.dir);
                        v3 t1 = muls(beta, tr);
                        t1 = mulv(t1, fExit);
                        t1 = muls(t1, wt);
                        f = add(f, t1);
                    }
                }
            }
        }
    }
    return mk(f.x / 5.0f, f.y / 5.0f, f.z / 5.0f);
}

static int layered_sample(uint32_t* seed, v3 albedo, float roughness, v3 wo, bsample* out) {
    /* :372-524 */
    const int mode = RADIANCE;
    const float thickness = 0.01f;
    const int maxDepth = 10;
    int flipWi = 0;
    if (wo.z < 0.0f) { wo = neg(wo); flipWi = 1; }
    const int enteredTop = 1;
    bsample bs;
    int ok = layer_sample(enteredTop, seed, albedo, roughness, wo, &bs, mode, 1, 1);
    if (bs_bad(ok, &bs)) return 0;
    if (bs.refl) {
        if (flipWi) bs.dir = neg(bs.dir);
        *out = bs;
        return 1;
    }
    v3 w = bs.dir;
    int specPath = bs.spec;
    uint32_t ns = orc_tea16(orc_f2u_sat(wo.x * 1000.0f), orc_f2u_sat(wo.y * 1000.0f));
    ns = orc_tea16(ns, *seed);
    v3 f = muls(bs.color, abscost(bs.dir));
    float pdf = bs.pdf;
    float z = enteredTop ? thickness : 0.0f;
    for (int depth = 0; depth < maxDepth; ++depth) {
        float rrBeta = savemax3(f) / pdf;
        if (depth > 3 && rrBeta < 0.25f) {
            float q = gmax(0.0f, 1.0f - rrBeta);
            if (rnd(&ns) < q) return 0;
            pdf *= 1.0f - q;
        }
        if (w.z == 0.0f) return 0;
        z = (z == thickness) ? 0.0f : thickness;
        f = muls(f, transmittance(thickness, w));
        int itop = (z == 0.0f) ? 0 : 1;
        ok = layer_sample(itop, seed, albedo, roughness, neg(w), &bs, mode, 1, 1);
        if (bs_bad(ok, &bs)) return 0;
        f = mulv(f, bs.color);
        pdf *= bs.pdf;
        specPath &= bs.spec;
        w = bs.dir;
        if (bs.trans) {
            if (flipWi) w = neg(w);
            out->color = f;
            out->dir = w;
            out->pdf = pdf;
            out->refl = samehemi(wo, w);
            out->trans = !out->refl;
            out->spec = specPath;
            out->glossy = !out->spec;
            return 1;
        }
        f = muls(f, abscost(bs.dir));
    }
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* Material dispatch — devicePrograms.cu:303-341 (+ commented alternatives)              */
/* ------------------------------------------------------------------------------------ */
typedef struct {
    v3 wo;  /* outgoingRay in shading space */
    v3 albedo;
    float roughness;
    int conductor;
} surf;

static int bsdf_sample_mode(int mode, uint32_t* seed, const surf* s, bsample* bs) {
    switch (mode) {
        case ORC_MAT_LAMBERT: return lambert_sample(seed, s->albedo, s->wo, bs, 1);
        case ORC_MAT_CONDUCTOR: return conductor_sample(seed, s->albedo, s->roughness, s->wo, bs);
        case ORC_MAT_DIELECTRIC: return dielectric_sample(seed, s->roughness, s->wo, bs, RADIANCE, 1, 1);
        case ORC_MAT_LAYERED: return layered_sample(seed, s->albedo, s->roughness, s->wo, bs);
        default:
            if (s->conductor) return conductor_sample(seed, s->albedo, s->roughness, s->wo, bs);
            return layered_sample(seed, s->albedo, s->roughness, s->wo, bs);
    }
}
static v3 bsdf_f_mode(int mode, uint32_t* seed, const surf* s, v3 wi) {
    switch (mode) {
        case ORC_MAT_LAMBERT: return lambert_f(s->albedo, s->wo, wi);
        case ORC_MAT_CONDUCTOR: return conductor_f(s->albedo, s->roughness, s->wo, wi);
        case ORC_MAT_DIELECTRIC: return dielectric_f(s->roughness, s->wo, wi, RADIANCE);
        case ORC_MAT_LAYERED: return layered_f(seed, s->albedo, s->roughness, s->wo, wi);
        default:
            if (s->conductor) return conductor_f(s->albedo, s->roughness, s->wo, wi);
            return layered_f(seed, s->albedo, s->roughness, s->wo, wi);
    }
}

static void fill_out(const bsample* b, float out[8]) {
    out[0] = b->color.x; out[1] = b->color.y; out[2] = b->color.z; out[3] = b->pdf;
    out[4] = b->dir.x; out[5] = b->dir.y; out[6] = b->dir.z;
    out[7] = (float)((b->refl ? 1 : 0) | (b->trans ? 2 : 0) | (b->spec ? 4 : 0) | (b->glossy ? 8 : 0));
}
int32_t orc_bsdf_sample(int32_t model, uint32_t* seed, const float albedo[3], float roughness,
                        const float wo[3], float out[8]) {
    bsample b;
    memset(&b, 0, sizeof b);
    v3 a = mk(albedo[0], albedo[1], albedo[2]), w = mk(wo[0], wo[1], wo[2]);
    int ok = 0;
    switch (model) {
        case ORC_BSDF_LAMBERT: ok = lambert_sample(seed, a, w, &b, 1); break;
        case ORC_BSDF_CONDUCTOR: ok = conductor_sample(seed, a, roughness, w, &b); break;
        case ORC_BSDF_DIELECTRIC: ok = dielectric_sample(seed, roughness, w, &b, RADIANCE, 1, 1); break;
        default: ok = layered_sample(seed, a, roughness, w, &b); break;
    }
    if (!ok) memset(&b, 0, sizeof b);
    fill_out(&b, out);
    return ok;
}
void orc_bsdf_eval(int32_t model, uint32_t* seed, const float albedo[3], float roughness,
                   const float wo[3], const float wi[3], float out[3]) {
    v3 a = mk(albedo[0], albedo[1], albedo[2]), o = mk(wo[0], wo[1], wo[2]), i = mk(wi[0], wi[1], wi[2]);
    v3 r;
    switch (model) {
        case ORC_BSDF_LAMBERT: r = lambert_f(a, o, i); break;
        case ORC_BSDF_CONDUCTOR: r = conductor_f(a, roughness, o, i); break;
        case ORC_BSDF_DIELECTRIC: r = dielectric_f(roughness, o, i, RADIANCE); break;
        default: r = layered_f(seed, a, roughness, o, i); break;
    }
    out[0] = r.x; out[1] = r.y; out[2] = r.z;
}
/* UnitTests/SpherGeom_Test.cpp:17-22 (PBRT::SpherGeom::CosTheta, SphericalGeometry.h:8) */
float orc_cos_theta(const float w[3]) { return w[2]; }

/* Furnace loop of UnitTests/SpherGeom_Test.cpp:28-252: mean over n samples of
 * f*|cos|/pdf (AbsDot(dir, (0,0,1))) for one wo, one shared seed (advanced in place). */
void orc_furnace(int32_t model, uint32_t* seed, const float albedo[3], float roughness, const float wo[3],
                 int32_t n, float out[3]) {
    v3 a = mk(albedo[0], albedo[1], albedo[2]), w = mk(wo[0], wo[1], wo[2]);
    v3 acc = mk(0, 0, 0);
    for (int32_t j = 0; j < n; ++j) {
        bsample b;
        memset(&b, 0, sizeof b);
        int ok = (model == ORC_BSDF_CONDUCTOR) ? conductor_sample(seed, a, roughness, w, &b)
                                                : layered_sample(seed, a, roughness, w, &b);
        if (ok) acc = add(acc, divs(muls(b.color, absdot(b.dir, ZAXIS)), b.pdf));
    }
    out[0] = acc.x / (float)n; out[1] = acc.y / (float)n; out[2] = acc.z / (float)n;
}

/* Density of Conductor::Sample_f's direction (Conductor.h:123-189 computes it for the sampled
 * wm: D(wo, wm) / (4 |wo.wm|)).  The reference has no Conductor::PDF; this is PBRT-v4's
 * ConductorBxDF::PDF (wm = the half vector of wo and wi, faced to +z), used by the chi-square
 * sampling test (tests/test_oracle_pins.py). */
static float conductor_pdf(float roughness, v3 wo, v3 wi) {
    float alpha = sqr(roughness);
    if (!(wo.z * wi.z > 0.0f) || alpha < 1e-3f) return 0.0f;
    v3 wm = add(wo, wi);
    if (lensqr3(wm) == 0.0f) return 0.0f;
    wm = normalize3(wm);
    if (wm.z < 0.0f) wm = neg(wm);
    return mf_pdf(wo, wm, alpha) / (4.0f * absdot(wo, wm));
}
float orc_bsdf_pdf(int32_t model, float roughness, const float wo[3], const float wi[3]) {
    v3 o = mk(wo[0], wo[1], wo[2]), i = mk(wi[0], wi[1], wi[2]);
    if (model == ORC_BSDF_LAMBERT) return lambert_pdf(o, i, 1);
    if (model == ORC_BSDF_DIELECTRIC) return dielectric_pdf(roughness, o, i, 1, 1);
    if (model == ORC_BSDF_CONDUCTOR) return conductor_pdf(roughness, o, i);
    return 0.0f;
}
/* Batched forms for the statistical tests: n samples from one wo and a running seed; the pdf
 * at n directions. */
void orc_bsdf_sample_n(int32_t model, uint32_t* seed, const float albedo[3], float roughness, const float wo[3],
                       int32_t n, float* out8, int32_t* ok) {
    for (int32_t k = 0; k < n; ++k) ok[k] = orc_bsdf_sample(model, seed, albedo, roughness, wo, out8 + 8 * (size_t)k);
}
void orc_bsdf_pdf_n(int32_t model, float roughness, const float wo[3], const float* wi3, int32_t n, float* out) {
    for (int32_t k = 0; k < n; ++k) out[k] = orc_bsdf_pdf(model, roughness, wo, wi3 + 3 * (size_t)k);
}

/* ------------------------------------------------------------------------------------ */
/* Camera — Camera.cpp:6-70, GlmHelperMethods.cpp:4-10, glm perspectiveRH_NO/lookAtRH/inverse */
/* ------------------------------------------------------------------------------------ */
static void glm_inverse4(const float* m, float* out) {  /* glm detail/func_matrix.inl:294-351 */
#define M(c, r) m[(c) * 4 + (r)]
    float C00 = M(2,2) * M(3,3) - M(3,2) * M(2,3);
    float C02 = M(1,2) * M(3,3) - M(3,2) * M(1,3);
    float C03 = M(1,2) * M(2,3) - M(2,2) * M(1,3);
    float C04 = M(2,1) * M(3,3) - M(3,1) * M(2,3);
    float C06 = M(1,1) * M(3,3) - M(3,1) * M(1,3);
    float C07 = M(1,1) * M(2,3) - M(2,1) * M(1,3);
    float C08 = M(2,1) * M(3,2) - M(3,1) * M(2,2);
    float C10 = M(1,1) * M(3,2) - M(3,1) * M(1,2);
    float C11 = M(1,1) * M(2,2) - M(2,1) * M(1,2);
    float C12 = M(2,0) * M(3,3) - M(3,0) * M(2,3);
    float C14 = M(1,0) * M(3,3) - M(3,0) * M(1,3);
    float C15 = M(1,0) * M(2,3) - M(2,0) * M(1,3);
    float C16 = M(2,0) * M(3,2) - M(3,0) * M(2,2);
    float C18 = M(1,0) * M(3,2) - M(3,0) * M(1,2);
    float C19 = M(1,0) * M(2,2) - M(2,0) * M(1,2);
    float C20 = M(2,0) * M(3,1) - M(3,0) * M(2,1);
    float C22 = M(1,0) * M(3,1) - M(3,0) * M(1,1);
    float C23 = M(1,0) * M(2,1) - M(2,0) * M(1,1);
    float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
    float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
    float V0[4] = {M(1,0), M(0,0), M(0,0), M(0,0)};
    float V1[4] = {M(1,1), M(0,1), M(0,1), M(0,1)};
    float V2[4] = {M(1,2), M(0,2), M(0,2), M(0,2)};
    float V3[4] = {M(1,3), M(0,3), M(0,3), M(0,3)};
    float I0[4], I1[4], I2[4], I3[4];
    const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
    for (int i = 0; i < 4; ++i) {
        I0[i] = (V1[i] * F0[i] - V2[i] * F1[i] + V3[i] * F2[i]) * SA[i];
        I1[i] = (V0[i] * F0[i] - V2[i] * F3[i] + V3[i] * F4[i]) * SB[i];
        I2[i] = (V0[i] * F1[i] - V1[i] * F3[i] + V3[i] * F5[i]) * SA[i];
        I3[i] = (V0[i] * F2[i] - V1[i] * F4[i] + V2[i] * F5[i]) * SB[i];
    }
    float row0[4] = {I0[0], I1[0], I2[0], I3[0]};
    float d0 = M(0,0) * row0[0], d1 = M(0,1) * row0[1], d2 = M(0,2) * row0[2], d3 = M(0,3) * row0[3];
    float det = (d0 + d1) + (d2 + d3);
    float one = 1.0f / det;
    for (int i = 0; i < 4; ++i) {
        out[0 * 4 + i] = I0[i] * one; out[1 * 4 + i] = I1[i] * one;
        out[2 * 4 + i] = I2[i] * one; out[3 * 4 + i] = I3[i] * one;
    }
#undef M
}
void orc_camera_from_blender(const float bp[3], const float br[3], float fov_deg, int32_t W,
                             int32_t H, float pos[3], float inv_view[16], float inv_proj[16]) {
    const float deg2rad = 0.01745329251994329576923690768489f;  /* glm::radians */
    v3 p = mk(bp[0], bp[2], -bp[1]);                                   /* BlenderToEnginePosition */
    v3 rot = mk(90.0f - br[0], 180.0f + br[2], br[1]);                 /* BlenderToEngineRotation */
    v3 rr = mk(rot.x * deg2rad, rot.y * deg2rad, rot.z * deg2rad);
    float x = sinf(rr.y);  /* Camera::GetForward :37-49 */
    x *= cosf(rr.x);
    float y = -sinf(rr.x);
    float z = cosf(rr.x);
    z *= cosf(rr.y);
    v3 fwd = normalize3(mk(x, y, z));
    /* lookAtRH(eye, center, up) */
    v3 center = add(p, fwd);
    v3 up = mk(0.0f, 1.0f, 0.0f);
    v3 f = normalize3(sub(center, p));
    v3 s = normalize3(cross3(f, up));
    v3 u = cross3(s, f);
    float V[16];
    for (int i = 0; i < 16; ++i) V[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    V[0 * 4 + 0] = s.x; V[1 * 4 + 0] = s.y; V[2 * 4 + 0] = s.z;
    V[0 * 4 + 1] = u.x; V[1 * 4 + 1] = u.y; V[2 * 4 + 1] = u.z;
    V[0 * 4 + 2] = -f.x; V[1 * 4 + 2] = -f.y; V[2 * 4 + 2] = -f.z;
    V[3 * 4 + 0] = -dot3(s, p); V[3 * 4 + 1] = -dot3(u, p); V[3 * 4 + 2] = dot3(f, p);
    /* perspectiveRH_NO(fovy, aspect, 0.1, 100) — fov used as fovy (quirk 1) */
    float fovy = fov_deg * deg2rad;
    float aspect = (float)W / (float)H;
    float zNear = (float)0.1, zFar = (float)100.0;
    float th = tanf(fovy / 2.0f);
    float P[16];
    memset(P, 0, sizeof P);
    P[0 * 4 + 0] = 1.0f / (aspect * th);
    P[1 * 4 + 1] = 1.0f / th;
    P[2 * 4 + 2] = -(zFar + zNear) / (zFar - zNear);
    P[2 * 4 + 3] = -1.0f;
    P[3 * 4 + 2] = -(2.0f * zFar * zNear) / (zFar - zNear);
    pos[0] = p.x; pos[1] = p.y; pos[2] = p.z;
    glm_inverse4(V, inv_view);
    glm_inverse4(P, inv_proj);
}
void orc_camera_ray(const orc_launch* lp, int32_t x, int32_t y, float origin[3], float dir[3]) {
    /* devicePrograms.cu:601-623 — pixel centre, no jitter */
    float xs = ((float)x + 0.5f) / (float)lp->width;
    float ys = ((float)y + 0.5f) / (float)lp->height;
    float ndc[4] = {xs * 2.0f - 1.0f, ys * 2.0f - 1.0f, 1.0f, 1.0f};
    float pv[4], pw[4];
    mat4_mul_vec4(lp->inv_proj, ndc, pv);
    float pv0[4] = {pv[0], pv[1], pv[2], 0.0f};
    mat4_mul_vec4(lp->inv_view, pv0, pw);
    /* glm normalize(vec4): dot4 = (x*x + y*y) + (z*z + w*w) */
    float d4 = (pw[0] * pw[0] + pw[1] * pw[1]) + (pw[2] * pw[2] + pw[3] * pw[3]);
    float inv = 1.0f / sqrtf(d4);
    dir[0] = pw[0] * inv; dir[1] = pw[1] * inv; dir[2] = pw[2] * inv;
    origin[0] = lp->cam_pos[0]; origin[1] = lp->cam_pos[1]; origin[2] = lp->cam_pos[2];
}

/* ------------------------------------------------------------------------------------ */
/* Scene + CPU BVH (independent of the GPU LBVH; results ordered by (t, prim))           */
/* ------------------------------------------------------------------------------------ */
typedef struct { float lo[3], hi[3]; int32_t left, right, first, count; } onode;

struct orc_scene {
    int32_t ntri;
    v3* v;          /* 3 per triangle, world space */
    v3* n;          /* 3 per triangle, object space (transformed at hit, as the reference) */
    int32_t* has_n;
    float* model;   /* 16 per triangle's mesh */
    int32_t* mesh;  /* mesh id per triangle */
    v3* albedo;     /* per mesh */
    float* metallic;
    float* roughness;
    int32_t nmesh;
    int32_t* order; /* BVH leaf order -> triangle index */
    onode* nodes;
    int32_t nnodes;
    float* uv;          /* 6 per triangle (uv0, uv1, uv2; zeros when the mesh has none) */
    int32_t* tex_ids;   /* 3 per mesh: albedo, normal, metal-rough (-1 = none) */
    orc_texture* tex;   /* copies of the caller's texture descriptors (pixels borrowed) */
    uint32_t** texpix;  /* owned pixel copies */
    int32_t ntex;
};

/* ---- textures: devicePrograms.cu:62-73 (SRGB8ToLinear), :143-166 (SampleTextures),
 * OptixRenderer.cpp:562-612 (CreateTextures: uchar4, cudaFilterModeLinear,
 * cudaAddressModeWrap, normalized coords, cudaReadModeNormalizedFloat).  Bilinear filtering
 * follows the CUDA programming guide's texture-fetch formula with the filter weight held in
 * 1.8 fixed point (8 fractional bits); the HIP kernels evaluate exactly the same expression. */
static inline float srgb_to_linear(float c) {
    float m = (c < 0.04045f) ? 0.0f : 1.0f;  /* glm::step(0.04045, c) */
    float a = c / 12.92f;
    float nom = c + 0.055f;
    float b = orc_powf_unit(nom / 1.055f, 2.4f);  /* SavePow */
    return a * (1.0f - m) + b * m;            /* SaveMix */
}
static inline int wrapi(int i, int n) { int r = i % n; return r < 0 ? r + n : r; }
void orc_tex_sample(const orc_texture* t, float x, float y, int32_t srgb, float out[4]) {
    const int W = t->width, H = t->height;
    x = x - floorf(x);
    y = y - floorf(y);
    float xb = x * (float)W - 0.5f, yb = y * (float)H - 0.5f;
    float fx = floorf(xb), fy = floorf(yb);
    float ax = rintf((xb - fx) * 256.0f) * (1.0f / 256.0f);
    float ay = rintf((yb - fy) * 256.0f) * (1.0f / 256.0f);
    int i0 = wrapi((int)fx, W), i1 = wrapi((int)fx + 1, W);
    int j0 = wrapi((int)fy, H), j1 = wrapi((int)fy + 1, H);
    uint32_t p00 = t->rgba8[(size_t)j0 * W + i0], p10 = t->rgba8[(size_t)j0 * W + i1];
    uint32_t p01 = t->rgba8[(size_t)j1 * W + i0], p11 = t->rgba8[(size_t)j1 * W + i1];
    for (int c = 0; c < 4; ++c) {
        float t00 = (float)((p00 >> (8 * c)) & 0xff) / 255.0f, t10 = (float)((p10 >> (8 * c)) & 0xff) / 255.0f;
        float t01 = (float)((p01 >> (8 * c)) & 0xff) / 255.0f, t11 = (float)((p11 >> (8 * c)) & 0xff) / 255.0f;
        float r0 = t00 * (1.0f - ax) + t10 * ax;
        float r1 = t01 * (1.0f - ax) + t11 * ax;
        float v = r0 * (1.0f - ay) + r1 * ay;
        out[c] = srgb ? srgb_to_linear(v) : v;
    }
}
/* GetTextureCoord (devicePrograms.cu:131-141) */
static inline void tri_uv(const orc_scene* s, int t, float u, float v, float* x, float* y) {
    const float* q = &s->uv[6 * t];
    float w = 1.0f - u - v;
    *x = (w * q[0] + u * q[2]) + v * q[4];
    *y = (w * q[1] + u * q[3]) + v * q[5];
}
/* AlphaCutout (devicePrograms.cu:518-543): albedo-textured meshes drop hits with alpha < 0.9 */
static int alpha_cut(const orc_scene* s, int t, float u, float v) {
    int m = s->mesh[t];
    int at = s->tex_ids ? s->tex_ids[3 * m] : -1;
    if (at < 0) return 0;
    float x, y, c[4];
    tri_uv(s, t, u, v, &x, &y);
    orc_tex_sample(&s->tex[at], x, y, 1, c);
    return c[3] < 0.9f;
}

/* ---- Closest-hit rule shared with the kernels (pt_device.h tri_accept / node_eval) ------
 * OptiX's closest hit comes from closed code (devicePrograms.cu:243-260); this restatement
 * defines it as the (t, global index) minimum over the ACCEPTABLE Moller-Trumbore hits: the
 * hit's t must lie in the slab interval of the triangle's own padded box, with relative slack
 * K = 1 + 2^-12.  The box uses the vertices as the hit test sees them (v0, v0 + e1, v0 + e2);
 * slab distances are fmaf(plane, inv, -o*inv) with inv = 1/d (a zero component -> +-1e30).
 * Every BVH box below is a union of these boxes, and the box cull keeps a box iff
 * max(tn, tmin) <= min(tf, best) * K, so no box holding an acceptable hit with t <= best is
 * culled: the answer is the same for any BVH and any visiting order (the kernels' BVH4 and
 * this binary median split agree bit for bit).  Without the rule a grazing ray could be
 * accepted at a point outside the triangle's own box and the answer depended on which
 * triangle set `best` first (one trace in 62 M of the config-5 band). */
/* The traversal and the path loop are compiled twice, with and without the FMA instruction set,
 * and the loader picks the FMA clone where the CPU has it: fmaf is then one instruction instead
 * of a libm call.  fmaf is exactly rounded either way, so both clones give the same bits. */
#if defined(__x86_64__) && defined(__GNUC__)
#define ORC_HOT __attribute__((target_clones("fma", "default")))
#else
#define ORC_HOT
#endif
static const float kSlabWiden = 1.000244140625f;
/* fminf / fmaxf without the libm call (gcc calls them unless NaNs and signed zeros are
 * excluded, and the traversal spent most of its time there).  No NaN reaches these: slab
 * distances are fmaf(plane, inv, -o*inv) with finite inv (a zero direction component maps to
 * +-1e30), and which zero a tie returns does not change a comparison or a padded box. */
static inline float mn(float a, float b) { return b < a ? b : a; }
static inline float mx(float a, float b) { return b > a ? b : a; }
static inline float ray_inv(float d) { return d != 0.0f ? 1.0f / d : copysignf(1e30f, d); }
static inline float box_pad(float x) { return fabsf(x) * 9.5367431640625e-7f + 1e-6f; }
static void tri_bounds(const orc_scene* s, int t, float lo[3], float hi[3]) {
    v3 v0 = s->v[3 * t], e1 = sub(s->v[3 * t + 1], v0), e2 = sub(s->v[3 * t + 2], v0);
    float a[3] = {v0.x, v0.y, v0.z}, b[3] = {e1.x, e1.y, e1.z}, c[3] = {e2.x, e2.y, e2.z};
    for (int k = 0; k < 3; ++k) {
        float p1 = a[k] + b[k], p2 = a[k] + c[k];
        float l = mn(mn(a[k], p1), p2), h = mx(mx(a[k], p1), p2);
        lo[k] = l - box_pad(l);
        hi[k] = h + box_pad(h);
    }
}
/* slab interval of a box; tn / tf without tmin / tmax */
static inline void slab_interval(const float lo[3], const float hi[3], v3 inv, v3 io, float* tn, float* tf) {
    float ax = fmaf(lo[0], inv.x, -io.x), bx = fmaf(hi[0], inv.x, -io.x);
    float ay = fmaf(lo[1], inv.y, -io.y), by = fmaf(hi[1], inv.y, -io.y);
    float az = fmaf(lo[2], inv.z, -io.z), bz = fmaf(hi[2], inv.z, -io.z);
    *tn = mx(mx(mn(ax, bx), mn(ay, by)), mn(az, bz));
    *tf = mn(mn(mx(ax, bx), mx(ay, by)), mx(az, bz));
}
static int tri_accept(const orc_scene* s, int t, v3 inv, v3 io, float th) {
    float lo[3], hi[3], tn, tf;
    tri_bounds(s, t, lo, hi);
    slab_interval(lo, hi, inv, io, &tn, &tf);
    float tfk = tf * kSlabWiden;
    return tn <= th * kSlabWiden && th <= tfk && tn <= tfk;
}
static float centroid(const orc_scene* s, int t, int a) {
    float lo[3], hi[3];
    tri_bounds(s, t, lo, hi);
    return 0.5f * (lo[a] + hi[a]);
}
static const orc_scene* g_sort_scene;
static int g_sort_axis;
static int cmp_cent(const void* A, const void* B) {
    float a = centroid(g_sort_scene, *(const int32_t*)A, g_sort_axis);
    float b = centroid(g_sort_scene, *(const int32_t*)B, g_sort_axis);
    return (a < b) ? -1 : (a > b) ? 1 : 0;
}
static int build_rec(orc_scene* s, int first, int count) {
    int id = s->nnodes++;
    onode* nd = &s->nodes[id];
    for (int a = 0; a < 3; ++a) { nd->lo[a] = INFINITY; nd->hi[a] = -INFINITY; }
    for (int i = first; i < first + count; ++i) {
        float lo[3], hi[3];
        tri_bounds(s, s->order[i], lo, hi);
        for (int a = 0; a < 3; ++a) {
            if (lo[a] < nd->lo[a]) nd->lo[a] = lo[a];
            if (hi[a] > nd->hi[a]) nd->hi[a] = hi[a];
        }
    }
    if (count <= 4) { nd->left = nd->right = -1; nd->first = first; nd->count = count; return id; }
    int axis = 0;
    float best = -1.0f;
    for (int a = 0; a < 3; ++a) if (nd->hi[a] - nd->lo[a] > best) { best = nd->hi[a] - nd->lo[a]; axis = a; }
    g_sort_scene = s;
    g_sort_axis = axis;
    qsort(s->order + first, (size_t)count, sizeof(int32_t), cmp_cent);
    int half = count / 2;
    int l = build_rec(s, first, half);
    int r = build_rec(s, first + half, count - half);
    nd = &s->nodes[id];
    nd->left = l; nd->right = r; nd->first = 0; nd->count = 0;
    return id;
}

orc_scene* orc_scene_create(const orc_mesh* meshes, int32_t n_meshes, const orc_texture* textures,
                            int32_t n_textures) {
    orc_scene* s = (orc_scene*)calloc(1, sizeof(orc_scene));
    int ntri = 0;
    for (int m = 0; m < n_meshes; ++m) ntri += meshes[m].n_triangles;
    s->ntri = ntri;
    s->nmesh = n_meshes;
    s->v = (v3*)malloc(sizeof(v3) * 3 * (size_t)(ntri ? ntri : 1));
    s->n = (v3*)malloc(sizeof(v3) * 3 * (size_t)(ntri ? ntri : 1));
    s->has_n = (int32_t*)malloc(sizeof(int32_t) * (size_t)(n_meshes ? n_meshes : 1));
    s->model = (float*)malloc(sizeof(float) * 16 * (size_t)(n_meshes ? n_meshes : 1));
    s->mesh = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ntri ? ntri : 1));
    s->albedo = (v3*)malloc(sizeof(v3) * (size_t)(n_meshes ? n_meshes : 1));
    s->metallic = (float*)malloc(sizeof(float) * (size_t)(n_meshes ? n_meshes : 1));
    s->roughness = (float*)malloc(sizeof(float) * (size_t)(n_meshes ? n_meshes : 1));
    s->uv = (float*)calloc(6 * (size_t)(ntri ? ntri : 1), sizeof(float));
    s->tex_ids = (int32_t*)malloc(sizeof(int32_t) * 3 * (size_t)(n_meshes ? n_meshes : 1));
    s->ntex = n_textures > 0 ? n_textures : 0;
    s->tex = (orc_texture*)calloc((size_t)(s->ntex ? s->ntex : 1), sizeof(orc_texture));
    s->texpix = (uint32_t**)calloc((size_t)(s->ntex ? s->ntex : 1), sizeof(uint32_t*));
    for (int k = 0; k < s->ntex; ++k) {
        size_t n = (size_t)textures[k].width * (size_t)textures[k].height;
        s->texpix[k] = (uint32_t*)malloc(sizeof(uint32_t) * (n ? n : 1));
        if (n) memcpy(s->texpix[k], textures[k].rgba8, sizeof(uint32_t) * n);
        s->tex[k].rgba8 = s->texpix[k];
        s->tex[k].width = textures[k].width;
        s->tex[k].height = textures[k].height;
    }
    int t = 0;
    for (int m = 0; m < n_meshes; ++m) {
        const orc_mesh* me = &meshes[m];
        memcpy(&s->model[16 * m], me->model, 16 * sizeof(float));
        s->albedo[m] = mk(me->albedo[0], me->albedo[1], me->albedo[2]);
        s->metallic[m] = me->metallic;
        s->roughness[m] = me->roughness;
        s->has_n[m] = me->normals != NULL;
        int at = me->albedo_tex, nt = me->normal_tex, mt = me->metal_rough_tex;
        s->tex_ids[3 * m] = (at >= 0 && at < s->ntex) ? at : -1;
        s->tex_ids[3 * m + 1] = (nt >= 0 && nt < s->ntex) ? nt : -1;
        s->tex_ids[3 * m + 2] = (mt >= 0 && mt < s->ntex) ? mt : -1;
        for (int i = 0; i < me->n_triangles; ++i, ++t) {
            s->mesh[t] = m;
            for (int k = 0; k < 3; ++k) {
                int vi = me->indices[3 * i + k];
                if (me->texcoords) {
                    s->uv[6 * t + 2 * k] = me->texcoords[2 * vi];
                    s->uv[6 * t + 2 * k + 1] = me->texcoords[2 * vi + 1];
                }
                /* GetVertices (devicePrograms.cu:77-81): modelMatrix * vec4(v, 1) */
                float in4[4] = {me->vertices[3 * vi], me->vertices[3 * vi + 1], me->vertices[3 * vi + 2], 1.0f};
                float o4[4];
                mat4_mul_vec4(me->model, in4, o4);
                s->v[3 * t + k] = mk(o4[0], o4[1], o4[2]);
                if (me->normals)
                    s->n[3 * t + k] = mk(me->normals[3 * vi], me->normals[3 * vi + 1], me->normals[3 * vi + 2]);
                else
                    s->n[3 * t + k] = mk(0, 0, 0);
            }
        }
    }
    s->order = (int32_t*)malloc(sizeof(int32_t) * (size_t)(ntri ? ntri : 1));
    for (int i = 0; i < ntri; ++i) s->order[i] = i;
    s->nodes = (onode*)malloc(sizeof(onode) * (size_t)(2 * ntri + 1));
    s->nnodes = 0;
    if (ntri > 0) build_rec(s, 0, ntri);
    return s;
}
void orc_scene_destroy(orc_scene* s) {
    if (!s) return;
    free(s->v); free(s->n); free(s->has_n); free(s->model); free(s->mesh);
    free(s->albedo); free(s->metallic); free(s->roughness); free(s->order); free(s->nodes);
    free(s->uv); free(s->tex_ids);
    for (int k = 0; k < s->ntex; ++k) free(s->texpix[k]);
    free(s->texpix); free(s->tex);
    free(s);
}
int32_t orc_scene_triangles(const orc_scene* s) { return s->ntri; }

/* Moller-Trumbore, OptiX barycentric convention (u -> v1, v -> v2); closed interval. */
static int tri_hit(const orc_scene* s, int t, v3 o, v3 d, float tmin, float tmax, float* th,
                   float* uh, float* vh, int* back) {
    v3 v0 = s->v[3 * t], v1 = s->v[3 * t + 1], v2 = s->v[3 * t + 2];
    v3 e1 = sub(v1, v0), e2 = sub(v2, v0);
    v3 p = cross3(d, e2);
    float det = dot3(e1, p);
    if (det == 0.0f) return 0;
    float inv = 1.0f / det;
    v3 tv = sub(o, v0);
    float u = dot3(tv, p) * inv;
    if (u < 0.0f || u > 1.0f) return 0;
    v3 q = cross3(tv, e1);
    float v = dot3(d, q) * inv;
    if (v < 0.0f || u + v > 1.0f) return 0;
    float tt = dot3(e2, q) * inv;
    if (!(tt >= tmin && tt <= tmax)) return 0;
    *th = tt; *uh = u; *vh = v; *back = det < 0.0f;
    return 1;
}
static int box_hit(const onode* nd, v3 inv, v3 io, float tmin, float tmax) {
    float tn, tf;
    slab_interval(nd->lo, nd->hi, inv, io, &tn, &tf);
    return mx(tn, tmin) <= mn(tf, tmax) * kSlabWiden;
}
static int trace_impl(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, int anyhit, float* th,
                      float* uh, float* vh, int* back, int cull);
/* Cull check (diagnostic): every closest-hit trace is repeated without culling boxes by the
 * current best t (only by [tmin, tmax]), i.e. the exhaustive (t, index) minimum over every
 * triangle whose padded box the ray passes, and disagreements are counted. */
static atomic_int g_cull_check;
static atomic_ullong g_cull_traces, g_cull_mismatch;
static float g_cull_first[16];
static atomic_int g_cull_first_set;
void orc_set_cull_check(int32_t on) {
    atomic_store(&g_cull_check, on);
    atomic_store(&g_cull_traces, 0);
    atomic_store(&g_cull_mismatch, 0);
    atomic_store(&g_cull_first_set, 0);
}
void orc_cull_check_stats(uint64_t out[2], float first[16]) {
    out[0] = atomic_load(&g_cull_traces);
    out[1] = atomic_load(&g_cull_mismatch);
    memcpy(first, g_cull_first, sizeof g_cull_first);
}
static int trace(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, int anyhit, float* th,
                 float* uh, float* vh, int* back) {
    float t0 = 0, u0 = 0, v0 = 0;
    int b0 = 0;
    int r = trace_impl(s, o, d, tmin, tmax, anyhit, &t0, &u0, &v0, &b0, 1);
    if (!anyhit && atomic_load_explicit(&g_cull_check, memory_order_relaxed)) {
        float t1 = 0, u1 = 0, v1 = 0;
        int b1 = 0;
        int r1 = trace_impl(s, o, d, tmin, tmax, 0, &t1, &u1, &v1, &b1, 0);
        atomic_fetch_add(&g_cull_traces, 1);
        if (r1 != r || (r >= 0 && (t1 != t0 || u1 != u0 || v1 != v0))) {
            atomic_fetch_add(&g_cull_mismatch, 1);
            if (atomic_exchange(&g_cull_first_set, 1) == 0) {
                float rec[16] = {o.x, o.y, o.z, d.x, d.y, d.z, tmin, tmax, (float)r, t0, (float)r1, t1,
                                 u0, v0, u1, v1};
                memcpy(g_cull_first, rec, sizeof rec);
            }
        }
    }
    if (r >= 0 && th) { *th = t0; *uh = u0; *vh = v0; *back = b0; }
    return r;
}
ORC_HOT static int trace_impl(const orc_scene* s, v3 o, v3 d, float tmin, float tmax, int anyhit, float* th,
                              float* uh, float* vh, int* back, int cull) {
    if (s->ntri == 0) return -1;
    v3 inv = mk(ray_inv(d.x), ray_inv(d.y), ray_inv(d.z));
    v3 io = mk(o.x * inv.x, o.y * inv.y, o.z * inv.z);
    int stack[128];
    int sp = 0;
    stack[sp++] = 0;
    int best = -1;
    float bt = tmax, bu = 0, bv = 0;
    int bb = 0;
    while (sp) {
        const onode* nd = &s->nodes[stack[--sp]];
        if (!box_hit(nd, inv, io, tmin, cull ? bt : tmax)) continue;
        if (nd->left < 0) {
            for (int i = nd->first; i < nd->first + nd->count; ++i) {
                int t = s->order[i];
                float tt, uu, vv;
                int bk;
                if (!tri_hit(s, t, o, d, tmin, bt, &tt, &uu, &vv, &bk)) continue;
                if (alpha_cut(s, t, uu, vv)) continue;  /* __anyhit__radiance/shadow */
                if (!tri_accept(s, t, inv, io, tt)) continue;
                if (anyhit) return t;
                if (best < 0 || tt < bt || (tt == bt && t < best)) {
                    best = t; bt = tt; bu = uu; bv = vv; bb = bk;
                }
            }
        } else {
            stack[sp++] = nd->left;
            stack[sp++] = nd->right;
        }
    }
    if (best >= 0 && th) { *th = bt; *uh = bu; *vh = bv; *back = bb; }
    return best;
}
int32_t orc_trace_closest(const orc_scene* s, const float o[3], const float d[3], float tmin,
                          float tmax, float* t, float* u, float* v, int32_t* backface) {
    int bk = 0;
    int r = trace(s, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), tmin, tmax, 0, t, u, v, &bk);
    if (backface) *backface = bk;
    return r;
}
int32_t orc_trace_any(const orc_scene* s, const float o[3], const float d[3], float tmin, float tmax) {
    return trace(s, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), tmin, tmax, 1, NULL, NULL, NULL, NULL) >= 0;
}

/* ------------------------------------------------------------------------------------ */
/* The path — SamplePath (devicePrograms.cu:625-664) + __closesthit__radiance (:343-514)  */
/* ------------------------------------------------------------------------------------ */
ORC_HOT static v3 sample_path(const orc_scene* s, const orc_launch* lp, v3 origin, v3 dir, uint32_t seed,
                      int* segs, float* dbg, int dbg_max) {
    v3 radiance = mk(0, 0, 0), beta = mk(1, 1, 1);
    int bounce = 0, endPath = 0;
    v3 o = origin, d = dir;
    while (!endPath && bounce < lp->max_bounces && length3(beta) > 0.00001f) {
        float th, u, v;
        int back;
        int prim = trace(s, o, d, 0.0f, 100.0f, 0, &th, &u, &v, &back);
        (*segs)++;
        if (prim < 0) {  /* __miss__radiance :576-583 */
            beta = mk(0, 0, 0);
            bounce = 100;
            continue;
        }
        bounce++;
        if (bounce > lp->max_bounces) { endPath = 1; continue; }
        int m = s->mesh[prim];
        v3 wo = normalize3(neg(d));
        v3 v0 = s->v[3 * prim], v1 = s->v[3 * prim + 1], v2 = s->v[3 * prim + 2];
        /* GetNormal :83-117 */
        v3 Ng = cross3(sub(v1, v0), sub(v2, v0));
        float w = 1.0f - u - v;
        v3 Ns = mk(0, 0, 0);
        if (s->has_n[m]) {
            v3 n0 = s->n[3 * prim], n1 = s->n[3 * prim + 1], n2 = s->n[3 * prim + 2];
            Ns = mk(w * n0.x + u * n1.x + v * n2.x, w * n0.y + u * n1.y + v * n2.y,
                    w * n0.z + u * n1.z + v * n2.z);
            float in4[4] = {Ns.x, Ns.y, Ns.z, 0.0f}, o4[4];
            mat4_mul_vec4(&s->model[16 * m], in4, o4);
            float d4 = (o4[0] * o4[0] + o4[1] * o4[1]) + (o4[2] * o4[2] + o4[3] * o4[3]);
            float inv = 1.0f / sqrtf(d4);
            Ns = mk(o4[0] * inv, o4[1] * inv, o4[2] * inv);
        }
        if (dot3(wo, Ng) < 0.0f) Ng = neg(Ng);
        Ng = normalize3(Ng);
        if (dot3(Ng, Ns) < 0.0f) Ns = neg(Ns);
        Ns = normalize3(Ns);
        if (back) { Ns = muls(Ns, -1.0f); Ng = muls(Ng, -1.0f); }  /* :379-382 */
        v3 pos = mk(w * v0.x + u * v1.x + v * v2.x, w * v0.y + u * v1.y + v * v2.y,
                    w * v0.z + u * v1.z + v * v2.z);  /* GetSurfacePos :119-129 */
        surf sf;
        sf.albedo = s->albedo[m];
        float metallic = s->metallic[m];
        sf.roughness = s->roughness[m];
        /* SampleTextures :143-166 (each texture by its own id: the reference's
         * hasNormalTexture/hasMetalRoughTexture = HasAlbedoTex() flag bug, OptixRenderer.cpp:535,540,
         * is not reproduced) */
        v3 normalTex = mk(0, 0, 0);
        const int32_t* tid = &s->tex_ids[3 * m];
        if (tid[0] >= 0 || tid[1] >= 0 || tid[2] >= 0) {
            float tx, ty, c[4];
            tri_uv(s, prim, u, v, &tx, &ty);
            if (tid[0] >= 0) {
                orc_tex_sample(&s->tex[tid[0]], tx, ty, 1, c);
                sf.albedo = mulv(sf.albedo, mk(c[0], c[1], c[2]));
            }
            if (tid[1] >= 0) {
                orc_tex_sample(&s->tex[tid[1]], tx, ty, 0, c);
                normalTex = mk(c[0], c[1], c[2]);
            }
            if (tid[2] >= 0) {
                orc_tex_sample(&s->tex[tid[2]], tx, ty, 0, c);
                metallic = c[0];
                sf.roughness = c[1];
            }
        }
        sf.conductor = rnd(&seed) < metallic;  /* :400 */
        if (!iszero3(normalTex)) {  /* normal mapping :403-409 in the a8 frame of Ns */
            v3 d1 = cross3(Ns, mk(0.0f, 0.0f, 1.0f));
            v3 d2 = cross3(Ns, mk(0.0f, 1.0f, 0.0f));
            v3 T0 = (length3(d1) > length3(d2)) ? d1 : d2;
            T0 = normalize3(T0);
            v3 B0 = cross3(T0, Ns);
            v3 tn = mk(normalTex.x * 2.0f - 1.0f, normalTex.y * 2.0f - 1.0f, normalTex.z * 2.0f - 1.0f);
            v3 wn = mk((T0.x * tn.x + B0.x * tn.y) + Ns.x * tn.z, (T0.y * tn.x + B0.y * tn.y) + Ns.y * tn.z,
                       (T0.z * tn.x + B0.z * tn.y) + Ns.z * tn.z);
            Ns = normalize3(wn);
        }
        if (dbg && bounce <= dbg_max) {  /* debug print of devicePrograms.cu:428-437, as data */
            float* r = dbg + (size_t)(bounce - 1) * ORC_DEBUG_FLOATS;
            int32_t ib = bounce, ip = prim;
            memcpy(&r[0], &ib, 4);
            memcpy(&r[1], &ip, 4);
            r[2] = pos.x; r[3] = pos.y; r[4] = pos.z;
            r[5] = sf.albedo.x; r[6] = sf.albedo.y; r[7] = sf.albedo.z;
            r[8] = Ns.x; r[9] = Ns.y; r[10] = Ns.z;
            r[11] = Ng.x; r[12] = Ng.y; r[13] = Ng.z;
            r[14] = sf.roughness; r[15] = metallic;
            r[16] = beta.x; r[17] = beta.y; r[18] = beta.z;
            r[19] = radiance.x; r[20] = radiance.y; r[21] = radiance.z;
        }
        /* GetTBN / BuildTangentSpace :168-212 */
        v3 c1 = cross3(Ns, mk(0.0f, 0.0f, 1.0f));
        v3 c2 = cross3(Ns, mk(0.0f, 1.0f, 0.0f));
        v3 T = (length3(c1) > length3(c2)) ? c1 : c2;
        T = normalize3(T);
        v3 B = cross3(T, Ns);
        v3 N = Ns;
        /* WorldToShading = transpose(mat3(T,B,N)) */
        sf.wo = mk(dot3(T, wo), dot3(B, wo), dot3(N, wo));
        /* NEE :446-472 */
        float P = 0.0f;
        int li = 0;
        if (lp->n_lights == 1) { P = 1.0f; li = 0; }
        else if (lp->n_lights > 1) {  /* LightMethods.h:25-40 */
            float r = rnd(&seed);
            li = (int)(r * (float)lp->n_lights);
            if (li >= lp->n_lights) li = lp->n_lights - 1;
            P = 1.0f / (float)lp->n_lights;
        }
        if (P > 0.0f) {
            const float* L = &lp->lights[6 * li];
            v3 lpos = mk(L[0], L[1], L[2]), lcol = mk(L[3], L[4], L[5]);
            v3 ldir = sub(lpos, pos);  /* LightVisibility :216-241 */
            v3 ldn = normalize3(ldir);
            v3 so = add(pos, smul(1e-3f, Ng));
            int occluded = trace(s, so, normalize3(ldir), 0.0f, length3(ldir), 1, NULL, NULL, NULL, NULL) >= 0;
            v3 lds = mk(dot3(T, ldn), dot3(B, ldn), dot3(N, ldn));
            if (!occluded) {
                v3 f = bsdf_f_mode(lp->material_mode, &seed, &sf, lds);
                float c = absdot(lds, ZAXIS);
                v3 spectrum = muls(f, c);
                if (!iszero3(spectrum)) {
                    v3 dd = sub(pos, lpos);
                    float d2 = dd.x * dd.x + dd.y * dd.y + dd.z * dd.z;
                    v3 Li = divs(lcol, d2);
                    v3 c3 = mulv(mulv(beta, spectrum), Li);
                    radiance = add(radiance, divs(c3, P * 1.0f));
                }
            }
        }
        bsample bs;
        memset(&bs, 0, sizeof bs);
        if (!bsdf_sample_mode(lp->material_mode, &seed, &sf, &bs)) { endPath = 1; continue; }
        float ac = absdot(bs.dir, ZAXIS);
        beta = mulv(beta, mk(bs.color.x * ac / bs.pdf, bs.color.y * ac / bs.pdf, bs.color.z * ac / bs.pdf));
        v3 off = smul(1e-3f, Ng);
        if (dot3(bs.dir, ZAXIS) < 0.0f) off = neg(off);
        o = add(pos, off);
        /* ShadingToWorld * dir = T*x + B*y + N*z */
        v3 wd = mk(T.x * bs.dir.x + B.x * bs.dir.y + N.x * bs.dir.z,
                   T.y * bs.dir.x + B.y * bs.dir.y + N.y * bs.dir.z,
                   T.z * bs.dir.x + B.z * bs.dir.y + N.z * bs.dir.z);
        d = normalize3(wd);
    }
    return radiance;
}

void orc_sample_path(const orc_scene* s, const orc_launch* lp, int32_t x, int32_t y, uint32_t frame,
                     float out_rgb[3], int32_t* segments) {
    float o[3], d[3];
    orc_camera_ray(lp, x, y, o, d);
    uint32_t seed = orc_tea16((uint32_t)(lp->width * y + x), frame);  /* :631 */
    int segs = 0;
    v3 r = sample_path(s, lp, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), seed, &segs, NULL, 0);
    out_rgb[0] = r.x; out_rgb[1] = r.y; out_rgb[2] = r.z;
    if (segments) *segments = segs;
}
int32_t orc_sample_path_debug(const orc_scene* s, const orc_launch* lp, int32_t x, int32_t y, uint32_t frame,
                              float* records, int32_t max_bounces, float out_rgb[3]) {
    float o[3], d[3];
    orc_camera_ray(lp, x, y, o, d);
    uint32_t seed = orc_tea16((uint32_t)(lp->width * y + x), frame);
    int segs = 0;
    memset(records, 0, sizeof(float) * ORC_DEBUG_FLOATS * (size_t)(max_bounces > 0 ? max_bounces : 0));
    v3 r = sample_path(s, lp, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), seed, &segs, records, max_bounces);
    out_rgb[0] = r.x; out_rgb[1] = r.y; out_rgb[2] = r.z;
    int n = 0;
    while (n < max_bounces) {
        int32_t b;
        memcpy(&b, &records[(size_t)n * ORC_DEBUG_FLOATS], 4);
        if (b != n + 1) break;
        ++n;
    }
    return n;
}

typedef struct {
    const orc_scene* s;
    const orc_launch* lp;
    uint32_t f0, nf;
    int x0, y0, x1, y1;
    float* sum;
    atomic_int next_row;
    atomic_ullong segs;
} job;

static void* worker(void* arg) {
    job* J = (job*)arg;
    unsigned long long local = 0;
    for (;;) {
        int y = atomic_fetch_add(&J->next_row, 1);
        if (y >= J->y1) break;
        for (int x = J->x0; x < J->x1; ++x) {
            float o[3], d[3];
            orc_camera_ray(J->lp, x, y, o, d);
            size_t idx = ((size_t)y * (size_t)J->lp->width + (size_t)x) * 3;
            float sx = J->sum[idx], sy = J->sum[idx + 1], sz = J->sum[idx + 2];
            for (uint32_t f = 0; f < J->nf; ++f) {
                uint32_t seed = orc_tea16((uint32_t)(J->lp->width * y + x), J->f0 + f);
                int segs = 0;
                v3 r = sample_path(J->s, J->lp, mk(o[0], o[1], o[2]), mk(d[0], d[1], d[2]), seed, &segs, NULL, 0);
                local += (unsigned long long)segs;
                sx += r.x; sy += r.y; sz += r.z;
            }
            J->sum[idx] = sx; J->sum[idx + 1] = sy; J->sum[idx + 2] = sz;
        }
    }
    atomic_fetch_add(&J->segs, local);
    return NULL;
}

void orc_render(const orc_scene* s, const orc_launch* lp, uint32_t first_frame, uint32_t n_frames,
                int32_t x0, int32_t y0, int32_t x1, int32_t y1, float* sum_rgb, int32_t n_threads,
                uint64_t* segments_out) {
    job J;
    J.s = s; J.lp = lp; J.f0 = first_frame; J.nf = n_frames;
    J.x0 = x0; J.y0 = y0; J.x1 = x1; J.y1 = y1; J.sum = sum_rgb;
    atomic_init(&J.next_row, y0);
    atomic_init(&J.segs, 0ull);
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 256) n_threads = 256;
    pthread_t th[256];
    for (int i = 0; i < n_threads; ++i) pthread_create(&th[i], NULL, worker, &J);
    for (int i = 0; i < n_threads; ++i) pthread_join(th[i], NULL);
    if (segments_out) *segments_out = (uint64_t)atomic_load(&J.segs);
}
