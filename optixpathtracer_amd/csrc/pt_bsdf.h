// pt_bsdf.h — the reference's BSDF models as gfx950 device code.
//
// Behaviour follows Renderer/OptiX/PBRT/{Microfacet,Conductor,LambertDiffuse,Dielectric,
// GlossyDiffuse}.h of Damo12320/OptixPathtracer (line numbers cited per function).  All
// evaluation happens in the shading frame (N = +z).  RNG draws consume the path seed in the
// reference order (SURVEY.md §8(a) "RNG draw order"); the Layered walk's Russian-roulette
// draws use the private TEA stream the reference derives from wo/wi.
#pragma once
#include "pt_math.h"

namespace pt {

constexpr float kInvPi = 0.31830988618379067154f;

struct BSample {
    f3 color;
    float pdf;
    f3 dir;
    bool refl, trans, spec;
};

// ---- sampling primitives ----------------------------------------------------------------
// random.h:76-84 (u0 then u1, left-to-right as in devicePrograms.cu.ptx)
__device__ __forceinline__ void disk_polar(uint32_t& seed, float& px, float& py) {
    const float pi = (float)3.14159265359;
    float u0 = rnd(seed);
    float u1 = rnd(seed);
    float r = fsqrt(u0);
    float theta = 2.0f * pi * u1;
    float st, ct;
    pt_sincosf(theta, st, ct);  // cosf / sinf (pt_math.h: bit-identical to the oracle)
    px = r * ct;
    py = r * st;
}
// LambertDiffuse.h:35-55
__device__ __forceinline__ void disk_concentric(uint32_t& seed, float& dx, float& dy) {
    const float PiOver4 = 0.78539816339744830961f;
    const float PiOver2 = 1.57079632679489661923f;
    float u0 = rnd(seed);
    float u1 = rnd(seed);
    float ox = 2.0f * u0 - 1.0f, oy = 2.0f * u1 - 1.0f;
    if (ox == 0.0f && oy == 0.0f) {
        dx = 0.0f;
        dy = 0.0f;
        return;
    }
    float theta, r;
    if (gabs(ox) > gabs(oy)) {
        r = ox;
        theta = PiOver4 * fdiv(oy, ox);
    } else {
        r = oy;
        theta = PiOver2 - PiOver4 * fdiv(ox, oy);
    }
    float st, ct;
    pt_sincosf(theta, st, ct);
    dx = r * ct;
    dy = r * st;
}

// ---- spherical geometry: SphericalGeometry.h:8-29 ----------------------------------------
__device__ __forceinline__ float cos2_theta(f3 w) { return sqr(w.z); }
__device__ __forceinline__ float abs_cos_theta(f3 w) { return gabs(w.z); }
__device__ __forceinline__ float sin2_theta(f3 w) { return gmax(0.0f, 1.0f - cos2_theta(w)); }
__device__ __forceinline__ float sin_theta(f3 w) { return fsqrt(sin2_theta(w)); }
__device__ __forceinline__ float tan2_theta(f3 w) { return fdiv(sin2_theta(w), cos2_theta(w)); }
__device__ __forceinline__ float cos_phi(f3 w) {
    float s = sin_theta(w);
    return (s == 0.0f) ? 1.0f : gclamp(fdiv(w.x, s), -1.0f, 1.0f);
}
__device__ __forceinline__ float sin_phi(f3 w) {
    float s = sin_theta(w);
    return (s == 0.0f) ? 0.0f : gclamp(fdiv(w.y, s), -1.0f, 1.0f);
}
__device__ __forceinline__ bool same_hemisphere(f3 w, f3 wp) { return w.z * wp.z > 0.0f; }

// ---- Trowbridge-Reitz: Microfacet.h:9-119 ------------------------------------------------
__device__ __forceinline__ float tr_D(f3 wm, float alpha) {
    const float pi = 3.14159265359f;
    float t2 = tan2_theta(wm);
    if (isinf(t2)) return 0.0f;
    float cos4 = sqr(cos2_theta(wm));
    if (cos4 < 1e-16f) return 0.0f;
    float e = t2 * (sqr(fdiv(cos_phi(wm), alpha)) + sqr(fdiv(sin_phi(wm), alpha)));
    return frcp(pi * alpha * alpha * cos4 * sqr(1.0f + e));
}
__device__ __forceinline__ float tr_lambda(f3 w, float alpha) {
    float t2 = tan2_theta(w);
    if (isinf(t2)) return 0.0f;
    float a2 = sqr(cos_phi(w) * alpha) + sqr(sin_phi(w) * alpha);
    return (fsqrt(1.0f + a2 * t2) - 1.0f) / 2.0f;  // / 2: an exact multiply
}
__device__ __forceinline__ float tr_G(f3 wo, f3 wi, float alpha) {
    return frcp(1.0f + tr_lambda(wo, alpha) + tr_lambda(wi, alpha));
}
__device__ __forceinline__ float tr_G1(f3 w, float alpha) { return frcp(1.0f + tr_lambda(w, alpha)); }
__device__ __forceinline__ float tr_pdf(f3 w, f3 wm, float alpha) {   // D(w, wm): :81-88
    return fdiv(tr_G1(w, alpha), abs_cos_theta(w)) * tr_D(wm, alpha) * abs_dot(w, wm);
}
// Trowbridge-Reitz quantities of one direction w that every sample or evaluation with w as
// the outgoing direction recomputes: tr_sample_wm's hemisphere frame, Lambda(w) and
// G1(w) / |cos w|.  The layered walk computes them once per direction and reuses them across
// its samples and depths; they are the same operations on the same inputs, so every result
// stays bit-identical to recomputing them inline.
// PT_TRDIR_LEAN = 1 keeps wh and T1 of the frame and recomputes T2 = cross(wh, T1) where a sample
// uses it (the same operations, so the same bits): three registers fewer per direction the walk
// holds.
#ifndef PT_TRDIR_LEAN
#define PT_TRDIR_LEAN 0  // Dielectric -1.2 %, Layered -0.3 %: not kept
#endif
struct TRDir {
#if PT_TRDIR_LEAN
    f3 wh, T1;      // tr_sample_wm frame (tr_dir_frame); T2 = cross(wh, T1)
#else
    f3 wh, T1, T2;  // tr_sample_wm frame (tr_dir_frame)
#endif
    float lam;      // tr_lambda(w, alpha) (tr_dir_lam)
    float g1c;      // tr_G1(w, alpha) / abs_cos_theta(w) (tr_dir_lam)
};
__device__ __forceinline__ void tr_dir_lam(TRDir& p, f3 w, float alpha) {
    p.lam = tr_lambda(w, alpha);
    p.g1c = fdiv(frcp(1.0f + p.lam), abs_cos_theta(w));
}
__device__ __forceinline__ void tr_dir_frame(TRDir& p, f3 w, float alpha) {  // Microfacet.h:90-98
    f3 wh = normalize(mk(alpha * w.x, alpha * w.y, w.z));
    if (wh.z < 0.0f) wh = -wh;
    p.T1 = (wh.z < 0.99999f) ? normalize(cross(mk(0.0f, 0.0f, 1.0f), wh)) : mk(1.0f, 0.0f, 0.0f);
#if !PT_TRDIR_LEAN
    p.T2 = cross(wh, p.T1);
#endif
    p.wh = wh;
}
__device__ __forceinline__ f3 tr_sample_wm_dir(uint32_t& seed, const TRDir& p, float alpha) {  // :99-119
#if PT_TRDIR_LEAN
    const f3 wh = p.wh, T1 = p.T1, T2 = cross(wh, T1);
#else
    const f3 wh = p.wh, T1 = p.T1, T2 = p.T2;
#endif
    float px, py;
    disk_polar(seed, px, py);
    float h = fsqrt(1.0f - sqr(px));
    float x = (1.0f + wh.z) / 2.0f;
    py = (1.0f - x) * h + x * py;
    float pz = fsqrt(gmax(0.0f, 1.0f - (sqr(px) + sqr(py))));
    f3 nh = mk(px * T1.x + py * T2.x + pz * wh.x, px * T1.y + py * T2.y + pz * wh.y,
               px * T1.z + py * T2.z + pz * wh.z);
    return normalize(mk(alpha * nh.x, alpha * nh.y, gmax(1e-6f, nh.z)));
}
__device__ __forceinline__ f3 tr_sample_wm(uint32_t& seed, f3 w, float alpha) {  // :90-119
    TRDir p;
    tr_dir_frame(p, w, alpha);
    return tr_sample_wm_dir(seed, p, alpha);
}

// ---- Conductor: Conductor.h:42-190, Complex.h:5-63 ---------------------------------------
struct cpx {
    float re, im;
};
__device__ __forceinline__ cpx c_add(cpx a, cpx b) { return cpx{a.re + b.re, a.im + b.im}; }
__device__ __forceinline__ cpx c_sub(cpx a, cpx b) { return cpx{a.re - b.re, a.im - b.im}; }
__device__ __forceinline__ cpx c_mul(cpx a, cpx b) {
    return cpx{a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ cpx c_div(cpx a, cpx z) {
    float scale = frcp(z.re * z.re + z.im * z.im);
    return cpx{scale * (a.re * z.re + a.im * z.im), scale * (a.im * z.re - a.re * z.im)};
}
__device__ __forceinline__ float c_norm(cpx z) { return z.re * z.re + z.im * z.im; }
__device__ __forceinline__ cpx c_sqrt(cpx z) {
    float n = fsqrt(c_norm(z));
    float t1 = fsqrt(0.5f * (n + gabs(z.re)));
    float t2 = fdiv(0.5f * z.im, t1);
    if (n == 0.0f) return cpx{0.0f, 0.0f};
    if (z.re >= 0.0f) return cpx{t1, t2};
    return cpx{gabs(t2), copysignf(t1, z.im)};
}
__device__ __forceinline__ float fr_complex(float cos_i, cpx eta) {  // :42-52
    cos_i = gclamp(cos_i, 0.0f, 1.0f);
    float sin2i = 1.0f - sqr(cos_i);
    cpx sin2t = c_div(cpx{sin2i, 0.0f}, c_mul(eta, eta));
    cpx cost = c_sqrt(c_sub(cpx{1.0f, 0.0f}, sin2t));
    cpx ec = c_mul(eta, cpx{cos_i, 0.0f});
    cpx r_parl = c_div(c_sub(ec, cost), c_add(ec, cost));
    cpx ect = c_mul(eta, cost);
    cpx r_perp = c_div(c_sub(cpx{cos_i, 0.0f}, ect), c_add(cpx{cos_i, 0.0f}, ect));
    return (c_norm(r_parl) + c_norm(r_perp)) / 2.0f;
}
__device__ __forceinline__ float fresnel_complex1(float cos_i, float refl) {  // :54-92, one channel
    float r = gclamp(refl, 0.0f, 0.9999f);
    float om = 1.0f - r;
    om = om > 0.0f ? om : 0.0f;
    float k = fdiv(2.0f * fsqrt(r), fsqrt(om));
    return fr_complex(cos_i, cpx{1.0f, k});
}
__device__ __forceinline__ f3 fresnel_complex(float cos_i, f3 refl) {
    return mk(fresnel_complex1(cos_i, refl.x), fresnel_complex1(cos_i, refl.y),
              fresnel_complex1(cos_i, refl.z));
}
__device__ __forceinline__ f3 conductor_f(f3 albedo, float roughness, f3 wo, f3 wi) {  // :97-120
    float alpha = sqr(roughness);
    if (!same_hemisphere(wo, wi)) return mk(0, 0, 0);
    if (alpha < 1e-3f) return mk(0, 0, 0);
    float co = abs_cos_theta(wo), ci = abs_cos_theta(wi);
    if (ci == 0.0f || co == 0.0f) return mk(0, 0, 0);
    f3 wm = wi + wo;
    if (length_sqr(wm) == 0.0f) return mk(0, 0, 0);
    wm = normalize(wm);
    f3 F = fresnel_complex(abs_dot(wo, wm), albedo);
    float D = tr_D(wm, alpha), G = tr_G(wo, wi, alpha);
    float den = 4.0f * ci * co;
    return mk(fdiv(D * F.x * G, den), fdiv(D * F.y * G, den), fdiv(D * F.z * G, den));
}
__device__ __forceinline__ bool conductor_sample(uint32_t& seed, f3 albedo, float roughness, f3 wo,
                                                 BSample& s) {  // :122-190
    float alpha = sqr(roughness);
    if (alpha < 1e-3f) {
        f3 wi = mk(-wo.x, -wo.y, wo.z);
        float ac = abs_cos_theta(wi);
        s.color = fresnel_complex(ac, albedo) / ac;  // f3 / float: fdiv per channel
        s.dir = wi;
        s.pdf = 1.0f;
        s.refl = true;
        s.trans = false;
        s.spec = true;
        return true;
    }
    if (wo.z == 0.0f) return false;
    f3 wm = tr_sample_wm(seed, wo, alpha);
    float d2 = 2.0f * dot(wo, wm);
    f3 wi = (-wo) + d2 * wm;
    if (!same_hemisphere(wo, wi)) return false;
    float pdf = fdiv(tr_pdf(wo, wm, alpha), 4.0f * abs_dot(wo, wm));
    float co = abs_cos_theta(wo), ci = abs_cos_theta(wi);
    if (ci == 0.0f || co == 0.0f) return false;
    f3 F = fresnel_complex(abs_dot(wo, wm), albedo);
    float D = tr_D(wm, alpha), G = tr_G(wo, wi, alpha);
    float den = 4.0f * ci * co;
    s.color = mk(fdiv(D * F.x * G, den), fdiv(D * F.y * G, den), fdiv(D * F.z * G, den));
    s.dir = wi;
    s.pdf = pdf;
    s.refl = true;
    s.trans = false;
    s.spec = false;
    return true;
}

// ---- Lambert: LambertDiffuse.h:86-140 ------------------------------------------------------
__device__ __forceinline__ f3 lambert_f(f3 albedo, f3 wo, f3 wi) {
    if (!same_hemisphere(wo, wi)) return mk(0, 0, 0);
    return albedo * kInvPi;
}
// z forced >= 0 whatever wo's hemisphere (:115-119)
__device__ __forceinline__ bool lambert_sample(uint32_t& seed, f3 albedo, bool reflection, BSample& s) {
    if (!reflection) return false;
    float dx, dy;
    disk_concentric(seed, dx, dy);
    float z = fsqrt(gmax(0.0f, 1.0f - sqr(dx) - sqr(dy)));
    f3 d = mk(dx, dy, z);
    if (d.z < 0.0f) d.z *= -1.0f;
    d = normalize(d);
    s.dir = d;
    s.pdf = abs_cos_theta(d) * kInvPi;
    s.color = albedo * kInvPi;
    s.refl = true;
    s.trans = false;
    s.spec = false;
    return true;
}
__device__ __forceinline__ float lambert_pdf(f3 wo, f3 wi, bool reflection) {
    if (!reflection || !same_hemisphere(wi, wo)) return 0.0f;
    return abs_cos_theta(wi) * kInvPi;
}

// ---- Dielectric (eta = 1.5): Dielectric.h:20-343 -------------------------------------------
enum { kRadiance = 0, kImportance = 1 };
__device__ __forceinline__ float fresnel_dielectric(float cos_i, float ior) {  // :20-42
    cos_i = gclamp(cos_i, -1.0f, 1.0f);
    if (cos_i < 0.0f) {
        ior = 1.0f / ior;
        cos_i = -cos_i;
    }
    float sin2i = 1.0f - sqr(cos_i);
    float sin2t = fdiv(sin2i, sqr(ior));
    if (sin2t >= 1.0f) return 1.0f;
    float cost = fsqrt(1.0f - sin2t);
    float r_parl = fdiv(ior * cos_i - cost, ior * cos_i + cost);
    float r_perp = fdiv(cos_i - ior * cost, cos_i + ior * cost);
    return (sqr(r_parl) + sqr(r_perp)) / 2.0f;
}
__device__ __forceinline__ bool refract(f3 wi, f3 n, float eta, float& etap, f3& wt) {  // :68-92
    float cos_i = dot(n, wi);
    if (cos_i < 0.0f) {
        eta = 1.0f / eta;
        cos_i = -cos_i;
        n = -n;
    }
    float sin2i = gmax(0.0f, 1.0f - sqr(cos_i));
    float sin2t = fdiv(sin2i, sqr(eta));
    if (sin2t >= 1.0f) return false;
    float cost = fsqrt(1.0f - sin2t);
    float k = fdiv(cos_i, eta) - cost;
    wt = ((-wi) / eta) + k * n;  // f3 / float: fdiv per channel
    etap = eta;
    return true;
}
// glm::faceforward(-normalize(wm), (0,0,1), normalize(wm))
__device__ __forceinline__ f3 faceforward_z(f3 wm) {
    f3 n = normalize(wm);
    return (dot(n, mk(0.0f, 0.0f, 1.0f)) < 0.0f) ? -n : n;
}
__device__ __forceinline__ float dielectric_f(float roughness, f3 wo, f3 wi, int mode) {  // :96-139
    const float eta = 1.5f;
    float alpha = sqr(roughness);
    if (alpha < 1e-3f) return 0.0f;
    float co = wo.z, ci = wi.z;
    bool reflect = ci * co > 0.0f;
    float etap = 1.0f;
    if (!reflect) etap = co > 0.0f ? eta : (1.0f / eta);
    f3 wm = wi * etap + wo;
    if (ci == 0.0f || co == 0.0f || sqr(length(wm)) == 0.0f) return 0.0f;
    wm = faceforward_z(wm);
    if (dot(wm, wi) * ci < 0.0f || dot(wm, wo) * co < 0.0f) return 0.0f;
    float F = fresnel_dielectric(dot(wo, wm), eta);
    if (reflect) return fdiv(tr_D(wm, alpha) * tr_G(wo, wi, alpha) * F, fabsf(4.0f * ci * co));
    float denom = sqr(dot(wi, wm) + fdiv(dot(wo, wm), etap)) * ci * co;
    float ft = tr_D(wm, alpha) * (1.0f - F) * tr_G(wo, wi, alpha) * fabsf(fdiv(dot(wi, wm) * dot(wo, wm), denom));
    if (mode == kRadiance) ft = fdiv(ft, sqr(etap));
    return ft;
}
// Dielectric.h:146-288 with the wo-only Trowbridge-Reitz terms taken from `p` (a full TRDir of
// wo when the surface is rough; unused when smooth).
__device__ __forceinline__ bool dielectric_sample_dir(uint32_t& seed, float roughness, f3 wo, const TRDir& p,
                                                      BSample& s, int mode, bool reflection, bool transmission) {
    const float eta = 1.5f;
    float alpha = sqr(roughness);
    float uc = rnd(seed);  // drawn first, always (:149)
    if (alpha < 1e-3f) {
        float R = fresnel_dielectric(wo.z, eta);
        float T = 1.0f - R;
        float pr = R, pt = T;
        if (!reflection) pr = 0.0f;
        if (!transmission) pt = 0.0f;
        if (pr == 0.0f && pt == 0.0f) return false;
        if (uc < fdiv(pr, pr + pt)) {
            f3 wi = mk(-wo.x, -wo.y, wo.z);
            float fr = fdiv(R, abs_cos_theta(wi));
            s.color = mk(fr, fr, fr);
            s.dir = wi;
            s.pdf = fdiv(pr, pr + pt);
            s.refl = true;
            s.trans = false;
            s.spec = true;
            return true;
        }
        f3 wi;
        float etap;
        if (!refract(wo, mk(0.0f, 0.0f, 1.0f), eta, etap, wi)) return false;
        float ft = fdiv(T, abs_cos_theta(wi));
        if (mode == kRadiance) ft = fdiv(ft, sqr(etap));
        s.color = mk(ft, ft, ft);
        s.dir = wi;
        s.pdf = fdiv(pt, pr + pt);
        s.refl = false;
        s.trans = true;
        s.spec = true;
        return true;
    }
    f3 wm = tr_sample_wm_dir(seed, p, alpha);
    float R = fresnel_dielectric(dot(wo, wm), eta);
    float T = 1.0f - R;
    float pr = R, pt = T;
    if (!reflection) pr = 0.0f;
    if (!transmission) pt = 0.0f;
    if (pr == 0.0f && pt == 0.0f) return false;
    // The reflection and transmission branches (:162-236) run in the same wave whenever its
    // lanes draw different lobes (nearly always: R is a few percent).  Both branches evaluate
    // D(wm) and Lambda(wi) and end in the same divisions, so they are computed once here, on the
    // lane's own wi and with each division's operands selected per lobe: every value is the one
    // its branch computes, with one copy of the expensive terms instead of two.
    const bool refl = uc < fdiv(pr, pr + pt);
    const f3 I = -wo;  // glm::reflect(I, N) = I - N*dot(N,I)*2
    const float dr = dot(wm, I);
    const f3 wr = mk(I.x - wm.x * dr * 2.0f, I.y - wm.y * dr * 2.0f, I.z - wm.z * dr * 2.0f);
    float etap_t = 1.0f;
    f3 wt = mk(0, 0, 0);
    const bool tir = !refract(wo, wm, eta, etap_t, wt);
    const f3 wi = refl ? wr : wt;
    if (refl ? !same_hemisphere(wo, wi) : (tir || same_hemisphere(wo, wi) || wi.z == 0.0f)) return false;
    const float etap = refl ? 1.0f : etap_t;
    const float D = tr_D(wm, alpha);
    const float G = frcp(1.0f + p.lam + tr_lambda(wi, alpha));
    const float adw = abs_dot(wo, wm);
    const float A = p.g1c * D * adw;
    const float denom = sqr(dot(wi, wm) + fdiv(dot(wo, wm), etap));            // transmission only
    const float q1 = fdiv(refl ? A : abs_dot(wi, wm), refl ? 4.0f * adw : denom);  // A/(4|wo.wm|) | dwm_dwi
    const float pdf = fdiv(refl ? q1 * pr : A * q1 * pt, pr + pt);
    const float q2 = fdiv(refl ? D * G * R : dot(wi, wm) * dot(wo, wm), refl ? 4.0f * wi.z * wo.z : wi.z * wo.z * denom);
    float f = refl ? q2 : T * D * G * fabsf(q2);
    const float fd = fdiv(f, sqr(etap));
    if (!refl && mode == kRadiance) f = fd;
    s.color = mk(f, f, f);
    s.dir = wi;
    s.pdf = pdf;
    s.refl = refl;
    s.trans = !refl;
    s.spec = false;
    return true;
}
__device__ __forceinline__ bool dielectric_sample(uint32_t& seed, float roughness, f3 wo, BSample& s,
                                                  int mode, bool reflection, bool transmission) {
    TRDir p{};
    const float alpha = sqr(roughness);
    if (!(alpha < 1e-3f)) {
        tr_dir_frame(p, wo, alpha);
        tr_dir_lam(p, wo, alpha);
    }
    return dielectric_sample_dir(seed, roughness, wo, p, s, mode, reflection, transmission);
}
__device__ __forceinline__ float dielectric_pdf(float roughness, f3 wo, f3 wi, bool reflection,
                                                bool transmission) {  // :290-343
    const float eta = 1.5f;
    float alpha = sqr(roughness);
    if (alpha < 1e-3f) return 0.0f;
    float co = wo.z, ci = wi.z;
    bool reflect = ci * co > 0.0f;
    float etap = 1.0f;
    if (!reflect) etap = co > 0.0f ? eta : (1.0f / eta);
    f3 wm = wi * etap + wo;
    if (ci == 0.0f || co == 0.0f || length_sqr(wm) == 0.0f) return 0.0f;
    wm = faceforward_z(wm);
    if (dot(wm, wi) * ci < 0.0f || dot(wm, wo) * co < 0.0f) return 0.0f;
    float R = fresnel_dielectric(dot(wo, wm), eta);
    float T = 1.0f - R;
    float pr = R, pt = T;
    if (!reflection) pr = 0.0f;
    if (!transmission) pt = 0.0f;
    if (pr == 0.0f && pt == 0.0f) return 0.0f;
    if (reflect) return fdiv(fdiv(tr_pdf(wo, wm, alpha), 4.0f * abs_dot(wo, wm)) * pr, pr + pt);
    float denom = sqr(dot(wi, wm) + fdiv(dot(wo, wm), etap));
    float dwm_dwi = fdiv(abs_dot(wi, wm), denom);
    return fdiv(tr_pdf(wo, wm, alpha) * dwm_dwi * pt, pr + pt);
}

// dielectric_f and dielectric_pdf at the same (wo, wi) in one pass: the half vector, the
// Fresnel term, D(wm) and the two Smith lambdas are computed once.  Each output keeps the
// arithmetic of its own function (tr_G = 1 / ((1 + L(wo)) + L(wi)), tr_pdf = G1(wo) / |cos wo|
// * D * |wo.wm|), so both are bit-identical to the separate calls; the layered walk evaluates
// f and pdf of one interface together at every NEE step (GlossyDiffuse.h:318-329, :342-352).
// `po` holds lam / g1c of wo (tr_dir_lam), `lam_i` = tr_lambda(wi, alpha).
__device__ __forceinline__ void dielectric_f_pdf_dir(float roughness, f3 wo, const TRDir& po, f3 wi, float lam_i,
                                                     int mode, bool reflection, bool transmission, float& f,
                                                     float& pdf) {
    const float eta = 1.5f;
    f = 0.0f;
    pdf = 0.0f;
    float alpha = sqr(roughness);
    if (alpha < 1e-3f) return;
    float co = wo.z, ci = wi.z;
    bool reflect = ci * co > 0.0f;
    float etap = 1.0f;
    if (!reflect) etap = co > 0.0f ? eta : (1.0f / eta);
    f3 wm = wi * etap + wo;
    if (ci == 0.0f || co == 0.0f) return;
    const bool f_ok = sqr(length(wm)) != 0.0f;  // dielectric_f's test
    const bool p_ok = length_sqr(wm) != 0.0f;   // dielectric_pdf's test
    if (!f_ok && !p_ok) return;
    wm = faceforward_z(wm);
    if (dot(wm, wi) * ci < 0.0f || dot(wm, wo) * co < 0.0f) return;
    const float F = fresnel_dielectric(dot(wo, wm), eta);
    const float D = tr_D(wm, alpha);
    const float G = frcp(1.0f + po.lam + lam_i);
    const float tp = po.g1c * D * abs_dot(wo, wm);
    float fv, pv;
    // reflection and transmission in one sequence (lanes of a wave disagree on `reflect`): each
    // division takes its lobe's operands, so every value equals its branch's below
    const float R = F, T = 1.0f - R;
    float pr = R, pt = T;
    if (!reflection) pr = 0.0f;
    if (!transmission) pt = 0.0f;
    const float s2 = sqr(dot(wi, wm) + fdiv(dot(wo, wm), etap));  // transmission only
    const float qf = fdiv(reflect ? D * G * F : dot(wi, wm) * dot(wo, wm), reflect ? fabsf(4.0f * ci * co) : s2 * ci * co);
    fv = reflect ? qf : D * (1.0f - F) * G * fabsf(qf);
    const float fd = fdiv(fv, sqr(etap));
    if (!reflect && mode == kRadiance) fv = fd;
    const float qp = fdiv(reflect ? tp : abs_dot(wi, wm), reflect ? 4.0f * abs_dot(wo, wm) : s2);
    pv = fdiv(reflect ? qp * pr : tp * qp * pt, pr + pt);
    if (pr == 0.0f && pt == 0.0f) pv = 0.0f;
    f = f_ok ? fv : 0.0f;
    pdf = p_ok ? pv : 0.0f;
}
__device__ __forceinline__ void dielectric_f_pdf(float roughness, f3 wo, f3 wi, int mode, bool reflection,
                                                 bool transmission, float& f, float& pdf) {
    TRDir po;
    const float alpha = sqr(roughness);
    tr_dir_lam(po, wo, alpha);
    dielectric_f_pdf_dir(roughness, wo, po, wi, tr_lambda(wi, alpha), mode, reflection, transmission, f, pdf);
}

// ---- Layered "GlossyDiffuse" (dielectric top, Lambert bottom): GlossyDiffuse.h:91-524 ------
__device__ __forceinline__ float power_heuristic(float fpdf, float gpdf) {  // :91-95 (nf=ng=1)
    float f = 1.0f * fpdf, g = 1.0f * gpdf;
    return fdiv(sqr(f), sqr(f) + sqr(g));
}
__device__ __forceinline__ float transmittance(float dz, f3 w) {  // :97-105
    if (gabs(dz) <= 1.17549435e-38f) return 1.0f;
    return pt_expf_neg(-gabs(fdiv(dz, w.z)));  // expf (pt_math.h)
}
__device__ __forceinline__ f3 layer_f(bool top, f3 albedo, float roughness, f3 wo, f3 wi, int mode) {
    if (top) {
        float v = dielectric_f(roughness, wo, wi, mode);
        return mk(v, v, v);
    }
    return lambert_f(albedo, wo, wi);
}
__device__ __forceinline__ bool layer_sample(bool top, uint32_t& seed, f3 albedo, float roughness, f3 wo,
                                             BSample& s, int mode, bool refl, bool trans) {
    if (top) return dielectric_sample(seed, roughness, wo, s, mode, refl, trans);
    return lambert_sample(seed, albedo, refl, s);
}
__device__ __forceinline__ float layer_pdf(bool top, float roughness, f3 wo, f3 wi, bool refl, bool trans) {
    return top ? dielectric_pdf(roughness, wo, wi, refl, trans) : lambert_pdf(wo, wi, refl);
}
// layer_f and layer_pdf of one interface at the same directions
__device__ __forceinline__ void layer_f_pdf(bool top, f3 albedo, float roughness, f3 wo, f3 wi, int mode, bool refl,
                                            bool trans, f3& f, float& pdf) {
    if (top) {
        float v;
        dielectric_f_pdf(roughness, wo, wi, mode, refl, trans, v, pdf);
        f = mk(v, v, v);
    } else {
        f = lambert_f(albedo, wo, wi);
        pdf = lambert_pdf(wo, wi, refl);
    }
}
__device__ __forceinline__ bool bs_bad(bool ok, const BSample& b) {
    return !ok || is_zero(b.color) || b.pdf == 0.0f || b.dir.z == 0.0f;
}
__device__ __forceinline__ f3 bs_weight(const BSample& b) {  // color * |cos| / pdf
    float c = abs_cos_theta(b.dir);
    return mk(fdiv(b.color.x * c, b.pdf), fdiv(b.color.y * c, b.pdf), fdiv(b.color.z * c, b.pdf));
}

// PT_LAYERED_F_INLINE / PT_LAYERED_SAMPLE_INLINE = 1 inline the layered eval / sample walk into
// their kernels (default; 0 = one call each)
#ifndef PT_LAYERED_F_INLINE
#define PT_LAYERED_F_INLINE 1  // with PT_LAYERED_SAMPLE_INLINE: Default +1.5 %, Sponza-class +1.2 %
#endif
#ifndef PT_LAYERED_SAMPLE_INLINE
#define PT_LAYERED_SAMPLE_INLINE 1
#endif
#if PT_LAYERED_F_INLINE
#define PT_LAYERED_FN_F __device__ __forceinline__
#else
#define PT_LAYERED_FN_F __device__ __noinline__
#endif
#if PT_LAYERED_SAMPLE_INLINE
#define PT_LAYERED_FN_S __device__ __forceinline__
#else
#define PT_LAYERED_FN_S __device__ __noinline__
#endif
// EXITK = 1: the caller guarantees same_hemisphere(wo, wi) (the light on the viewer's side of the
// shading plane, nearly every NEE item), so the exit interface is the top one and the walk
// alternates bottom (even depths) and top (odd depths) at compile time; EXITK = 0 decides at run
// time.  Both run the same operations on the same values as GlossyDiffuse::f.
// TOPK = 1 / 2: the caller guarantees a rough / smooth (alpha < 1e-3) top interface for every lane
// of the wave (the bucketed NEE queue groups them), so the other kind's code is compiled out.
template <int EXITK, int TOPK = 0>
PT_LAYERED_FN_F f3 layered_f_t(uint32_t& seed, f3 albedo, float roughness, f3 wo, f3 wi) {
    // GlossyDiffuse.h:141-367 (mediaAlbedo = 0: the medium branch :269-312 is dead code).
    // The top interface is the rough or smooth dielectric, the bottom the Lambertian.  Terms
    // that depend on one direction only are computed once per direction (TRDir): wo and wi
    // for the whole walk, -w from the exit NEE term of one depth for the sample of the next
    // (same direction), so every value is the one the inline calls would produce.
    const int mode = kRadiance;
    const float thickness = 0.01f;
    const float alpha = sqr(roughness);
    const bool topSpec = TOPK == 1 ? false : TOPK == 2 ? true : alpha < 1e-3f;
    // the dielectric helpers test alpha < 1e-3 themselves: the known answer folds their branches
    if (TOPK == 1) __builtin_assume(!(alpha < 1e-3f));
    if (TOPK == 2) __builtin_assume(alpha < 1e-3f);
    const bool botSpec = false;
    f3 f = mk(0, 0, 0);
    if (wo.z < 0.0f) {
        wo = -wo;
        wi = -wi;
    }
    const bool enteredTop = true;
    const bool same = EXITK == 1 ? true : same_hemisphere(wo, wi);
    bool exitTop, nonExitTop, exitSpec, nonExitSpec;
    if (same ^ enteredTop) {
        exitSpec = botSpec; nonExitSpec = topSpec; exitTop = false; nonExitTop = true;
    } else {
        exitSpec = topSpec; nonExitSpec = botSpec; exitTop = true; nonExitTop = false;
    }
    TRDir pwo{}, pwi{};
    if (!topSpec) {
        tr_dir_frame(pwo, wo, alpha);
        tr_dir_lam(pwo, wo, alpha);
        if (exitTop) {
            tr_dir_frame(pwi, wi, alpha);
            tr_dir_lam(pwi, wi, alpha);
        }
    }
    if (same) {  // layer_f(enteredTop = top, wo, wi)
        float v, unused;
        dielectric_f_pdf_dir(roughness, wo, pwo, wi, pwi.lam, mode, true, true, v, unused);
        f = mk(5.0f, 5.0f, 5.0f) * mk(v, v, v);
    }

    uint32_t ns = tea16(f2u_sat(wo.x * 1000.0f), f2u_sat(wo.y * 1000.0f));
    ns = tea16(ns, f2u_sat(wi.x * 1000.0f));
    ns = tea16(ns, f2u_sat(wi.y * 1000.0f));
    ns = tea16(ns, seed);

    for (int s = 0; s < 5; ++s) {
        BSample wos, wis, bs;
        bool ok = dielectric_sample_dir(seed, roughness, wo, pwo, wos, mode, false, true);  // enteredTop
        if (bs_bad(ok, wos)) continue;
        ok = exitTop ? dielectric_sample_dir(seed, roughness, wi, pwi, wis, kImportance, false, true)
                     : lambert_sample(seed, albedo, false, wis);
        if (bs_bad(ok, wis)) continue;
        f3 beta = bs_weight(wos);
        f3 w = wos.dir;
        const float tr_wis = transmittance(thickness, wis.dir);
        float tr_w = transmittance(thickness, w);
        // NEE through the top as the non-exit interface (wi below the surface)
        const float lam_nwis = (nonExitTop && !topSpec) ? tr_lambda(-wis.dir, alpha) : 0.0f;
        TRDir cw{};  // lam / g1c (and, for a top sample, the frame) of -w
        bool cw_ok = false;
// PT_LAYERED_UNROLL 2 (round 6): the depth loop unrolled by two, so the compile-time walk of
// layered_f_split (bottom at even depths, top at odd ones) needs no per-depth interface select.
// Interleaved A/B against round 5 (profiles/r06e_ab_spec_*.log): config 3 +2.3 %, Layered +2.4 %,
// Sponza-class +1.3 %; the walk alone unrolled +1.6 / +1.5 %; the top interface's kind
// specialised as well (PT_LAYERED_SPLIT 2) +2.5 / +3.1 / 0.0 %
#ifndef PT_LAYERED_UNROLL
#define PT_LAYERED_UNROLL 2
#endif
#if PT_LAYERED_UNROLL > 1
#pragma unroll PT_LAYERED_UNROLL
#endif
        for (int depth = 0; depth < 10; ++depth) {
            if (depth > 3 && save_max(beta) < 0.25f) {
                float q = gmax(0.0f, 1.0f - save_max(beta));
                if (rnd(ns) < q) break;
                beta = beta / (1.0f - q);  // f3 / float: fdiv per channel
            }
            beta = beta * tr_w;
            // The reference branches on z == exitZ (GlossyDiffuse.h:315-360); lanes of a wave
            // disagree on exitZ, so both branches would run every depth.  Here the two
            // layer_sample calls are one call on the selected layer, with the NEE terms of the
            // non-exit branch predicated around it: the same operations and random numbers.
            // (Flattening the sample and depth loops into one loop of steps, so lanes start
            // their next sample early, was 40 % slower: DESIGN.md §5.)
            // z starts at the top (enteredTop) and flips every depth, so it is 0 at even depths
            // and `thickness` at odd ones; exitZ is `thickness` when wo and wi share a hemisphere
            // (the top exits) and 0 otherwise: z == exitZ is a parity test.
            const bool atExit = same ? (depth & 1) != 0 : (depth & 1) == 0;
            const bool itop = atExit ? exitTop : nonExitTop;
            if (itop && !topSpec && !cw_ok) {
                tr_dir_lam(cw, -w, alpha);
                cw_ok = true;
            }
            if (!atExit && !nonExitSpec) {
                float wt = 1.0f;
                f3 lf;
                float lpdf;
                if (nonExitTop) {
                    float v;
                    dielectric_f_pdf_dir(roughness, -w, cw, -wis.dir, lam_nwis, mode, true, true, v, lpdf);
                    lf = mk(v, v, v);
                } else {
                    lf = lambert_f(albedo, -w, -wis.dir);
                    lpdf = lambert_pdf(-w, -wis.dir, true);
                }
                if (!exitSpec) wt = power_heuristic(wis.pdf, lpdf);
                float ac = abs_cos_theta(wis.dir);
                f3 t1 = beta * lf;
                t1 = t1 * ac;
                t1 = t1 * wt;
                t1 = t1 * tr_wis;
                t1 = t1 * wis.color;
                t1 = t1 / wis.pdf;  // f3 / float: fdiv per channel
                f = f + t1;
            }
            if (itop) {
                if (!topSpec) tr_dir_frame(cw, -w, alpha);
                ok = dielectric_sample_dir(seed, roughness, -w, cw, bs, mode, true, false);
            } else {
                ok = lambert_sample(seed, albedo, true, bs);
            }
            if (bs_bad(ok, bs)) break;
            beta = beta * bs_weight(bs);
            w = bs.dir;
            cw_ok = false;
            tr_w = transmittance(thickness, w);  // this NEE term's and the next depth's factor
            if (!atExit && !exitSpec) {
                f3 fExit;
                float epdf;
                if (exitTop) {
                    tr_dir_lam(cw, -w, alpha);  // reused by the next depth's top sample
                    cw_ok = true;
                    float v;
                    dielectric_f_pdf_dir(roughness, -w, cw, wi, pwi.lam, mode, false, true, v, epdf);
                    fExit = mk(v, v, v);
                } else {
                    fExit = lambert_f(albedo, -w, wi);
                    epdf = lambert_pdf(-w, wi, false);
                }
                if (!is_zero(fExit)) {
                    float wt = 1.0f;
                    if (!nonExitSpec) wt = power_heuristic(bs.pdf, epdf);
                    f3 t1 = beta * tr_w;
                    t1 = t1 * fExit;
                    t1 = t1 * wt;
                    f = f + t1;
                }
            }
        }
    }
    return mk(fdiv(f.x, 5.0f), fdiv(f.y, 5.0f), fdiv(f.z, 5.0f));
}
__device__ __forceinline__ f3 layered_f(uint32_t& seed, f3 albedo, float roughness, f3 wo, f3 wi) {
    return layered_f_t<0>(seed, albedo, roughness, wo, wi);
}
// The NEE kernel's entry (PT_LAYERED_SPLIT): a wave whose lanes all have the light on the viewer's
// side takes the compile-time walk, any other wave the run-time one (same_hemisphere is invariant
// under the walk's flip of both directions).
#ifndef PT_LAYERED_SPLIT
#define PT_LAYERED_SPLIT 3
#endif
__device__ __forceinline__ f3 layered_f_split(uint32_t& seed, f3 albedo, float roughness, f3 wo, f3 wi) {
    if (PT_LAYERED_SPLIT >= 4) {  // as 3, a wave with both top kinds runs both compiled walks, masked
        if (__builtin_amdgcn_ballot_w64(!same_hemisphere(wo, wi)) == 0) {
            if (sqr(roughness) < 1e-3f) return layered_f_t<1, 2>(seed, albedo, roughness, wo, wi);
            return layered_f_t<1, 1>(seed, albedo, roughness, wo, wi);
        }
        return layered_f_t<0>(seed, albedo, roughness, wo, wi);
    }
    if (PT_LAYERED_SPLIT >= 3) {  // two specialised walks and the run-time one: no third copy
        if (__builtin_amdgcn_ballot_w64(!same_hemisphere(wo, wi)) == 0) {
            const bool spec = sqr(roughness) < 1e-3f;
            if (__builtin_amdgcn_ballot_w64(spec) == 0) return layered_f_t<1, 1>(seed, albedo, roughness, wo, wi);
            if (__builtin_amdgcn_ballot_w64(!spec) == 0) return layered_f_t<1, 2>(seed, albedo, roughness, wo, wi);
        }
        return layered_f_t<0>(seed, albedo, roughness, wo, wi);
    }
    if (PT_LAYERED_SPLIT && __builtin_amdgcn_ballot_w64(!same_hemisphere(wo, wi)) == 0) {
        if (PT_LAYERED_SPLIT >= 2) {  // the top interface's kind, wave-uniform in all but a bucket's last wave
            const bool spec = sqr(roughness) < 1e-3f;
            if (__builtin_amdgcn_ballot_w64(spec) == 0) return layered_f_t<1, 1>(seed, albedo, roughness, wo, wi);
            if (__builtin_amdgcn_ballot_w64(!spec) == 0) return layered_f_t<1, 2>(seed, albedo, roughness, wo, wi);
        }
        return layered_f_t<1>(seed, albedo, roughness, wo, wi);
    }
    return layered_f_t<0>(seed, albedo, roughness, wo, wi);
}

// TOPK = 1 / 2: the caller guarantees a rough / smooth top interface for every lane of the wave
// (layered_sample_split), so the dielectric helpers' alpha tests fold
template <int TOPK = 0>
PT_LAYERED_FN_S bool layered_sample_t(uint32_t& seed, f3 albedo, float roughness, f3 wo, BSample& out) {
    // GlossyDiffuse.h:372-524
    const float alpha = sqr(roughness);
    if (TOPK == 1) __builtin_assume(!(alpha < 1e-3f));
    if (TOPK == 2) __builtin_assume(alpha < 1e-3f);
    const int mode = kRadiance;
    const float thickness = 0.01f;
    bool flipWi = false;
    if (wo.z < 0.0f) {
        wo = -wo;
        flipWi = true;
    }
    BSample bs;
    bool ok = layer_sample(true, seed, albedo, roughness, wo, bs, mode, true, true);
    if (bs_bad(ok, bs)) return false;
    if (bs.refl) {
        if (flipWi) bs.dir = -bs.dir;
        out = bs;
        return true;
    }
    f3 w = bs.dir;
    bool specPath = bs.spec;
    uint32_t ns = tea16(f2u_sat(wo.x * 1000.0f), f2u_sat(wo.y * 1000.0f));
    ns = tea16(ns, seed);
    f3 f = bs.color * abs_cos_theta(bs.dir);
    float pdf = bs.pdf;
    // z starts at the top and flips every depth (GlossyDiffuse.h:441-447): the bottom at even
    // depths, the top at odd ones, so the interface is a parity test and, with the loop unrolled
    // by two (PT_LAYERED_SAMPLE_UNROLL), known at compile time in each copy
// (unrolled by two since round 6: Layered +0.6 %, config 3 +0.5 %, Sponza-class -0.1 %,
// profiles/r06_ab/r06m_ab_smp_*.log)
#ifndef PT_LAYERED_SAMPLE_UNROLL
#define PT_LAYERED_SAMPLE_UNROLL 2
#endif
#if PT_LAYERED_SAMPLE_UNROLL > 1
#pragma unroll PT_LAYERED_SAMPLE_UNROLL
#endif
    for (int depth = 0; depth < 10; ++depth) {
        float rrBeta = fdiv(save_max(f), pdf);
        if (depth > 3 && rrBeta < 0.25f) {
            float q = gmax(0.0f, 1.0f - rrBeta);
            if (rnd(ns) < q) return false;
            pdf *= 1.0f - q;
        }
        if (w.z == 0.0f) return false;
        f = f * transmittance(thickness, w);
        const bool itop = (depth & 1) != 0;
        ok = layer_sample(itop, seed, albedo, roughness, -w, bs, mode, true, true);
        if (bs_bad(ok, bs)) return false;
        f = f * bs.color;
        pdf *= bs.pdf;
        specPath = specPath && bs.spec;
        w = bs.dir;
        if (bs.trans) {
            if (flipWi) w = -w;
            out.color = f;
            out.dir = w;
            out.pdf = pdf;
            out.refl = same_hemisphere(wo, w);
            out.trans = !out.refl;
            out.spec = specPath;
            return true;
        }
        f = f * abs_cos_theta(bs.dir);
    }
    return false;
}
__device__ __forceinline__ bool layered_sample(uint32_t& seed, f3 albedo, float roughness, f3 wo, BSample& out) {
    return layered_sample_t<0>(seed, albedo, roughness, wo, out);
}
// The sample kernel's entry (PT_LAYERED_SAMPLE_SPLIT): a wave whose lanes share the top
// interface's kind (all but a bucket's last wave) takes that kind's compiled walk
#ifndef PT_LAYERED_SAMPLE_SPLIT
#define PT_LAYERED_SAMPLE_SPLIT 0
#endif
__device__ __forceinline__ bool layered_sample_split(uint32_t& seed, f3 albedo, float roughness, f3 wo, BSample& out) {
    if (PT_LAYERED_SAMPLE_SPLIT >= 2) {  // the two compiled walks only: a mixed wave runs both, masked
        if (sqr(roughness) < 1e-3f) return layered_sample_t<2>(seed, albedo, roughness, wo, out);
        return layered_sample_t<1>(seed, albedo, roughness, wo, out);
    }
    if (PT_LAYERED_SAMPLE_SPLIT) {
        const bool spec = sqr(roughness) < 1e-3f;
        if (__builtin_amdgcn_ballot_w64(spec) == 0) return layered_sample_t<1>(seed, albedo, roughness, wo, out);
        if (__builtin_amdgcn_ballot_w64(!spec) == 0) return layered_sample_t<2>(seed, albedo, roughness, wo, out);
    }
    return layered_sample_t<0>(seed, albedo, roughness, wo, out);
}

// ---- material dispatch: devicePrograms.cu:303-341 (+ commented alternatives) ---------------
enum MaterialMode { kModeDefault = 0, kModeLambert = 1, kModeConductor = 2, kModeDielectric = 3, kModeLayered = 4 };

// SPLIT: the layered sample through layered_sample_split (the bucketed sample kernel)
template <int MODE, bool SPLIT = false>
__device__ __forceinline__ bool bsdf_sample(uint32_t& seed, f3 albedo, float roughness, bool conductor, f3 wo,
                                            BSample& bs) {
    if (MODE == kModeLambert) return lambert_sample(seed, albedo, true, bs);
    if (MODE == kModeConductor) return conductor_sample(seed, albedo, roughness, wo, bs);
    if (MODE == kModeDielectric) return dielectric_sample(seed, roughness, wo, bs, kRadiance, true, true);
    if (MODE == kModeLayered)
        return SPLIT ? layered_sample_split(seed, albedo, roughness, wo, bs) : layered_sample(seed, albedo, roughness, wo, bs);
    if (conductor) return conductor_sample(seed, albedo, roughness, wo, bs);
    return SPLIT ? layered_sample_split(seed, albedo, roughness, wo, bs) : layered_sample(seed, albedo, roughness, wo, bs);
}
// SPLIT: the layered eval through layered_f_split (the bucketed NEE kernel)
template <int MODE, bool SPLIT = false>
__device__ __forceinline__ f3 bsdf_f(uint32_t& seed, f3 albedo, float roughness, bool conductor, f3 wo, f3 wi) {
    if (MODE == kModeLambert) return lambert_f(albedo, wo, wi);
    if (MODE == kModeConductor) return conductor_f(albedo, roughness, wo, wi);
    if (MODE == kModeDielectric) {
        float v = dielectric_f(roughness, wo, wi, kRadiance);
        return mk(v, v, v);
    }
    if (MODE == kModeLayered)
        return SPLIT ? layered_f_split(seed, albedo, roughness, wo, wi) : layered_f(seed, albedo, roughness, wo, wi);
    if (conductor) return conductor_f(albedo, roughness, wo, wi);
    return SPLIT ? layered_f_split(seed, albedo, roughness, wo, wi) : layered_f(seed, albedo, roughness, wo, wi);
}

}  // namespace pt
