// pt_device.h — HBM layout of the scene, LBVH traversal and the path integrator for gfx950.
//
// Replaces, for the render path of Damo12320/OptixPathtracer:
//   * optixTrace + the closed OptiX 7.3 traversal / triangle test (devicePrograms.cu:216-260)
//   * __closesthit__radiance (devicePrograms.cu:343-514), __miss__radiance/__miss__shadow
//     (:576-591), SamplePath (:625-664) and the camera of __raygen__renderFrame (:601-623).
//
// HBM layout (all arrays in LBVH leaf order, 16-byte aligned records):
//   nodes  : BNode[N-1], 64 B — both children's AABBs + child links (leaf = ~triangle)
//   tri    : float4[3N]       — v0.xyz|orig index, v1.xyz|material, v2.xyz|0 (world space)
//   nrm    : float4[3N]       — world-space vertex normals of the triangle
//   mats   : float4[2M]       — albedo.xyz|metallic, roughness|has_normals|0|0
#pragma once
#include "pt_bsdf.h"

namespace pt {

struct __align__(16) BNode {
    float4 a;  // c0.lo.x c0.hi.x c0.lo.y c0.hi.y
    float4 b;  // c1.lo.x c1.hi.x c1.lo.y c1.hi.y
    float4 c;  // c0.lo.z c0.hi.z c1.lo.z c1.hi.z
    int4 d;    // child0 child1 (>=0 internal node, <0 leaf = ~tri)
};

struct DevScene {
    const BNode* nodes;
    const float4* tri;
    const float4* nrm;
    const float4* mats;
    int ntri;
};

struct DevLight {
    float px, py, pz, cr, cg, cb;
};

struct DevLaunch {
    int width, height;
    float cam_pos[3];
    float inv_view[16];
    float inv_proj[16];
    const DevLight* lights;
    int n_lights;
    int max_bounces;
    uint32_t frame_base;
    uint32_t n_frames;
    float* accum;                    // W*H*3 fp32 sum
    unsigned long long* counters;    // [0] segments
};

struct Hit {
    float t, u, v;
    int tri;     // leaf-order triangle index, -1 = miss
    int orig;    // global (original) triangle index, tie-break key
    bool back;
};

// Moller-Trumbore; OptiX barycentric convention (u weights v1, v weights v2); closed
// interval [tmin, tmax]; det < 0 <=> back face (ray along the CCW normal).  Same
// arithmetic order as the oracle's tri_hit.
__device__ __forceinline__ bool tri_intersect(const float4 a, const float4 b, const float4 c, f3 o, f3 d,
                                              float tmin, float tmax, float& th, float& uh, float& vh,
                                              bool& back) {
    f3 v0 = mk(a.x, a.y, a.z), v1 = mk(b.x, b.y, b.z), v2 = mk(c.x, c.y, c.z);
    f3 e1 = v1 - v0, e2 = v2 - v0;
    f3 p = cross(d, e2);
    float det = dot(e1, p);
    if (det == 0.0f) return false;
    float inv = 1.0f / det;
    f3 tv = o - v0;
    float u = dot(tv, p) * inv;
    if (u < 0.0f || u > 1.0f) return false;
    f3 q = cross(tv, e1);
    float v = dot(d, q) * inv;
    if (v < 0.0f || u + v > 1.0f) return false;
    float t = dot(e2, q) * inv;
    if (!(t >= tmin && t <= tmax)) return false;
    th = t;
    uh = u;
    vh = v;
    back = det < 0.0f;
    return true;
}

// Slab test of both children; boxes are padded at build time so the fma form is conservative.
__device__ __forceinline__ void box2(const BNode& n, f3 io, f3 inv, float tmin, float tmax, float& t0n,
                                     float& t1n, bool& h0, bool& h1) {
    const float k = 1.0000004f;
    float ax = __fmaf_rn(n.a.x, inv.x, -io.x), bx = __fmaf_rn(n.a.y, inv.x, -io.x);
    float ay = __fmaf_rn(n.a.z, inv.y, -io.y), by = __fmaf_rn(n.a.w, inv.y, -io.y);
    float az = __fmaf_rn(n.c.x, inv.z, -io.z), bz = __fmaf_rn(n.c.y, inv.z, -io.z);
    float n0 = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fmaxf(fminf(az, bz), tmin));
    float f0 = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fminf(fmaxf(az, bz), tmax)) * k;
    float cx = __fmaf_rn(n.b.x, inv.x, -io.x), dx = __fmaf_rn(n.b.y, inv.x, -io.x);
    float cy = __fmaf_rn(n.b.z, inv.y, -io.y), dy = __fmaf_rn(n.b.w, inv.y, -io.y);
    float cz = __fmaf_rn(n.c.z, inv.z, -io.z), dz = __fmaf_rn(n.c.w, inv.z, -io.z);
    float n1 = fmaxf(fmaxf(fminf(cx, dx), fminf(cy, dy)), fmaxf(fminf(cz, dz), tmin));
    float f1 = fminf(fminf(fmaxf(cx, dx), fmaxf(cy, dy)), fminf(fmaxf(cz, dz), tmax)) * k;
    t0n = n0;
    t1n = n1;
    h0 = n0 <= f0;
    h1 = n1 <= f1;
}

// Reciprocal direction; zero components map to a huge finite value so the fma slab form
// never produces 0*inf.
__device__ __forceinline__ f3 safe_inv(f3 d) {
    const float big = 1e30f;
    return mk(d.x != 0.0f ? 1.0f / d.x : copysignf(big, d.x), d.y != 0.0f ? 1.0f / d.y : copysignf(big, d.y),
              d.z != 0.0f ? 1.0f / d.z : copysignf(big, d.z));
}

constexpr int kStack = 64;

// Closest hit ordered by (t, original triangle index): independent of BVH shape.
template <bool ANY>
__device__ __forceinline__ bool traverse(const DevScene& S, f3 o, f3 d, float tmin, float tmax, Hit& h) {
    h.tri = -1;
    h.orig = 0x7fffffff;
    if (S.ntri <= 0) return false;
    if (S.ntri == 1) {
        float t, u, v;
        bool bk;
        if (!tri_intersect(S.tri[0], S.tri[1], S.tri[2], o, d, tmin, tmax, t, u, v, bk)) return false;
        h.t = t; h.u = u; h.v = v; h.back = bk; h.tri = 0;
        h.orig = __float_as_int(S.tri[0].w);
        return true;
    }
    f3 inv = safe_inv(d);
    f3 io = mk(o.x * inv.x, o.y * inv.y, o.z * inv.z);
    int stack[kStack];
    int sp = 0;
    int node = 0;
    float best = tmax;
    while (true) {
        const BNode n = S.nodes[node];
        float t0, t1;
        bool h0, h1;
        box2(n, io, inv, tmin, best, t0, t1, h0, h1);
        int c0 = n.d.x, c1 = n.d.y;
        if (h0 && c0 < 0) {
            int ti = ~c0;
            float t, u, v;
            bool bk;
            float4 A = S.tri[3 * ti], B = S.tri[3 * ti + 1], C = S.tri[3 * ti + 2];
            if (tri_intersect(A, B, C, o, d, tmin, best, t, u, v, bk)) {
                int oi = __float_as_int(A.w);
                if (ANY) { h.tri = ti; h.orig = oi; return true; }
                if (t < best || oi < h.orig) {
                    best = t; h.t = t; h.u = u; h.v = v; h.back = bk; h.tri = ti; h.orig = oi;
                }
            }
            h0 = false;
        }
        if (h1 && c1 < 0) {
            int ti = ~c1;
            float t, u, v;
            bool bk;
            float4 A = S.tri[3 * ti], B = S.tri[3 * ti + 1], C = S.tri[3 * ti + 2];
            if (tri_intersect(A, B, C, o, d, tmin, best, t, u, v, bk)) {
                int oi = __float_as_int(A.w);
                if (ANY) { h.tri = ti; h.orig = oi; return true; }
                if (t < best || oi < h.orig) {
                    best = t; h.t = t; h.u = u; h.v = v; h.back = bk; h.tri = ti; h.orig = oi;
                }
            }
            h1 = false;
        }
        if (h0 && h1) {
            int nearc = (t0 <= t1) ? c0 : c1;
            int farc = (t0 <= t1) ? c1 : c0;
            if (sp < kStack) stack[sp++] = farc;
            node = nearc;
        } else if (h0) {
            node = c0;
        } else if (h1) {
            node = c1;
        } else {
            if (sp == 0) break;
            node = stack[--sp];
        }
    }
    return h.tri >= 0;
}

// devicePrograms.cu:601-623 — pixel-centre primary ray.
__device__ __forceinline__ void camera_ray(const DevLaunch& L, int x, int y, f3& o, f3& d) {
    float xs = ((float)x + 0.5f) / (float)L.width;
    float ys = ((float)y + 0.5f) / (float)L.height;
    float ndc[4] = {xs * 2.0f - 1.0f, ys * 2.0f - 1.0f, 1.0f, 1.0f};
    float pv[4], pw[4];
    mat4_mul_vec4(L.inv_proj, ndc, pv);
    float pv0[4] = {pv[0], pv[1], pv[2], 0.0f};
    mat4_mul_vec4(L.inv_view, pv0, pw);
    float d4 = (pw[0] * pw[0] + pw[1] * pw[1]) + (pw[2] * pw[2] + pw[3] * pw[3]);
    float inv = 1.0f / sqrtf(d4);
    d = mk(pw[0] * inv, pw[1] * inv, pw[2] * inv);
    o = mk(L.cam_pos[0], L.cam_pos[1], L.cam_pos[2]);
}

// Surface reconstruction at a hit: GetNormal / GetSurfacePos (devicePrograms.cu:83-129),
// back-face flip (:379-382), BuildTangentSpace (:168-212).
struct SurfaceHit {
    f3 pos, ng;
    Frame fr;
    f3 wo;        // shading space
    f3 albedo;
    float metallic, roughness;
};

__device__ __forceinline__ void reconstruct(const DevScene& S, const Hit& h, f3 d, SurfaceHit& s) {
    const int ti = h.tri;
    const float4 A = S.tri[3 * ti], B = S.tri[3 * ti + 1], C = S.tri[3 * ti + 2];
    const float4 NA = S.nrm[3 * ti], NB = S.nrm[3 * ti + 1], NC = S.nrm[3 * ti + 2];
    const int mi = __float_as_int(B.w);
    const float4 M0 = S.mats[2 * mi], M1 = S.mats[2 * mi + 1];
    f3 wo_w = normalize(-d);
    f3 v0 = mk(A.x, A.y, A.z), v1 = mk(B.x, B.y, B.z), v2 = mk(C.x, C.y, C.z);
    f3 Ng = cross(v1 - v0, v2 - v0);
    const float u = h.u, v = h.v;
    float w = 1.0f - u - v;
    f3 Ns = mk(w * NA.x + u * NB.x + v * NC.x, w * NA.y + u * NB.y + v * NC.y, w * NA.z + u * NB.z + v * NC.z);
    if (M1.y != 0.0f) Ns = normalize(Ns);  // has normals: normalize(modelMatrix * vec4(Ns, 0))
    if (dot(wo_w, Ng) < 0.0f) Ng = -Ng;
    Ng = normalize(Ng);
    if (dot(Ng, Ns) < 0.0f) Ns = -Ns;
    Ns = normalize(Ns);
    if (h.back) {
        Ns = Ns * -1.0f;
        Ng = Ng * -1.0f;
    }
    s.pos = mk(w * v0.x + u * v1.x + v * v2.x, w * v0.y + u * v1.y + v * v2.y, w * v0.z + u * v1.z + v * v2.z);
    s.ng = Ng;
    f3 c1 = cross(Ns, mk(0.0f, 0.0f, 1.0f));
    f3 c2 = cross(Ns, mk(0.0f, 1.0f, 0.0f));
    f3 T = (length(c1) > length(c2)) ? c1 : c2;
    T = normalize(T);
    s.fr.t = T;
    s.fr.b = cross(T, Ns);
    s.fr.n = Ns;
    s.wo = to_local(s.fr, wo_w);
    s.albedo = mk(M0.x, M0.y, M0.z);
    s.metallic = M0.w;
    s.roughness = M1.x;
}

// One camera path: SamplePath (devicePrograms.cu:625-664) with the closest-hit program inlined.
template <int MODE>
__device__ __forceinline__ f3 sample_path(const DevScene& S, const DevLaunch& L, f3 o, f3 d, uint32_t seed,
                                          uint32_t& segs) {
    f3 radiance = mk(0, 0, 0), beta = mk(1, 1, 1);
    int bounce = 0;
    bool endPath = false;
    while (!endPath && bounce < L.max_bounces && length(beta) > 0.00001f) {
        Hit h;
        bool hit = traverse<false>(S, o, d, 0.0f, 100.0f, h);
        segs++;
        if (!hit) {  // __miss__radiance :576-583
            beta = mk(0, 0, 0);
            bounce = 100;
            continue;
        }
        bounce++;
        if (bounce > L.max_bounces) {
            endPath = true;
            continue;
        }
        SurfaceHit sf;
        reconstruct(S, h, d, sf);
        const bool conductor = rnd(seed) < sf.metallic;  // :400
        // NEE (:446-472), Lighting::GetRandomPointLight (LightMethods.h:25-40)
        float P = 0.0f;
        int li = 0;
        if (L.n_lights == 1) {
            P = 1.0f;
        } else if (L.n_lights > 1) {
            float r = rnd(seed);
            li = (int)(r * (float)L.n_lights);
            if (li >= L.n_lights) li = L.n_lights - 1;
            P = 1.0f / (float)L.n_lights;
        }
        if (P > 0.0f) {
            const DevLight lt = L.lights[li];
            f3 lpos = mk(lt.px, lt.py, lt.pz);
            f3 ldir = lpos - sf.pos;
            f3 ldn = normalize(ldir);
            f3 so = sf.pos + 1e-3f * sf.ng;
            Hit sh;
            bool occluded = traverse<true>(S, so, normalize(ldir), 0.0f, length(ldir), sh);
            f3 lds = to_local(sf.fr, ldn);
            if (!occluded) {
                f3 f = bsdf_f<MODE>(seed, sf.albedo, sf.roughness, conductor, sf.wo, lds);
                float c = abs_dot(lds, mk(0.0f, 0.0f, 1.0f));
                f3 spectrum = f * c;
                if (!is_zero(spectrum)) {
                    f3 dd = sf.pos - lpos;
                    float d2 = dd.x * dd.x + dd.y * dd.y + dd.z * dd.z;
                    f3 Li = mk(lt.cr, lt.cg, lt.cb) / d2;
                    radiance = radiance + ((beta * spectrum) * Li) / (P * 1.0f);
                }
            }
        }
        BSample bs;
        if (!bsdf_sample<MODE>(seed, sf.albedo, sf.roughness, conductor, sf.wo, bs)) {
            endPath = true;
            continue;
        }
        float ac = abs_dot(bs.dir, mk(0.0f, 0.0f, 1.0f));
        beta = beta * mk(bs.color.x * ac / bs.pdf, bs.color.y * ac / bs.pdf, bs.color.z * ac / bs.pdf);
        f3 off = 1e-3f * sf.ng;
        if (dot(bs.dir, mk(0.0f, 0.0f, 1.0f)) < 0.0f) off = -off;
        o = sf.pos + off;
        d = normalize(to_world(sf.fr, bs.dir));
    }
    return radiance;
}

}  // namespace pt
