// pt_device.h — HBM layout of the scene, BVH4 traversal and the path integrator for gfx950.
//
// Replaces, for the render path of Damo12320/OptixPathtracer:
//   * optixTrace + the closed OptiX 7.3 traversal / triangle test (devicePrograms.cu:216-260)
//   * __closesthit__radiance (devicePrograms.cu:343-514), __miss__radiance/__miss__shadow
//     (:576-591), SamplePath (:625-664) and the camera of __raygen__renderFrame (:601-623).
//
// HBM layout (triangle arrays in LBVH leaf order, 16-byte aligned records):
//   nodes4 : BNode4[<N], 128 B — 4 child AABBs as SoA float4s + child links; one cache line
//   isect  : float4[3N]         — v0.xyz|orig index, e1.xyz|material, e2.xyz|0  (e = v - v0,
//                                  the same fp32 subtraction the oracle performs)
//   shade  : float4[4N]         — v1.xyz|n0.x, v2.xyz|n0.y, n0.z n1.xyz, n2.xyz|0
//   mats   : float4[3M]         — albedo.xyz|metallic, roughness|has_normals|texture ids, ... (kMatStride)
// Leaves reference up to 4 consecutive triangles (a BVH subtree is a contiguous range of the
// leaf-ordered triangles, so no index indirection is needed).
#pragma once
#include "pt_bsdf.h"

namespace pt {

constexpr int kEmptyChild = (int)0x80000000;

struct __align__(16) BNode4 {
    float4 lox, hix, loy, hiy, loz, hiz;  // children 0..3
    int4 child;                           // >=0 inner node; <0 leaf ~(first<<3 | count-1); kEmptyChild
    int4 pad;
};

__device__ __forceinline__ int leaf_first(int c) { return (~c) >> 3; }
__device__ __forceinline__ int leaf_count(int c) { return ((~c) & 7) + 1; }

struct DevScene {
    const BNode4* nodes;
    const float4* isect;
    const float4* shade;
    const float4* mats;      // kMatStride per mesh
    const float4* tuv;       // 2 per triangle (uv0, uv1 | uv2, 0), leaf order; NULL without textures
    const uint32_t* texels;  // all textures' RGBA8 texels, concatenated
    const int4* texinfo;     // per texture: texel offset, width, height, 0
    int ntri;
    int n_nodes;             // BVH4 nodes (breadth-first: the top levels are nodes 0 .. k)
    // the first n_lds nodes staged in the workgroup's LDS by a trace kernel (stage_top_nodes);
    // n_lds = 0 everywhere else
    const BNode4* lds_nodes;
    int n_lds;
};

// Material record (3 x float4 per mesh):
//   [0] albedo.rgb | metallic     [1] roughness | has_normals | albedo_tex | normal_tex
//   [2] metal_rough_tex | any texture | 0 | 0          (texture ids as int bits, -1 = none)
constexpr int kMatStride = 3;

struct DevLight {
    float px, py, pz, cr, cg, cb;
};

struct DevLaunch {
    int width, height;  // height: the rows of this launch (a band of the image, see row0)
    // A launch may render a band of rows [row0, row0 + height) of an image image_height rows high
    // (the one-frame path splits a frame into two bands on the two wavefront streams): the camera
    // ray, the path seed and the debug pixel use the image's row and pixel index, everything else
    // the band's own pixel index p (image pixel = p + width * row0), and accum points at the band.
    int row0, image_height;
    float cam_pos[3];
    float inv_view[16];
    float inv_proj[16];
    const DevLight* lights;
    int n_lights;
    int max_bounces;
    uint32_t frame_base;
    uint32_t n_frames;
    float* accum;                    // W*H*3 fp32 sum
    double* accum64;                 // pt_set_accum_fp64: W*H*3 fp64 sum (accum then holds its
                                     // fp32 rounding); NULL = fp32 accumulation
    size_t frame_stride;             // 0: the frames add into accum; else frame f of the launch is
                                     // written alone to accum + f * frame_stride (pt_render's
                                     // render-ahead ring, wavefront k_accum only)
    unsigned long long* counters;    // [0] segments [1] nodes visited [2] triangle tests [3] rays
    // debug path (pt_set_debug_pixel; the reference's isDebugRay, devicePrograms.cu:637-644):
    // the path of pixel debug_pixel (W*y + x, -1 = off) at frame debug_frame records every
    // bounce's surface into debug[bounce - 1] (kDebugRecordFloats floats each)
    int debug_pixel;
    uint32_t debug_frame;
    float* debug;
};
constexpr int kDebugMaxBounces = 64;
constexpr int kDebugRecordFloats = 22;  // ptamd.h pt_debug_bounce

// Wavefront path id of the debug path in the batch of L (path = frame offset * pixels + pixel, in
// the launch's band), or -1.
__device__ __forceinline__ int debug_path_id(const DevLaunch& L) {
    const uint32_t f = L.debug_frame - L.frame_base;
    const int P = L.width * L.height, p = L.debug_pixel - L.width * L.row0;  // the band's pixel index
    return (L.debug_pixel >= 0 && p >= 0 && p < P && f < L.n_frames) ? (int)f * P + p : -1;
}

struct Hit {
    float t, u, v;
    int tri;     // leaf-order triangle index, -1 = miss
    int orig;    // global (original) triangle index, tie-break key
    bool back;
};

// PT_CYCLE_PROBE (timing probe of the wavefront trace loop, with traversal stats on): the
// wave_active_lanes / wave_node_steps / wave_tri_steps / wave_refills counters hold the shader
// cycles each wave spent waiting for the node half's loads, in the rest of the node half, in the
// triangle batches and in the refill blocks (s_memtime around each section; a section's end
// waits for a value it produced, so its memory operations have landed).
#ifndef PT_CYCLE_PROBE
#define PT_CYCLE_PROBE 0
#endif
__device__ __forceinline__ uint64_t probe_clock() {
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    return t;
}
template <class T>
__device__ __forceinline__ uint64_t probe_clock(const T& dep) {  // once `dep` is available
    T v = dep;
    __asm__ volatile("" : "+v"(v));
    __builtin_amdgcn_s_waitcnt(0);
    return probe_clock();
}

struct TravStats {
    uint32_t nodes = 0, tris = 0, rays = 0, overflow = 0, retrace = 0;
    uint32_t lds_nodes = 0;  // node visits served from the staged top levels (stage_top_nodes)
    uint32_t unocc = 0;      // k_trace_pair: shadow rays that found their light unoccluded
    // wave schedule (trace_range, lane 0 of each wave): iterations, active lanes summed over
    // them, iterations running the node half / the triangle half, refill blocks
    uint32_t steps = 0, active = 0, node_steps = 0, tri_steps = 0, refills = 0;
    // coherence of the global (non-LDS) node loads: per wave step with
    // such loads, the number of distinct nodes its lanes load, in buckets 1, 2, 3-4, 5-8, 9-16,
    // 17-64 (wave-uniform, counted by every lane alike), and the lanes that loaded one
    uint32_t coh[6] = {0, 0, 0, 0, 0, 0};
    uint32_t coh_lanes = 0;
#if PT_CYCLE_PROBE
    uint64_t probe_t = 0;  // s_memtime when the node half's loads landed
#endif
};

// ---- ray / box arithmetic shared bit for bit with the oracle ---------------------------------
// The slab distance of a plane p on axis a is fma(p, inv_a, -io_a) with inv = 1/d (IEEE
// division; a zero component maps to +-1e30) and io = o * inv.  oracle/pt_oracle.c evaluates
// the same expressions, so both sides agree bit for bit on every slab distance, and with it on
// the hit-acceptance rule below.
constexpr float kSlabWiden = 1.000244140625f;  // 1 + 2^-12, see tri_accept
__device__ __forceinline__ float ray_inv(float d) { return d != 0.0f ? 1.0f / d : copysignf(1e30f, d); }
__device__ __forceinline__ f3 safe_inv(f3 d) { return mk(ray_inv(d.x), ray_inv(d.y), ray_inv(d.z)); }

// Padded box of one triangle, from the vertices exactly as the hit test sees them (v0, v0 + e1,
// v0 + e2, with e = v - v0 rounded once).  The BVH builder (pt_build.hip) unions these boxes,
// so every BVH box holding a triangle contains this box bit for bit.
PT_HD float box_pad(float x) { return fabsf(x) * 9.5367431640625e-7f + 1e-6f; }
PT_HD void tri_box_padded(f3 v0, f3 e1, f3 e2, float lo[3], float hi[3]) {
    const float a[3] = {v0.x, v0.y, v0.z}, b[3] = {e1.x, e1.y, e1.z}, c[3] = {e2.x, e2.y, e2.z};
    for (int k = 0; k < 3; ++k) {
        const float p1 = a[k] + b[k], p2 = a[k] + c[k];
        const float l = fminf(fminf(a[k], p1), p2), h = fmaxf(fmaxf(a[k], p1), p2);
        lo[k] = l - box_pad(l);
        hi[k] = h + box_pad(h);
    }
}

// Hit acceptance.  A Moller-Trumbore hit at t on triangle T counts only if t lies in the slab
// interval [tn, tf] of T's padded box, with relative slack K = kSlabWiden:
//     tn <= t*K,   t <= tf*K,   tn <= tf*K.
// A node keeps a child box B iff max(tn_B, tmin) <= min(tf_B, best)*K (node_eval).  B contains
// T's padded box and the slab distance is monotone in the plane coordinate, so tn_B <= tn and
// tf_B >= tf: a box holding an acceptable hit with t <= best is never culled.  The closest hit
// is therefore the (t, original index) minimum over the acceptable hits for ANY BVH and ANY
// visiting order -- the oracle's binary median-split BVH and this BVH4 give the same answer.
// Without the rule (round 1), a grazing ray could be accepted by Moller-Trumbore at a point
// outside the triangle's own box (barycentric rounding at cos = 0.038), whose box the cull then
// dropped or kept depending on which triangle had set `best` first -- a visiting-order, hence
// wave-neighbour, dependence ("Closest-hit determinism").
__device__ __forceinline__ bool tri_accept(const float4 A, const float4 E1, const float4 E2, f3 inv, f3 io, float t) {
    float lo[3], hi[3];
    tri_box_padded(mk(A.x, A.y, A.z), mk(E1.x, E1.y, E1.z), mk(E2.x, E2.y, E2.z), lo, hi);
    const float ax = __fmaf_rn(lo[0], inv.x, -io.x), bx = __fmaf_rn(hi[0], inv.x, -io.x);
    const float ay = __fmaf_rn(lo[1], inv.y, -io.y), by = __fmaf_rn(hi[1], inv.y, -io.y);
    const float az = __fmaf_rn(lo[2], inv.z, -io.z), bz = __fmaf_rn(hi[2], inv.z, -io.z);
    const float tn = fmaxf(fmaxf(fminf(ax, bx), fminf(ay, by)), fminf(az, bz));
    const float tfk = fminf(fminf(fmaxf(ax, bx), fmaxf(ay, by)), fmaxf(az, bz)) * kSlabWiden;
    return tn <= t * kSlabWiden && t <= tfk && tn <= tfk;
}

__device__ __forceinline__ void cswap(float& ta, int& ca, float& tb, int& cb) {
    bool s = tb < ta;
    float t0 = s ? tb : ta, t1 = s ? ta : tb;
    int c0 = s ? cb : ca, c1 = s ? ca : cb;
    ta = t0; tb = t1; ca = c0; cb = c1;
}

// LDS stack: entry s of thread tid at stk[s * stride] with stk = base + tid, so the 64
// lanes of a wave always touch 64 consecutive dwords (conflict-free for any sp mix).  Pushes
// and pops only ever address LDS: when a push would overflow it, the bottom half moves to a
// private spill array, and a pop from an empty LDS stack brings the newest spilled half
// back (both rare, separate branches — a pop that may read either memory compiles to a
// slow flat load on every step).
// The LDS depth is a template parameter (DEPTH): it trades LDS per workgroup against
// occupancy per kernel (see pt_render.hip / pt_wavefront.hip).  A traversal holds at most
// 3 entries per BVH4 level; pt_create rejects trees deeper than the smallest traversal
// stack holds (stack_capacity).
constexpr int kSpillDepth = 64;
// LDS stack depths of the wavefront trace kernels and of the megakernel / k_trace (A/B builds
// override them with -D; every translation unit sees the same value)
#ifndef PT_WF_STACK
#define PT_WF_STACK 11  // 6 trace workgroups per CU (14 at 5 per CU before)
#endif
#ifndef PT_MK_STACK
#define PT_MK_STACK 32
#endif
// Entries a traversal with an LDS stack of `lds` entries holds without losing one: the spill
// moves chunks of lds/2 entries, so only whole chunks of kSpillDepth are usable, and the LDS
// part fills up to `lds` (a push of <= 3 happens at sp <= lds - 3).
constexpr int stack_capacity(int lds) { return (kSpillDepth / (lds / 2)) * (lds / 2) + lds; }

// ---- textures: devicePrograms.cu:62-73 (SRGB8ToLinear), :131-166 (GetTextureCoord,
// SampleTextures), :518-543 (AlphaCutout); CreateTextures (OptixRenderer.cpp:562-612) sets up
// bilinear / wrap / normalized-coordinate / normalized-float uchar4 textures.  Filtering is
// done here in software with the CUDA texture-fetch formula (filter weight in 1.8 fixed
// point), the same expression as the oracle's orc_tex_sample, instead of the texture unit
// whose filter precision is not specified bit for bit.
__device__ __forceinline__ float srgb_to_linear(float c) {
    const float m = (c < 0.04045f) ? 0.0f : 1.0f;  // glm::step
    const float a = c / 12.92f;
    const float b = pt_powf_unit((c + 0.055f) / 1.055f, 2.4f);  // SavePow (powf, pt_math.h)
    return a * (1.0f - m) + b * m;                      // SaveMix
}
__device__ __forceinline__ int wrapi(int i, int n) {
    const int r = i % n;
    return r < 0 ? r + n : r;
}
__device__ __forceinline__ float4 tex_sample(const DevScene& S, int tex, float x, float y, bool srgb) {
    const int4 ti = S.texinfo[tex];
    const int W = ti.y, H = ti.z;
    x = x - floorf(x);
    y = y - floorf(y);
    const float xb = x * (float)W - 0.5f, yb = y * (float)H - 0.5f;
    const float fx = floorf(xb), fy = floorf(yb);
    const float ax = rintf((xb - fx) * 256.0f) * (1.0f / 256.0f);
    const float ay = rintf((yb - fy) * 256.0f) * (1.0f / 256.0f);
    const int i0 = wrapi((int)fx, W), i1 = wrapi((int)fx + 1, W);
    const int j0 = wrapi((int)fy, H), j1 = wrapi((int)fy + 1, H);
    const uint32_t* px = S.texels + ti.x;
    const uint32_t p00 = px[(size_t)j0 * W + i0], p10 = px[(size_t)j0 * W + i1];
    const uint32_t p01 = px[(size_t)j1 * W + i0], p11 = px[(size_t)j1 * W + i1];
    float o[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
        const float t00 = (float)((p00 >> (8 * c)) & 0xff) / 255.0f, t10 = (float)((p10 >> (8 * c)) & 0xff) / 255.0f;
        const float t01 = (float)((p01 >> (8 * c)) & 0xff) / 255.0f, t11 = (float)((p11 >> (8 * c)) & 0xff) / 255.0f;
        const float r0 = t00 * (1.0f - ax) + t10 * ax;
        const float r1 = t01 * (1.0f - ax) + t11 * ax;
        const float v = r0 * (1.0f - ay) + r1 * ay;
        o[c] = srgb ? srgb_to_linear(v) : v;
    }
    return make_float4(o[0], o[1], o[2], o[3]);
}
// GetTextureCoord: (1-u-v)*uv0 + u*uv1 + v*uv2 (zeros when the mesh has no texcoords)
__device__ __forceinline__ void tri_texcoord(const DevScene& S, int ti, float u, float v, float& x, float& y) {
    const float4 a = S.tuv[2 * ti], b = S.tuv[2 * ti + 1];
    const float w = 1.0f - u - v;
    x = (w * a.x + u * a.z) + v * b.x;
    y = (w * a.y + u * a.w) + v * b.y;
}
// AlphaCutout: a hit on an albedo-textured mesh is ignored when the decoded alpha < 0.9
// (__anyhit__radiance / __anyhit__shadow, devicePrograms.cu:545-561).
__device__ __forceinline__ bool alpha_cut(const DevScene& S, int ti, int mi, float u, float v) {
    const int at = __float_as_int(S.mats[kMatStride * mi + 1].z);
    float x, y;
    tri_texcoord(S, ti, u, v, x, y);
    return tex_sample(S, at, x, y, true).w < 0.9f;
}

// ---- BVH4 traversal -----------------------------------------------------------------------
// A per-lane state machine.  A lane carries one node (`cur`) and one leaf (`leaf`), and one
// step visits the node (4 slab tests, sorted push of the far hits, descend) AND tests one
// triangle of the leaf: a wave whose lanes are split between nodes and triangles executes
// both halves anyway, so most lanes do useful work in both.  Written
// branch-reduced for 64-wide waves: the three pushes are unconditional LDS stores with
// predicated stack-pointer increments and the triangle test is predicated (same arithmetic
// and NaN behaviour as the oracle's tri_hit, without the early exits).  Closest hit is
// ordered by (t, original triangle index) over the acceptable hits (tri_accept), so the
// result is independent of BVH shape and visit order.
struct TravState {
    f3 o, d, inv, io;
    float tmin, best;
    int cur, sp, spc;  // current node/leaf, LDS stack depth, entries spilled
    int leaf;          // leaf whose triangles are tested alongside node steps
    int nx, ny, nz;    // byte offset (0 or 16) of the near slab plane per axis within the node
    bool any;          // any-hit ray (only read by kRayMixed traversals)
    bool strict;       // re-trace: only acceptable hits are taken (trav_restart_strict)
    int path;          // closest-hit wavefront rays: the path id for the hit record; any-hit
                       // rays: the bits of the hit's t once they stop (trav_result_ok)
    Hit h;
};

// Ray kinds of a traversal (the ANY template argument): closest hit, any hit (shadow rays,
// stop at the first hit), or mixed queues where TravState::any decides per lane.
enum { kRayClosest = 0, kRayAny = 1, kRayMixed = 2 };

__device__ __forceinline__ void trav_init(TravState& s, f3 o, f3 d, float tmin, float tmax) {
    s.o = o;
    s.d = d;
    s.inv = safe_inv(d);
    s.io = mk(o.x * s.inv.x, o.y * s.inv.y, o.z * s.inv.z);
    s.nx = s.inv.x < 0.0f ? 16 : 0;
    s.ny = s.inv.y < 0.0f ? 16 : 0;
    s.nz = s.inv.z < 0.0f ? 16 : 0;
    s.tmin = tmin;
    s.best = tmax;
    s.cur = 0;  // root (always an inner node)
    s.sp = 0;
    s.spc = 0;
    s.leaf = kEmptyChild;
    s.any = false;
    s.strict = false;
    s.h.tri = -1;
    s.h.orig = 0x7fffffff;
}

template <int ANY>
__device__ __forceinline__ bool is_any(const TravState& s) {
    return ANY == kRayAny || (ANY == kRayMixed && s.any);
}

// Moller-Trumbore; OptiX barycentric convention (u weights v1, v weights v2); closed
// interval [tmin, tmax]; det < 0 <=> back face (ray along the CCW normal).  Same
// arithmetic order and NaN behaviour as the oracle's tri_hit (edges precomputed with the
// same subtraction); predicated instead of early exits (no divergent branches per test).
__device__ __forceinline__ bool tri_test(const float4 A, const float4 E1, const float4 E2, f3 o, f3 d, float tmin,
                                         float tmax, float& th, float& uh, float& vh, bool& back) {
    f3 v0 = mk(A.x, A.y, A.z), e1 = mk(E1.x, E1.y, E1.z), e2 = mk(E2.x, E2.y, E2.z);
    f3 p = cross(d, e2);
    float det = dot(e1, p);
    float inv = 1.0f / det;
    f3 tv = o - v0;
    float u = dot(tv, p) * inv;
    f3 q = cross(tv, e1);
    float v = dot(d, q) * inv;
    float t = dot(e2, q) * inv;
    th = t;
    uh = u;
    vh = v;
    back = det < 0.0f;
    return (det != 0.0f) & !(u < 0.0f || u > 1.0f) & !(v < 0.0f || u + v > 1.0f) & (t >= tmin && t <= tmax);
}

// Move the bottom (DEPTH / 2) LDS entries to the spill array (rare).  pt_create bounds the
// BVH depth so the spill never fills (kMaxBvhDepth); a full spill is still counted.
template <int DEPTH, bool STATS>
__device__ __forceinline__ void stack_spill(TravState& s, int* __restrict__ stk, int stride, int* spill,
                                         TravStats& ts) {
    if (s.spc + (DEPTH / 2) <= kSpillDepth) {
        for (int k = 0; k < (DEPTH / 2); ++k) spill[s.spc + k] = stk[k * stride];
        s.spc += (DEPTH / 2);
    } else if (STATS) {
        ts.overflow++;
    }
    for (int k = (DEPTH / 2); k < s.sp; ++k) stk[(k - (DEPTH / 2)) * stride] = stk[k * stride];
    s.sp -= (DEPTH / 2);
}

// LDS stack empty but entries spilled: bring the newest chunk back (rare).
template <int DEPTH>
__device__ __forceinline__ void stack_refill(TravState& s, int* __restrict__ stk, int stride, const int* spill) {
    s.spc -= (DEPTH / 2);
    for (int k = 0; k < (DEPTH / 2); ++k) stk[k * stride] = spill[s.spc + k];
    s.sp = (DEPTH / 2);
}

typedef float pt_f2 __attribute__((ext_vector_type(2)));

// The six sign-selected planes and the child links of one node, as loaded.
struct NodeLoad {
    float4 ax, bx, ay, by, az, bz;
    int4 ch;
};

__device__ __forceinline__ NodeLoad node_load(const DevScene& S, const TravState& s, int ni) {
    NodeLoad n;
    if (ni < S.n_lds) {  // a top-level node staged in LDS (north_star: "BVH nodes ... staged through LDS")
        const char* b = reinterpret_cast<const char*>(S.lds_nodes + ni);
        auto ld = [&](int off) { return *reinterpret_cast<const float4*>(b + off); };
        n.ax = ld(s.nx);
        n.bx = ld(16 - s.nx);
        n.ay = ld(32 + s.ny);
        n.by = ld(48 - s.ny);
        n.az = ld(64 + s.nz);
        n.bz = ld(80 - s.nz);
        n.ch = *reinterpret_cast<const int4*>(b + 96);
        return n;
    }
    // raw buffer loads: one 32-bit offset add per plane instead of a 64-bit address
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)S.nodes, 0, 0x7fffffff, 0x00020000);
    const int nb = ni << 7;
    auto ld = [&](int off) {
        return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, nb + off, 0, 0));
    };
    n.ax = ld(s.nx);
    n.bx = ld(16 - s.nx);
    n.ay = ld(32 + s.ny);
    n.by = ld(48 - s.ny);
    n.az = ld(64 + s.nz);
    n.bz = ld(80 - s.nz);
    n.ch = __builtin_bit_cast(int4, __builtin_amdgcn_raw_buffer_load_b128(rs, nb + 96, 0, 0));
    return n;
}

// Copy the first min(n_nodes, K) BVH4 nodes (the top levels: nodes are numbered breadth-first)
// into the workgroup's LDS and point the scene view at them.  Every thread of the block calls it
// before any early exit.
template <int K>
__device__ __forceinline__ void stage_top_nodes(DevScene& S, BNode4* top) {
    const int n = K > 0 ? min(S.n_nodes, K) : 0;
    const float4* src = reinterpret_cast<const float4*>(S.nodes);
    float4* dst = reinterpret_cast<float4*>(top);
    for (int i = (int)threadIdx.x; i < n * 8; i += (int)blockDim.x) dst[i] = src[i];
    __syncthreads();
    S.lds_nodes = top;
    S.n_lds = n;
}

// Slab test of the four children of a loaded node, hits as (t_near, child) with misses and
// empty slots as (inf, kEmptyChild).  The ray's direction signs picked the near and far plane
// of every axis at load time (per-lane byte offsets into the node), so each child needs no
// min/max per axis, and the plane distances are two children per packed v_pk_fma.  The planes
// are the ones min/max would choose (fma is monotone in the plane coordinate), so the slab
// distances equal tri_accept's and the oracle's box_hit's bit for bit.
__device__ __forceinline__ void node_eval(const NodeLoad& n, const TravState& s, float& t0, float& t1, float& t2,
                                          float& t3, int& c0, int& c1, int& c2, int& c3) {
    bool h0, h1, h2, h3;
    const float4 ax = n.ax, bx = n.bx, ay = n.ay, by = n.by, az = n.az, bz = n.bz;
    const int4 ch = n.ch;
    const pt_f2 ix = {s.inv.x, s.inv.x}, iy = {s.inv.y, s.inv.y}, iz = {s.inv.z, s.inv.z};
    const pt_f2 ox = {-s.io.x, -s.io.x}, oy = {-s.io.y, -s.io.y}, oz = {-s.io.z, -s.io.z};
    const pt_f2 nx01 = __builtin_elementwise_fma(pt_f2{ax.x, ax.y}, ix, ox);
    const pt_f2 nx23 = __builtin_elementwise_fma(pt_f2{ax.z, ax.w}, ix, ox);
    const pt_f2 fx01 = __builtin_elementwise_fma(pt_f2{bx.x, bx.y}, ix, ox);
    const pt_f2 fx23 = __builtin_elementwise_fma(pt_f2{bx.z, bx.w}, ix, ox);
    const pt_f2 ny01 = __builtin_elementwise_fma(pt_f2{ay.x, ay.y}, iy, oy);
    const pt_f2 ny23 = __builtin_elementwise_fma(pt_f2{ay.z, ay.w}, iy, oy);
    const pt_f2 fy01 = __builtin_elementwise_fma(pt_f2{by.x, by.y}, iy, oy);
    const pt_f2 fy23 = __builtin_elementwise_fma(pt_f2{by.z, by.w}, iy, oy);
    const pt_f2 nz01 = __builtin_elementwise_fma(pt_f2{az.x, az.y}, iz, oz);
    const pt_f2 nz23 = __builtin_elementwise_fma(pt_f2{az.z, az.w}, iz, oz);
    const pt_f2 fz01 = __builtin_elementwise_fma(pt_f2{bz.x, bz.y}, iz, oz);
    const pt_f2 fz23 = __builtin_elementwise_fma(pt_f2{bz.z, bz.w}, iz, oz);
    const float tmin = s.tmin, tmax = s.best;
    t0 = fmaxf(fmaxf(nx01.x, ny01.x), fmaxf(nz01.x, tmin));
    t1 = fmaxf(fmaxf(nx01.y, ny01.y), fmaxf(nz01.y, tmin));
    t2 = fmaxf(fmaxf(nx23.x, ny23.x), fmaxf(nz23.x, tmin));
    t3 = fmaxf(fmaxf(nx23.y, ny23.y), fmaxf(nz23.y, tmin));
    pt_f2 f01 = {fminf(fminf(fx01.x, fy01.x), fminf(fz01.x, tmax)), fminf(fminf(fx01.y, fy01.y), fminf(fz01.y, tmax))};
    pt_f2 f23 = {fminf(fminf(fx23.x, fy23.x), fminf(fz23.x, tmax)), fminf(fminf(fx23.y, fy23.y), fminf(fz23.y, tmax))};
    f01 = f01 * pt_f2{kSlabWiden, kSlabWiden};
    f23 = f23 * pt_f2{kSlabWiden, kSlabWiden};
    h0 = t0 <= f01.x;
    h1 = t1 <= f01.y;
    h2 = t2 <= f23.x;
    h3 = t3 <= f23.y;
    // empty slots hold inverted boxes (pt_build.hip k_collapse_sah): they never hit
    const float inf = __int_as_float(0x7f800000);
    t0 = h0 ? t0 : inf;
    t1 = h1 ? t1 : inf;
    t2 = h2 ? t2 : inf;
    t3 = h3 ? t3 : inf;
    c0 = h0 ? ch.x : kEmptyChild;
    c1 = h1 ? ch.y : kEmptyChild;
    c2 = h2 ? ch.z : kEmptyChild;
    c3 = h3 ? ch.w : kEmptyChild;
}

// Test one triangle of the leaf s.leaf and advance it; true when an any-hit ray is done.
// Closest-hit lanes take a hit by the (t, original index) order; in strict mode
// (trav_restart_strict) only acceptable hits count.  Any-hit lanes stop at the first hit and
// record only h.tri (the shadow queue carries the path and contribution in h's other fields).
template <int ANY, bool STATS, bool TEX>
__device__ __forceinline__ bool leaf_tri_eval(const DevScene& S, TravState& s, TravStats& ts, const float4 A,
                                              const float4 E1, const float4 E2) {
    const int first = leaf_first(s.leaf), cnt = leaf_count(s.leaf);
    const int ti = first;
    if (STATS) ts.tris++;
    float t, u, v;
    bool bk;
    bool hit = tri_test(A, E1, E2, s.o, s.d, s.tmin, s.best, t, u, v, bk);
    if (TEX && hit && __float_as_int(E2.w) != 0) hit = !alpha_cut(S, ti, __float_as_int(E1.w), u, v);
    if (s.strict && hit) hit = tri_accept(A, E1, E2, s.inv, s.io, t);  // rare re-trace lanes only
    const int oi = __float_as_int(A.w);
    s.leaf = cnt > 1 ? ~(((first + 1) << 3) | (cnt - 2)) : kEmptyChild;  // rest of the leaf
    if (is_any<ANY>(s)) {
        if (hit) {
            s.h.tri = ti;
            s.path = __float_as_int(t);
            return true;
        }
    } else {
        const bool take = hit && (t < s.best || oi < s.h.orig);
        s.best = take ? t : s.best;
        s.h.t = take ? t : s.h.t;
        s.h.u = take ? u : s.h.u;
        s.h.v = take ? v : s.h.v;
        s.h.back = take ? bk : s.h.back;
        s.h.tri = take ? ti : s.h.tri;
        s.h.orig = take ? oi : s.h.orig;
    }
    return false;
}

template <int ANY, bool STATS, bool TEX>
__device__ __forceinline__ bool leaf_tri_step(const DevScene& S, TravState& s, TravStats& ts) {
    const int ti = leaf_first(s.leaf);
    return leaf_tri_eval<ANY, STATS, TEX>(S, s, ts, S.isect[3 * ti], S.isect[3 * ti + 1], S.isect[3 * ti + 2]);
}

// Next stack entry into s.cur (kEmptyChild when the stack is empty).
template <int DEPTH>
__device__ __forceinline__ void stack_pop(TravState& s, int* __restrict__ stk, int stride, const int* spill) {
    if (s.sp == 0 && s.spc > 0) stack_refill<DEPTH>(s, stk, stride, spill);
    const int sp = s.sp - 1;
    const int e = stk[max(sp, 0) * stride];
    s.cur = sp >= 0 ? e : kEmptyChild;
    s.sp = max(sp, 0);
}

// One traversal step (one triangle of the pending leaf AND one node); true when the ray is
// finished.  Leaves are tested out of front-to-back order, which the (t, index) closest-hit
// rule makes harmless; culling stays conservative (best only shrinks).  `tri_ok`
// (wave-uniform) lets the caller postpone the triangle half of the step until enough lanes
// hold a leaf (trace_range); lanes keep traversing nodes meanwhile.
template <int ANY, bool STATS, int DEPTH, bool TEX>
__device__ __forceinline__ bool trav_step(const DevScene& S, TravState& s, int* __restrict__ stk, int stride,
                                          int* spill, TravStats& ts, bool tri_ok = true) {
    // (issuing the triangle and node loads before either test overlaps their round trips but
    // needs 116 VGPRs, one wave per SIMD fewer: -1.5 % Lambert, -22 % Dielectric)
    if (tri_ok && s.leaf != kEmptyChild) {
        if (leaf_tri_step<ANY, STATS, TEX>(S, s, ts)) return true;
    }
    if (s.cur >= 0) {
        if (STATS) ts.nodes++;
        float t0, t1, t2, t3;
        int c0, c1, c2, c3;
        node_eval(node_load(S, s, s.cur), s, t0, t1, t2, t3, c0, c1, c2, c3);  // misses: t = inf
        if (ANY != kRayAny) {  // nearest first; an any-hit ray's answer does not depend on order
            cswap(t0, c0, t1, c1);
            cswap(t2, c2, t3, c3);
            cswap(t0, c0, t2, c2);  // c0 nearest
            cswap(t1, c1, t3, c3);
            cswap(t1, c1, t2, c2);
        }
        if (s.sp > DEPTH - 3) stack_spill<DEPTH, STATS>(s, stk, stride, spill, ts);
        {  // unconditional stores, predicated sp: an empty child's store lands in the slot the
           // next valid one overwrites
            int sp = s.sp;
            stk[sp * stride] = c3;
            sp += c3 != kEmptyChild;
            stk[sp * stride] = c2;
            sp += c2 != kEmptyChild;
            stk[sp * stride] = c1;
            sp += c1 != kEmptyChild;
            s.sp = sp;
        }
        s.cur = c0;
    }
    // hand-off: a leaf in the node slot moves to a free leaf slot; refill the node slot
    if (s.cur == kEmptyChild) stack_pop<DEPTH>(s, stk, stride, spill);
    if (s.cur < 0 && s.cur != kEmptyChild && s.leaf == kEmptyChild) {
        s.leaf = s.cur;
        stack_pop<DEPTH>(s, stk, stride, spill);
    }
    return s.cur == kEmptyChild && s.leaf == kEmptyChild;
}

// ---- wave-batched triangle tests (the lane-refilling wavefront trace loop) -----------------
// The triangle half of the per-lane step (trav_step) tests one triangle of a lane's leaf per
// step, and only about a third of the lanes hold a leaf when it runs (DESIGN.md §4 "Wave
// schedule").  Here the wave instead lists every triangle of every pending leaf as (triangle,
// owner lane) pairs in LDS and tests them 64 at a time, each lane taking one pair and fetching
// the owner's ray with cross-lane reads.  A pair's hit competes for its owner by the key
// (t, original index) -- t >= 0, so its bits order as an unsigned integer -- through an LDS
// 64-bit atomic min; the owner then takes the winner by the closest-hit rule of leaf_tri_eval.
// The answer is the same (t, index) minimum over acceptable hits as in trav_step.
constexpr int kTriPairsPerWave = 256;  // 64 lanes x <= 4 triangles per leaf
struct TriBatchLds {                    // one per wave
    uint32_t pair[kTriPairsPerWave];    // (leaf-order triangle << 6) | owner lane
    unsigned long long key[64];         // per owner: min over this round's hits of (t bits << 32 | orig)
    float2 res_uv[64];                  // per owner: the winning pair's u, v
    int res_code[64];                   //   and tri | back << 31 (2.25 KB per wave in all)
};

__device__ __forceinline__ int lane_prefix(unsigned long long m) {
    return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Every lane of the wave calls this (wave-uniform control flow); `has` = the lane holds a
// pending leaf.  Tests all those leaves' triangles, empties the leaf slots and updates the
// owners' hits.  The trace loop's rays have tmin = 0.
template <int ANY, bool STATS, bool TEX>
__device__ __forceinline__ void wave_tri_batch(const DevScene& S, TravState& s, bool has, TriBatchLds* L,
                                               TravStats& ts) {
    const int lane = (int)(threadIdx.x & 63);
    const int c1 = has ? leaf_count(s.leaf) - 1 : 0;  // 0..3
    const int first = leaf_first(s.leaf);
    const unsigned long long m0 = __ballot(has), m1 = __ballot(has && (c1 & 1)), m2 = __ballot(has && (c1 & 2));
    const int pre = lane_prefix(m0) + lane_prefix(m1) + 2 * lane_prefix(m2);
    const int total = (int)(__popcll(m0) + __popcll(m1) + 2 * __popcll(m2));
    if (has) {
        L->pair[pre] = ((uint32_t)first << 6) | (uint32_t)lane;
        if (c1 >= 1) L->pair[pre + 1] = ((uint32_t)(first + 1) << 6) | (uint32_t)lane;
        if (c1 >= 2) L->pair[pre + 2] = ((uint32_t)(first + 2) << 6) | (uint32_t)lane;
        if (c1 >= 3) L->pair[pre + 3] = ((uint32_t)(first + 3) << 6) | (uint32_t)lane;
        s.leaf = kEmptyChild;
    }
    L->key[lane] = ~0ull;
    const int flags = is_any<ANY>(s) ? 2 : 0;
    __builtin_amdgcn_wave_barrier();
    for (int base = 0; base < total; base += 64) {  // total is wave-uniform
        const int k = base + lane;
        const bool valid = k < total;
        const uint32_t pair = L->pair[valid ? k : 0];
        const int owner = (int)(pair & 63u), ti = (int)(pair >> 6);
        const f3 o = mk(__shfl(s.o.x, owner, 64), __shfl(s.o.y, owner, 64), __shfl(s.o.z, owner, 64));
        const f3 d = mk(__shfl(s.d.x, owner, 64), __shfl(s.d.y, owner, 64), __shfl(s.d.z, owner, 64));
        const float tmax = __shfl(s.best, owner, 64);
        // every lane tests a triangle: a lane past the end repeats pair 0 (a real pair) and
        // discards its result, so the round needs no branch and no zeroed registers
        bool bk = false;
        float t, u, v;
        if (STATS && valid) ts.tris++;
        const float4 A = S.isect[3 * ti], E1 = S.isect[3 * ti + 1], E2 = S.isect[3 * ti + 2];
        bool hit = tri_test(A, E1, E2, o, d, 0.0f, tmax, t, u, v, bk) && valid;
        if (TEX && hit && __float_as_int(E2.w) != 0) hit = !alpha_cut(S, ti, __float_as_int(E1.w), u, v);
        const int oi = __float_as_int(A.w);
        // Every candidate is held to the acceptance rule here (tri_accept with the owner's inv / io,
        // read across lanes by the whole wave), so the batch only ever takes acceptable hits: the
        // traversal is strict from the start and its finished rays need no check and no re-trace.
        // (Round 2 checked the finished rays' hits in the trace loop's refill block instead, which
        // loaded each hit triangle again and stalled the block: +3.3 % Lambert)
        if (__ballot(hit)) {  // wave-uniform
            const f3 inv = mk(__shfl(s.inv.x, owner, 64), __shfl(s.inv.y, owner, 64), __shfl(s.inv.z, owner, 64));
            const f3 io = mk(__shfl(s.io.x, owner, 64), __shfl(s.io.y, owner, 64), __shfl(s.io.z, owner, 64));
            if (hit) hit = tri_accept(A, E1, E2, inv, io, t);
        }
        // t >= tmin = 0: with the sign bit cleared (t = -0), its bits order as an unsigned integer
        const unsigned long long key =
            ((unsigned long long)(__float_as_uint(t) & 0x7fffffffu) << 32) | (unsigned long long)(uint32_t)oi;
        if (hit) atomicMin(&L->key[owner], key);
        __builtin_amdgcn_wave_barrier();
        if (hit && L->key[owner] == key)  // the owner's winning pair (a triangle is in one leaf only)
        {
            L->res_uv[owner] = make_float2(u, v);
            L->res_code[owner] = ti | (bk ? (int)0x80000000 : 0);
        }
        __builtin_amdgcn_wave_barrier();
        const unsigned long long w = L->key[lane];
        if (w != ~0ull) {
            const float tw = __uint_as_float((uint32_t)(w >> 32));
            const int ow = (int)(uint32_t)w;
            const float2 ruv = L->res_uv[lane];
            const float4 r = make_float4(ruv.x, ruv.y, __int_as_float(L->res_code[lane]), 0.0f);
            const int code = __float_as_int(r.z);
            if (flags & 2) {  // (this lane's own kind) any hit: done; only h.tri (the record's other fields carry the path)
                s.h.tri = code & 0x7fffffff;
                s.path = __float_as_int(tw);
            } else if (tw < s.best || (tw == s.best && ow < s.h.orig)) {
                s.best = tw;
                s.h.t = tw;
                s.h.u = r.x;
                s.h.v = r.y;
                s.h.tri = code & 0x7fffffff;
                s.h.back = code < 0;
                s.h.orig = ow;
            }
            L->key[lane] = ~0ull;
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// The node half and hand-off of trav_step (the wavefront loop tests triangles in wave batches).
template <int ANY, bool STATS, int DEPTH>
__device__ __forceinline__ bool trav_node_step(const DevScene& S, TravState& s, int* __restrict__ stk, int stride,
                                               int* spill, TravStats& ts) {
    if (s.cur >= 0) {
        if (STATS) {
            ts.nodes++;
            ts.lds_nodes += s.cur < S.n_lds;
        }
        float t0, t1, t2, t3;
        int c0, c1, c2, c3;
        const NodeLoad nl = node_load(S, s, s.cur);
#if PT_CYCLE_PROBE
        if (STATS) ts.probe_t = probe_clock(nl.ch.x);
#endif
        node_eval(nl, s, t0, t1, t2, t3, c0, c1, c2, c3);
        if (ANY != kRayAny) {
            cswap(t0, c0, t1, c1);
            cswap(t2, c2, t3, c3);
            cswap(t0, c0, t2, c2);
            cswap(t1, c1, t3, c3);
            cswap(t1, c1, t2, c2);
        }
        if (s.sp > DEPTH - 3) stack_spill<DEPTH, STATS>(s, stk, stride, spill, ts);
        {
            int sp = s.sp;
            stk[sp * stride] = c3;
            sp += c3 != kEmptyChild;
            stk[sp * stride] = c2;
            sp += c2 != kEmptyChild;
            stk[sp * stride] = c1;
            sp += c1 != kEmptyChild;
            s.sp = sp;
        }
        s.cur = c0;
    }
    if (s.cur == kEmptyChild) stack_pop<DEPTH>(s, stk, stride, spill);
    if (s.cur < 0 && s.cur != kEmptyChild && s.leaf == kEmptyChild) {
        s.leaf = s.cur;
        stack_pop<DEPTH>(s, stk, stride, spill);
    }
    return s.cur == kEmptyChild && s.leaf == kEmptyChild;
}

// Per-lane traversals (trav_step: the megakernel and k_trace; the wavefront's triangle batches
// are strict throughout): a finished traversal's answer stands unless its hit is not acceptable
// (tri_accept) -- then the ray is traced again in strict mode.  If the final hit is acceptable it IS the minimum
// over the acceptable hits: every acceptable hit ordered before it had t <= best throughout,
// so its boxes were never culled and it was tested and taken.  It runs once per finished ray,
// on the hit's t kept by the traversal and the hit triangle's record (A, E1, E2).
template <int ANY>
__device__ __forceinline__ bool trav_hit_acceptable(const TravState& s, const float4 A, const float4 E1,
                                                    const float4 E2) {
    const float t = is_any<ANY>(s) ? __int_as_float(s.path) : s.h.t;
    return tri_accept(A, E1, E2, s.inv, s.io, t);
}
template <int ANY, bool TEX>
__device__ __forceinline__ bool trav_result_ok(const DevScene& S, const TravState& s) {
    if (s.strict || s.h.tri < 0) return true;
    const int ti = s.h.tri;
    return trav_hit_acceptable<ANY>(s, S.isect[3 * ti], S.isect[3 * ti + 1], S.isect[3 * ti + 2]);
}

// Trace the ray again from the root, taking acceptable hits only.  Closest-hit lanes restart
// from tmax_closest; any-hit lanes keep their tmax (best never shrinks for them) and their
// carried fields.
template <int ANY>
__device__ __forceinline__ void trav_restart_strict(TravState& s, float tmax_closest) {
    s.cur = 0;
    s.sp = 0;
    s.spc = 0;
    s.leaf = kEmptyChild;
    s.strict = true;
    s.h.tri = -1;
    if (!is_any<ANY>(s)) {
        s.best = tmax_closest;
        s.h.orig = 0x7fffffff;
    }
}

// Whole traversal of one ray (megakernel, k_trace).
template <int ANY, bool STATS, int DEPTH, bool TEX>
__device__ __forceinline__ bool traverse(const DevScene& S, f3 o, f3 d, float tmin, float tmax, Hit& h,
                                         int* __restrict__ stk, int stride, TravStats& ts) {
    if (STATS) ts.rays++;
    TravState s;
    trav_init(s, o, d, tmin, tmax);
    if (S.ntri > 0) {
        int spill[kSpillDepth];
        while (true) {
            while (!trav_step<ANY, STATS, DEPTH, TEX>(S, s, stk, stride, spill, ts)) {
            }
            if (trav_result_ok<ANY, TEX>(S, s)) break;
            if (STATS) ts.retrace++;
            trav_restart_strict<ANY>(s, tmax);
        }
    }
    h = s.h;
    return s.h.tri >= 0;
}

// devicePrograms.cu:601-623 — pixel-centre primary ray (y: the launch's row, row0 + y the image's).
__device__ __forceinline__ void camera_ray(const DevLaunch& L, int x, int y, f3& o, f3& d) {
    float xs = ((float)x + 0.5f) / (float)L.width;
    float ys = ((float)(y + L.row0) + 0.5f) / (float)L.image_height;
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
// back-face flip (:379-382), SampleTextures + normal mapping (:392-409), BuildTangentSpace
// (:168-212).  The texture ids are used as given (the reference's hasNormalTexture /
// hasMetalRoughTexture = HasAlbedoTex() flag bug, OptixRenderer.cpp:535,540, is not kept).
struct SurfaceHit {
    f3 pos, ng;
    Frame fr;
    f3 wo;        // shading space
    f3 albedo;
    float metallic, roughness;
};

__device__ __forceinline__ void apply_textures(const DevScene& S, int ti, float u, float v, const float4 M1,
                                               const float4 M2, f3& albedo, float& metallic, float& roughness,
                                               f3& Ns) {
    const int at = __float_as_int(M1.z), nt = __float_as_int(M1.w), mt = __float_as_int(M2.x);
    float x, y;
    tri_texcoord(S, ti, u, v, x, y);
    f3 ntex = mk(0.0f, 0.0f, 0.0f);
    if (at >= 0) {
        const float4 c = tex_sample(S, at, x, y, true);
        albedo = albedo * mk(c.x, c.y, c.z);
    }
    if (nt >= 0) {
        const float4 c = tex_sample(S, nt, x, y, false);
        ntex = mk(c.x, c.y, c.z);
    }
    if (mt >= 0) {
        const float4 c = tex_sample(S, mt, x, y, false);
        metallic = c.x;
        roughness = c.y;
    }
    if (ntex.x != 0.0f || ntex.y != 0.0f || ntex.z != 0.0f) {  // normal mapping in the a8 frame of Ns
        f3 d1 = cross(Ns, mk(0.0f, 0.0f, 1.0f));
        f3 d2 = cross(Ns, mk(0.0f, 1.0f, 0.0f));
        f3 T0 = (length(d1) > length(d2)) ? d1 : d2;
        T0 = normalize(T0);
        const f3 B0 = cross(T0, Ns);
        const f3 tn = mk(ntex.x * 2.0f - 1.0f, ntex.y * 2.0f - 1.0f, ntex.z * 2.0f - 1.0f);
        Ns = normalize(mk((T0.x * tn.x + B0.x * tn.y) + Ns.x * tn.z, (T0.y * tn.x + B0.y * tn.y) + Ns.y * tn.z,
                          (T0.z * tn.x + B0.z * tn.y) + Ns.z * tn.z));
    }
}

// TEX: the scene has textures (kernels are instantiated both ways so untextured scenes keep
// the texture code out of their register budget).
template <bool TEX>
__device__ __forceinline__ void reconstruct(const DevScene& S, const Hit& h, f3 d, SurfaceHit& s) {
    const int ti = h.tri;
    const float4 A = S.isect[3 * ti];
    const float4 S0 = S.shade[4 * ti], S1 = S.shade[4 * ti + 1], S2 = S.shade[4 * ti + 2], S3 = S.shade[4 * ti + 3];
    // the edges again from the vertices: e = v - v0 is the one fp32 subtraction k_gather stored in
    // isect, so Ng is bit-identical, and the hit costs five gathers instead of seven
    const float4 E1 = make_float4(S0.x - A.x, S0.y - A.y, S0.z - A.z, 0.0f);
    const float4 E2 = make_float4(S1.x - A.x, S1.y - A.y, S1.z - A.z, 0.0f);
    const int mi = __float_as_int(S3.w);
    const float4 M0 = S.mats[kMatStride * mi], M1 = S.mats[kMatStride * mi + 1];
    f3 wo_w = normalize(-d);
    f3 v0 = mk(A.x, A.y, A.z), v1 = mk(S0.x, S0.y, S0.z), v2 = mk(S1.x, S1.y, S1.z);
    f3 n0 = mk(S0.w, S1.w, S2.x), n1 = mk(S2.y, S2.z, S2.w), n2 = mk(S3.x, S3.y, S3.z);
    f3 Ng = cross(mk(E1.x, E1.y, E1.z), mk(E2.x, E2.y, E2.z));
    const float u = h.u, v = h.v;
    float w = 1.0f - u - v;
    f3 Ns = mk(w * n0.x + u * n1.x + v * n2.x, w * n0.y + u * n1.y + v * n2.y, w * n0.z + u * n1.z + v * n2.z);
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
    s.albedo = mk(M0.x, M0.y, M0.z);
    s.metallic = M0.w;
    s.roughness = M1.x;
    if (TEX) {
        const float4 M2 = S.mats[kMatStride * mi + 2];
        if (M2.y != 0.0f) apply_textures(S, ti, u, v, M1, M2, s.albedo, s.metallic, s.roughness, Ns);
    }
    f3 c1 = cross(Ns, mk(0.0f, 0.0f, 1.0f));
    f3 c2 = cross(Ns, mk(0.0f, 1.0f, 0.0f));
    f3 T = (length(c1) > length(c2)) ? c1 : c2;
    T = normalize(T);
    s.fr.t = T;
    s.fr.b = cross(T, Ns);
    s.fr.n = Ns;
    s.wo = to_local(s.fr, wo_w);
}

// Path state of one camera sample (RadianceRayData, RayData.h:5-21).
struct PathState {
    f3 o, d, beta, radiance;
    uint32_t seed;
    int bounce;
    bool end;
};

__device__ __forceinline__ void path_start(PathState& p, f3 o, f3 d, uint32_t seed) {  // SamplePath :626-635
    p.o = o;
    p.d = d;
    p.beta = mk(1.0f, 1.0f, 1.0f);
    p.radiance = mk(0.0f, 0.0f, 0.0f);
    p.seed = seed;
    p.bounce = 0;
    p.end = false;
}

// The reference's debug print of one bounce of the debug path (devicePrograms.cu:428-437:
// position, albedo, shading and geometry normal, roughness, metallic, at bounceCounter), plus
// the hit triangle's global index, the throughput entering the bounce and the radiance so far.
// Record layout: ptamd.h pt_debug_bounce.
__device__ __forceinline__ void debug_record(const DevLaunch& L, int bounce, int prim, const SurfaceHit& sf, f3 beta,
                                             f3 radiance) {
    if (bounce < 1 || bounce > kDebugMaxBounces) return;
    float* r = L.debug + (size_t)(bounce - 1) * kDebugRecordFloats;
    const float v[kDebugRecordFloats] = {__int_as_float(bounce), __int_as_float(prim),
                                         sf.pos.x, sf.pos.y, sf.pos.z, sf.albedo.x, sf.albedo.y, sf.albedo.z,
                                         sf.fr.n.x, sf.fr.n.y, sf.fr.n.z, sf.ng.x, sf.ng.y, sf.ng.z,
                                         sf.roughness, sf.metallic, beta.x, beta.y, beta.z,
                                         radiance.x, radiance.y, radiance.z};
    for (int k = 0; k < kDebugRecordFloats; ++k) r[k] = v[k];
}

// loop test of SamplePath (devicePrograms.cu:646)
__device__ __forceinline__ bool path_alive(const DevLaunch& L, const PathState& p) {
    return !p.end && p.bounce < L.max_bounces && length(p.beta) > 0.00001f;
}

// One iteration of SamplePath's loop: TraceRadiance + __closesthit__radiance
// (devicePrograms.cu:343-514) or __miss__radiance (:576-583).  Returns false on a miss.
template <int MODE, bool STATS, int DEPTH, bool TEX>
__device__ __forceinline__ void path_segment(const DevScene& S, const DevLaunch& L, PathState& p, int* stk,
                                             int stride, TravStats& ts, bool debug_path) {
    Hit h;
    bool hit = traverse<false, STATS, DEPTH, TEX>(S, p.o, p.d, 0.0f, 100.0f, h, stk, stride, ts);
    if (!hit) {
        p.beta = mk(0, 0, 0);
        p.bounce = 100;
        return;
    }
    p.bounce++;
    if (p.bounce > L.max_bounces) {
        p.end = true;
        return;
    }
    SurfaceHit sf;
    reconstruct<TEX>(S, h, p.d, sf);
    if (debug_path) debug_record(L, p.bounce, __float_as_int(S.isect[3 * h.tri].w), sf, p.beta, p.radiance);
    const bool conductor = rnd(p.seed) < sf.metallic;  // :400
    // NEE (:446-472), Lighting::GetRandomPointLight (LightMethods.h:25-40)
    float P = 0.0f;
    int li = 0;
    if (L.n_lights == 1) {
        P = 1.0f;
    } else if (L.n_lights > 1) {
        float r = rnd(p.seed);
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
        bool occluded = traverse<true, STATS, DEPTH, TEX>(S, so, normalize(ldir), 0.0f, length(ldir), sh, stk, stride, ts);
        f3 lds = to_local(sf.fr, ldn);
        if (!occluded) {
            f3 f = bsdf_f<MODE>(p.seed, sf.albedo, sf.roughness, conductor, sf.wo, lds);
            float c = abs_dot(lds, mk(0.0f, 0.0f, 1.0f));
            f3 spectrum = f * c;
            if (!is_zero(spectrum)) {
                f3 dd = sf.pos - lpos;
                float d2 = dd.x * dd.x + dd.y * dd.y + dd.z * dd.z;
                f3 Li = mk(lt.cr, lt.cg, lt.cb) / d2;
                p.radiance = p.radiance + ((p.beta * spectrum) * Li) / (P * 1.0f);
            }
        }
    }
    BSample bs;
    // the last segment's sampled direction is never traced (SamplePath's loop test, :646):
    // skipping the sample leaves every traced value unchanged
    if (p.bounce >= L.max_bounces) {
        p.end = true;
        return;
    }
    if (!bsdf_sample<MODE>(p.seed, sf.albedo, sf.roughness, conductor, sf.wo, bs)) {
        p.end = true;
        return;
    }
    float ac = abs_dot(bs.dir, mk(0.0f, 0.0f, 1.0f));
    p.beta = p.beta * mk(bs.color.x * ac / bs.pdf, bs.color.y * ac / bs.pdf, bs.color.z * ac / bs.pdf);
    f3 off = 1e-3f * sf.ng;
    if (dot(bs.dir, mk(0.0f, 0.0f, 1.0f)) < 0.0f) off = -off;
    p.o = sf.pos + off;
    p.d = normalize(to_world(sf.fr, bs.dir));
}

}  // namespace pt
