// pt_trace_group.h — BVH4 traversal with a group of lanes per ray, for the wavefront trace
// kernels (PT_TRACE_GROUP = 4; the default per-lane loop is trace_range in pt_wavefront.hip).
//
// Why.  A node visit of the per-lane traversal (node_load, pt_device.h) is seven 16-B loads per
// lane from one 128-B line.  A wave whose 64 lanes sit on different nodes touches 64 lines per
// load instruction, and the CU's texture data path pays about one cycle per distinct line
// (tools/td_probe.hip); in k_trace_pair TA / TD are 81 / 94 % busy (DESIGN.md §4 "Roofline").
// Here the four lanes of a ray's group each load ONE child of the node (32 B, two 16-B loads)
// from a child-major copy of the BVH, so a visit touches one line per group: two load
// instructions per wave, 16 lines each, instead of seven of up to 64.  A leaf's <= 4 triangles
// are tested one per lane, and each lane checks its own hit against its own ray (no cross-lane
// ray fetches as in wave_tri_batch).  The price: a wave carries 16 rays instead of 64, so the
// per-ray control work (stack, refill) is replicated over the group's lanes.
//
// Same answers bit for bit.  Each child's slab distances are node_eval's expressions (the
// sign-selected planes, the same fma / fmaxf / fminf nesting and widening); the triangle test
// and the acceptance rule are tri_test / tri_accept; the closest hit is the (t, original index)
// minimum over acceptable hits, which does not depend on the order the nodes are visited in
// (DESIGN.md §2); an any-hit ray is occluded iff an acceptable hit exists.  The children are
// ordered near to far as in trav_node_step (ties by child slot), so the tree is walked in the
// same order as the per-lane traversal.
#pragma once
#include <algorithm>
#include <type_traits>

#include "pt_device.h"

namespace pt {

#ifndef PT_TRACE_GROUP
#define PT_TRACE_GROUP 1
#endif
constexpr int kTraceGroup = PT_TRACE_GROUP;
static_assert(kTraceGroup == 1 || kTraceGroup == 4, "PT_TRACE_GROUP: 1 (one ray per lane) or 4 (lane groups)");

// LDS stack entries per ray.  The group traversal has no spill path, so its stack holds every
// stack a BVH accepted by pt_create can need (3 entries per BVH4 level, kMinTraversalStack).
constexpr int kGrpStack = 72;
static_assert(kGrpStack >= std::min(stack_capacity(PT_WF_STACK), stack_capacity(PT_MK_STACK)),
              "the group stack must hold the deepest BVH pt_create accepts");

// Idle groups before a wave refills, and groups holding a leaf before it runs its triangle step
// (the per-lane loop's PT_REFILL_MIN = 16 and PT_TRI_BATCH = 20 lanes, in groups of four).
#ifndef PT_GRP_REFILL
#define PT_GRP_REFILL 4
#endif
#ifndef PT_GRP_TRI
#define PT_GRP_TRI 5
#endif

// quad_perm DPP controls: the lane of the quad at index (lane ^ 1), (lane ^ 2), (lane ^ 3)
constexpr int kDppX1 = 0xB1, kDppX2 = 0x4E, kDppX3 = 0x1B;
template <int CTRL>
__device__ __forceinline__ int qperm(int v) {
    return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint32_t qperm(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float qperm(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}

// Child-major copy of the first K nodes into the workgroup's LDS (every thread calls it).
template <int K>
__device__ __forceinline__ void stage_top_cm(DevScene& S, float4* top) {
    const int n = K > 0 ? min(S.n_nodes, K) : 0;
    for (int i = (int)threadIdx.x; i < n * 8; i += (int)blockDim.x) top[i] = S.nodes_cm[i];
    __syncthreads();
    S.lds_cm = top;
    S.n_lds = n;
}

__device__ __forceinline__ void grp_pop(TravState& s, const int* __restrict__ stk, int stride) {
    const int sp = s.sp - 1;
    const int e = stk[max(sp, 0) * stride];
    s.cur = sp >= 0 ? e : kEmptyChild;
    s.sp = max(sp, 0);
}

// Node half of a group step: lane gc tests child gc of s.cur, the group ranks its hits near to
// far, the nearest becomes s.cur and the others go on the ray's stack (farthest deepest); then
// the hand-off of trav_node_step.  Called by all four lanes of a group together.  True when the
// ray has nothing left to visit.
template <bool STATS>
__device__ __forceinline__ bool grp_node_step(const DevScene& S, TravState& s, int* __restrict__ stk, int stride,
                                              int gc, TravStats& ts) {
    if (s.cur >= 0) {
        const int ni = s.cur;
        if (STATS && gc == 0) {
            ts.nodes++;
            ts.lds_nodes += ni < S.n_lds;
        }
        float4 A, B;
        if (ni < S.n_lds) {
            const float4* p = S.lds_cm + ni * 8 + gc * 2;
            A = p[0];
            B = p[1];
        } else {
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void*)S.nodes_cm, 0, 0x7fffffff, 0x00020000);
            const int off = (ni << 7) + (gc << 5);
            A = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
            B = __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16, 0, 0));
        }
        const int link = __float_as_int(A.w);
        // node_eval's arithmetic for one child: near / far plane by the direction's sign
        const float nx = __fmaf_rn(s.nx ? B.x : A.x, s.inv.x, -s.io.x), fx = __fmaf_rn(s.nx ? A.x : B.x, s.inv.x, -s.io.x);
        const float ny = __fmaf_rn(s.ny ? B.y : A.y, s.inv.y, -s.io.y), fy = __fmaf_rn(s.ny ? A.y : B.y, s.inv.y, -s.io.y);
        const float nz = __fmaf_rn(s.nz ? B.z : A.z, s.inv.z, -s.io.z), fz = __fmaf_rn(s.nz ? A.z : B.z, s.inv.z, -s.io.z);
        const float tn = fmaxf(fmaxf(nx, ny), fmaxf(nz, s.tmin));
        const float tf = fminf(fminf(fx, fy), fminf(fz, s.best)) * kSlabWiden;
        const bool hit = tn <= tf;  // empty slots hold inverted boxes: never
        const float tk = hit ? tn : __int_as_float(0x7f800000);
        // rank among the group's children: nearer ones, ties by slot (lane gc ^ m precedes gc
        // iff that lane index is smaller)
        const float t1 = qperm<kDppX1>(tk), t2 = qperm<kDppX2>(tk), t3 = qperm<kDppX3>(tk);
        const int rank = (int)((t1 < tk) | ((t1 == tk) & ((gc & 1) != 0))) +
                         (int)((t2 < tk) | ((t2 == tk) & ((gc & 2) != 0))) +
                         (int)((t3 < tk) | ((t3 == tk) & ((gc & 2) != 0)));
        int nh = hit ? 1 : 0;
        nh += qperm<kDppX1>(nh);
        nh += qperm<kDppX2>(nh);
        int near = (hit && rank == 0) ? link : 0;  // exactly one lane contributes when nh > 0
        near += qperm<kDppX1>(near);
        near += qperm<kDppX2>(near);
        if (hit && rank > 0) stk[(s.sp + nh - 1 - rank) * stride] = link;
        s.sp += max(nh - 1, 0);
        s.cur = nh > 0 ? near : kEmptyChild;
    }
    if (s.cur == kEmptyChild) grp_pop(s, stk, stride);
    if (s.cur < 0 && s.cur != kEmptyChild && s.leaf == kEmptyChild) {
        s.leaf = s.cur;
        grp_pop(s, stk, stride);
    }
    return s.cur == kEmptyChild && s.leaf == kEmptyChild;
}

// One round of the group minimum of (key hi, key lo) carrying the winner's u, v and code.
template <int CTRL>
__device__ __forceinline__ void grp_min_round(uint32_t& khi, uint32_t& klo, float& u, float& v, int& code) {
    const uint32_t ohi = qperm<CTRL>(khi), olo = qperm<CTRL>(klo);
    const float ou = qperm<CTRL>(u), ov = qperm<CTRL>(v);
    const int oc = qperm<CTRL>(code);
    const bool take = ohi < khi || (ohi == khi && olo < klo);
    khi = take ? ohi : khi;
    klo = take ? olo : klo;
    u = take ? ou : u;
    v = take ? ov : v;
    code = take ? oc : code;
}

// Triangle half of a group step (the group's ray holds a pending leaf): lane gc tests triangle
// gc of the leaf against its own copy of the ray and holds a hit to the acceptance rule; the
// group takes the (t, original index) minimum, which the ray then takes by the closest-hit rule
// of wave_tri_batch (any-hit rays: any acceptable hit ends them).
template <int ANY, bool STATS, bool TEX>
__device__ __forceinline__ void grp_tri_step(const DevScene& S, TravState& s, int gc, TravStats& ts) {
    const int cnt = leaf_count(s.leaf), first = leaf_first(s.leaf);
    const bool valid = gc < cnt;
    const int ti = first + min(gc, cnt - 1);  // lanes past the leaf repeat its last triangle
    if (STATS) ts.tris += valid;
    const float4 A = S.isect[3 * ti], E1 = S.isect[3 * ti + 1], E2 = S.isect[3 * ti + 2];
    float t, u, v;
    bool bk = false;
    bool hit = tri_test(A, E1, E2, s.o, s.d, 0.0f, s.best, t, u, v, bk) && valid;
    if (TEX && hit && __float_as_int(E2.w) != 0) hit = !alpha_cut(S, ti, __float_as_int(E1.w), u, v);
    if (hit) hit = tri_accept(A, E1, E2, s.inv, s.io, t);
    // key (t bits | original index): t >= 0, so with the sign cleared (t = -0) it orders as an integer
    uint32_t khi = hit ? (__float_as_uint(t) & 0x7fffffffu) : 0xffffffffu;
    uint32_t klo = hit ? __float_as_uint(A.w) : 0xffffffffu;
    int code = ti | (bk ? (int)0x80000000 : 0);
    grp_min_round<kDppX1>(khi, klo, u, v, code);
    grp_min_round<kDppX2>(khi, klo, u, v, code);
    s.leaf = kEmptyChild;
    if ((khi & klo) != 0xffffffffu) {
        const float tw = __uint_as_float(khi);
        const int ow = (int)klo;
        if (is_any<ANY>(s)) {  // only h.tri (the record's other fields carry the path)
            s.h.tri = code & 0x7fffffff;
            s.path = __float_as_int(tw);
        } else if (tw < s.best || (tw == s.best && ow < s.h.orig)) {
            s.best = tw;
            s.h.t = tw;
            s.h.u = u;
            s.h.v = v;
            s.h.tri = code & 0x7fffffff;
            s.h.back = code < 0;
            s.h.orig = ow;
        }
    }
}

}  // namespace pt
