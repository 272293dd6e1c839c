// pt_build.hip — BVH construction on gfx950 (replaces optixAccelBuild + compaction,
// Renderer/OptiX/OptixRenderer.cpp:306-456 of Damo12320/OptixPathtracer).
//
//   1. k_morton   : per triangle AABB centroid -> 30-bit Morton key (10 bits/axis)
//   2. radix sort : (key, triangle) pairs, hipCUB device radix sort
//   3. k_gather   : triangle records into leaf order (isect: v0,e1,e2; shade: v1,v2,normals);
//                   level 0 of an AABB sparse table over the sorted leaves
//   4. k_sparse   : sparse-table level l = union of two level l-1 boxes (log2 N launches)
//   5. k_karras   : binary LBVH, one thread per internal node (Karras 2012 split search);
//                   each node's AABB = O(1) sparse-table range query over its leaf range
//   6. SAH-optimal BVH4 collapse: a bottom-up dynamic programme (k_sah_dp) picks every binary
//                   node's cheapest cover by 1-4 BVH4 children, a top-down pass replays it one
//                   BVH4 level at a time (k_collapse_count -> scan -> k_collapse_emit), numbering
//                   the nodes breadth-first by a prefix sum: the node array is the same on every
//                   build (no atomic slot order), and the top levels are a contiguous prefix.
// PLOC builder (Meister & Bittner 2018, "Parallel Locally-Ordered Clustering for Bounding
// Volume Hierarchy Construction"), the default: starting from the Morton-sorted leaves, each
// iteration finds every cluster's nearest neighbour (smallest merged surface area) within
// +-kPlocRadius positions, merges mutual pairs and compacts (hipCUB scan).  A top-down pass
// then numbers the leaves in depth-first order, so every subtree is again a contiguous
// leaf range, and the same collapse turns it into BVH4.  Its SAH quality is close to a
// full sweep build, which cuts traversal steps against the Karras tree.
// Apart from the DP's bottom-up hand-off, every kernel reads only what earlier launches wrote.
// The build is deterministic: the same scene gives the same node and triangle arrays bit for
// bit (tests/test_gpu_parity.py::test_bvh_build_deterministic).  The sparse
// table costs N*log2(N)*32 B (~150 MB at 250k triangles) — trivial against 288 GB HBM.
#include <hipcub/hipcub.hpp>

#include <vector>

#include "pt_internal.h"

namespace pt {

namespace {

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}

__device__ __forceinline__ void tri_box(const float4* tri, int i, float lo[3], float hi[3]) {
    float4 a = tri[3 * i], b = tri[3 * i + 1], c = tri[3 * i + 2];
    lo[0] = fminf(fminf(a.x, b.x), c.x);
    lo[1] = fminf(fminf(a.y, b.y), c.y);
    lo[2] = fminf(fminf(a.z, b.z), c.z);
    hi[0] = fmaxf(fmaxf(a.x, b.x), c.x);
    hi[1] = fmaxf(fmaxf(a.y, b.y), c.y);
    hi[2] = fmaxf(fmaxf(a.z, b.z), c.z);
}

// The box the traversal's hit-acceptance rule uses for triangle i (pt_device.h tri_accept): the
// vertices as the hit test sees them (v0, v0 + (v1 - v0), v0 + (v2 - v0)), padded.  The boxes
// stored in the BVH4 nodes are exact unions of these (k_sah_dp's refit), so they contain every
// acceptance box bit for bit; the tree itself (PLOC clustering, SAH choices) is built on the
// plain triangle boxes.
__device__ __forceinline__ void tri_box_accept(const float4* tri, int i, float lo[3], float hi[3]) {
    const float4 a = tri[3 * i], b = tri[3 * i + 1], c = tri[3 * i + 2];
    const f3 v0 = mk(a.x, a.y, a.z);
    tri_box_padded(v0, mk(b.x - a.x, b.y - a.y, b.z - a.z), mk(c.x - a.x, c.y - a.y, c.z - a.z), lo, hi);
}

__global__ void k_morton(const float4* tri, int n, float3 cmin, float3 cinv, uint32_t* keys, uint32_t* vals) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float lo[3], hi[3];
    tri_box(tri, i, lo, hi);
    float cx = (0.5f * (lo[0] + hi[0]) - cmin.x) * cinv.x;
    float cy = (0.5f * (lo[1] + hi[1]) - cmin.y) * cinv.y;
    float cz = (0.5f * (lo[2] + hi[2]) - cmin.z) * cinv.z;
    uint32_t qx = (uint32_t)fminf(fmaxf(cx * 1024.0f, 0.0f), 1023.0f);
    uint32_t qy = (uint32_t)fminf(fmaxf(cy * 1024.0f, 0.0f), 1023.0f);
    uint32_t qz = (uint32_t)fminf(fmaxf(cz * 1024.0f, 0.0f), 1023.0f);
    keys[i] = (expand_bits(qx) << 2) | (expand_bits(qy) << 1) | expand_bits(qz);
    vals[i] = (uint32_t)i;
}

// Leaf-order gather.  isect: v0|orig, (v1-v0)|material, (v2-v0)|alpha flag — the edge subtraction
// is the same single fp32 op the oracle performs, so the hit arithmetic stays identical.
// shade: v1|n0.x, v2|n0.y, n0.z n1, n2|material.
__global__ void k_gather(const float4* tri_orig, const float4* nrm_orig, const float4* uv_orig, const uint32_t* order,
                         int n, float4* isect, float4* shade, float4* tuv, float4* st0, float4* pleaf) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int i = (int)order[k];
    const float4 a = tri_orig[3 * i], b = tri_orig[3 * i + 1], c = tri_orig[3 * i + 2];
    const float4 na = nrm_orig[3 * i], nb = nrm_orig[3 * i + 1], nc = nrm_orig[3 * i + 2];
    isect[3 * k] = a;
    isect[3 * k + 1] = make_float4(b.x - a.x, b.y - a.y, b.z - a.z, b.w);
    isect[3 * k + 2] = make_float4(c.x - a.x, c.y - a.y, c.z - a.z, c.w);  // w: alpha-cut-out flag
    if (tuv) {
        tuv[2 * k] = uv_orig[2 * i];
        tuv[2 * k + 1] = uv_orig[2 * i + 1];
    }
    shade[4 * k] = make_float4(b.x, b.y, b.z, na.x);
    shade[4 * k + 1] = make_float4(c.x, c.y, c.z, na.y);
    shade[4 * k + 2] = make_float4(na.z, nb.x, nb.y, nb.z);
    shade[4 * k + 3] = make_float4(nc.x, nc.y, nc.z, b.w);  // w: material (as isect's e1.w) for reconstruct
    float lo[3], hi[3];
    tri_box(tri_orig, i, lo, hi);
    st0[2 * k] = make_float4(lo[0], lo[1], lo[2], 0.0f);
    st0[2 * k + 1] = make_float4(hi[0], hi[1], hi[2], 0.0f);
    tri_box_accept(tri_orig, i, lo, hi);
    pleaf[2 * k] = make_float4(lo[0], lo[1], lo[2], 0.0f);
    pleaf[2 * k + 1] = make_float4(hi[0], hi[1], hi[2], 0.0f);
}

__global__ void k_sparse(const float4* prev, float4* cur, int count, int half) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    float4 a0 = prev[2 * i], a1 = prev[2 * i + 1];
    float4 b0 = prev[2 * (i + half)], b1 = prev[2 * (i + half) + 1];
    cur[2 * i] = make_float4(fminf(a0.x, b0.x), fminf(a0.y, b0.y), fminf(a0.z, b0.z), 0.0f);
    cur[2 * i + 1] = make_float4(fmaxf(a1.x, b1.x), fmaxf(a1.y, b1.y), fmaxf(a1.z, b1.z), 0.0f);
}

struct SparseTable {
    const float4* level[32];
    int n;
};

__device__ __forceinline__ void range_box(const SparseTable& st, int a, int b, float4& lo, float4& hi) {
    int len = b - a + 1;
    int l = 31 - __clz(len);
    const float4* L = st.level[l];
    int c = b - (1 << l) + 1;
    float4 a0 = L[2 * a], a1 = L[2 * a + 1], b0 = L[2 * c], b1 = L[2 * c + 1];
    lo = make_float4(fminf(a0.x, b0.x), fminf(a0.y, b0.y), fminf(a0.z, b0.z), 0.0f);
    hi = make_float4(fmaxf(a1.x, b1.x), fmaxf(a1.y, b1.y), fmaxf(a1.z, b1.z), 0.0f);
}

__device__ __forceinline__ int delta(const uint32_t* keys, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    uint32_t ki = keys[i], kj = keys[j];
    if (ki == kj) return 32 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clz(ki ^ kj);
}

// Binary LBVH node i: child codes (>= 0 internal, < 0 leaf ~k), leaf range, AABB.
__global__ void k_karras(const uint32_t* keys, int n, SparseTable st, int2* bchild, int2* brange, float4* bbox) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n - 1) return;
    int d = (delta(keys, n, i, i + 1) - delta(keys, n, i, i - 1)) >= 0 ? 1 : -1;
    int dmin = delta(keys, n, i, i - d);
    int lmax = 2;
    while (delta(keys, n, i, i + lmax * d) > dmin) lmax *= 2;
    int l = 0;
    for (int t = lmax / 2; t >= 1; t /= 2)
        if (delta(keys, n, i, i + (l + t) * d) > dmin) l += t;
    int j = i + l * d;
    int dnode = delta(keys, n, i, j);
    int s = 0, t = l;
    do {
        t = (t + 1) >> 1;
        if (delta(keys, n, i, i + (s + t) * d) > dnode) s += t;
    } while (t > 1);
    int gamma = i + s * d + (d < 0 ? -1 : 0);
    int first = min(i, j), last = max(i, j);
    int c0 = (first == gamma) ? ~gamma : gamma;
    int c1 = (last == gamma + 1) ? ~(gamma + 1) : (gamma + 1);
    bchild[i] = make_int2(c0, c1);
    brange[i] = make_int2(first, last);
    float4 lo, hi;
    range_box(st, first, last, lo, hi);
    bbox[2 * i] = lo;
    bbox[2 * i + 1] = hi;
}

struct BinTree {
    const int2* child;
    const int2* range;
    const float4* box;  // internal node boxes (2 per node)
    const float4* leafbox;  // sparse table level 0 (2 per leaf)
    const float4* pleaf;  // padded acceptance box per leaf (2 per leaf)
    float4* pbox;         // union of the padded leaf boxes per internal node (k_sah_dp)
};
// Node box for the BVH4: the exact union of the padded acceptance boxes below `code`.
__device__ __forceinline__ void code_box_padded(const BinTree& B, int code, float4& lo, float4& hi) {
    if (code >= 0) {
        lo = B.pbox[2 * code];
        hi = B.pbox[2 * code + 1];
    } else {
        lo = B.pleaf[2 * ~code];
        hi = B.pleaf[2 * ~code + 1];
    }
}

__device__ __forceinline__ void code_box(const BinTree& B, int code, float4& lo, float4& hi) {
    if (code >= 0) {
        lo = B.box[2 * code];
        hi = B.box[2 * code + 1];
    } else {
        lo = B.leafbox[2 * ~code];
        hi = B.leafbox[2 * ~code + 1];
    }
}
__device__ __forceinline__ int code_count(const BinTree& B, int code) {
    if (code < 0) return 1;
    int2 r = B.range[code];
    return r.y - r.x + 1;
}
__device__ __forceinline__ int code_first(const BinTree& B, int code) { return code < 0 ? ~code : B.range[code].x; }
__device__ __forceinline__ float half_area(float4 lo, float4 hi) {
    float x = hi.x - lo.x, y = hi.y - lo.y, z = hi.z - lo.z;
    return x * y + y * z + z * x;
}
// ---- SAH-optimal BVH4 collapse -------------------------------------------------------------
// Bottom-up dynamic programme over the binary tree (the wide-BVH collapse of Ylitie, Karras &
// Laine 2017, "Efficient Incoherent Ray Traversal on GPUs Through Compressed Wide BVHs",
// for 4-wide nodes): cost[n][j] = cheapest SAH cost of covering subtree n with at most j
// BVH4 children, each one a BVH4 node or a leaf of <= kSahLeafMax consecutive triangles:
//   single(n)  = min(A(n) * cTri * count(n)            [leaf, count <= kSahLeafMax],
//                   A(n) * cNode + min_a cost[L][a] + cost[R][4 - a])   [BVH4 node]
//   cost[n][1] = single(n);  cost[n][j] = min(single(n), min_a cost[L][a] + cost[R][j - a])
// The top-down k_collapse_sah then replays the recorded choices.  With the dual traversal
// step (pt_device.h) a triangle test overlaps a node visit, hence cTri < cNode.
#ifndef PT_SAH_LEAF_MAX
#define PT_SAH_LEAF_MAX 4
#endif
#ifndef PT_SAH_CTRI
#define PT_SAH_CTRI 0.5f
#endif
constexpr int kSahLeafMax = PT_SAH_LEAF_MAX;
static_assert(kSahLeafMax >= 1 && kSahLeafMax <= 8, "leaf count is encoded in 3 bits");
constexpr float kSahCNode = 1.0f;
constexpr float kSahCTri = PT_SAH_CTRI;

// Decision word of an internal node: bits 2(j-2)..2(j-2)+1 for j = 2..4 = left pieces a of the
// best split into j (0 = keep single); bits 6..7 = left pieces of the node's own 4-way split;
// bit 8 = single is a leaf.
__device__ __forceinline__ int dp_split(int dec, int j) { return (dec >> (2 * (j - 2))) & 3; }
__device__ __forceinline__ int dp_node_split(int dec) { return (dec >> 6) & 3; }
__device__ __forceinline__ bool dp_is_leaf(int dec) { return (dec >> 8) & 1; }

__global__ void k_parents(const int2* bchild, int nb, int* parent, int* leafparent) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nb) return;
    const int2 c = bchild[i];
    if (c.x >= 0) parent[c.x] = i; else leafparent[~c.x] = i;
    if (c.y >= 0) parent[c.y] = i; else leafparent[~c.y] = i;
}

__device__ __forceinline__ float4 dp_load(const float4* p) {
    const float* f = reinterpret_cast<const float*>(p);
    return make_float4(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load(f + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load(f + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                       __hip_atomic_load(f + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// One thread per triangle walks up; the second child to finish computes the parent (the
// usual bottom-up refit hand-off through a per-node arrival counter).
__global__ void k_sah_dp(BinTree B, int n, const int* parent, const int* leafparent, int* visits, float4* dpc,
                         int* dpd) {
    int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    int node = leafparent[t];
    while (node >= 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        if (atomicAdd(&visits[node], 1) == 0) return;  // the sibling subtree is not done yet
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const int2 ch = B.child[node];
        float cl[5], cr[5];
        float4 plo = make_float4(INFINITY, INFINITY, INFINITY, 0.0f), phi = make_float4(-INFINITY, -INFINITY, -INFINITY, 0.0f);
        const int kids[2] = {ch.x, ch.y};
        for (int k = 0; k < 2; ++k) {
            float* c = k == 0 ? cl : cr;
            const int code = kids[k];
            float4 klo, khi;  // the child's padded box
            if (code < 0) {  // one triangle: always a leaf
                float4 lo = B.leafbox[2 * ~code], hi = B.leafbox[2 * ~code + 1];
                float v = half_area(lo, hi) * kSahCTri;
                c[1] = c[2] = c[3] = c[4] = v;
                klo = B.pleaf[2 * ~code];
                khi = B.pleaf[2 * ~code + 1];
            } else {
                float4 v = dp_load(dpc + code);
                c[1] = v.x; c[2] = v.y; c[3] = v.z; c[4] = v.w;
                klo = dp_load(B.pbox + 2 * code);
                khi = dp_load(B.pbox + 2 * code + 1);
            }
            plo = make_float4(fminf(plo.x, klo.x), fminf(plo.y, klo.y), fminf(plo.z, klo.z), 0.0f);
            phi = make_float4(fmaxf(phi.x, khi.x), fmaxf(phi.y, khi.y), fmaxf(phi.z, khi.z), 0.0f);
        }
        B.pbox[2 * node] = plo;
        B.pbox[2 * node + 1] = phi;
        const float area = half_area(B.box[2 * node], B.box[2 * node + 1]);
        const int2 r = B.range[node];
        const int count = r.y - r.x + 1;
        const float inf = __int_as_float(0x7f800000);
        float best4 = inf;
        int a4 = 1;
        for (int a = 1; a <= 3; ++a) {
            const float v = cl[a] + cr[4 - a];
            if (v < best4) { best4 = v; a4 = a; }
        }
        const float node_cost = area * kSahCNode + best4;
        const float leaf_cost = count <= kSahLeafMax ? area * kSahCTri * (float)count : inf;
        const bool leaf = leaf_cost <= node_cost;
        const float single = leaf ? leaf_cost : node_cost;
        float out[5];
        int dec = (a4 << 6) | (leaf ? 256 : 0);
        out[1] = single;
        for (int j = 2; j <= 4; ++j) {
            float bj = single;
            int aj = 0;
            for (int a = 1; a < j; ++a) {
                const float v = cl[a] + cr[j - a];
                if (v < bj) { bj = v; aj = a; }
            }
            out[j] = bj;
            dec |= aj << (2 * (j - 2));
        }
        dpc[node] = make_float4(out[1], out[2], out[3], out[4]);
        dpd[node] = dec;
        node = parent[node];
    }
}

// Children of one BVH4 node (work item: binary code) from the DP choices, in DFS order of the
// binary tree; returns the count (1..4).
__device__ __forceinline__ int collapse_children(const BinTree& B, const int* dpd, int code, int c[4]) {
    int n = 0;
    if (code < 0) {  // degenerate scene: the root is a single leaf
        c[n++] = code;
        return n;
    }
    int st_code[8], st_j[8], sp = 0;
    const int2 ch = B.child[code];
    const int a = dp_node_split(dpd[code]);
    st_code[sp] = ch.y; st_j[sp++] = 4 - a;
    st_code[sp] = ch.x; st_j[sp++] = a;
    while (sp > 0) {
        --sp;
        const int x = st_code[sp], j = st_j[sp];
        const int s = (x < 0 || j < 2) ? 0 : dp_split(dpd[x], j);
        if (s == 0) {
            c[n++] = x;
        } else {
            const int2 xc = B.child[x];
            st_code[sp] = xc.y; st_j[sp++] = j - s;
            st_code[sp] = xc.x; st_j[sp++] = s;
        }
    }
    return n;
}
__device__ __forceinline__ bool child_is_leaf(const BinTree& B, const int* dpd, int code) {
    return code < 0 || dp_is_leaf(dpd[code]);
}

// Top-down collapse, one BVH4 level per launch pair.  k_collapse_count: inner (non-leaf)
// children per work item; an exclusive scan of the counts gives every inner child its slot
// (level base + offset) and its position in the next level's work list, so the numbering is
// breadth-first and the same on every build.
__global__ void k_collapse_count(BinTree B, const int* dpd, const int* work, int nwork, int* cnt) {
    int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwork) return;
    int c[4];
    const int n = collapse_children(B, dpd, work[w], c);
    int inner = 0;
    for (int k = 0; k < n; ++k) inner += child_is_leaf(B, dpd, c[k]) ? 0 : 1;
    cnt[w] = inner;
}

// k_collapse_emit: node of work item w goes to slot level_base + w (the parent assigned it
// in this order), its inner children to next_base + off[w] + j.
__global__ void k_collapse_emit(BinTree B, const int* dpd, const int* work, int nwork, const int* off,
                                int level_base, int next_base, BNode4* out, int* next) {
    int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwork) return;
    int c[4];
    const int n = collapse_children(B, dpd, work[w], c);
    float lo[3][4], hi[3][4];
    int cc[4];
    int j = off[w];
    for (int k = 0; k < 4; ++k) {
        if (k >= n) {
            cc[k] = kEmptyChild;
            // inverted box: misses for every ray direction (the sign-selected slab test of
            // pt_device.h node_eval relies on it instead of testing the child id)
            for (int a = 0; a < 3; ++a) {
                lo[a][k] = __int_as_float(0x7f800000);
                hi[a][k] = -__int_as_float(0x7f800000);
            }
            continue;
        }
        float4 l4, h4;  // the exact union of the padded acceptance boxes below the child
        code_box_padded(B, c[k], l4, h4);
        lo[0][k] = l4.x; lo[1][k] = l4.y; lo[2][k] = l4.z;
        hi[0][k] = h4.x; hi[1][k] = h4.y; hi[2][k] = h4.z;
        if (child_is_leaf(B, dpd, c[k])) {
            cc[k] = ~((code_first(B, c[k]) << 3) | (code_count(B, c[k]) - 1));
        } else {
            cc[k] = next_base + j;
            next[j] = c[k];
            ++j;
        }
    }
    BNode4 nd;
    nd.lox = make_float4(lo[0][0], lo[0][1], lo[0][2], lo[0][3]);
    nd.hix = make_float4(hi[0][0], hi[0][1], hi[0][2], hi[0][3]);
    nd.loy = make_float4(lo[1][0], lo[1][1], lo[1][2], lo[1][3]);
    nd.hiy = make_float4(hi[1][0], hi[1][1], hi[1][2], hi[1][3]);
    nd.loz = make_float4(lo[2][0], lo[2][1], lo[2][2], lo[2][3]);
    nd.hiz = make_float4(hi[2][0], hi[2][1], hi[2][2], hi[2][3]);
    nd.child = make_int4(cc[0], cc[1], cc[2], cc[3]);
    nd.pad = make_int4(0, 0, 0, 0);
    out[level_base + w] = nd;
}

// ---- PLOC ---------------------------------------------------------------------------------
#ifndef PT_PLOC_RADIUS
#define PT_PLOC_RADIUS 8
#endif
constexpr int kPlocRadius = PT_PLOC_RADIUS;

__device__ __forceinline__ float merged_area(float4 alo, float4 ahi, float4 blo, float4 bhi) {
    float x = fmaxf(ahi.x, bhi.x) - fminf(alo.x, blo.x);
    float y = fmaxf(ahi.y, bhi.y) - fminf(alo.y, blo.y);
    float z = fmaxf(ahi.z, bhi.z) - fminf(alo.z, blo.z);
    return x * y + y * z + z * x;
}

// Leaf boxes in Morton order.
__global__ void k_leafbox(const float4* tri_orig, const uint32_t* order, int n, float4* box, int* code, int* cnt) {
    int m = blockIdx.x * blockDim.x + threadIdx.x;
    if (m >= n) return;
    float lo[3], hi[3];
    tri_box(tri_orig, (int)order[m], lo, hi);
    box[2 * m] = make_float4(lo[0], lo[1], lo[2], 0.0f);
    box[2 * m + 1] = make_float4(hi[0], hi[1], hi[2], 0.0f);
    code[m] = ~m;
    cnt[m] = 1;
}

// Nearest neighbour of every cluster within the window.  Ties go to the lower position,
// which makes the globally best pair mutual (progress every iteration).
__global__ void k_ploc_nn(const float4* box, int n, int* nn) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4 lo = box[2 * i], hi = box[2 * i + 1];
    unsigned long long best = ~0ull;
    const int a = max(0, i - kPlocRadius), b = min(n - 1, i + kPlocRadius);
    for (int j = a; j <= b; ++j) {
        if (j == i) continue;
        float c = merged_area(lo, hi, box[2 * j], box[2 * j + 1]);
        unsigned long long key = ((unsigned long long)__float_as_uint(c) << 32) | (unsigned)j;
        best = key < best ? key : best;
    }
    nn[i] = (int)(best & 0xffffffffu);
}

// flags: low 32 bits = cluster survives, high 32 bits = cluster creates a node.
__global__ void k_ploc_flags(const int* nn, int n, unsigned long long* flags) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int j = nn[i];
    const bool mutual = n > 1 && nn[j] == i;
    const bool keep = !(mutual && i > j);
    const bool merge = mutual && i < j;
    flags[i] = ((unsigned long long)(merge ? 1 : 0) << 32) | (keep ? 1ull : 0ull);
}

__global__ void k_ploc_compact(const float4* box, const int* code, const int* cnt, const int* nn,
                               const unsigned long long* scan, const unsigned long long* flags, int n,
                               int node_base, float4* obox, int* ocode, int* ocnt, int2* bchild, float4* bbox,
                               int* bcount) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long f = flags[i];
    if (!(f & 1ull)) return;
    const unsigned long long sc = scan[i];
    const int pos = (int)(sc & 0xffffffffu);
    float4 lo = box[2 * i], hi = box[2 * i + 1];
    int c = code[i], k = cnt[i];
    if (f >> 32) {
        const int j = nn[i];
        const float4 lj = box[2 * j], hj = box[2 * j + 1];
        lo = make_float4(fminf(lo.x, lj.x), fminf(lo.y, lj.y), fminf(lo.z, lj.z), 0.0f);
        hi = make_float4(fmaxf(hi.x, hj.x), fmaxf(hi.y, hj.y), fmaxf(hi.z, hj.z), 0.0f);
        const int node = node_base + (int)(sc >> 32);
        bchild[node] = make_int2(c, code[j]);
        bbox[2 * node] = lo;
        bbox[2 * node + 1] = hi;
        bcount[node] = k + cnt[j];
        c = node;
        k += cnt[j];
    }
    obox[2 * pos] = lo;
    obox[2 * pos + 1] = hi;
    ocode[pos] = c;
    ocnt[pos] = k;
}

// Depth-first leaf numbering, one launch per tree level: item = (node, first leaf).  Writes
// the node's leaf range, rewrites leaf child codes from Morton positions to DFS positions
// and records the triangle order.
__global__ void k_ploc_dfs(const int2* work, int nwork, int2* bchild, const int* bcount, int2* brange,
                           const uint32_t* morton_order, uint32_t* dfs_order, int2* next, int* nnext) {
    int w = blockIdx.x * blockDim.x + threadIdx.x;
    if (w >= nwork) return;
    const int2 it = work[w];
    const int node = it.x, first = it.y;
    brange[node] = make_int2(first, first + bcount[node] - 1);
    int2 ch = bchild[node];
    int c[2] = {ch.x, ch.y};
    int f = first;
    for (int k = 0; k < 2; ++k) {
        if (c[k] < 0) {
            dfs_order[f] = morton_order[~c[k]];
            c[k] = ~f;
            f += 1;
        } else {
            int q = atomicAdd(nnext, 1);
            next[q] = make_int2(c[k], f);
            f += bcount[c[k]];
        }
    }
    bchild[node] = make_int2(c[0], c[1]);
}

inline unsigned grid_for(int n, int b) { return (unsigned)((n + b - 1) / b); }

__global__ void k_ploc_total(const unsigned long long* scan, const unsigned long long* flags, int n, int* out) {
    const unsigned long long t = scan[n - 1] + flags[n - 1];
    out[0] = (int)(t & 0xffffffffu);  // surviving clusters
    out[1] = (int)(t >> 32);          // nodes created
}

// Host sequencing of the PLOC iterations and the DFS numbering; fills B, the triangle
// records in DFS leaf order and the binary root code.  One host sync per iteration / level
// (the loop bounds come from device counts); allocations are appended to `owned`.
hipError_t ploc_build(const BuildInput& in, const uint32_t* morton_order, BuildOutput& out, hipStream_t stream,
                      BinTree& B, int& root, std::vector<void*>& owned) {
    const int n = in.n;
    hipError_t err = hipSuccess;
    auto alloc = [&](void** p, size_t bytes) {
        if (err == hipSuccess) err = hipMalloc(p, bytes > 0 ? bytes : 16);
        if (err == hipSuccess) owned.push_back(*p);
    };
    const int nb = n > 1 ? n - 1 : 1;
    float4 *box[2] = {nullptr, nullptr}, *bbox = nullptr, *leafbox = nullptr, *pleaf = nullptr;
    int *code[2] = {nullptr, nullptr}, *ccnt[2] = {nullptr, nullptr}, *nn = nullptr, *bcount = nullptr,
        *tot = nullptr;
    unsigned long long *flags = nullptr, *scan = nullptr;
    int2 *bchild = nullptr, *brange = nullptr, *work[2] = {nullptr, nullptr};
    uint32_t* dfs = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    for (int k = 0; k < 2; ++k) {
        alloc((void**)&box[k], sizeof(float4) * 2 * (size_t)n);
        alloc((void**)&code[k], sizeof(int) * (size_t)n);
        alloc((void**)&ccnt[k], sizeof(int) * (size_t)n);
        alloc((void**)&work[k], sizeof(int2) * (size_t)n);
    }
    alloc((void**)&nn, sizeof(int) * (size_t)n);
    alloc((void**)&flags, sizeof(unsigned long long) * (size_t)n);
    alloc((void**)&scan, sizeof(unsigned long long) * (size_t)n);
    alloc((void**)&bchild, sizeof(int2) * (size_t)nb);
    alloc((void**)&brange, sizeof(int2) * (size_t)nb);
    alloc((void**)&bbox, sizeof(float4) * 2 * (size_t)nb);
    alloc((void**)&bcount, sizeof(int) * (size_t)nb);
    alloc((void**)&leafbox, sizeof(float4) * 2 * (size_t)n);
    alloc((void**)&pleaf, sizeof(float4) * 2 * (size_t)n);
    alloc((void**)&dfs, sizeof(uint32_t) * (size_t)n);
    alloc((void**)&tot, sizeof(int) * 2);
    if (err != hipSuccess) return err;
    if ((err = hipcub::DeviceScan::ExclusiveSum(nullptr, temp_bytes, flags, scan, n, stream)) != hipSuccess)
        return err;
    alloc(&temp, temp_bytes);
    if (err != hipSuccess) return err;
    hipLaunchKernelGGL(k_leafbox, dim3(grid_for(n, 256)), dim3(256), 0, stream, in.tri_orig, morton_order, n, box[0],
                       code[0], ccnt[0]);
    if ((err = hipGetLastError()) != hipSuccess) return err;
    int cur = 0, m = n, node_base = 0;
    while (m > 1) {
        hipLaunchKernelGGL(k_ploc_nn, dim3(grid_for(m, 256)), dim3(256), 0, stream, box[cur], m, nn);
        hipLaunchKernelGGL(k_ploc_flags, dim3(grid_for(m, 256)), dim3(256), 0, stream, nn, m, flags);
        if ((err = hipGetLastError()) != hipSuccess) return err;
        if ((err = hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, flags, scan, m, stream)) != hipSuccess)
            return err;
        hipLaunchKernelGGL(k_ploc_compact, dim3(grid_for(m, 256)), dim3(256), 0, stream, box[cur], code[cur],
                           ccnt[cur], nn, scan, flags, m, node_base, box[cur ^ 1], code[cur ^ 1], ccnt[cur ^ 1],
                           bchild, bbox, bcount);
        hipLaunchKernelGGL(k_ploc_total, dim3(1), dim3(1), 0, stream, scan, flags, m, tot);
        if ((err = hipGetLastError()) != hipSuccess) return err;
        int h[2] = {0, 0};
        if ((err = hipMemcpyAsync(h, tot, sizeof h, hipMemcpyDeviceToHost, stream)) != hipSuccess) return err;
        if ((err = hipStreamSynchronize(stream)) != hipSuccess) return err;
        if (h[1] <= 0) return hipErrorUnknown;  // cannot happen: the best pair is always mutual
        m = h[0];
        node_base += h[1];
        cur ^= 1;
    }
    int rc = ~0;
    if ((err = hipMemcpyAsync(&rc, code[cur], sizeof(int), hipMemcpyDeviceToHost, stream)) != hipSuccess) return err;
    if ((err = hipStreamSynchronize(stream)) != hipSuccess) return err;
    root = rc;
    if (rc < 0) {  // single triangle
        if ((err = hipMemcpyAsync(dfs, morton_order, sizeof(uint32_t), hipMemcpyDeviceToDevice, stream)) !=
            hipSuccess)
            return err;
        root = ~0;
    } else {
        int2 w0 = make_int2(rc, 0);
        int nwork = 1, c = 0;
        int* nnext = tot;
        if ((err = hipMemcpyAsync(work[0], &w0, sizeof(int2), hipMemcpyHostToDevice, stream)) != hipSuccess)
            return err;
        while (nwork > 0) {
            if ((err = hipMemsetAsync(nnext, 0, sizeof(int), stream)) != hipSuccess) return err;
            hipLaunchKernelGGL(k_ploc_dfs, dim3(grid_for(nwork, 128)), dim3(128), 0, stream, work[c], nwork, bchild,
                               bcount, brange, morton_order, dfs, work[c ^ 1], nnext);
            if ((err = hipGetLastError()) != hipSuccess) return err;
            if ((err = hipMemcpyAsync(&nwork, nnext, sizeof(int), hipMemcpyDeviceToHost, stream)) != hipSuccess)
                return err;
            if ((err = hipStreamSynchronize(stream)) != hipSuccess) return err;
            c ^= 1;
        }
    }
    hipLaunchKernelGGL(k_gather, dim3(grid_for(n, 256)), dim3(256), 0, stream, in.tri_orig, in.nrm_orig, in.uv_orig, dfs,
                       n, out.isect, out.shade, out.tuv, leafbox, pleaf);
    if ((err = hipGetLastError()) != hipSuccess) return err;
    B.child = bchild;
    B.range = brange;
    B.box = bbox;
    B.leafbox = leafbox;
    B.pleaf = pleaf;
    return hipSuccess;
}

}  // namespace

#define PT_TRY(x)                          \
    do {                                   \
        hipError_t e_ = (x);               \
        if (e_ != hipSuccess) {            \
            err = e_;                      \
            goto done;                     \
        }                                  \
    } while (0)

hipError_t lbvh_build(const BuildInput& in, BuildOutput& out, hipStream_t stream, float* ms) {
    const int n = in.n;
    hipError_t err = hipSuccess;
    uint32_t *keys = nullptr, *vals = nullptr, *keys2 = nullptr, *vals2 = nullptr;
    float4 *st = nullptr, *bbox = nullptr;
    int2 *bchild = nullptr, *brange = nullptr;
    int *work = nullptr, *work2 = nullptr, *wcnt = nullptr, *woff = nullptr;
    int *dp_parent = nullptr, *dp_leafparent = nullptr, *dp_visits = nullptr, *dp_dec = nullptr;
    float4 *dp_cost = nullptr, *lb_pleaf = nullptr, *pbox = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0, scan_bytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int levels = 1;
    SparseTable table{};
    BinTree B{};
    int nwork = 1, depth = 0, root = 0, node_count = 1, level_base = 0;
    const int nbin = n > 1 ? n - 1 : 1;
    const bool ploc = in.builder != kBuilderLBVH;
    std::vector<void*> owned;
    if (ms) *ms = 0.0f;
    out.n_nodes = 0;
    out.depth = 0;
    if (n <= 0) return hipSuccess;
    while ((1 << levels) <= n) ++levels;  // levels 0..levels-1 with 2^l <= n
    PT_TRY(hipEventCreate(&e0));
    PT_TRY(hipEventCreate(&e1));
    PT_TRY(hipMalloc(&keys, sizeof(uint32_t) * n));
    PT_TRY(hipMalloc(&vals, sizeof(uint32_t) * n));
    PT_TRY(hipMalloc(&keys2, sizeof(uint32_t) * n));
    PT_TRY(hipMalloc(&vals2, sizeof(uint32_t) * n));
    if (!ploc) {
        PT_TRY(hipMalloc(&st, sizeof(float4) * 2 * (size_t)n * (size_t)levels));
        PT_TRY(hipMalloc(&bchild, sizeof(int2) * nbin));
        PT_TRY(hipMalloc(&brange, sizeof(int2) * nbin));
        PT_TRY(hipMalloc(&bbox, sizeof(float4) * 2 * nbin));
        PT_TRY(hipMalloc(&lb_pleaf, sizeof(float4) * 2 * (size_t)n));
    }
    PT_TRY(hipMalloc(&work, sizeof(int) * n));
    PT_TRY(hipMalloc(&work2, sizeof(int) * n));
    PT_TRY(hipMalloc(&wcnt, sizeof(int) * n));
    PT_TRY(hipMalloc(&woff, sizeof(int) * n));
    PT_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys, keys2, vals, vals2, n, 0, 30, stream));
    PT_TRY(hipcub::DeviceScan::ExclusiveSum(nullptr, scan_bytes, wcnt, woff, n, stream));
    temp_bytes = std::max(temp_bytes, scan_bytes);
    PT_TRY(hipMalloc(&temp, temp_bytes > 0 ? temp_bytes : 16));
    PT_TRY(hipEventRecord(e0, stream));
    if ((in.builder == kBuilderSAH || in.builder == kBuilderSAHGPU) && n > 1) {
        // host binned-SAH binary tree, then the same leaf gather and SAH-optimal collapse
        std::vector<uint32_t> order;
        std::vector<int2> hchild, hrange;
        std::vector<float4> hbox;
        const bool on_gpu = in.builder == kBuilderSAHGPU;
        if (!on_gpu) sah_binary_tree(in.tri_host, n, order, hchild, hrange, hbox);
        if (!on_gpu && PT_SAH_REINSERT > 0) {
            // kept only when it cuts the binary tree's cost by 2 % or more: Sponza-class 8.9 % ->
            // +0.5 % Msamples/s; the sphere box 0.13 % -> one level deeper and -1.1 to -1.6 %
            // (profiles/r04u_ab_reinsert_sponza.log)
            std::vector<uint32_t> order2 = order;
            std::vector<int2> child2 = hchild, range2 = hrange;
            std::vector<float4> box2 = hbox;
            if (sah_reinsert(order2, child2, range2, box2, in.tri_host, PT_SAH_REINSERT) >= 0.02) {
                order.swap(order2);
                hchild.swap(child2);
                hrange.swap(range2);
                hbox.swap(box2);
            }
        }
        uint32_t* dfs = nullptr;
        float4 *sbox = nullptr, *sleaf = nullptr, *spleaf = nullptr;
        int2 *schild = nullptr, *srange = nullptr;
        for (auto pr : {std::make_pair((void**)&dfs, sizeof(uint32_t) * (size_t)n),
                        std::make_pair((void**)&schild, sizeof(int2) * (size_t)nbin),
                        std::make_pair((void**)&srange, sizeof(int2) * (size_t)nbin),
                        std::make_pair((void**)&sbox, sizeof(float4) * 2 * (size_t)nbin),
                        std::make_pair((void**)&sleaf, sizeof(float4) * 2 * (size_t)n),
                        std::make_pair((void**)&spleaf, sizeof(float4) * 2 * (size_t)n)}) {
            PT_TRY(hipMalloc(pr.first, pr.second));
            owned.push_back(*pr.first);
        }
        if (on_gpu) {
            PT_TRY(sah_build_gpu(in.tri_orig, n, dfs, schild, srange, sbox, stream));
        } else {
            PT_TRY(hipMemcpyAsync(dfs, order.data(), sizeof(uint32_t) * (size_t)n, hipMemcpyHostToDevice, stream));
            PT_TRY(hipMemcpyAsync(schild, hchild.data(), sizeof(int2) * (size_t)nbin, hipMemcpyHostToDevice, stream));
            PT_TRY(hipMemcpyAsync(srange, hrange.data(), sizeof(int2) * (size_t)nbin, hipMemcpyHostToDevice, stream));
            PT_TRY(hipMemcpyAsync(sbox, hbox.data(), sizeof(float4) * 2 * (size_t)nbin, hipMemcpyHostToDevice, stream));
        }
        hipLaunchKernelGGL(k_gather, dim3(grid_for(n, 256)), dim3(256), 0, stream, in.tri_orig, in.nrm_orig,
                           in.uv_orig, dfs, n, out.isect, out.shade, out.tuv, sleaf, spleaf);
        PT_TRY(hipGetLastError());
        PT_TRY(hipStreamSynchronize(stream));  // the host vectors go out of scope
        B.child = schild;
        B.range = srange;
        B.box = sbox;
        B.leafbox = sleaf;
        B.pleaf = spleaf;
        root = 0;
    }
    if ((in.builder != kBuilderSAH && in.builder != kBuilderSAHGPU) || n <= 1) {
        float3 cmin = make_float3(in.cmin[0], in.cmin[1], in.cmin[2]);
        float ex = in.cmax[0] - in.cmin[0], ey = in.cmax[1] - in.cmin[1], ez = in.cmax[2] - in.cmin[2];
        float3 cinv = make_float3(ex > 0.0f ? 1.0f / ex : 0.0f, ey > 0.0f ? 1.0f / ey : 0.0f,
                                  ez > 0.0f ? 1.0f / ez : 0.0f);
        hipLaunchKernelGGL(k_morton, dim3(grid_for(n, 256)), dim3(256), 0, stream, in.tri_orig, n, cmin, cinv, keys,
                           vals);
        PT_TRY(hipGetLastError());
        PT_TRY(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys, keys2, vals, vals2, n, 0, 30, stream));
        if (ploc) {
            PT_TRY(ploc_build(in, vals2, out, stream, B, root, owned));
        } else {
            hipLaunchKernelGGL(k_gather, dim3(grid_for(n, 256)), dim3(256), 0, stream, in.tri_orig, in.nrm_orig,
                               in.uv_orig, vals2, n, out.isect, out.shade, out.tuv, st, lb_pleaf);
            PT_TRY(hipGetLastError());
            table.n = n;
            table.level[0] = st;
            for (int l = 1; l < levels; ++l) {
                float4* prev = st + 2 * (size_t)n * (size_t)(l - 1);
                float4* cur = st + 2 * (size_t)n * (size_t)l;
                int count = n - (1 << l) + 1;
                hipLaunchKernelGGL(k_sparse, dim3(grid_for(count, 256)), dim3(256), 0, stream, prev, cur, count,
                                   1 << (l - 1));
                PT_TRY(hipGetLastError());
                table.level[l] = cur;
            }
            if (n > 1) {
                hipLaunchKernelGGL(k_karras, dim3(grid_for(n - 1, 256)), dim3(256), 0, stream, keys2, n, table,
                                   bchild, brange, bbox);
                PT_TRY(hipGetLastError());
            }
            B.child = bchild;
            B.range = brange;
            B.box = bbox;
            B.leafbox = st;
            B.pleaf = lb_pleaf;
            root = n > 1 ? 0 : ~0;
        }
    }
    {
        if (root >= 0) {  // SAH DP over the binary tree (n >= 2)
            PT_TRY(hipMalloc(&dp_parent, sizeof(int) * nbin));
            PT_TRY(hipMalloc(&dp_leafparent, sizeof(int) * n));
            PT_TRY(hipMalloc(&dp_visits, sizeof(int) * nbin));
            PT_TRY(hipMalloc(&dp_cost, sizeof(float4) * nbin));
            PT_TRY(hipMalloc(&dp_dec, sizeof(int) * nbin));
            PT_TRY(hipMalloc(&pbox, sizeof(float4) * 2 * nbin));
            B.pbox = pbox;
            PT_TRY(hipMemsetAsync(dp_visits, 0, sizeof(int) * nbin, stream));
            PT_TRY(hipMemsetAsync(dp_parent, 0xff, sizeof(int) * nbin, stream));  // root: -1
            hipLaunchKernelGGL(k_parents, dim3(grid_for(nbin, 256)), dim3(256), 0, stream, B.child, nbin, dp_parent,
                               dp_leafparent);
            PT_TRY(hipGetLastError());
            hipLaunchKernelGGL(k_sah_dp, dim3(grid_for(n, 256)), dim3(256), 0, stream, B, n, dp_parent, dp_leafparent,
                               dp_visits, dp_cost, dp_dec);
            PT_TRY(hipGetLastError());
        }
        // level 0: the binary root (or the single leaf ~0) -> BVH4 slot 0
        PT_TRY(hipMemcpyAsync(work, &root, sizeof(int), hipMemcpyHostToDevice, stream));
        while (nwork > 0) {
            hipLaunchKernelGGL(k_collapse_count, dim3(grid_for(nwork, 128)), dim3(128), 0, stream, B, dp_dec, work,
                               nwork, wcnt);
            PT_TRY(hipGetLastError());
            PT_TRY(hipcub::DeviceScan::ExclusiveSum(temp, temp_bytes, wcnt, woff, nwork, stream));
            hipLaunchKernelGGL(k_collapse_emit, dim3(grid_for(nwork, 128)), dim3(128), 0, stream, B, dp_dec, work,
                               nwork, woff, level_base, node_count, out.nodes, work2);
            PT_TRY(hipGetLastError());
            int tail[2] = {0, 0};  // offset and count of the level's last item: the next level's size
            PT_TRY(hipMemcpyAsync(&tail[0], woff + nwork - 1, sizeof(int), hipMemcpyDeviceToHost, stream));
            PT_TRY(hipMemcpyAsync(&tail[1], wcnt + nwork - 1, sizeof(int), hipMemcpyDeviceToHost, stream));
            PT_TRY(hipStreamSynchronize(stream));
            nwork = tail[0] + tail[1];
            level_base = node_count;
            node_count += nwork;
            ++depth;
            std::swap(work, work2);
        }
    }
    PT_TRY(hipEventRecord(e1, stream));
    PT_TRY(hipEventSynchronize(e1));
    if (ms) PT_TRY(hipEventElapsedTime(ms, e0, e1));
    out.n_nodes = node_count;
    out.depth = depth;
done:
    (void)hipStreamSynchronize(stream);
    for (void* p : {(void*)keys, (void*)vals, (void*)keys2, (void*)vals2, (void*)st, (void*)bchild, (void*)brange,
                    (void*)bbox, (void*)work, (void*)work2, (void*)wcnt, (void*)woff, temp, (void*)dp_parent,
                    (void*)dp_leafparent, (void*)dp_visits, (void*)dp_cost, (void*)dp_dec, (void*)lb_pleaf,
                    (void*)pbox})
        if (p) (void)hipFree(p);
    for (void* p : owned) (void)hipFree(p);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return err;
}

}  // namespace pt
