// pt_sah_gpu.hip — the binned-SAH binary BVH of pt_sah.cpp, built on the GPU (pt_options.bvh_builder =
// PT_BVH_SAH_GPU, the default through PT_BVH_AUTO).  Replaces optixAccelBuild
// (OptixRenderer.cpp:306-456), which builds its acceleration structure on the device.
//
// The tree is the host builder's, node for node: every node splits its triangles at the
// surface-area-heuristic minimum over 64 centroid bins per axis (first minimum in axis-then-bin
// order, strict `<`), the split is a stable partition (so a node's range stays in original
// triangle order), and a node with no usable split (coincident centroids, or every centroid on
// one side) is cut in the middle of its range.  Every quantity the decisions depend on is
// computed with the host's operations in the host's order -- the centroid, the bin index
// (c - lo) * (64 / ext), the boxes' unions (exact in any order), half_area x*y + y*z + z*x and
// the cost A_L * n_L + A_R * n_R -- so the binary tree, the DFS leaf order and, after the shared
// collapse, the BVH4 are identical to PT_BVH_SAH's bit for bit (tests/test_gpu_sah_builder.py).
// Only the internal node numbering differs, which the collapse never sees.
//
// Two phases.  Large nodes (more than kSmallMax triangles) are processed level by level, one
// 512-thread workgroup per node: block reductions for the node and centroid boxes, bins in LDS
// (ordered-int atomics), one wave per axis for the sweep, a tiled stable partition; the host reads
// back the split positions of the level, numbers the children and launches the next level.
// Nodes of at most kSmallMax triangles are subtrees built to the end by one wave each: the same
// steps at wave scale (wave-private LDS bins, shuffle scans for the sweep, ballot/mbcnt for the
// partition), with the smaller child processed next and the larger one stacked, so the stack
// stays within log2(kSmallMax) entries.  Buffers alternate between two copies of the triangle
// order per partition level; a leaf writes its triangle to the output order.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <vector>

#include "pt_internal.h"

namespace pt {

namespace {

constexpr int kSBins = 64;       // centroid bins per axis: pt_sah.cpp kBins
constexpr int kSmallMax = 512;   // subtree size built by one wave
constexpr int kLargeBlock = 512;  // 2 waves per SIMD: room for the sweep's registers
constexpr int kLargeWaves = kLargeBlock / 64;
constexpr int kSmallBlock = 256;
constexpr int kSmallWaves = kSmallBlock / 64;
constexpr int kSmallStack = 16;  // > log2(kSmallMax): the larger child is stacked, the smaller one goes on

// Order-preserving int encoding of a (non-NaN) float, for atomic min / max.
__device__ __forceinline__ int f2o(float f) {
    const int i = __float_as_int(f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// pt_sah.cpp Box::grow (std::min / std::max: a NaN operand never replaces the bound)
__device__ __forceinline__ float gmin_h(float a, float p) { return p < a ? p : a; }
__device__ __forceinline__ float gmax_h(float a, float p) { return a < p ? p : a; }

// pt_sah.cpp Box::half_area
__device__ __forceinline__ float box_half_area(float lx, float ly, float lz, float hx, float hy, float hz) {
    if (lx > hx) return 0.0f;
    const float x = hx - lx, y = hy - ly, z = hz - lz;
    return x * y + y * z + z * x;
}

// pt_sah.cpp bin_of
__device__ __forceinline__ int bin_of(float c, float lo, float scale) {
    const float f = (c - lo) * scale;
    if (!(f > 0.0f)) return 0;
    return f < (float)(kSBins - 1) ? (int)f : kSBins - 1;
}

// Per triangle (original order): box lo | hi and centroid, as pt_sah.cpp sah_binary_tree computes them.
__global__ void k_sah_prep(const float4* tri, int n, float4* tlo, float4* thi, float4* cen, uint32_t* order) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int v = 0; v < 3; ++v) {
        const float4 p = tri[3 * (size_t)i + v];
        const float q[3] = {p.x, p.y, p.z};
        for (int a = 0; a < 3; ++a) {
            lo[a] = gmin_h(lo[a], q[a]);
            hi[a] = gmax_h(hi[a], q[a]);
        }
    }
    tlo[i] = make_float4(lo[0], lo[1], lo[2], 0.0f);
    thi[i] = make_float4(hi[0], hi[1], hi[2], 0.0f);
    cen[i] = make_float4(0.5f * (lo[0] + hi[0]), 0.5f * (lo[1] + hi[1]), 0.5f * (lo[2] + hi[2]), 0.0f);
    order[i] = (uint32_t)i;
}

struct SahTris {
    const float4 *tlo, *thi, *cen;
};
struct SahOut {
    int2* child;
    int2* range;
    float4* box;
    uint32_t* order;  // DFS leaf order (the output)
};

// One node's split decision from its 3 x 64 bins (ordered ints: lo xyz, hi xyz, count per bin),
// by one wave: the host's two sweeps as shuffle scans (unions are exact in any order, counts are
// integers), then the first minimum in axis-then-bin order.  Returns the split code
// axis * 64 + bin, or -1 (no usable split).  `valid_axis` bit a: the axis has a finite positive
// centroid extent (pt_sah.cpp skips the others).
__device__ int wave_sweep(const int* bins, int valid_axis) {
    const int lane = threadIdx.x & 63;
    float best = FLT_MAX;
    int best_code = -1;
    for (int a = 0; a < 3; ++a) {
        if (!((valid_axis >> a) & 1)) continue;  // wave-uniform
        const int* bb = bins + (a * kSBins + lane) * 8;
        int L[7], R[7];
        for (int k = 0; k < 7; ++k) L[k] = R[k] = bb[k];
        for (int o = 1; o < 64; o <<= 1) {
            int tl[7], tr[7];
            for (int k = 0; k < 7; ++k) {
                tl[k] = __shfl_up(L[k], o, 64);
                tr[k] = __shfl_down(R[k], o, 64);
            }
            if (lane >= o) {
                for (int k = 0; k < 3; ++k) L[k] = min(L[k], tl[k]);
                for (int k = 3; k < 6; ++k) L[k] = max(L[k], tl[k]);
                L[6] += tl[6];
            }
            if (lane + o < 64) {
                for (int k = 0; k < 3; ++k) R[k] = min(R[k], tr[k]);
                for (int k = 3; k < 6; ++k) R[k] = max(R[k], tr[k]);
                R[6] += tr[6];
            }
        }
        // lane b: left = bins 0..b, right = bins b+1..63 (the right scan of lane b + 1)
        const float ra = box_half_area(o2f(R[0]), o2f(R[1]), o2f(R[2]), o2f(R[3]), o2f(R[4]), o2f(R[5]));
        const float right_area = __shfl_down(ra, 1, 64);
        const int right_cnt = __shfl_down(R[6], 1, 64);
        const float la = box_half_area(o2f(L[0]), o2f(L[1]), o2f(L[2]), o2f(L[3]), o2f(L[4]), o2f(L[5]));
        float cost = FLT_MAX;
        if (lane < kSBins - 1 && L[6] != 0 && right_cnt != 0) {
            const float c = la * (float)L[6] + right_area * (float)right_cnt;
            if (c < FLT_MAX) cost = c;  // NaN and +inf never beat the host's FLT_MAX start
        }
        float bc = cost;
        int bi = cost < FLT_MAX ? lane : 64;
        for (int o = 32; o >= 1; o >>= 1) {
            const float oc = __shfl_xor(bc, o, 64);
            const int oi = __shfl_xor(bi, o, 64);
            if (oc < bc || (oc == bc && oi < bi)) {
                bc = oc;
                bi = oi;
            }
        }
        if (bi < 64 && bc < best) {  // strictly smaller than the earlier axes' best (host order)
            best = bc;
            best_code = a * kSBins + bi;
        }
    }
    return best_code;
}

// ---- large nodes: one 512-thread workgroup per node, one level per launch ------------------
struct LargeNode {
    int begin, end;  // [begin, end) of the level's source order buffer
    int id;          // binary node id
};

__device__ __forceinline__ int block_sum(int v, int* lds) {  // every thread gets the block total
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    const int wave = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds[wave] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < kLargeWaves; ++w) t += lds[w];
    return t;
}

__global__ __launch_bounds__(kLargeBlock) void k_sah_large(SahTris T, SahOut O, const LargeNode* nodes,
                                                           const uint32_t* src, uint32_t* dst, int* mid_out) {
    const LargeNode nd = nodes[blockIdx.x];
    const int m = nd.end - nd.begin;
    __shared__ int s_box[kLargeWaves][12];    // per wave: node box lo/hi, centroid box lo/hi (ordered ints)
    __shared__ int s_bins[3 * kSBins * 8];    // lo xyz, hi xyz, count, pad per bin
    __shared__ int s_red[kLargeWaves];
    __shared__ int s_split;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // node box and centroid box (pt_sah.cpp: nb.grow(tb), cb.grow(cen) over the range)
    float nb[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    float cb[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int k = nd.begin + (int)threadIdx.x; k < nd.end; k += kLargeBlock) {
        const uint32_t t = src[k];
        const float4 l = T.tlo[t], h = T.thi[t], c = T.cen[t];
        nb[0] = gmin_h(nb[0], l.x); nb[1] = gmin_h(nb[1], l.y); nb[2] = gmin_h(nb[2], l.z);
        nb[3] = gmax_h(nb[3], h.x); nb[4] = gmax_h(nb[4], h.y); nb[5] = gmax_h(nb[5], h.z);
        cb[0] = gmin_h(cb[0], c.x); cb[1] = gmin_h(cb[1], c.y); cb[2] = gmin_h(cb[2], c.z);
        cb[3] = gmax_h(cb[3], c.x); cb[4] = gmax_h(cb[4], c.y); cb[5] = gmax_h(cb[5], c.z);
    }
    int ob[12];
    for (int k = 0; k < 6; ++k) {
        ob[k] = f2o(nb[k]);
        ob[6 + k] = f2o(cb[k]);
    }
    for (int o = 32; o >= 1; o >>= 1)
        for (int k = 0; k < 12; ++k) {
            const int v = __shfl_xor(ob[k], o, 64);
            ob[k] = (k % 6) < 3 ? min(ob[k], v) : max(ob[k], v);
        }
    if (lane == 0)
        for (int k = 0; k < 12; ++k) s_box[wave][k] = ob[k];
    for (int i = threadIdx.x; i < 3 * kSBins * 8; i += kLargeBlock) {
        const int f = i & 7;
        s_bins[i] = f < 3 ? f2o(FLT_MAX) : f < 6 ? f2o(-FLT_MAX) : 0;
    }
    __syncthreads();
    for (int k = 0; k < 12; ++k) {
        int v = s_box[0][k];
        for (int w = 1; w < kLargeWaves; ++w) v = (k % 6) < 3 ? min(v, s_box[w][k]) : max(v, s_box[w][k]);
        ob[k] = v;
    }
    float clo[3], scale[3];
    int valid = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        clo[a] = o2f(ob[6 + a]);
        const float ext = o2f(ob[9 + a]) - clo[a];
        scale[a] = 1.0f;
        if (ext > 0.0f && isfinite(ext)) {
            valid |= 1 << a;
            scale[a] = (float)kSBins / ext;
        }
    }
    // bins of the valid axes
    for (int k = nd.begin + (int)threadIdx.x; k < nd.end; k += kLargeBlock) {
        const uint32_t t = src[k];
        const float4 l = T.tlo[t], h = T.thi[t], c = T.cen[t];
        const float cc[3] = {c.x, c.y, c.z};
        for (int a = 0; a < 3; ++a) {
            if (!((valid >> a) & 1)) continue;
            int* b = s_bins + (a * kSBins + bin_of(cc[a], clo[a], scale[a])) * 8;
            atomicMin(b + 0, f2o(l.x)); atomicMin(b + 1, f2o(l.y)); atomicMin(b + 2, f2o(l.z));
            atomicMax(b + 3, f2o(h.x)); atomicMax(b + 4, f2o(h.y)); atomicMax(b + 5, f2o(h.z));
            atomicAdd(b + 6, 1);
        }
    }
    __syncthreads();
    if (wave == 0) {
        const int code = wave_sweep(s_bins, valid);
        if (lane == 0) s_split = code;
    }
    __syncthreads();
    const int code = s_split;
    const int axis = code >= 0 ? code / kSBins : 0, split = code >= 0 ? code % kSBins : 0;
    const float lo_ax = axis == 0 ? clo[0] : axis == 1 ? clo[1] : clo[2];  // no dynamic indexing (scratch)
    const float sc_ax = axis == 0 ? scale[0] : axis == 1 ? scale[1] : scale[2];
    // left count, then the tiled stable partition
    int nl_part = 0;
    if (code >= 0)
        for (int k = nd.begin + (int)threadIdx.x; k < nd.end; k += kLargeBlock) {
            const float4 c = T.cen[src[k]];
            const float ca = axis == 0 ? c.x : axis == 1 ? c.y : c.z;
            nl_part += bin_of(ca, lo_ax, sc_ax) <= split ? 1 : 0;
        }
    const int nl = code >= 0 ? block_sum(nl_part, s_red) : 0;
    const bool cut_middle = code < 0 || nl == 0 || nl == m;
    const int mid = cut_middle ? nd.begin + m / 2 : nd.begin + nl;
    if (threadIdx.x == 0) {
        mid_out[blockIdx.x] = mid;
        O.range[nd.id] = make_int2(nd.begin, nd.end - 1);
        O.box[2 * (size_t)nd.id] = make_float4(o2f(ob[0]), o2f(ob[1]), o2f(ob[2]), 0.0f);
        O.box[2 * (size_t)nd.id + 1] = make_float4(o2f(ob[3]), o2f(ob[4]), o2f(ob[5]), 0.0f);
    }
    int lbase = nd.begin, rbase = mid;
    for (int k0 = nd.begin; k0 < nd.end; k0 += kLargeBlock) {  // block-uniform trip count
        const int k = k0 + (int)threadIdx.x;
        const bool in = k < nd.end;
        const uint32_t t = in ? src[k] : 0u;
        bool left = false;
        if (in && !cut_middle) {
            const float4 c = T.cen[t];
            const float ca = axis == 0 ? c.x : axis == 1 ? c.y : c.z;
            left = bin_of(ca, lo_ax, sc_ax) <= split;
        }
        const unsigned long long ml = __ballot(in && left), mr = __ballot(in && !left);
        __syncthreads();
        if (lane == 0) {
            s_box[wave][0] = __popcll(ml);
            s_box[wave][1] = __popcll(mr);
        }
        __syncthreads();
        int pl = 0, pr = 0, tl = 0, tr = 0;
        for (int w = 0; w < kLargeWaves; ++w) {
            if (w < wave) {
                pl += s_box[w][0];
                pr += s_box[w][1];
            }
            tl += s_box[w][0];
            tr += s_box[w][1];
        }
        if (in) {
            if (cut_middle) {
                dst[k] = t;
            } else {
                const unsigned long long mm = left ? ml : mr;
                const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
                dst[left ? lbase + pl + r : rbase + pr + r] = t;
            }
        }
        lbase += tl;
        rbase += tr;
    }
}

// child codes of the large nodes, numbered on the host: pairs (id, 0), (code 0, code 1)
__global__ void k_sah_fix(const int2* fix, int n, int2* child) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) child[fix[2 * i].x] = fix[2 * i + 1];
}

// ---- small subtrees: one wave each, to the leaves --------------------------------------------
struct SmallTree {
    int begin, end;  // [begin, end) of the source order buffer `parity`
    int id;          // id of its root (unused for a single triangle); its nodes take id .. id + size - 2
    int parity;      // which order buffer holds its triangles
};
struct StackEntry {
    int begin, end, id, parity;
};

__global__ __launch_bounds__(kSmallBlock) void k_sah_small(SahTris T, SahOut O, const SmallTree* trees, int ntrees,
                                                           uint32_t* buf0, uint32_t* buf1) {
    __shared__ int s_bins[kSmallWaves][3 * kSBins * 8];
    __shared__ StackEntry s_stack[kSmallWaves][kSmallStack];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int ti = blockIdx.x * kSmallWaves + wave;
    if (ti >= ntrees) return;  // no barrier below
    const SmallTree tr = trees[ti];
    int* bins = s_bins[wave];
    StackEntry* stk = s_stack[wave];
    if (tr.end - tr.begin == 1) {  // a leaf child of a large node
        if (lane == 0) O.order[tr.begin] = (tr.parity ? buf1 : buf0)[tr.begin];
        return;
    }
    int sp = 0;
    int next_id = tr.id + 1;
    StackEntry cur{tr.begin, tr.end, tr.id, tr.parity};
    while (true) {
        const uint32_t* src = cur.parity ? buf1 : buf0;
        uint32_t* dst = cur.parity ? buf0 : buf1;
        const int m = cur.end - cur.begin;
        float nb[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
        float cb[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
        for (int k = cur.begin + lane; k < cur.end; k += 64) {
            const uint32_t t = src[k];
            const float4 l = T.tlo[t], h = T.thi[t], c = T.cen[t];
            nb[0] = gmin_h(nb[0], l.x); nb[1] = gmin_h(nb[1], l.y); nb[2] = gmin_h(nb[2], l.z);
            nb[3] = gmax_h(nb[3], h.x); nb[4] = gmax_h(nb[4], h.y); nb[5] = gmax_h(nb[5], h.z);
            cb[0] = gmin_h(cb[0], c.x); cb[1] = gmin_h(cb[1], c.y); cb[2] = gmin_h(cb[2], c.z);
            cb[3] = gmax_h(cb[3], c.x); cb[4] = gmax_h(cb[4], c.y); cb[5] = gmax_h(cb[5], c.z);
        }
        int ob[12];
        for (int k = 0; k < 6; ++k) {
            ob[k] = f2o(nb[k]);
            ob[6 + k] = f2o(cb[k]);
        }
        for (int o = 32; o >= 1; o >>= 1)
            for (int k = 0; k < 12; ++k) {
                const int v = __shfl_xor(ob[k], o, 64);
                ob[k] = (k % 6) < 3 ? min(ob[k], v) : max(ob[k], v);
            }
        float clo[3], scale[3];
        int valid = 0;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            clo[a] = o2f(ob[6 + a]);
            const float ext = o2f(ob[9 + a]) - clo[a];
            scale[a] = 1.0f;
            if (ext > 0.0f && isfinite(ext)) {
                valid |= 1 << a;
                scale[a] = (float)kSBins / ext;
            }
        }
        for (int i = lane; i < 3 * kSBins * 8; i += 64) {
            const int f = i & 7;
            bins[i] = f < 3 ? f2o(FLT_MAX) : f < 6 ? f2o(-FLT_MAX) : 0;
        }
        __builtin_amdgcn_wave_barrier();
        for (int k = cur.begin + lane; k < cur.end; k += 64) {
            const uint32_t t = src[k];
            const float4 l = T.tlo[t], h = T.thi[t], c = T.cen[t];
            const float cc[3] = {c.x, c.y, c.z};
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                if (!((valid >> a) & 1)) continue;
                int* b = bins + (a * kSBins + bin_of(cc[a], clo[a], scale[a])) * 8;
                atomicMin(b + 0, f2o(l.x)); atomicMin(b + 1, f2o(l.y)); atomicMin(b + 2, f2o(l.z));
                atomicMax(b + 3, f2o(h.x)); atomicMax(b + 4, f2o(h.y)); atomicMax(b + 5, f2o(h.z));
                atomicAdd(b + 6, 1);
            }
        }
        __builtin_amdgcn_wave_barrier();
        const int code = wave_sweep(bins, valid);
        const int axis = code >= 0 ? code / kSBins : 0, split = code >= 0 ? code % kSBins : 0;
        const float lo_ax = axis == 0 ? clo[0] : axis == 1 ? clo[1] : clo[2];
        const float sc_ax = axis == 0 ? scale[0] : axis == 1 ? scale[1] : scale[2];
        int nl = 0;
        if (code >= 0)
            for (int k0 = cur.begin; k0 < cur.end; k0 += 64) {
                const int k = k0 + lane;
                bool left = false;
                if (k < cur.end) {
                    const float4 c = T.cen[src[k]];
                    const float ca = axis == 0 ? c.x : axis == 1 ? c.y : c.z;
                    left = bin_of(ca, lo_ax, sc_ax) <= split;
                }
                nl += __popcll(__ballot(left));
            }
        const bool cut_middle = code < 0 || nl == 0 || nl == m;
        const int mid = cut_middle ? cur.begin + m / 2 : cur.begin + nl;
        if (!cut_middle) {
            int lb = cur.begin, rb = mid;
            for (int k0 = cur.begin; k0 < cur.end; k0 += 64) {
                const int k = k0 + lane;
                const bool in = k < cur.end;
                const uint32_t t = in ? src[k] : 0u;
                bool left = false;
                if (in) {
                    const float4 c = T.cen[t];
                    const float ca = axis == 0 ? c.x : axis == 1 ? c.y : c.z;
                    left = bin_of(ca, lo_ax, sc_ax) <= split;
                }
                const unsigned long long ml = __ballot(in && left), mr = __ballot(in && !left);
                const unsigned long long mm = left ? ml : mr;
                const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
                if (in) dst[left ? lb + r : rb + r] = t;
                lb += __popcll(ml);
                rb += __popcll(mr);
            }
        }
        // the children's data: the partitioned copy, or the same buffer when cut in the middle
        const int cpar = cut_middle ? cur.parity : 1 - cur.parity;
        const uint32_t* cdata = cut_middle ? src : dst;
        // children [begin, mid) and [mid, end): a single triangle is a leaf (its DFS position),
        // anything larger an internal node numbered in creation order (left first)
        const bool leaf0 = mid - cur.begin == 1, leaf1 = cur.end - mid == 1;
        const int code0 = leaf0 ? ~cur.begin : next_id;
        next_id += leaf0 ? 0 : 1;
        const int code1 = leaf1 ? ~mid : next_id;
        next_id += leaf1 ? 0 : 1;
        if (lane == 0) {
            if (leaf0) O.order[cur.begin] = cdata[cur.begin];
            if (leaf1) O.order[mid] = cdata[mid];
            O.child[cur.id] = make_int2(code0, code1);
            O.range[cur.id] = make_int2(cur.begin, cur.end - 1);
            O.box[2 * (size_t)cur.id] = make_float4(o2f(ob[0]), o2f(ob[1]), o2f(ob[2]), 0.0f);
            O.box[2 * (size_t)cur.id + 1] = make_float4(o2f(ob[3]), o2f(ob[4]), o2f(ob[5]), 0.0f);
        }
        if (!leaf0 && !leaf1) {
            // the smaller child next, the larger one on the stack (depth <= log2 of the subtree);
            // fields selected one by one (a struct select went through scratch)
            const bool fs = mid - cur.begin <= cur.end - mid;
            if (lane == 0) stk[sp] = StackEntry{fs ? mid : cur.begin, fs ? cur.end : mid, fs ? code1 : code0, cpar};
            ++sp;
            cur = StackEntry{fs ? cur.begin : mid, fs ? mid : cur.end, fs ? code0 : code1, cpar};
        } else if (!leaf0) {
            cur = StackEntry{cur.begin, mid, code0, cpar};
        } else if (!leaf1) {
            cur = StackEntry{mid, cur.end, code1, cpar};
        } else {
            if (sp == 0) break;
            __builtin_amdgcn_wave_barrier();
            cur = stk[--sp];
        }
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace

hipError_t sah_build_gpu(const float4* tri, int n, uint32_t* order, int2* child, int2* range, float4* box,
                         hipStream_t stream) {
    if (n < 2) return hipSuccess;
    hipError_t err = hipSuccess;
    float4 *tlo = nullptr, *thi = nullptr, *cen = nullptr;
    uint32_t *buf[2] = {nullptr, nullptr};
    LargeNode* d_large = nullptr;
    SmallTree* d_small = nullptr;
    int* d_mid = nullptr;
    int2* d_fix = nullptr;
    std::vector<LargeNode> level;
    std::vector<SmallTree> small;
    std::vector<int> mids;
    std::vector<int2> fix;  // per large node: (id, 0), (child code 0, child code 1), written at the end
    int next_id = 1, parity = 0;
    auto alloc = [&](void** p, size_t bytes) {
        if (err == hipSuccess) err = hipMalloc(p, bytes);
    };
    alloc((void**)&tlo, sizeof(float4) * (size_t)n);
    alloc((void**)&thi, sizeof(float4) * (size_t)n);
    alloc((void**)&cen, sizeof(float4) * (size_t)n);
    alloc((void**)&buf[0], sizeof(uint32_t) * (size_t)n);
    alloc((void**)&buf[1], sizeof(uint32_t) * (size_t)n);
    alloc((void**)&d_mid, sizeof(int) * (size_t)n);
    alloc((void**)&d_large, sizeof(LargeNode) * (size_t)n);
    if (err != hipSuccess) goto done;
    hipLaunchKernelGGL(k_sah_prep, dim3((n + 255) / 256), dim3(256), 0, stream, tri, n, tlo, thi, cen, buf[0]);
    if ((err = hipGetLastError()) != hipSuccess) goto done;
    {
        const SahTris T{tlo, thi, cen};
        const SahOut O{child, range, box, order};
        if (n > kSmallMax) level.push_back(LargeNode{0, n, 0});
        else small.push_back(SmallTree{0, n, 0, 0});
        while (!level.empty()) {
            const int nn = (int)level.size();
            if ((err = hipMemcpyAsync(d_large, level.data(), sizeof(LargeNode) * nn, hipMemcpyHostToDevice, stream)) !=
                hipSuccess)
                goto done;
            hipLaunchKernelGGL(k_sah_large, dim3(nn), dim3(kLargeBlock), 0, stream, T, O, d_large, buf[parity],
                               buf[1 - parity], d_mid);
            if ((err = hipGetLastError()) != hipSuccess) goto done;
            mids.resize(nn);
            if ((err = hipMemcpyAsync(mids.data(), d_mid, sizeof(int) * nn, hipMemcpyDeviceToHost, stream)) != hipSuccess)
                goto done;
            if ((err = hipStreamSynchronize(stream)) != hipSuccess) goto done;
            // every node of the level was partitioned into buf[1 - parity] (a middle cut copies)
            std::vector<LargeNode> next;
            for (int i = 0; i < nn; ++i) {
                const LargeNode& nd = level[i];
                const int b0[2] = {nd.begin, mids[i]}, e0[2] = {mids[i], nd.end};
                int codes[2];
                for (int s = 0; s < 2; ++s) {
                    const int sz = e0[s] - b0[s];
                    if (sz == 1) {
                        codes[s] = ~b0[s];
                        small.push_back(SmallTree{b0[s], e0[s], -1, 1 - parity});
                    } else if (sz > kSmallMax) {
                        codes[s] = next_id++;
                        next.push_back(LargeNode{b0[s], e0[s], codes[s]});
                    } else {
                        codes[s] = next_id;
                        small.push_back(SmallTree{b0[s], e0[s], next_id, 1 - parity});
                        next_id += sz - 1;
                    }
                }
                fix.push_back(make_int2(nd.id, 0));
                fix.push_back(make_int2(codes[0], codes[1]));
            }
            level.swap(next);
            parity = 1 - parity;
        }
        // a large level's node ids were handed out before the small subtrees that follow it, so the
        // subtrees' ranges [id, id + size - 1) and the large ids never overlap (the total is n - 1)
        if (!fix.empty()) {
            alloc((void**)&d_fix, sizeof(int2) * fix.size());
            if (err != hipSuccess) goto done;
            if ((err = hipMemcpyAsync(d_fix, fix.data(), sizeof(int2) * fix.size(), hipMemcpyHostToDevice, stream)) !=
                hipSuccess)
                goto done;
            const int nf = (int)fix.size() / 2;
            hipLaunchKernelGGL(k_sah_fix, dim3((nf + 255) / 256), dim3(256), 0, stream, d_fix, nf, child);
            if ((err = hipGetLastError()) != hipSuccess) goto done;
        }
        if (!small.empty()) {
            alloc((void**)&d_small, sizeof(SmallTree) * small.size());
            if (err != hipSuccess) goto done;
            if ((err = hipMemcpyAsync(d_small, small.data(), sizeof(SmallTree) * small.size(), hipMemcpyHostToDevice,
                                      stream)) != hipSuccess)
                goto done;
            const int nt = (int)small.size();
            hipLaunchKernelGGL(k_sah_small, dim3((nt + kSmallWaves - 1) / kSmallWaves), dim3(kSmallBlock), 0, stream, T,
                               O, d_small, nt, buf[0], buf[1]);
            if ((err = hipGetLastError()) != hipSuccess) goto done;
        }
        err = hipStreamSynchronize(stream);
    }
done:
    (void)hipStreamSynchronize(stream);
    for (void* p : {(void*)tlo, (void*)thi, (void*)cen, (void*)buf[0], (void*)buf[1], (void*)d_large, (void*)d_small,
                    (void*)d_mid, (void*)d_fix})
        if (p) (void)hipFree(p);
    return err;
}

}  // namespace pt
