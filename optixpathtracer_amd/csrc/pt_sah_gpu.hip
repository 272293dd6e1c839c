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
// Two phases.  Large nodes (more than kSmallMax triangles) are processed level by level, each cut
// into chunks of 4096 triangles with one workgroup per chunk: block reductions for the node and
// centroid boxes and LDS bins (ordered-int atomics) merged into the node's with global atomics, one
// wave per node for the sweep, a tiled stable partition after the node's earlier chunks; the host
// reads back the split positions of the level, numbers the children and launches the next level.
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
#ifndef PT_SAH_SMALL
#define PT_SAH_SMALL 64  // 512 / 128 / 64 / 32: 7.9 / 5.9 / 5.6 / 5.8 ms warm at 250k triangles
#endif
constexpr int kSmallMax = PT_SAH_SMALL;  // subtree size built by one wave
constexpr int kSmallBlock = 256;
constexpr int kSmallWaves = kSmallBlock / 64;
constexpr int kSmallStack = 16;  // > log2(kSmallMax): the larger child is stacked, the smaller one goes on

// Order-preserving int encoding of a (non-NaN) float, for atomic min / max.
// -0 is taken as +0 first (f + 0 under round-to-nearest): the ordered encoding puts -0 below +0,
// where the host's std::min / std::max keep whichever zero came first; both
// builders now see only +0, so their boxes agree in the sign of zero as well.
__device__ __forceinline__ int f2o(float f) {
    const int i = __float_as_int(f + 0.0f);
    return i >= 0 ? i : i ^ 0x7fffffff;
}
__device__ __forceinline__ float o2f(int i) { return __int_as_float(i >= 0 ? i : i ^ 0x7fffffff); }

// pt_sah.cpp Box::grow (std::min / std::max: a NaN operand never replaces the bound)
// (-0 taken as +0, as Box::grow does since round 6)
__device__ __forceinline__ float gmin_h(float a, float p) { p += 0.0f; return p < a ? p : a; }
__device__ __forceinline__ float gmax_h(float a, float p) { p += 0.0f; return a < p ? p : a; }

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

// ---- large nodes: one level per pass, several workgroups per node ---------------------------
// A level's nodes are cut into chunks of kChunk consecutive triangles, one 256-thread workgroup
// each: the node and centroid boxes and the bins are reduced per chunk in LDS and merged into the
// node's global copy with atomics (min / max / add: exact and order-independent), one wave per
// node takes the split decision, and the stable partition writes every chunk's left triangles
// after the left triangles of the node's earlier chunks (a prefix over the chunks' counts).
struct LargeNode {
    int begin, end;  // [begin, end) of the level's source order buffer
    int id;          // binary node id
    int chunk0;      // its first chunk
};
struct Chunk {
    int node, begin, end;
};
constexpr int kChunk = 4096;
constexpr int kChunkBlock = 256;
constexpr int kChunkWaves = kChunkBlock / 64;
constexpr int kAcc = 12;                // node box lo / hi, centroid box lo / hi (ordered ints)
constexpr int kBinInts = 3 * kSBins * 8;  // lo xyz, hi xyz, count, pad per bin

__global__ void k_lg_init(int nn, int* acc, int* bins) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nn * kAcc) {
        const int k = i % kAcc;
        acc[i] = (k % 6) < 3 ? f2o(FLT_MAX) : f2o(-FLT_MAX);
    }
    if (i < nn * kBinInts) {
        const int f = i & 7;
        bins[i] = f < 3 ? f2o(FLT_MAX) : f < 6 ? f2o(-FLT_MAX) : 0;
    }
}

__device__ __forceinline__ void block_reduce_acc(int ob[kAcc], int (*lds)[kAcc]) {
    for (int o = 32; o >= 1; o >>= 1)
        for (int k = 0; k < kAcc; ++k) {
            const int v = __shfl_xor(ob[k], o, 64);
            ob[k] = (k % 6) < 3 ? min(ob[k], v) : max(ob[k], v);
        }
    if ((threadIdx.x & 63) == 0)
        for (int k = 0; k < kAcc; ++k) lds[threadIdx.x >> 6][k] = ob[k];
    __syncthreads();
    for (int k = 0; k < kAcc; ++k) {
        int v = lds[0][k];
        for (int w = 1; w < kChunkWaves; ++w) v = (k % 6) < 3 ? min(v, lds[w][k]) : max(v, lds[w][k]);
        ob[k] = v;
    }
}

// node box and centroid box of each chunk, merged into the node's (pt_sah.cpp nb / cb)
__global__ __launch_bounds__(kChunkBlock) void k_lg_bounds(SahTris T, const Chunk* chunks, const uint32_t* src,
                                                           int* acc) {
    const Chunk ch = chunks[blockIdx.x];
    __shared__ int s_red[kChunkWaves][kAcc];
    float nb[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    float cb[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int k = ch.begin + (int)threadIdx.x; k < ch.end; k += kChunkBlock) {
        const uint32_t t = src[k];
        const float4 l = T.tlo[t], h = T.thi[t], c = T.cen[t];
        nb[0] = gmin_h(nb[0], l.x); nb[1] = gmin_h(nb[1], l.y); nb[2] = gmin_h(nb[2], l.z);
        nb[3] = gmax_h(nb[3], h.x); nb[4] = gmax_h(nb[4], h.y); nb[5] = gmax_h(nb[5], h.z);
        cb[0] = gmin_h(cb[0], c.x); cb[1] = gmin_h(cb[1], c.y); cb[2] = gmin_h(cb[2], c.z);
        cb[3] = gmax_h(cb[3], c.x); cb[4] = gmax_h(cb[4], c.y); cb[5] = gmax_h(cb[5], c.z);
    }
    int ob[kAcc];
    for (int k = 0; k < 6; ++k) {
        ob[k] = f2o(nb[k]);
        ob[6 + k] = f2o(cb[k]);
    }
    block_reduce_acc(ob, s_red);
    if (threadIdx.x < kAcc) {
        const int k = threadIdx.x;
        int v = ob[0];
        for (int j = 1; j < kAcc; ++j) v = j == k ? ob[j] : v;  // ob[k] without dynamic indexing
        if ((k % 6) < 3) atomicMin(acc + ch.node * kAcc + k, v);
        else atomicMax(acc + ch.node * kAcc + k, v);
    }
}

// the axes with a usable centroid extent, their lower bound and bin scale (pt_sah.cpp)
__device__ __forceinline__ int axis_setup(const int* a, float clo[3], float scale[3]) {
    int valid = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        clo[k] = o2f(a[6 + k]);
        const float ext = o2f(a[9 + k]) - clo[k];
        scale[k] = 1.0f;
        if (ext > 0.0f && isfinite(ext)) {
            valid |= 1 << k;
            scale[k] = (float)kSBins / ext;
        }
    }
    return valid;
}

__global__ __launch_bounds__(kChunkBlock) void k_lg_bins(SahTris T, const Chunk* chunks, const uint32_t* src,
                                                         const int* acc, int* bins) {
    const Chunk ch = chunks[blockIdx.x];
    __shared__ int s_bins[kBinInts];
    float clo[3], scale[3];
    const int valid = axis_setup(acc + ch.node * kAcc, clo, scale);
    for (int i = threadIdx.x; i < kBinInts; i += kChunkBlock) {
        const int f = i & 7;
        s_bins[i] = f < 3 ? f2o(FLT_MAX) : f < 6 ? f2o(-FLT_MAX) : 0;
    }
    __syncthreads();
    for (int k = ch.begin + (int)threadIdx.x; k < ch.end; k += kChunkBlock) {
        const uint32_t t = src[k];
        const float4 l = T.tlo[t], h = T.thi[t], c = T.cen[t];
        const float cc[3] = {c.x, c.y, c.z};
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            if (!((valid >> a) & 1)) continue;
            int* b = s_bins + (a * kSBins + bin_of(cc[a], clo[a], scale[a])) * 8;
            atomicMin(b + 0, f2o(l.x)); atomicMin(b + 1, f2o(l.y)); atomicMin(b + 2, f2o(l.z));
            atomicMax(b + 3, f2o(h.x)); atomicMax(b + 4, f2o(h.y)); atomicMax(b + 5, f2o(h.z));
            atomicAdd(b + 6, 1);
        }
    }
    __syncthreads();
    int* g = bins + (size_t)ch.node * kBinInts;
    for (int i = threadIdx.x; i < 3 * kSBins; i += kChunkBlock) {
        const int* b = s_bins + i * 8;
        if (b[6] == 0) continue;  // an empty bin adds nothing to the union
        int* d = g + i * 8;
        atomicMin(d + 0, b[0]); atomicMin(d + 1, b[1]); atomicMin(d + 2, b[2]);
        atomicMax(d + 3, b[3]); atomicMax(d + 4, b[4]); atomicMax(d + 5, b[5]);
        atomicAdd(d + 6, b[6]);
    }
}

// one wave per node: the split decision, the node's box and range
__global__ void k_lg_sweep(SahOut O, const LargeNode* nodes, int nn, const int* acc, const int* bins, int* code) {
    const int i = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (i >= nn) return;
    const int* a = acc + i * kAcc;
    float clo[3], scale[3];
    const int valid = axis_setup(a, clo, scale);
    const int c = wave_sweep(bins + (size_t)i * kBinInts, valid);
    if ((threadIdx.x & 63) == 0) {
        const LargeNode nd = nodes[i];
        code[i] = c;
        O.range[nd.id] = make_int2(nd.begin, nd.end - 1);
        O.box[2 * (size_t)nd.id] = make_float4(o2f(a[0]), o2f(a[1]), o2f(a[2]), 0.0f);
        O.box[2 * (size_t)nd.id + 1] = make_float4(o2f(a[3]), o2f(a[4]), o2f(a[5]), 0.0f);
    }
}

__device__ __forceinline__ bool goes_left(const SahTris& T, uint32_t t, int axis, float lo, float sc, int split) {
    const float4 c = T.cen[t];
    const float ca = axis == 0 ? c.x : axis == 1 ? c.y : c.z;
    return bin_of(ca, lo, sc) <= split;
}
__device__ __forceinline__ void split_of(const int* acc, int code, int& axis, int& split, float& lo, float& sc) {
    float clo[3], scale[3];
    (void)axis_setup(acc, clo, scale);
    axis = code >= 0 ? code / kSBins : 0;
    split = code >= 0 ? code % kSBins : 0;
    lo = axis == 0 ? clo[0] : axis == 1 ? clo[1] : clo[2];  // no dynamic indexing (scratch)
    sc = axis == 0 ? scale[0] : axis == 1 ? scale[1] : scale[2];
}

__device__ __forceinline__ int block_total(int v, int* lds) {  // every thread gets the block total
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
    __syncthreads();
    int t = 0;
    for (int w = 0; w < kChunkWaves; ++w) t += lds[w];
    return t;
}

__global__ __launch_bounds__(kChunkBlock) void k_lg_count(SahTris T, const Chunk* chunks, const uint32_t* src,
                                                          const int* acc, const int* code, int* chunk_left) {
    const Chunk ch = chunks[blockIdx.x];
    __shared__ int s_red[kChunkWaves];
    const int cd = code[ch.node];
    int axis, split;
    float lo, sc;
    split_of(acc + ch.node * kAcc, cd, axis, split, lo, sc);
    int n = 0;
    if (cd >= 0)
        for (int k = ch.begin + (int)threadIdx.x; k < ch.end; k += kChunkBlock)
            n += goes_left(T, src[k], axis, lo, sc, split) ? 1 : 0;
    n = block_total(n, s_red);
    if (threadIdx.x == 0) chunk_left[blockIdx.x] = n;
}

// Stable partition of each chunk into dst; a node with no usable split is cut in the middle of its
// range and copied unchanged.
__global__ __launch_bounds__(kChunkBlock) void k_lg_scatter(SahTris T, const LargeNode* nodes, const Chunk* chunks,
                                                            const uint32_t* src, uint32_t* dst, const int* acc,
                                                            const int* code, const int* chunk_left, int* mid_out) {
    const Chunk ch = chunks[blockIdx.x];
    const LargeNode nd = nodes[ch.node];
    __shared__ int s_cnt[kChunkWaves][2];
    const int cd = code[ch.node];
    int axis, split;
    float lo, sc;
    split_of(acc + ch.node * kAcc, cd, axis, split, lo, sc);
    int loff = 0, nl = 0;  // left triangles of the node's earlier chunks, of all its chunks
    for (int c = nd.chunk0; chunks[c].node == ch.node; ++c) {
        if (c == (int)blockIdx.x) loff = nl;
        nl += chunk_left[c];
        if (chunks[c].end == nd.end) break;
    }
    const int m = nd.end - nd.begin;
    const bool cut_middle = cd < 0 || nl == 0 || nl == m;
    const int mid = cut_middle ? nd.begin + m / 2 : nd.begin + nl;
    if (threadIdx.x == 0 && (int)blockIdx.x == nd.chunk0) mid_out[ch.node] = mid;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int lbase = nd.begin + loff, rbase = mid + (ch.begin - nd.begin - loff);
    for (int k0 = ch.begin; k0 < ch.end; k0 += kChunkBlock) {  // block-uniform trip count
        const int k = k0 + (int)threadIdx.x;
        const bool in = k < ch.end;
        const uint32_t t = in ? src[k] : 0u;
        if (cut_middle) {
            if (in) dst[k] = t;
            continue;  // block-uniform
        }
        const bool left = in && goes_left(T, t, axis, lo, sc, split);
        const unsigned long long ml = __ballot(in && left), mr = __ballot(in && !left);
        __syncthreads();
        if (lane == 0) {
            s_cnt[wave][0] = __popcll(ml);
            s_cnt[wave][1] = __popcll(mr);
        }
        __syncthreads();
        int pl = 0, pr = 0, tl = 0, tr = 0;
        for (int w = 0; w < kChunkWaves; ++w) {
            if (w < wave) {
                pl += s_cnt[w][0];
                pr += s_cnt[w][1];
            }
            tl += s_cnt[w][0];
            tr += s_cnt[w][1];
        }
        if (in) {
            const unsigned long long mm = left ? ml : mr;
            const int r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
            dst[left ? lbase + pl + r : rbase + pr + r] = t;
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
    Chunk* d_chunks = nullptr;
    SmallTree* d_small = nullptr;
    int *d_mid = nullptr, *d_acc = nullptr, *d_bins = nullptr, *d_code = nullptr, *d_cleft = nullptr;
    int2* d_fix = nullptr;
    std::vector<LargeNode> level;
    std::vector<Chunk> chunks;
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
    {
        // a level holds at most n / (kSmallMax + 1) nodes, and a node of m triangles m / kChunk + 1 chunks
        const size_t max_nodes = (size_t)n / (kSmallMax + 1) + 1, max_chunks = (size_t)n / kChunk + max_nodes;
        alloc((void**)&d_mid, sizeof(int) * max_nodes);
        alloc((void**)&d_code, sizeof(int) * max_nodes);
        alloc((void**)&d_acc, sizeof(int) * kAcc * max_nodes);
        alloc((void**)&d_bins, sizeof(int) * kBinInts * max_nodes);
        alloc((void**)&d_large, sizeof(LargeNode) * max_nodes);
        alloc((void**)&d_chunks, sizeof(Chunk) * max_chunks);
        alloc((void**)&d_cleft, sizeof(int) * max_chunks);
    }
    if (err != hipSuccess) goto done;
    hipLaunchKernelGGL(k_sah_prep, dim3((n + 255) / 256), dim3(256), 0, stream, tri, n, tlo, thi, cen, buf[0]);
    if ((err = hipGetLastError()) != hipSuccess) goto done;
    {
        const SahTris T{tlo, thi, cen};
        const SahOut O{child, range, box, order};
        if (n > kSmallMax) level.push_back(LargeNode{0, n, 0, 0});
        else small.push_back(SmallTree{0, n, 0, 0});
        while (!level.empty()) {
            const int nn = (int)level.size();
            chunks.clear();
            for (int i = 0; i < nn; ++i) {
                level[i].chunk0 = (int)chunks.size();
                for (int b = level[i].begin; b < level[i].end; b += kChunk)
                    chunks.push_back(Chunk{i, b, std::min(level[i].end, b + kChunk)});
            }
            const int nc = (int)chunks.size();
            if ((err = hipMemcpyAsync(d_large, level.data(), sizeof(LargeNode) * nn, hipMemcpyHostToDevice, stream)) !=
                    hipSuccess ||
                (err = hipMemcpyAsync(d_chunks, chunks.data(), sizeof(Chunk) * nc, hipMemcpyHostToDevice, stream)) !=
                    hipSuccess)
                goto done;
            const uint32_t* src = buf[parity];
            uint32_t* dst = buf[1 - parity];
            hipLaunchKernelGGL(k_lg_init, dim3((nn * kBinInts + 255) / 256), dim3(256), 0, stream, nn, d_acc, d_bins);
            hipLaunchKernelGGL(k_lg_bounds, dim3(nc), dim3(kChunkBlock), 0, stream, T, d_chunks, src, d_acc);
            hipLaunchKernelGGL(k_lg_bins, dim3(nc), dim3(kChunkBlock), 0, stream, T, d_chunks, src, d_acc, d_bins);
            hipLaunchKernelGGL(k_lg_sweep, dim3((nn + 3) / 4), dim3(256), 0, stream, O, d_large, nn, d_acc, d_bins,
                               d_code);
            hipLaunchKernelGGL(k_lg_count, dim3(nc), dim3(kChunkBlock), 0, stream, T, d_chunks, src, d_acc, d_code,
                               d_cleft);
            hipLaunchKernelGGL(k_lg_scatter, dim3(nc), dim3(kChunkBlock), 0, stream, T, d_large, d_chunks, src, dst,
                               d_acc, d_code, d_cleft, d_mid);
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
                        next.push_back(LargeNode{b0[s], e0[s], codes[s], 0});
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
                    (void*)d_mid, (void*)d_fix, (void*)d_chunks, (void*)d_acc, (void*)d_bins, (void*)d_code,
                    (void*)d_cleft})
        if (p) (void)hipFree(p);
    return err;
}

}  // namespace pt
