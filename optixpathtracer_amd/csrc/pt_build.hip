// pt_build.hip — LBVH construction on gfx950 (replaces optixAccelBuild + compaction,
// Renderer/OptiX/OptixRenderer.cpp:306-456 of Damo12320/OptixPathtracer).
//
//   1. k_morton   : per triangle AABB centroid -> 30-bit Morton key (10 bits/axis)
//   2. radix sort : (key, triangle) pairs, hipCUB device radix sort
//   3. k_gather   : triangles + normals into leaf order; level 0 of an AABB sparse table
//   4. k_sparse   : sparse-table level l = union of two level l-1 boxes (log2 N launches)
//   5. k_karras   : one thread per internal node (Karras 2012 split search); each child's
//                   AABB = O(1) sparse-table range query over its sorted leaf range
// No inter-workgroup hand-offs: every kernel reads only what earlier launches wrote, so
// the build needs no atomics or agent-scope fences and is deterministic.  The sparse
// table costs N*log2(N)*32 B (≈150 MB at 250k triangles) — trivial against 288 GB HBM.
#include <hipcub/hipcub.hpp>

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

// leaf order gather + sparse-table level 0 (box = {lo.xyz,0},{hi.xyz,0})
__global__ void k_gather(const float4* tri_orig, const float4* nrm_orig, const uint32_t* order, int n, float4* tri,
                         float4* nrm, float4* st0) {
    int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int i = (int)order[k];
    tri[3 * k] = tri_orig[3 * i];
    tri[3 * k + 1] = tri_orig[3 * i + 1];
    tri[3 * k + 2] = tri_orig[3 * i + 2];
    nrm[3 * k] = nrm_orig[3 * i];
    nrm[3 * k + 1] = nrm_orig[3 * i + 1];
    nrm[3 * k + 2] = nrm_orig[3 * i + 2];
    float lo[3], hi[3];
    tri_box(tri_orig, i, lo, hi);
    st0[2 * k] = make_float4(lo[0], lo[1], lo[2], 0.0f);
    st0[2 * k + 1] = make_float4(hi[0], hi[1], hi[2], 0.0f);
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

__device__ __forceinline__ void range_box(const SparseTable& st, int a, int b, float lo[3], float hi[3]) {
    int len = b - a + 1;
    int l = 31 - __clz(len);
    const float4* L = st.level[l];
    int c = b - (1 << l) + 1;
    float4 a0 = L[2 * a], a1 = L[2 * a + 1], b0 = L[2 * c], b1 = L[2 * c + 1];
    lo[0] = fminf(a0.x, b0.x);
    lo[1] = fminf(a0.y, b0.y);
    lo[2] = fminf(a0.z, b0.z);
    hi[0] = fmaxf(a1.x, b1.x);
    hi[1] = fmaxf(a1.y, b1.y);
    hi[2] = fmaxf(a1.z, b1.z);
}

// Conservative padding so the traversal's fma slab test never culls a true hit.
__device__ __forceinline__ float pad_amount(float x) { return fabsf(x) * 9.5367431640625e-7f + 1e-6f; }

__device__ __forceinline__ int delta(const uint32_t* keys, int n, int i, int j) {
    if (j < 0 || j >= n) return -1;
    uint32_t ki = keys[i], kj = keys[j];
    if (ki == kj) return 32 + __clz((uint32_t)i ^ (uint32_t)j);
    return __clz(ki ^ kj);
}

__global__ void k_karras(const uint32_t* keys, int n, SparseTable st, BNode* nodes) {
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
    float lo0[3], hi0[3], lo1[3], hi1[3];
    range_box(st, first, gamma, lo0, hi0);
    range_box(st, gamma + 1, last, lo1, hi1);
    for (int a = 0; a < 3; ++a) {
        lo0[a] -= pad_amount(lo0[a]);
        hi0[a] += pad_amount(hi0[a]);
        lo1[a] -= pad_amount(lo1[a]);
        hi1[a] += pad_amount(hi1[a]);
    }
    BNode nd;
    nd.a = make_float4(lo0[0], hi0[0], lo0[1], hi0[1]);
    nd.b = make_float4(lo1[0], hi1[0], lo1[1], hi1[1]);
    nd.c = make_float4(lo0[2], hi0[2], lo1[2], hi1[2]);
    nd.d = make_int4(c0, c1, 0, 0);
    nodes[i] = nd;
}

inline unsigned grid_for(int n, int b) { return (unsigned)((n + b - 1) / b); }

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
    float4* st = nullptr;
    void* temp = nullptr;
    size_t temp_bytes = 0;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    int levels = 1;
    SparseTable table{};
    if (ms) *ms = 0.0f;
    if (n <= 0) return hipSuccess;
    while ((1 << levels) <= n) ++levels;  // levels 0..levels-1 with 2^l <= n
    PT_TRY(hipEventCreate(&e0));
    PT_TRY(hipEventCreate(&e1));
    PT_TRY(hipMalloc(&keys, sizeof(uint32_t) * n));
    PT_TRY(hipMalloc(&vals, sizeof(uint32_t) * n));
    PT_TRY(hipMalloc(&keys2, sizeof(uint32_t) * n));
    PT_TRY(hipMalloc(&vals2, sizeof(uint32_t) * n));
    PT_TRY(hipMalloc(&st, sizeof(float4) * 2 * (size_t)n * (size_t)levels));
    PT_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, temp_bytes, keys, keys2, vals, vals2, n, 0, 30, stream));
    PT_TRY(hipMalloc(&temp, temp_bytes > 0 ? temp_bytes : 16));
    PT_TRY(hipEventRecord(e0, stream));
    {
        float3 cmin = make_float3(in.cmin[0], in.cmin[1], in.cmin[2]);
        float ex = in.cmax[0] - in.cmin[0], ey = in.cmax[1] - in.cmin[1], ez = in.cmax[2] - in.cmin[2];
        float3 cinv = make_float3(ex > 0.0f ? 1.0f / ex : 0.0f, ey > 0.0f ? 1.0f / ey : 0.0f,
                                  ez > 0.0f ? 1.0f / ez : 0.0f);
        hipLaunchKernelGGL(k_morton, dim3(grid_for(n, 256)), dim3(256), 0, stream, in.tri_orig, n, cmin, cinv, keys,
                           vals);
        PT_TRY(hipGetLastError());
        PT_TRY(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys, keys2, vals, vals2, n, 0, 30, stream));
        hipLaunchKernelGGL(k_gather, dim3(grid_for(n, 256)), dim3(256), 0, stream, in.tri_orig, in.nrm_orig, vals2,
                           n, out.tri, out.nrm, st);
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
                               out.nodes);
            PT_TRY(hipGetLastError());
        }
    }
    PT_TRY(hipEventRecord(e1, stream));
    PT_TRY(hipEventSynchronize(e1));
    if (ms) PT_TRY(hipEventElapsedTime(ms, e0, e1));
done:
    if (keys) (void)hipFree(keys);
    if (vals) (void)hipFree(vals);
    if (keys2) (void)hipFree(keys2);
    if (vals2) (void)hipFree(vals2);
    if (st) (void)hipFree(st);
    if (temp) (void)hipFree(temp);
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    return err;
}

}  // namespace pt
