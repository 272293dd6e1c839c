// pt_render.hip — render kernels for gfx950 (replaces optixLaunch of __raygen__renderFrame,
// Renderer/OptiX/OptixRenderer.cpp:617-647, and the per-spp GL accumulation of
// Renderer/OptixView.cpp:212-255).
//
// k_render_mega<MODE>: one thread per pixel; a 256-thread workgroup covers a 16x16 pixel
// tile, each wave64 an 8x8 quadrant (primary-ray coherence inside the wave).  The thread
// loads its fp32 sum, adds the radiance of frame ids frame_base .. frame_base+n_frames-1
// in order (identical rounding to sequential per-frame accumulation), and stores it once:
// no per-spp HBM round trip of the 24.9 MB colour buffer.  The BVH4 traversal stack lives
// in LDS (32 entries x 256 threads = 32 KB per workgroup).
#include "pt_internal.h"

namespace pt {

namespace {

constexpr int kBlock = 256;
// LDS traversal stack entries per lane (PT_MK_STACK, pt_device.h; the megakernel is
// VGPR-limited, not LDS-limited).
constexpr int kStack = PT_MK_STACK;
// Minimum waves per SIMD the register allocator must allow (caps VGPRs at 512/N).
#ifndef PT_MK_WAVES
#define PT_MK_WAVES 1
#endif

__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

template <bool STATS>
__device__ __forceinline__ void flush_stats(const DevLaunch& L, uint32_t segs, const TravStats& ts, int lane) {
    unsigned long long a = wave_sum((unsigned long long)segs);
    if (STATS) {
        unsigned long long b = wave_sum((unsigned long long)ts.nodes);
        unsigned long long c = wave_sum((unsigned long long)ts.tris);
        unsigned long long d = wave_sum((unsigned long long)ts.rays);
        unsigned long long e = wave_sum((unsigned long long)ts.overflow);
        unsigned long long g = wave_sum((unsigned long long)ts.retrace);
        if (lane == 0 && L.counters) {
            atomicAdd(&L.counters[1], b);
            atomicAdd(&L.counters[2], c);
            atomicAdd(&L.counters[3], d);
            atomicAdd(&L.counters[4], e);
            atomicAdd(&L.counters[8], g);
        }
    }
    if (lane == 0 && L.counters) atomicAdd(&L.counters[0], a);
}

template <int MODE, bool STATS, bool TEX>
__global__ __launch_bounds__(kBlock, PT_MK_WAVES) void k_render_mega(DevScene S, DevLaunch L) {
    __shared__ int stack[kStack * kBlock];
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int x = blockIdx.x * 16 + (wave & 1) * 8 + (lane & 7);
    const int y = blockIdx.y * 16 + (wave >> 1) * 8 + (lane >> 3);
    int* stk = stack + threadIdx.x;
    uint32_t segs = 0;
    TravStats ts;
    if (x < L.width && y < L.height && L.n_frames > 0) {
        f3 co, cd;
        camera_ray(L, x, y, co, cd);
        const size_t idx = ((size_t)y * (size_t)L.width + (size_t)x) * 3;
        float sx = L.accum[idx], sy = L.accum[idx + 1], sz = L.accum[idx + 2];
        const uint32_t pix = (uint32_t)(L.width * y + x);
        // Path regeneration: a lane whose path ends starts its next frame at once instead of
        // idling until the wave's longest path of the frame finishes.  Each lane still adds
        // its frames in order, so the sum is bit-identical to the sequential accumulation.
        uint32_t f = 0;
        PathState p;
        path_start(p, co, cd, tea16(pix, L.frame_base));  // devicePrograms.cu:631
        const bool debug_pixel = L.debug_pixel == (int)pix;
        while (true) {
            if (path_alive(L, p)) {
                path_segment<MODE, STATS, kStack, TEX>(S, L, p, stk, kBlock, ts,
                                                       debug_pixel && L.frame_base + f == L.debug_frame);
                segs++;
                continue;
            }
            sx += p.radiance.x;
            sy += p.radiance.y;
            sz += p.radiance.z;
            if (++f == L.n_frames) break;
            path_start(p, co, cd, tea16(pix, L.frame_base + f));
        }
        L.accum[idx] = sx;
        L.accum[idx + 1] = sy;
        L.accum[idx + 2] = sz;
    }
    flush_stats<STATS>(L, segs, ts, lane);
}

template <bool TEX>
__global__ __launch_bounds__(kBlock) void k_trace(DevScene S, const float* rays, int n, int* prim, float* th,
                                                  float* uh, float* vh, int* back, int any_hit) {
    __shared__ int stack[kStack * kBlock];
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float* r = rays + 8 * (size_t)i;
    f3 o = mk(r[0], r[1], r[2]), d = mk(r[3], r[4], r[5]);
    Hit h;
    TravStats ts;
    int* stk = stack + threadIdx.x;
    bool hit = any_hit ? traverse<true, false, kStack, TEX>(S, o, d, r[6], r[7], h, stk, kBlock, ts)
                       : traverse<false, false, kStack, TEX>(S, o, d, r[6], r[7], h, stk, kBlock, ts);
    // any-hit: the occluder's original index (an any-hit traversal records only its leaf slot)
    prim[i] = hit ? (any_hit ? __float_as_int(S.isect[3 * h.tri].w) : h.orig) : -1;
    th[i] = hit && !any_hit ? h.t : 0.0f;
    uh[i] = hit && !any_hit ? h.u : 0.0f;
    vh[i] = hit && !any_hit ? h.v : 0.0f;
    back[i] = hit && !any_hit ? (h.back ? 1 : 0) : 0;
}

template <int MODE>
hipError_t launch_mega(const DevScene& S, const DevLaunch& L, bool stats, hipStream_t stream) {
    dim3 grid((unsigned)((L.width + 15) / 16), (unsigned)((L.height + 15) / 16));
    const bool tex = S.texinfo != nullptr;
    if (tex) {
        if (stats)
            hipLaunchKernelGGL((k_render_mega<MODE, true, true>), grid, dim3(kBlock), 0, stream, S, L);
        else
            hipLaunchKernelGGL((k_render_mega<MODE, false, true>), grid, dim3(kBlock), 0, stream, S, L);
    } else if (stats) {
        hipLaunchKernelGGL((k_render_mega<MODE, true, false>), grid, dim3(kBlock), 0, stream, S, L);
    } else {
        hipLaunchKernelGGL((k_render_mega<MODE, false, false>), grid, dim3(kBlock), 0, stream, S, L);
    }
    return hipGetLastError();
}

}  // namespace

hipError_t launch_render(int kernel, int mode, bool stats, const DevScene& S, const DevLaunch& L,
                         hipStream_t stream) {
    (void)kernel;
    switch (mode) {
        case kModeLambert: return launch_mega<kModeLambert>(S, L, stats, stream);
        case kModeConductor: return launch_mega<kModeConductor>(S, L, stats, stream);
        case kModeDielectric: return launch_mega<kModeDielectric>(S, L, stats, stream);
        case kModeLayered: return launch_mega<kModeLayered>(S, L, stats, stream);
        default: return launch_mega<kModeDefault>(S, L, stats, stream);
    }
}

hipError_t launch_trace(const DevScene& S, const float* d_rays, int n, int* d_prim, float* d_thit, float* d_u,
                        float* d_v, int* d_back, int any_hit, hipStream_t stream) {
    if (n <= 0) return hipSuccess;
    if (S.texinfo)
        hipLaunchKernelGGL(k_trace<true>, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, S, d_rays, n,
                       d_prim, d_thit, d_u, d_v, d_back, any_hit);
    else
        hipLaunchKernelGGL(k_trace<false>, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, stream, S, d_rays, n,
                       d_prim, d_thit, d_u, d_v, d_back, any_hit);
    return hipGetLastError();
}

}  // namespace pt
