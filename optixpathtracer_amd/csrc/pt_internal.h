// pt_internal.h — host-side declarations shared by the C-ABI (pt_capi.cpp) and the kernel
// translation units (pt_build.hip, pt_render.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <vector>

#include "pt_device.h"

namespace pt {

// Scene triangle soup in ORIGINAL order (meshes concatenated), world space.
struct BuildInput {
    const float4* tri_orig;  // 3 per triangle: v0|orig idx bits, v1|material bits, v2|0
    const float4* nrm_orig;  // 3 per triangle
    const float4* uv_orig;   // 2 per triangle (uv0, uv1 | uv2, 0) or NULL (no textures)
    int n;
    float cmin[3], cmax[3];  // centroid bounds (Morton quantisation range)
    int builder;             // kBuilderPLOC (default), kBuilderLBVH or kBuilderSAH
    const float4* tri_host;  // the same triangles on the host (kBuilderSAH builds there)
};
constexpr int kBuilderPLOC = 0;
constexpr int kBuilderLBVH = 1;
constexpr int kBuilderSAH = 2;     // host binned SAH (pt_sah.cpp)
constexpr int kBuilderSAHGPU = 3;  // the same tree built on the GPU (pt_sah_gpu.hip)

// Host binned-SAH binary tree (pt_sah.cpp) in the GPU builders' layout: order = original triangle
// per DFS leaf, child codes (>= 0 internal, ~k DFS leaf k), leaf ranges and plain boxes; root 0.
void sah_binary_tree(const float4* tri, int n, std::vector<uint32_t>& order, std::vector<int2>& child,
                     std::vector<int2>& range, std::vector<float4>& box);
// The same binary tree built on the GPU (pt_sah_gpu.hip): order, child, range and box are device
// arrays of n, n - 1, n - 1 and 2 (n - 1) entries; identical to sah_binary_tree's up to the
// internal node numbering (root 0).  Synchronises `stream`.
hipError_t sah_build_gpu(const float4* tri, int n, uint32_t* order, int2* child, int2* range, float4* box,
                         hipStream_t stream);
// Insertion-based optimisation of that tree in place (pt_sah.cpp); returns the relative cost cut.
// PT_SAH_REINSERT = the most rounds kBuilderSAH runs (0: off, the default since round 5: it measured
// 0.0 % on Sponza-class for 30-55 ms of host build, profiles/r04v_ab_reinsert_undo_sponza.log, and
// the GPU builder reproduces the unrefined tree).
#ifndef PT_SAH_REINSERT
#define PT_SAH_REINSERT 0
#endif
double sah_reinsert(std::vector<uint32_t>& order, std::vector<int2>& child, std::vector<int2>& range,
                    std::vector<float4>& box, const float4* tri, int rounds);

// BVH4 (collapsed LBVH) + triangle records in leaf order.
struct BuildOutput {
    BNode4* nodes;  // capacity max(1, n) nodes
    float4* isect;  // 3n
    float4* shade;  // 4n
    float4* tuv;    // 2n or NULL
    int n_nodes;    // written by lbvh_build
    int depth;      // BVH4 levels
};

// GPU LBVH build (Morton codes -> radix sort -> Karras 2012 hierarchy -> AABBs from a sparse
// table over the sorted leaves).  Replaces optixAccelBuild (OptixRenderer.cpp:306-456).
// Returns hipSuccess or the first error; *ms = device time of the build.
hipError_t lbvh_build(const BuildInput& in, BuildOutput& out, hipStream_t stream, float* ms);

// Wavefront path state: SoA queues in HBM, capacity = paths (one path per pixel per frame).
struct WFState {
    float4* ray_o[2] = {nullptr, nullptr};  // queue b&1: origin.xyz | path id
    float4* ray_d[2] = {nullptr, nullptr};  // direction.xyz | 0
    float4* hit = nullptr;                  // path, u, v, tri | back<<31 (-1 = miss), queue order
    float4* beta = nullptr;                 // path throughput.xyz | seed: path order (Default / Layered),
                                            // queue order of the even bounces (fused modes)
    float4* beta_q = nullptr;               // fused modes: throughput | seed of the odd bounces' queues
    float4* L = nullptr;                    // path radiance of the frame, path order
    float4* sh_o = nullptr;                 // shadow queue: origin | path
    float4* sh_d = nullptr;                 // direction | tmax
    float4* sh_c = nullptr;                 // deferred NEE contribution (fused modes)
    int* aux = nullptr;                     // light index << 1 | conductor (RNG-coupled modes)
    int* vis = nullptr;                     // shadow result per shadow ray (RNG-coupled modes)
    int* nq = nullptr;                      // NEE items (RNG-coupled modes): kShadeBuckets regions of `paths`
    int* sq = nullptr;                      // BSDF-sample items, same layout
    int* count = nullptr;                   // per bounce: queue, shadow, NEE and sample bucket lengths
    int paths = 0;
    int max_bounces = 0;
    // Look-ahead cancellation (pt_capi.cpp cancel_look_ahead), set per batch: a speculative
    // render-ahead batch carries the renderer's cancel words and the epoch it was enqueued under,
    // and its kernels stop early once the host has published a newer epoch (wf_cancelled,
    // trace_range).  Null for every other batch: no polling.
    const unsigned* cancel_host = nullptr;  // pinned host word: the newest cancel epoch (PCIe reads)
    unsigned* cancel_seen = nullptr;        // device relay of it (agent-scope loads, L2-served)
    unsigned cancel_epoch = 0;
    // pt_set_debug_hold (tests only): a speculative batch with this pinned word starts with k_hold,
    // which returns once the batch is cancelled, the word is set, or 10 s have passed
    const unsigned* hold_release = nullptr;
};
size_t wavefront_bytes(int paths, int max_bounces);
// sum32[i] = (float)sum64[i] (the multi-device fp64 reduce's result -> the fp32 sum buffer)
hipError_t accum_f64_to_f32(const double* sum64, float* sum32, size_t n, hipStream_t stream);
hipError_t wavefront_alloc(WFState& W, int paths, int max_bounces);
void wavefront_free(WFState& W);
// Enqueue one frame (all bounces) of the wavefront pipeline; adds the frame into L.accum.
// trace_events (optional): up to 2 * (L.max_bounces + 1) events recorded around the trace
// launches; *n_timed (optional) receives the number of event pairs recorded.  shade_events /
// n_shade_timed: the same for the bounce's dominant shading kernel (k_shade_fused / k_shade0_pixel
// in the fused modes, k_shade_nee in Default / Layered), up to 2 * L.max_bounces events.
// nf frames (frame .. frame + nf - 1) are traced together; W must hold nf * W * H paths.
// primary_dedup: trace the batch's identical camera rays once per pixel (k_extend `dup`).
// accum_wait / accum_done (optional): the batch's k_accum waits for accum_wait and records
// accum_done, so batches on different streams still add into the sum in frame order.
// wide_trace: the call runs on one stream, so the untextured trace kernels take the wide
// workgroups (pt_wavefront.hip kBlockTraceWide).
hipError_t launch_wavefront_frame(int mode, bool stats, const DevScene& S, const DevLaunch& L, const WFState& W,
                                  uint32_t frame, int nf, bool primary_dedup, int cus, hipStream_t stream,
                                  const hipEvent_t* trace_events,
                                  int* n_timed = nullptr, hipEvent_t accum_wait = nullptr,
                                  hipEvent_t accum_done = nullptr, const hipEvent_t* shade_events = nullptr,
                                  int* n_shade_timed = nullptr, bool wide_trace = false);

// Render launches.
hipError_t launch_render(int kernel, int mode, bool stats, const DevScene& S, const DevLaunch& L,
                         hipStream_t stream);
hipError_t launch_trace(const DevScene& S, const float* d_rays, int n, int* d_prim, float* d_thit, float* d_u,
                        float* d_v, int* d_back, int any_hit, hipStream_t stream);

// Progressive view buffer (pt_display.hip).
hipError_t display_fill(float* p, size_t n, float v, hipStream_t stream);
hipError_t display_blend(float* fb, const float* frame, size_t n, float w, bool continuous, hipStream_t stream);

}  // namespace pt
