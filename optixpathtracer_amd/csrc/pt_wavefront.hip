// pt_wavefront.hip — wavefront path tracer for gfx950 (PT_KERNEL_WAVEFRONT).
//
// The reference runs one OptiX thread per pixel that loops over bounces
// (SamplePath, devicePrograms.cu:625-664).  Here each bounce of a frame is a sequence of
// persistent, grid-stride kernels over SoA queues in HBM, so the traversal kernels carry
// only a ray (low VGPR count -> high occupancy) and the BSDF code runs in its own kernel:
//
//   k_camera            : path q = f * P + pixel for the nf frames of the batch; camera ray ->
//                         queue 0, state init
//   per bounce b:
//     k_extend          : closest hit of queue b (BVH4 traversal, LDS stack) -> hit records
//                         (fused modes: bounce 0 only; later bounces ride in k_trace_pair)
//     fused modes (Lambert / Conductor / Dielectric: BRDF eval draws no random numbers):
//       k_shade_fused   : surface, metallic coin, light pick, f*|cos|, BSDF sample; NEE
//                         contribution + shadow ray -> shadow queue (only if f != 0);
//                         continuation ray -> queue b+1 (wave-ballot compaction)
//       k_trace_pair    : one launch tracing the shadow rays of bounce b (any hit; unoccluded ->
//                         L[path] += contribution) and the extension rays of bounce b+1
//                         (closest hit), which start at the same hit points
//     RNG-coupled modes (Default / Layered: GlossyDiffuse::f consumes the path seed only
//     when the light is visible, GlossyDiffuse.h:230-343):
//       k_shade_a       : surface, coin, light pick -> shadow ray queue; item -> bucketed
//                         sample queue (and NEE queue at bounce 0, from the visibility table)
//       k_shadow_vis    : any-hit -> vis[shadow ray]; k_nee_compact: visible -> NEE queue
//       k_shade_nee     : f (may draw), NEE, over the bucketed NEE queue
//       k_shade_smp     : BSDF sample -> queue b+1, over the bucketed sample queue
//   k_accum             : accum[pixel] += L[f * P + pixel] for f = 0 .. nf-1 in order (the same
//                         fp32 order as the sequential reference accumulation)
//
// Every kernel reads queue lengths from device memory written by an earlier launch (kernel
// boundaries order the hand-off), so a whole batch of frames is enqueued without host round trips.
#include <type_traits>
#include <unordered_map>

#include "pt_internal.h"

namespace pt {

namespace {

constexpr int kBlockWF = 256;
// Trace kernels (k_extend, k_trace_pair, k_shadow_vis): workgroup size.  Every workgroup holds its
// own copy of the staged top BVH levels in LDS, so fewer, larger workgroups per CU leave room for
// more staged nodes at the same waves per SIMD: 512 threads with 100 nodes / 768 with 150 lost
// 2.9 / 7.0 % Lambert and 1.7 / 3.8 % Dielectric, Sponza-class +0.6 %.
#ifndef PT_TRACE_BLOCK
#define PT_TRACE_BLOCK 256
#endif
constexpr int kBlockTrace = PT_TRACE_BLOCK;
// LDS traversal stack entries per lane (PT_WF_STACK, pt_device.h): 11 KB per workgroup.
constexpr int kStack = PT_WF_STACK;
// Top BVH4 levels staged in LDS per trace workgroup (nodes 0 .. kLdsNodes-1, breadth-first: 49 =
// the three top levels (21) and 28 of the fourth, 6.1 KB).  With the 11-KB stack and the 9-KB
// triangle batches (below) a workgroup takes 26.1 KB, so a CU holds 6 workgroups, the 6 waves per
// SIMD the kernels' 80 VGPRs allow (v39, DESIGN.md §5: Lambert +2.4 %, Conductor +7.7 %,
// Dielectric +4.5 % over 5 waves with 14 entries and 57 nodes; the kernels wait on memory in
// more than half their cycles, and a sixth wave covers more of it).  Earlier sweeps at 5 waves
// (v34 tree): 0 / 21 / 41 / 85 nodes with a 16-entry stack -8.6 / -1.2 / 0 / -7.5 % Lambert.
#ifndef PT_LDS_NODES
#define PT_LDS_NODES 49
#endif
constexpr int kLdsNodes = PT_LDS_NODES;
// Wide trace workgroups (round 6): on one wavefront stream (Lambert, Default, Layered) the untextured
// trace kernels run 768-thread workgroups, two per CU, each staging 150 top nodes (levels 0-3 and 65
// of level 4) in LDS instead of six 256-thread workgroups with 49 each: the same 6 waves per SIMD,
// three times the staged nodes per workgroup.  Lambert +2.5 %, Default +0.6 %, Sponza-class +1.0 %;
// beside a second stream's shading kernels (Conductor, Dielectric) the 256-thread workgroups stay
// (Dielectric 3404 on two streams vs 3362 with wide workgroups on one).
#ifndef PT_TRACE_BLOCK_WIDE
#define PT_TRACE_BLOCK_WIDE 768
#endif
#ifndef PT_LDS_NODES_WIDE
#define PT_LDS_NODES_WIDE 150
#endif
constexpr int kBlockTraceWide = PT_TRACE_BLOCK_WIDE;
template <int BLK>
constexpr int lds_nodes_of() { return BLK == kBlockTrace ? kLdsNodes : PT_LDS_NODES_WIDE; }
// wave-batched triangle tests (pt_device.h wave_tri_batch): 2.25 KB of LDS per wave
// Trace kernels: 6 waves per SIMD (80 VGPRs, 3 spilled in cold paths); the textured variants
// keep 4.
#ifndef PT_WF_WAVES
#define PT_WF_WAVES 6
#endif
// the textured variants: 6 waves as well since round 6 (4 before; the textured atrium, config 5t,
// +1.6 % at 6, ±0 at 5, profiles/r06_ab/r06m_ab_tex_c5t.log)
#ifndef PT_WF_WAVES_TEX
#define PT_WF_WAVES_TEX 6
#endif
// PT_WIDE_TEX 1: the textured trace kernels take the wide workgroups as well on one-stream calls
#ifndef PT_WIDE_TEX
#define PT_WIDE_TEX 1  // +0.7 % config 5t, +1.0 % on the small textured scene (profiles/r06_ab/r06n_ab_widetex_*.log)
#endif
constexpr int wf_waves(bool tex) { return tex ? PT_WF_WAVES_TEX : PT_WF_WAVES; }
constexpr int kMissTri = -1;

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Look-ahead cancellation.  pt_render renders up to 64 frames ahead of
// the caller on speculation (pt_capi.cpp render_frame_image); when the camera or any other
// render state changes, those frames are useless and the next call must not wait behind them.
// The host publishes a new cancel epoch in pinned host memory (cancel_look_ahead); a batch
// enqueued under an older epoch then stops: every wave of the shading kernels checks at its
// start and returns, and the trace kernels stop refilling (trace_range), so what is still
// enqueued of the batch drains in launch gaps.  The host word is read over PCIe by few lanes
// (`relay`: the first lane of one block in 64, or of one wave per trace workgroup now and
// then), which raise the device word cancel_seen with an atomic max; everyone else polls that
// word with agent-scope loads (sc1: L2-served, MI355X_MICROARCH "visibility").  Epochs only
// grow, so a stale read never cancels a batch enqueued after the cancel.  A cancelled batch's
// queues stay consistent (every counted entry is written), its ring slot is discarded, and the
// next batch starts from zeroed counters.
__device__ __forceinline__ bool wf_cancel_poll(const WFState& W, bool relay) {
    if (relay) {
        const unsigned h = __hip_atomic_load(W.cancel_host, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_fetch_max(W.cancel_seen, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    const unsigned v = __hip_atomic_load(W.cancel_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(v) > W.cancel_epoch;  // wave-uniform
}
// Entry check of the shading and setup kernels: the wave returns when its batch is cancelled
// (a barrier later in the kernel waits only on the surviving waves of the workgroup).
__device__ __forceinline__ bool wf_cancelled(const WFState& W) {
    if (!W.cancel_seen) return false;  // not a speculative batch (kernel argument: uniform)
    return wf_cancel_poll(W, (blockIdx.x & 63) == 0 && threadIdx.x == 0);
}

// pt_set_debug_hold (tests only): the first kernel of a held speculative
// batch.  One lane waits until the host cancels the batch (a newer epoch in the pinned cancel
// word, relayed into cancel_seen as wf_cancel_poll does), releases the hold (the pinned release
// word), or 10 s of the 100-MHz wall clock pass, with an iteration bound behind that.  Every later
// kernel of the batch is queued behind it, so a test can move the camera while the batch is
// provably in flight, whatever the speed of the GPU.
__global__ void k_hold(WFState W) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    const unsigned long long t0 = wall_clock64();
    for (int it = 0; it < (1 << 22); ++it) {
        const unsigned h = __hip_atomic_load(W.cancel_host, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (h > W.cancel_epoch) {
            __hip_atomic_fetch_max(W.cancel_seen, h, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            return;
        }
        if (__hip_atomic_load(W.hold_release, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0u) return;
        if (wall_clock64() - t0 > 1000000000ull) return;
        __builtin_amdgcn_s_sleep(64);
    }
}

// Hit record of a finished extension ray: (path, u, v, tri | back << 31), or a miss.  The
// shading kernels reconstruct the surface from (tri, u, v) and never read t, so the first word
// carries the path id and they skip the ray_o read.
__device__ __forceinline__ float4 hit_record(const Hit& h, int path) {
    const float x = __int_as_float(path);
    return h.tri >= 0 ? make_float4(x, h.u, h.v, __int_as_float(h.tri | (h.back ? (int)0x80000000 : 0)))
                      : make_float4(x, 0.0f, 0.0f, __int_as_float(kMissTri));
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// Traversal statistics of a wave into the renderer's counters ([1] nodes, [2] triangle tests,
// [3] rays, [4] stack overflows, [8] strict re-traces, [14] node visits served from LDS).
template <bool STATS>
__device__ __forceinline__ void flush_trav_stats(unsigned long long* counters, const TravStats& ts) {
    if (!STATS || !counters) return;
    const unsigned long long a = wave_sum_u64(ts.nodes), c = wave_sum_u64(ts.tris), d = wave_sum_u64(ts.rays);
    const unsigned long long e = wave_sum_u64(ts.overflow), r = wave_sum_u64(ts.retrace);
    const unsigned long long l = wave_sum_u64(ts.lds_nodes), u = wave_sum_u64(ts.unocc);
    if (lane_id() == 0) {  // the wave-schedule counts are kept by every lane alike: lane 0's
        atomicAdd(&counters[1], a);
        atomicAdd(&counters[2], c);
        atomicAdd(&counters[3], d);
        atomicAdd(&counters[4], e);
        atomicAdd(&counters[8], r);
        atomicAdd(&counters[9], (unsigned long long)ts.steps);
        atomicAdd(&counters[10], (unsigned long long)ts.active);
        atomicAdd(&counters[11], (unsigned long long)ts.node_steps);
        atomicAdd(&counters[12], (unsigned long long)ts.tri_steps);
        atomicAdd(&counters[13], (unsigned long long)ts.refills);
        atomicAdd(&counters[14], l);
        atomicAdd(&counters[18], u);
        for (int k = 0; k < 6; ++k) atomicAdd(&counters[20 + k], (unsigned long long)ts.coh[k]);
        atomicAdd(&counters[26], (unsigned long long)ts.coh_lanes);
    }
}

// Per-bounce counters: queue length and shadow-queue length, each on its own 128-B line
// (appends from different queues never contend for one L2 line).  Zeroed per frame.
// Default / Layered shading items are queued per bucket (shade_bucket): kNeeBuckets NEE and
// kShadeBuckets BSDF-sample counters follow the two queue counters.
constexpr int kShadeBuckets = 3;
// NEE buckets (round 6): 0 = conductor; 1 = kNeeCross, layered items whose light lies across the
// shading plane from the viewer (PT_NEE_CROSS), so that every other layered NEE wave runs the
// walk's compile-time path (layered_f_split; without it 70 % of Sponza-class's and 45 % of
// Layered's walk waves held such a lane, 4.2 / 1.6 % of the lanes, tools/nee_probe.py); then per
// albedo class k (kNeeClasses) the layered items with a smooth (2 + 2k) and a rough (3 + 2k) top.
// The walk's Russian roulette ends walks over a dark bottom layer early, so a wave that mixes
// them with bright ones runs as long as its brightest lane: the class of an item is the largest
// channel of its albedo against PT_NEE_MID (classes >= 3) and PT_NEE_DARK (classes >= 2).
// Bucket q fills region q / 2 of W.nq from the front (q even) or the back (q odd): a bounce
// queues at most W.paths NEE items in all, so the two ends of a region never meet.
#ifndef PT_NEE_CROSS
#define PT_NEE_CROSS 1
#endif
#ifndef PT_NEE_CLASSES
#define PT_NEE_CLASSES 2
#endif
#ifndef PT_NEE_DARK
#define PT_NEE_DARK 0.5f
#endif
#ifndef PT_NEE_MID
#define PT_NEE_MID 0.7f
#endif
constexpr int kNeeClasses = PT_NEE_CLASSES;
constexpr int kNeeBuckets = 2 + 2 * kNeeClasses;
constexpr int kNeeRegions = kNeeBuckets / 2;
constexpr int kNeeCross = 1;
static_assert(kNeeBuckets <= 8, "a shadow ray's item code holds the NEE bucket in bits 28-30");
// PT_SMP_DARK (> 0): a dark class of the BSDF-sample items, as PT_NEE_DARK (not kept):
// kSmpDark0 + 0 / 1 beside buckets 1 / 2, from the back of regions 1 / 2 of W.sq
#ifndef PT_SMP_DARK
#define PT_SMP_DARK 0.0f
#endif
constexpr bool kSmpDark = PT_SMP_DARK > 0.0f;
constexpr int kSmpBuckets = kShadeBuckets + (kSmpDark ? 2 : 0);
constexpr int kSmpDark0 = kShadeBuckets;
constexpr int kCnt = 5 + kNeeBuckets + kSmpBuckets;
constexpr int kCntStride = 32;  // ints per counter = 128 B
// kPool*: the run-time ray pools of k_trace_pair, k_extend and k_shadow_vis (RayPool)
enum { kQueue = 0, kShadowQ = 1, kNee0 = 2, kSmp0 = 2 + kNeeBuckets, kPool = 2 + kNeeBuckets + kSmpBuckets, kPoolExt, kPoolSh };
__device__ __forceinline__ int* cnt(const WFState& W, int b, int k) { return W.count + (kCnt * b + k) * kCntStride; }
// Slot `slot` of NEE bucket q in W.nq
__device__ __forceinline__ size_t nee_index(const WFState& W, int q, int slot) {
    const size_t r = (size_t)(q >> 1) * W.paths;
    return (q & 1) ? r + W.paths - 1 - slot : r + slot;
}
// NEE bucket of a layered item (sample bucket bk 1 / 2: smooth / rough top) from its albedo
__device__ __forceinline__ int nee_layered_bucket(int bk, f3 albedo) {
    const float m = fmaxf(fmaxf(albedo.x, albedo.y), albedo.z);
    int cls = 0;
    if (kNeeClasses >= 3 && m < PT_NEE_MID) cls = 1;
    if (kNeeClasses >= 2 && m < PT_NEE_DARK) cls = kNeeClasses - 1;
    return 2 + 2 * cls + (bk - 1);
}
// Slot `slot` of sample bucket q in W.sq: region q from the front, the dark buckets from the back
// of regions 1 / 2
__device__ __forceinline__ size_t smp_index(const WFState& W, int q, int slot) {
    if (q < kShadeBuckets) return (size_t)q * W.paths + slot;
    return (size_t)(q - kSmpDark0 + 2) * W.paths - 1 - slot;
}
// Path throughput | seed.  W.beta in path order (the phases of a bounce read it by path), except
// in the Lambert mode: in queue order next to the ray, ping-pong like ray_o / ray_d (queue b
// in W.beta for even b, W.beta_q for odd b), so k_shade_fused streams it instead of gathering it
// by path: a random 16-B read costs a 64-B line fetch (DESIGN.md §4 counter calibration).
// Queue 0 is in path order, so k_camera's W.beta[q] serves both layouts.
__device__ __forceinline__ float4* queue_beta(const WFState& W, int b) { return (b & 1) ? W.beta_q : W.beta; }
inline size_t count_bytes(int max_bounces) { return sizeof(int) * kCntStride * kCnt * (size_t)(max_bounces + 2); }

// Shading kernels: 1024-thread blocks, one queue item per thread over a grid sized to the
// queue capacity; blocks past the live queue length exit at once.  Queue appends are
// aggregated per block (one atomic per 1024 items): same-address atomics serialise at the
// L2 (≈90 per µs per word, MI355X_MICROARCH.md "dequeue"), and one atomic per wave cost
// ≈0.4 ms per shading launch at 2 M paths.  (Measured alternatives, see DESIGN.md:
// persistent grids with one atomic fetch head serialise the same way, and chunked fetching
// starves waves.)
constexpr int kBlockSh = 1024;
constexpr int kWavesSh = kBlockSh / 64;
#ifndef PT_SHA_BLOCK
#define PT_SHA_BLOCK 1024  // k_shade_a (Default / Layered); 512 / 256: +0.7 % / -3 %, DESIGN.md §5
#endif
constexpr int kBlockShA = PT_SHA_BLOCK, kWavesShA = kBlockShA / 64;
// k_shade_fused waves per SIMD: a CU holds two 1024-thread blocks only at <= 64 VGPRs (8 waves
// per SIMD); at 65..128 VGPRs one block per CU halves the occupancy (measured: 66 VGPRs made
// the Lambert shade 37 % slower).  Lambert fits 64 VGPRs untextured; Dielectric spills ~22
// VGPRs at 64 and still runs 6 % faster (1,795 -> 1,905 Msamples/s); Conductor spills ~41
// and is 1.4 % slower, so it keeps its natural allocation.
#ifndef PT_SHF_WAVES
#define PT_SHF_WAVES 8
#endif
#ifndef PT_SHF_WAVES_OTHER
#define PT_SHF_WAVES_OTHER 1
#endif
constexpr int shf_waves(int mode) { return (mode == 1 || mode == 3) /*Lambert, Dielectric*/ ? PT_SHF_WAVES : PT_SHF_WAVES_OTHER; }
// k_shade_fused / k_shade0_pixel block size per mode.  Conductor and Dielectric run in 256-thread
// blocks: +12.6 % and +6.1 % with the two wavefront streams; Lambert loses 5 % at
// 256, so it keeps 1024.
#ifndef PT_SHF_BLOCK_DIELECTRIC
#define PT_SHF_BLOCK_DIELECTRIC 256
#endif
#ifndef PT_SHF_BLOCK_CONDUCTOR
#define PT_SHF_BLOCK_CONDUCTOR 256
#endif
#ifndef PT_SHF_BLOCK_LAMBERT
#define PT_SHF_BLOCK_LAMBERT 1024
#endif
constexpr int shf_block(int mode) {
    return mode == 3 ? PT_SHF_BLOCK_DIELECTRIC : mode == 2 ? PT_SHF_BLOCK_CONDUCTOR : PT_SHF_BLOCK_LAMBERT;
}
// k_shade_nee / k_shade_smp (Default / Layered: the stochastic GlossyDiffuse eval, the sample)
// run in 256-thread blocks at 4 waves per SIMD (128 VGPRs).  (Round 2 before the bucketed
// queues: one kernel with both phases behind a block barrier, where 256-thread blocks beat
// 1024 / 512 / 128 / 64 threads: Layered 433 vs 375 / 431 / 427 / 425 Msamples/s)
#ifndef PT_SHB_BLOCK
#define PT_SHB_BLOCK 256
#endif
#ifndef PT_SHB_WAVES
#define PT_SHB_WAVES 4  // waves per SIMD the register allocator must allow (128 VGPRs)
#endif
#ifndef PT_SMP_WAVES
#define PT_SMP_WAVES 5  // k_shade_smp: 96 VGPRs, 4-12 spilled; configs 3 / 5 / Layered +0.6 / +0.5 / +0.9 % over 4
#endif
constexpr int kBlockShB = PT_SHB_BLOCK;

#ifndef PT_NEE_LEAN
#define PT_NEE_LEAN 1  // k_shade_nee keeps four values live across the walk
#endif

// Block-wide compaction: every thread of the block calls this (uniform control flow);
// threads with pred get consecutive slots.  `lds` is kWavesSh + 1 ints of shared memory
// private to this call site.
template <int WAVES>
__device__ __forceinline__ int block_append(int* counter, bool pred, int* lds) {
    const unsigned long long m = __ballot(pred ? 1 : 0);
    const int prefix = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const int wave = threadIdx.x >> 6;
    if (lane_id() == 0) lds[wave] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int tot = 0;
        for (int w = 0; w < WAVES; ++w) {
            const int c = lds[w];
            lds[w] = tot;
            tot += c;
        }
        lds[WAVES] = tot > 0 ? atomicAdd(counter, tot) : 0;
    }
    __syncthreads();
    return lds[WAVES] + lds[wave] + prefix;
}

// Block-wide append with one atomic per block whose slots are ordered by key: the block's range
// holds its key-0 items first, then key 1, ... (thread order within a key); key < 0 appends
// nothing.  Consecutive queue entries then share their key (the shadow rays' light, the
// continuation rays' direction octant), so the trace kernels' waves trace rays that take similar
// paths through the BVH.  `lds` holds K * WAVES + K + 1 ints.
template <int WAVES, int K>
__device__ __forceinline__ int block_append_sorted(int* counter, int key, int* lds) {
    const int wave = threadIdx.x >> 6;
    unsigned long long mine = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const unsigned long long m = __ballot(key == k ? 1 : 0);
        if (key == k) mine = m;
        if (lane_id() == 0) lds[k * WAVES + wave] = __popcll(m);
    }
    __syncthreads();
    if ((int)threadIdx.x < K) {  // per key: the waves' exclusive prefix and the key's total
        const int k = threadIdx.x;
        int tot = 0;
        for (int w = 0; w < WAVES; ++w) {
            const int c = lds[k * WAVES + w];
            lds[k * WAVES + w] = tot;
            tot += c;
        }
        lds[K * WAVES + 1 + k] = tot;
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // the keys' exclusive prefix, one atomic for the block
        int tot = 0;
        for (int k = 0; k < K; ++k) {
            const int c = lds[K * WAVES + 1 + k];
            lds[K * WAVES + 1 + k] = tot;
            tot += c;
        }
        lds[K * WAVES] = tot > 0 ? atomicAdd(counter, tot) : 0;
    }
    __syncthreads();
    if (key < 0) return 0;
    const int pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
    return lds[K * WAVES] + lds[K * WAVES + 1 + key] + lds[key * WAVES + wave] + pre;
}
// PT_SORT_SHADOW / PT_SORT_EXT: the fused shading kernels append their shadow rays ordered by light
// and their continuation rays ordered by direction octant within each block (block_append_sorted)
#ifndef PT_SORT_SHADOW
#define PT_SORT_SHADOW 0
#endif
#ifndef PT_SORT_EXT
#define PT_SORT_EXT 0
#endif
constexpr int kSortKeys = 8;
__device__ __forceinline__ int octant(f3 d) { return (d.x < 0.0f ? 1 : 0) | (d.y < 0.0f ? 2 : 0) | (d.z < 0.0f ? 4 : 0); }

// Block-wide append into K bucket regions (counter of bucket k at counter0 + k * kCntStride):
// threads with bucket k in [0, K) get consecutive slots of region k in thread order, bucket < 0
// appends nothing.  One atomic per non-empty bucket per block.  `lds` holds K * (WAVES + 1) ints.
template <int WAVES, int K>
__device__ __forceinline__ int block_append_k(int* counter0, int bucket, int* lds) {
    const int wave = threadIdx.x >> 6;
    unsigned long long mine = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const unsigned long long m = __ballot(bucket == k ? 1 : 0);
        if (bucket == k) mine = m;
        if (lane_id() == 0) lds[k * WAVES + wave] = __popcll(m);
    }
    __syncthreads();
    if ((int)threadIdx.x < K) {
        const int k = threadIdx.x;
        int tot = 0;
        for (int w = 0; w < WAVES; ++w) {
            const int c = lds[k * WAVES + w];
            lds[k * WAVES + w] = tot;
            tot += c;
        }
        lds[K * WAVES + k] = tot > 0 ? atomicAdd(counter0 + k * kCntStride, tot) : 0;
    }
    __syncthreads();
    if (bucket < 0) return 0;
    const int pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(mine >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mine, 0u));
    return lds[K * WAVES + bucket] + lds[bucket * WAVES + wave] + pre;
}

// Bucket of a Default / Layered shading item.  The items of one bucket run the same BSDF code
// path, so the NEE and sample kernels take them from per-bucket queue regions and their waves
// hold one kind of item: 0 = conductor (Default mode's metallic coin, devicePrograms.cu:400),
// 1 / 2 = the layered BSDF with a smooth / rough top interface (layered_f's topSpec: alpha =
// roughness^2 < 1e-3, GlossyDiffuse.h).  These are the sample buckets; the NEE items split the
// layered ones further (nee_layered_bucket, kNeeCross).
template <int MODE>
__device__ __forceinline__ int shade_bucket(bool conductor, float roughness) {
    if (MODE == kModeDefault && conductor) return 0;
    return sqr(roughness) < 1e-3f ? 1 : 2;
}
constexpr int kItemBits = 28;  // a queue item index is < 2^28 (kMaxWFPaths); the bucket sits above it

// Paths of nf consecutive frames are in flight together (path q = f * P + pixel), so every
// launch works on nf frames' queues: fewer launches and one SIMT tail per nf frames.
// lean (fused modes with the primary dedup): k_extend traces only frame 0's camera rays and the
// bounce-0 k_shade_fused derives the rest of the path state itself (shade0), so only frame 0's
// rays are written -- the other frames' copies, throughputs and radiances are never read.
__global__ __launch_bounds__(kBlockWF) void k_camera(WFState W, DevLaunch L, uint32_t frame0, int nf, int lean) {
    const int P = L.width * L.height;
    const int Q = P * nf;
    if (wf_cancelled(W)) return;  // no barrier below; the queue count stays 0 if wave 0 of block 0 returns
    if (lean) {
        for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < P; q += gridDim.x * blockDim.x) {
            f3 o, d;
            camera_ray(L, q % L.width, q / L.width, o, d);
            W.ray_o[0][q] = make_float4(o.x, o.y, o.z, __int_as_float(q));
            W.ray_d[0][q] = make_float4(d.x, d.y, d.z, 0.0f);
        }
        if (blockIdx.x == 0 && threadIdx.x == 0) *cnt(W, 0, kQueue) = Q;
        return;
    }
    for (int q = blockIdx.x * blockDim.x + threadIdx.x; q < Q; q += gridDim.x * blockDim.x) {
        const int f = q / P, p = q - f * P;
        const int x = p % L.width, y = p / L.width;
        f3 o, d;
        camera_ray(L, x, y, o, d);
        W.ray_o[0][q] = make_float4(o.x, o.y, o.z, __int_as_float(q));
        W.ray_d[0][q] = make_float4(d.x, d.y, d.z, 0.0f);
        const uint32_t seed = tea16((uint32_t)(L.width * (y + L.row0) + x), frame0 + (uint32_t)f);  // devicePrograms.cu:631
        W.beta[q] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(seed));
        W.L[q] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *cnt(W, 0, kQueue) = Q;
}

// This wave's static slice of a queue of length n (grid sized to residency, so every wave
// is resident and slices balance statistically; no fetch atomics).
#ifndef PT_REFILL_MIN
#define PT_REFILL_MIN 16  // idle lanes before a wave refills (24 before the triangle batches;
                          // with them 12 / 16 / 20 / 32: -1 / 0 / -0 / -5 %)
#endif
constexpr int kRefillMin = PT_REFILL_MIN;
#ifndef PT_SPLIT_FINISH  // k_trace_pair's deferred NEE add as load + store around the refill:
#define PT_SPLIT_FINISH 1  // +2.2 % Lambert, +1.3 % Conductor, +0.4 % Dielectric
#endif

#ifndef PT_TRI_BATCH
#define PT_TRI_BATCH 20  // lanes with a pending leaf before a wave runs its triangle batch (8 / 12 / 16 /
                         // 20 / 24 / 32: -7 / -2 / -0.3 / 0 / -0.3 / -5 %)
#endif

// chunk_log = k > 0: the queue is cut into chunks of 2^k rays dealt round-robin to the waves,
// so every wave's share samples the whole queue instead of one contiguous stretch of image rows
// (whose cost differs from the next stretch's).  A wave then walks a virtual range [0, count) of
// its chunks, and slice_ray maps a virtual index to the queue index.  k_extend and k_shadow_vis
// use PT_SLICE_CHUNK_LOG_X, k_trace_pair contiguous slices.
#ifndef PT_SLICE_CHUNK_LOG
#define PT_SLICE_CHUNK_LOG 0
#endif
#ifndef PT_SLICE_CHUNK_LOG_X
#define PT_SLICE_CHUNK_LOG_X PT_SLICE_CHUNK_LOG
#endif
__device__ __forceinline__ void wave_slice(int n, int& first, int& end, int chunk_log = 0) {
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nwaves = (int)((gridDim.x * blockDim.x) >> 6);
    if (chunk_log > 0) {
        const int K = 1 << chunk_log;
        const int chunks = (n + K - 1) / K;
        const int mine = chunks > wave ? (chunks - 1 - wave) / nwaves + 1 : 0;
        first = 0;
        // only the queue's last chunk is partial, and it is the last chunk of its wave
        end = mine * K - ((chunks > 0 && (chunks - 1) % nwaves == wave) ? chunks * K - n : 0);
        return;
    }
    const int per = (n + nwaves - 1) / nwaves;
    first = min(n, wave * per);
    end = min(n, first + per);
}
// queue index of the wave's virtual index v (identity without chunks)
__device__ __forceinline__ int slice_ray(int v, int chunk_log) {
    if (chunk_log == 0) return v;
    const int wave = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6);
    const int nwaves = (int)((gridDim.x * blockDim.x) >> 6);
    return (((v >> chunk_log) * nwaves + wave) << chunk_log) + (v & ((1 << chunk_log) - 1));
}

typedef float pt_v4f __attribute__((ext_vector_type(4)));
// k_shade_fused (the memory-bound kernel of a fused-mode frame, ≈ 66 % of HBM peak) streams
// its queue records and the path state once: non-temporal loads and stores keep them from
// evicting the triangle and material lines its gathers reuse.  Lambert +2 %, Dielectric and
// Conductor +0.4 %.  (The same hint on the trace kernels' queues: ±0.5 %, not
// used -- they are not memory-bound.)
__device__ __forceinline__ float4 ldqs(const float4* p) {
    const pt_v4f v = __builtin_nontemporal_load(reinterpret_cast<const pt_v4f*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void stqs(float4* p, float4 v) {
    __builtin_nontemporal_store(pt_v4f{v.x, v.y, v.z, v.w}, reinterpret_cast<pt_v4f*>(p));
}

// k_trace_pair's queue records (DESIGN.md §5 "Where k_trace_pair's memory traffic goes"):
// PT_TRACE_NTQ = 1 loads and stores them non-temporally; PT_PROBE_NO_NEE_ADD = 1 drops the deferred
// NEE add (a measurement probe: wrong images, same rays).
#ifndef PT_TRACE_NTQ
#define PT_TRACE_NTQ 1  // 19 % less k_trace_pair traffic, rate ±0.2 %
#endif
#ifndef PT_PROBE_NO_NEE_ADD
#define PT_PROBE_NO_NEE_ADD 0
#endif
// How an unoccluded shadow ray of k_trace_pair adds its contribution to W.L[path]: 0 = load in
// finish + store in commit (v37); 1 = three no-return float atomics; 2 = the ray only writes its
// path (or -1) into its own sh_c record and k_nee_add adds in shadow-queue order after the launch.
#ifndef PT_NEE_MODE
#define PT_NEE_MODE 0
#endif
__device__ __forceinline__ float4 ldq_pair(const float4* p) { return PT_TRACE_NTQ ? ldqs(p) : *p; }
// the same for k_extend and k_shadow_vis (PT_TRACE_NTQ_X)
#ifndef PT_TRACE_NTQ_X
#define PT_TRACE_NTQ_X 0  // configs 3 / 5 +0.1 / +0.3 %, Lambert -0.6 %: not kept
#endif
__device__ __forceinline__ float4 ldq_x(const float4* p) { return PT_TRACE_NTQ_X ? ldqs(p) : *p; }
__device__ __forceinline__ void stq_x(float4* p, float4 v) {
    if (PT_TRACE_NTQ_X)
        stqs(p, v);
    else
        *p = v;
}
__device__ __forceinline__ void stq_pair(float4* p, float4 v) {
    if (PT_TRACE_NTQ)
        stqs(p, v);
    else
        *p = v;
}

// PT_TAIL_PROBE = 1 (measurement only): every k_trace_pair wave adds its start and end times
// (s_memrealtime, 100 MHz) to module counters, and the last wave of the launch prints the launch
// span, the waves' mean lifetime and the spread of their end times, so the static slices' tail
// can be read off.
#ifndef PT_TAIL_PROBE
#define PT_TAIL_PROBE 0
#endif
#if PT_TAIL_PROBE
__device__ unsigned long long g_tail[5];  // ~min start, max end, sum end, finished waves, sum start
__device__ __forceinline__ void tail_probe_begin(unsigned long long& t0) {
    t0 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) == 0) {
        atomicMax(&g_tail[0], ~t0);
        atomicAdd(&g_tail[4], t0);
    }
}
__device__ __forceinline__ void tail_probe_end(int b) {
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    if ((threadIdx.x & 63) != 0) return;
    atomicMax(&g_tail[1], t1);
    atomicAdd(&g_tail[2], t1);
    __threadfence();
    const unsigned long long nw = (unsigned long long)gridDim.x * (blockDim.x / 64);
    if (atomicAdd(&g_tail[3], 1ull) == nw - 1) {
        __threadfence();
        const unsigned long long t0 = ~atomicAdd(&g_tail[0], 0ull), te = atomicAdd(&g_tail[1], 0ull);
        const unsigned long long se = atomicAdd(&g_tail[2], 0ull), ss = atomicAdd(&g_tail[4], 0ull);
        const double mean_end = (double)se / (double)nw - (double)t0, mean_start = (double)ss / (double)nw - (double)t0;
        printf("TAIL b=%d waves=%llu span_us=%.1f mean_start_us=%.1f mean_end_us=%.1f idle_frac=%.4f\n", b, nw,
               (double)(te - t0) / 100.0, mean_start / 100.0, mean_end / 100.0,
               1.0 - (mean_end - mean_start) / (double)(te - t0));
        for (int k = 0; k < 5; ++k) atomicExch(&g_tail[k], 0ull);  // vector atomics, no plain stores
        __threadfence();
    }
}
#endif

// Lane-refilling trace loop over a queue slice: `fetch(ri, state)` initialises lane state
// for ray ri, `finish(ri, state)` consumes a finished ray.  A finish that returns a token is
// split in two: its loads are issued before the refill's record loads and `commit(token)` (its
// stores) runs after them, so the two memory round trips of a batch block overlap
// (PT_SPLIT_FINISH).  A lane whose traversal ends parks
// (`done`) until enough lanes are idle; then the wave runs one batch block that finishes the
// parked rays and refills the idle lanes with the next rays of the slice.  The triangle
// batches take acceptable hits only (wave_tri_batch), so a finished ray's answer is final.
// The rays of a trace launch dealt at run time (PT_TRACE_POOL): queue range [begin, end), handed
// out in chunks of PT_POOL_CHUNK through the counter ctr (zeroed with the queue counters) to the
// waves whose static slices ran out.
#ifndef PT_TRACE_POOL
#define PT_TRACE_POOL 60  // percent of k_trace_pair's rays in the pool (0: static slices only)
#endif
#ifndef PT_TRACE_POOL_X
#define PT_TRACE_POOL_X 60  // the same for k_extend and k_shadow_vis
#endif
#ifndef PT_POOL_CHUNK
#define PT_POOL_CHUNK 512
#endif
// launches of fewer rays than this many per wave keep static slices only: a one-frame call's
// launches (about 300 rays per wave) ran 40 % slower with the pool
#ifndef PT_POOL_MIN_PER_WAVE
#define PT_POOL_MIN_PER_WAVE 2048
#endif
__device__ __forceinline__ bool pool_pays(int n) {
    const long long nwaves = (long long)((gridDim.x * blockDim.x) >> 6);
    return (long long)n >= nwaves * PT_POOL_MIN_PER_WAVE;
}
struct RayPool {
    int* ctr = nullptr;
    int begin = 0, end = 0;
    int chunk_log = 0;  // the static slices' chunk interleave (wave_slice)
};

struct NoCommit {
    template <class T>
    __device__ void operator()(const T&) const {}
};
template <int ANY, bool STATS, bool TEX, int BLK, class Fetch, class Finish, class Commit = NoCommit>
__device__ __forceinline__ void trace_range(const DevScene& S, int next, int end, int* stk, TriBatchLds* tri_lds,
                                            TravStats& ts, const WFState& W, Fetch fetch, Finish finish,
                                            Commit commit = Commit{}, RayPool pool = RayPool{}) {
    using Tok = decltype(finish(0, *static_cast<const TravState*>(nullptr)));
    constexpr bool kSplit = !std::is_void_v<Tok>;
    using TokS = std::conditional_t<kSplit, Tok, int>;
    int spill[kSpillDepth];
    TravState st;
    int ri = -1;
    bool done = false;
    // the slice bounds are wave-uniform: keeping them (and the refill bookkeeping) in SGPRs
    // makes the per-step refill test scalar work (it was VALU, with an f64 min from the
    // unsigned popcount; ±0.3 %)
    next = __builtin_amdgcn_readfirstlane(next);
    end = __builtin_amdgcn_readfirstlane(end);
    // look-ahead cancellation (wf_cancel_poll): a cancelled batch's wave stops taking rays from its
    // slice (it finishes the ones in flight), at the start and at every 16th batch block; one wave
    // in eight workgroups relays the host word at every 64th
    uint32_t npoll = 0;
    int* pctr = pool.ctr;
    int vlog = pool.chunk_log;  // the static slice walks chunk-interleaved virtual indices
    if (W.cancel_seen && wf_cancel_poll(W, false)) {
        end = next;
        pctr = nullptr;
    }
    while (true) {
        // batch block once enough lanes idle (it costs the wave about as much as a step), and
        // at every step once the slice is drained
        if ((int)__popcll(__ballot(ri < 0 || done)) >= kRefillMin || next >= end) {
            if (W.cancel_seen && (++npoll & 15) == 0 &&
                wf_cancel_poll(W, (npoll & 63) == 0 && (blockIdx.x & 7) == 0 && threadIdx.x == 0)) {
                end = next;
                pctr = nullptr;
            }
            if (pctr && next >= end) {  // static share drained: the next chunk of the pool
                int base = 0;
                if ((threadIdx.x & 63) == 0) base = atomicAdd(pctr, PT_POOL_CHUNK);
                base = __builtin_amdgcn_readfirstlane(__shfl(base, 0, 64));
                vlog = 0;
                next = min(pool.begin + base, pool.end);
                end = min(next + PT_POOL_CHUNK, pool.end);
                if (next >= pool.end) pctr = nullptr;
            }
#if PT_CYCLE_PROBE
            const uint64_t c0 = probe_clock();
#else
            if (STATS) ts.refills++;
#endif
            TokS tok{};
            const bool fin = done;
            if (done) {  // the triangle batches took acceptable hits only: the answer stands
                if constexpr (kSplit)
                    tok = finish(ri, st);
                else
                    finish(ri, st);
                ri = -1;
                done = false;
            }
            const unsigned long long m = __ballot(ri < 0);
            const int pre = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (ri < 0 && next + pre < end) {
                ri = vlog ? slice_ray(next + pre, vlog) : next + pre;
                fetch(ri, st);
                if (STATS) ts.rays++;
                done = S.ntri <= 0;  // empty scene: no BVH root, every ray misses
            }
            next = min(next + (int)__popcll(m), end);
            if constexpr (kSplit) {
                if (fin) commit(tok);
            }
#if PT_CYCLE_PROBE
            if (STATS) ts.refills += (uint32_t)(probe_clock(st.best) - c0);
#endif
        }
        const bool active = ri >= 0 && !done;
        const unsigned long long act = __ballot(active);
        // only parked lanes left: the next batch block finishes them.  The loop keeps a single
        // back edge (no `continue`): with two latch paths the compiler copied ~20 registers of lane
        // state between them every iteration (12 % of the kernel's VALU instructions)
        if (!act && !__ballot(ri >= 0)) break;
        // postponed leaves: test the pending leaves once enough lanes hold one, or when too few
        // lanes have a node left to visit (then the leaves are the work)
        const int n_act = __popcll(act);
        const int n_leaf = __popcll(__ballot(active && st.leaf != kEmptyChild));
        const int n_node = __popcll(__ballot(active && st.cur >= 0));
        const bool tri_ok = n_leaf >= min(PT_TRI_BATCH, n_act) || 2 * n_node < n_act;
        if (STATS) {
            ts.steps++;
#if !PT_CYCLE_PROBE
            ts.active += n_act;
            ts.node_steps += n_node > 0;
            ts.tri_steps += tri_ok && n_leaf > 0;
#endif
        }
#if PT_CYCLE_PROBE
        const uint64_t c1 = probe_clock();
#endif
        // the triangles of every pending leaf in one wave batch (pt_device.h wave_tri_batch),
        // then the node half of the step
        if (tri_ok && n_leaf > 0) {  // wave-uniform
            wave_tri_batch<ANY, STATS, TEX>(S, st, active && st.leaf != kEmptyChild, tri_lds, ts);
            if (active && is_any<ANY>(st) && st.h.tri >= 0) done = true;
        }
#if PT_CYCLE_PROBE
        const uint64_t c2 = probe_clock(st.best);
        if (STATS) ts.tri_steps += (uint32_t)(c2 - c1);
#endif
        if (STATS) {  // distinct global nodes among the lanes about to load one (pt_get_trace_coherence)
            const bool g = active && !done && st.cur >= S.n_lds;
            unsigned long long rem = __ballot(g);
            if (rem) {
                ts.coh_lanes += (uint32_t)__popcll(rem);
                int distinct = 0;
                while (rem) {
                    const int node = __shfl(st.cur, __ffsll((long long)rem) - 1, 64);
                    rem &= ~__ballot(g && st.cur == node);
                    ++distinct;
                }
                ts.coh[distinct <= 2 ? distinct - 1 : distinct <= 4 ? 2 : distinct <= 8 ? 3 : distinct <= 16 ? 4 : 5]++;
            }
        }
        if (active && !done && trav_node_step<ANY, STATS, kStack>(S, st, stk, BLK, spill, ts)) done = true;
#if PT_CYCLE_PROBE
        if (STATS) {  // node half: until its loads landed (active), the rest (node_steps)
            const uint64_t c4 = probe_clock(st.cur);
            const unsigned long long ml = __ballot(ts.probe_t > c2);
            const uint64_t tl = ml ? (uint64_t)__shfl((long long)ts.probe_t, __ffsll((long long)ml) - 1, 64) : c2;
            ts.active += (uint32_t)(tl - c2);
            ts.node_steps += (uint32_t)(c4 - tl);
        }
#endif
    }
}

// A trace kernel's queue range [first, end): the workgroup's LDS (per-lane stacks, the staged top
// BVH levels, the triangle batches), then the lane-refilling loop.
template <int ANY, bool STATS, bool TEX, int BLK, class Fetch, class Finish, class Commit = NoCommit>
__device__ __forceinline__ void trace_queue(DevScene S, int first, int end, TravStats& ts, const WFState& W, Fetch fetch,
                                            Finish finish, Commit commit = Commit{}, RayPool pool = RayPool{}) {
    constexpr int kNodes = lds_nodes_of<BLK>();
    __shared__ int stack[kStack * BLK];
    __shared__ BNode4 top[kNodes > 0 ? kNodes : 1];
    __shared__ TriBatchLds tri_batch[BLK / 64];
    stage_top_nodes<kNodes>(S, top);
    trace_range<ANY, STATS, TEX, BLK>(S, first, end, stack + threadIdx.x, tri_batch + (threadIdx.x >> 6), ts, W, fetch,
                                      finish, commit, pool);
}

template <int ANY, bool STATS, bool TEX, int BLK, class Fetch, class Finish>
__device__ __forceinline__ void trace_slice(const DevScene& S, int n, TravStats& ts, const WFState& W, Fetch fetch,
                                            Finish finish, int* pool_ctr) {
    int next, end;
    RayPool pool;
    pool.chunk_log = PT_SLICE_CHUNK_LOG_X;
    pool.end = n;
    if (PT_TRACE_POOL_X > 0 && pool_pays(n)) {
        pool.ctr = pool_ctr;
        pool.begin = n - (int)((long long)n * PT_TRACE_POOL_X / 100);
    } else {
        pool.begin = n;
    }
    wave_slice(pool.begin, next, end, pool.chunk_log);
    trace_queue<ANY, STATS, TEX, BLK>(S, next, end, ts, W, fetch, finish, NoCommit{}, pool);
}

// Closest hit of queue b.  `dup` > 1 (bounce 0 only): the queue holds `dup` copies of the same
// camera rays (one per frame of the batch: the reference has no pixel jitter, so a pixel's ray
// is identical in every frame, devicePrograms.cu:601-623), so only the first n / dup are traced
// and each hit record is written to all copies.  The records are bit-identical to tracing every
// copy; DESIGN.md §5 gives the A/B.
template <bool STATS, bool TEX, int BLK = kBlockTrace>
__global__ __launch_bounds__(BLK, wf_waves(TEX)) void k_extend(DevScene S, WFState W, int b, int dup,
                                                                  int copies, unsigned long long* counters) {
    const int n = *cnt(W, b, kQueue);
    const int n_trace = n / dup;
    const float4* ro = W.ray_o[b & 1];
    const float4* rd = W.ray_d[b & 1];
    TravStats ts;
    trace_slice<kRayClosest, STATS, TEX, BLK>(
        S, n_trace, ts, W,
        [&](int ri, TravState& st) {
            const float4 a = ldq_x(ro + ri), c = ldq_x(rd + ri);
            trav_init(st, mk(a.x, a.y, a.z), mk(c.x, c.y, c.z), 0.0f, 100.0f);
            st.path = __float_as_int(a.w);
        },
        [&](int ri, const TravState& st) {
            // copy k of a bounce-0 ray is path st.path + k * n_trace (queue 0 is in path order);
            // copies = 1: k_shade0_pixel reads the pixel's one record for all its frames
            for (int k = 0; k < copies; ++k)
                stq_x(W.hit + ri + (size_t)k * n_trace, hit_record(st.h, st.path + k * n_trace));
        }, cnt(W, b, kPoolExt));
    if (blockIdx.x == 0 && threadIdx.x == 0 && counters) {
        atomicAdd(&counters[0], (unsigned long long)n);        // path segments
        atomicAdd(&counters[6], (unsigned long long)n_trace);  // rays traced by the timed trace kernels
        atomicAdd(&counters[7], (32ull + 16ull * (unsigned long long)copies) * (unsigned long long)n_trace);  // bytes
    }
    flush_trav_stats<STATS>(counters, ts);
}

__device__ __forceinline__ Hit decode_hit(float4 hv) {
    Hit h;
    const int code = __float_as_int(hv.w);
    h.t = hv.x;
    h.u = hv.y;
    h.v = hv.z;
    h.back = code != kMissTri && (code & (int)0x80000000);
    h.tri = code == kMissTri ? -1 : (code & 0x7fffffff);
    return h;
}

// light choice: Lighting::GetRandomPointLight (LightMethods.h:25-40)
__device__ __forceinline__ float pick_light(const DevLaunch& L, uint32_t& seed, int& li) {
    li = 0;
    if (L.n_lights == 1) return 1.0f;
    if (L.n_lights <= 0) return 0.0f;
    float r = rnd(seed);
    li = (int)(r * (float)L.n_lights);
    if (li >= L.n_lights) li = L.n_lights - 1;
    return 1.0f / (float)L.n_lights;
}

// continuation (devicePrograms.cu:501-509) + loop test of SamplePath (:646)
__device__ __forceinline__ bool continue_path(const SurfaceHit& sf, const BSample& bs, f3& beta, f3& o, f3& d,
                                              int next_bounce, int max_bounces) {
    float ac = abs_dot(bs.dir, mk(0.0f, 0.0f, 1.0f));
    beta = beta * mk(bs.color.x * ac / bs.pdf, bs.color.y * ac / bs.pdf, bs.color.z * ac / bs.pdf);
    f3 off = 1e-3f * sf.ng;
    if (dot(bs.dir, mk(0.0f, 0.0f, 1.0f)) < 0.0f) off = -off;
    o = sf.pos + off;
    d = normalize(to_world(sf.fr, bs.dir));
    return next_bounce < max_bounces && length(beta) > 0.00001f;
}

// Bounce-0 shadow dedup (with primary dedup): a pixel's first hit is the same in every frame
// of the batch, so its shadow ray toward light li is too.  k_shadow0_setup builds one shadow
// ray per (pixel, light) from the frame-0 hit, k_shadow_vis traces them into W.vis[light *
// pixels + pixel], and the bounce-0 shading reads that table instead of tracing a shadow ray
// per path.  Same rays, same any-hit answers: the images stay bit-identical.
__device__ __forceinline__ int vis0_index(const DevLaunch& L, int path, int li) {
    const int P1 = L.width * L.height;
    return li * P1 + path % P1;  // light-major (coherent shadow rays); path = frame * P1 + pixel
}

template <bool TEX>
__global__ __launch_bounds__(kBlockWF) void k_shadow0_setup(DevScene S, DevLaunch L, WFState W) {
    const int P1 = L.width * L.height;
    const int nl = L.n_lights;
    const int n = P1 * nl;
    if (wf_cancelled(W)) return;  // no barrier below
    for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) {
        const int li = k / P1, p = k - li * P1;
        const Hit h = decode_hit(W.hit[p]);  // frame 0's copy (queue 0 is in path order)
        float4 so = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(k)), sd = make_float4(0.0f, 0.0f, 1.0f, 0.0f);
        if (h.tri >= 0) {  // same arithmetic as the shading kernels' shadow rays
            const float4 c = W.ray_d[0][p];
            SurfaceHit sf;
            reconstruct<TEX>(S, h, mk(c.x, c.y, c.z), sf);
            const DevLight lt = L.lights[li];
            const f3 ldir = mk(lt.px, lt.py, lt.pz) - sf.pos;
            const f3 o = sf.pos + 1e-3f * sf.ng;
            const f3 d = normalize(ldir);
            so = make_float4(o.x, o.y, o.z, __int_as_float(k));
            sd = make_float4(d.x, d.y, d.z, length(ldir));
        }
        W.sh_o[k] = so;
        W.sh_d[k] = sd;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) *cnt(W, 0, kShadowQ) = n;
}

// shade0 (bounce 0 after a lean k_camera): the path state is the camera's -- throughput 1, seed
// tea16(pixel, frame) (devicePrograms.cu:631), radiance 0, direction that of the pixel's frame-0
// ray (queue 0 is in path order) -- so it is derived here instead of read, and every path's
// radiance is written rather than updated.
template <int MODE, bool TEX, bool SHADE0>
__global__ __launch_bounds__(shf_block(MODE), shf_waves(MODE)) void k_shade_fused(DevScene S, DevLaunch L, WFState W, int b, int vis0) {
    constexpr bool shade0 = SHADE0;
    // Lambert (memory-bound, 56 VGPRs): the throughput in queue order (queue_beta), +1.6 %; the
    // Conductor and Dielectric kernels are register-bound, and holding it across the appends
    // cost them 1-2 %, so they gather it by path
    constexpr bool kBetaQ = MODE == kModeLambert;
    constexpr bool kShareOrigin = MODE == kModeLambert;
    constexpr int kBlock = shf_block(MODE), kWaves = kBlock / 64;
    const int n = *cnt(W, b, kQueue);
    const float4* rd = W.ray_d[b & 1];
    float4* no = W.ray_o[(b + 1) & 1];
    float4* nd = W.ray_d[(b + 1) & 1];
    __shared__ int lds_sh[kSortKeys * kWaves + kSortKeys + 1], lds_q[kSortKeys * kWaves + kSortKeys + 1];
    if (blockIdx.x == 0 && threadIdx.x == 0 && L.counters) atomicAdd(&L.counters[15], (unsigned long long)n);
    if ((int)(blockIdx.x * kBlock) >= n) return;  // block-uniform
    {
        const int i = (int)(blockIdx.x * kBlock + threadIdx.x);
        // a cancelled wave takes no item but still joins the block's appends (block_append)
        const bool valid = i < n && !wf_cancelled(W);
        bool emit_shadow = false, emit_next = false;
        f3 so, sdir, contrib, o, d, beta;
        uint32_t seed = 0;
        float stmax = 0.0f;
        int path = 0;
        int shadow_light = 0;
        const int P1 = L.width * L.height;
        float4 l0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // shade0: the path's radiance after bounce 0
        if (valid) {
            const float4 hv = ldqs(W.hit + i);
            // the queue-order records go out beside the hit record instead of after it: they do not
            // depend on it, and waiting for the hit first put two HBM round trips in a row (Lambert
            // +2 %)
            const float4 c_q = shade0 ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : ldqs(rd + i);
            const float4 bv_q = (!shade0 && kBetaQ) ? ldqs(queue_beta(W, b) + i) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            path = __float_as_int(hv.x);
            const Hit h = decode_hit(hv);
            if (h.tri >= 0) {  // a miss ends the path (__miss__radiance :576-583)
                const float4 c = shade0 ? ldqs(rd + path % P1) : c_q;
                d = mk(c.x, c.y, c.z);
                SurfaceHit sf;
                reconstruct<TEX>(S, h, d, sf);
                if (shade0) {
                    seed = tea16((uint32_t)(path % P1 + L.width * L.row0), L.frame_base + (uint32_t)(path / P1));
                    beta = mk(1.0f, 1.0f, 1.0f);
                } else {
                    float4 bv = kBetaQ ? bv_q : ldqs(W.beta + path);
                    seed = __float_as_uint(bv.w);
                    beta = mk(bv.x, bv.y, bv.z);
                }
                if (path == debug_path_id(L)) {  // pt_set_debug_pixel (devicePrograms.cu:637-644)
                    const float4 l = shade0 ? l0 : W.L[path];
                    debug_record(L, b + 1, __float_as_int(S.isect[3 * h.tri].w), sf, beta, mk(l.x, l.y, l.z));
                }
                const bool conductor = rnd(seed) < sf.metallic;  // :400
                int li;
                const float P = pick_light(L, seed, li);
                if (P > 0.0f) {
                    const DevLight lt = L.lights[li];
                    f3 lpos = mk(lt.px, lt.py, lt.pz);
                    f3 ldir = lpos - sf.pos;
                    f3 ldn = normalize(ldir);
                    f3 lds = to_local(sf.fr, ldn);
                    // f has no RNG side effects in these modes: evaluate before the shadow test
                    f3 f = bsdf_f<MODE>(seed, sf.albedo, sf.roughness, conductor, sf.wo, lds);
                    f3 spectrum = f * abs_dot(lds, mk(0.0f, 0.0f, 1.0f));
                    if (!is_zero(spectrum)) {
                        f3 dd = sf.pos - lpos;
                        float d2 = dd.x * dd.x + dd.y * dd.y + dd.z * dd.z;
                        f3 Li = mk(lt.cr, lt.cg, lt.cb) / d2;
                        contrib = ((beta * spectrum) * Li) / (P * 1.0f);
                        if (vis0) {  // bounce 0: the (pixel, light) visibility is already known
                            if (W.vis[vis0_index(L, path, li)]) {
                                const float4 l = shade0 ? l0 : W.L[path];
                                l0 = make_float4(l.x + contrib.x, l.y + contrib.y, l.z + contrib.z, 0.0f);
                                if (!shade0) W.L[path] = l0;
                            }
                        } else {
                            so = sf.pos + 1e-3f * sf.ng;
                            sdir = normalize(ldir);
                            stmax = length(ldir);
                            emit_shadow = true;
                            shadow_light = li;
                        }
                    }
                }
                BSample bs;
                // the last bounce's sampled direction is never traced (SamplePath :646)
                if (b + 1 < L.max_bounces &&
                    bsdf_sample<MODE>(seed, sf.albedo, sf.roughness, conductor, sf.wo, bs)) {
                    emit_next = continue_path(sf, bs, beta, o, d, b + 1, L.max_bounces);
                    if (!kBetaQ) stqs(W.beta + path, make_float4(beta.x, beta.y, beta.z, __uint_as_float(seed)));
                }
            }
        }
        if (shade0 && valid) W.L[path] = l0;  // every path of the batch, hit or miss
        const int qi = PT_SORT_EXT ? block_append_sorted<kWaves, kSortKeys>(cnt(W, b + 1, kQueue), emit_next ? octant(d) : -1, lds_q)
                                   : block_append<kWaves>(cnt(W, b + 1, kQueue), emit_next, lds_q);
        if (emit_next) {
            stqs(no + qi, make_float4(o.x, o.y, o.z, __int_as_float(path)));
            stqs(nd + qi, make_float4(d.x, d.y, d.z, 0.0f));
            if (kBetaQ) stqs(queue_beta(W, b + 1) + qi, make_float4(beta.x, beta.y, beta.z, __uint_as_float(seed)));
        }
        const int si = PT_SORT_SHADOW ? block_append_sorted<kWaves, kSortKeys>(cnt(W, b, kShadowQ),
                                                                              emit_shadow ? (shadow_light & (kSortKeys - 1)) : -1, lds_sh)
                                      : block_append<kWaves>(cnt(W, b, kShadowQ), emit_shadow, lds_sh);
        if (emit_shadow) {
            // Lambert: a sampled direction is never below the surface (lambert_sample forces z >= 0),
            // so the continuation ray starts at the shadow ray's origin (sf.pos + 1e-3 * Ng, the
            // same expression): the shadow record names that ray (qi) instead of repeating origin
            // and path, and k_trace_pair reads them from the extension queue.  -1: own sh_o record.
            const bool share = kShareOrigin && emit_next;
            if (!share) stqs(W.sh_o + si, make_float4(so.x, so.y, so.z, __int_as_float(path)));
            stqs(W.sh_d + si, make_float4(sdir.x, sdir.y, sdir.z, stmax));
            stqs(W.sh_c + si, make_float4(contrib.x, contrib.y, contrib.z, __int_as_float(share ? qi : -1)));
        }
    }
}

// Bounce 0 of a fused-mode batch with the primary dedup and the (pixel, light) visibility table:
// the nf paths of a pixel start from the same hit (no pixel jitter, devicePrograms.cu:601-623),
// so one thread reconstructs the pixel's surface once and shades its paths in frame order (k_extend
// wrote one hit record per pixel).  Per path: the operations of k_shade_fused<SHADE0> (throughput
// 1, seed tea16(pixel, frame), radiance written, continuation appended to queue 1).
template <int MODE, bool TEX>
__global__ __launch_bounds__(shf_block(MODE), 1) void k_shade0_pixel(DevScene S, DevLaunch L, WFState W, int nf) {
    constexpr bool kBetaQ = MODE == kModeLambert;  // as k_shade_fused
    constexpr int kBlock = shf_block(MODE), kWaves = kBlock / 64;
    const int P1 = L.width * L.height;
    __shared__ int lds_q[kSortKeys * kWaves + kSortKeys + 1];
    if (blockIdx.x == 0 && threadIdx.x == 0 && L.counters)
        atomicAdd(&L.counters[15], (unsigned long long)P1 * (unsigned long long)nf);
    if ((int)(blockIdx.x * kBlock) >= P1) return;  // block-uniform
    const int p = (int)(blockIdx.x * kBlock + threadIdx.x);
    const bool valid = p < P1 && !wf_cancelled(W);  // a cancelled wave still joins the appends
    int tri = -1;
    SurfaceHit sf;
    if (valid) {
        const float4 hv = W.hit[p];
        const Hit h = decode_hit(hv);
        tri = h.tri;
        if (tri >= 0) {
            const float4 c = W.ray_d[0][p];
            reconstruct<TEX>(S, h, mk(c.x, c.y, c.z), sf);
        }
    }
    const int dbg = debug_path_id(L);
    float4* no = W.ray_o[1];
    float4* nd = W.ray_d[1];
    for (int f = 0; f < nf; ++f) {  // uniform trip count (block_append below)
        const int path = f * P1 + p;
        bool emit_next = false;
        f3 o, d, beta = mk(1.0f, 1.0f, 1.0f);
        uint32_t seed = 0;
        float4 l0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (valid && tri >= 0) {
            seed = tea16((uint32_t)(p + L.width * L.row0), L.frame_base + (uint32_t)f);  // devicePrograms.cu:631
            if (path == dbg) debug_record(L, 1, __float_as_int(S.isect[3 * tri].w), sf, beta, mk(0.0f, 0.0f, 0.0f));
            const bool conductor = rnd(seed) < sf.metallic;  // :400
            int li;
            const float P = pick_light(L, seed, li);
            if (P > 0.0f) {
                const DevLight lt = L.lights[li];
                f3 lpos = mk(lt.px, lt.py, lt.pz);
                f3 lds = to_local(sf.fr, normalize(lpos - sf.pos));
                f3 fv = bsdf_f<MODE>(seed, sf.albedo, sf.roughness, conductor, sf.wo, lds);
                f3 spectrum = fv * abs_dot(lds, mk(0.0f, 0.0f, 1.0f));
                if (!is_zero(spectrum) && W.vis[vis0_index(L, path, li)]) {
                    f3 dd = sf.pos - lpos;
                    float d2 = dd.x * dd.x + dd.y * dd.y + dd.z * dd.z;
                    f3 Li = mk(lt.cr, lt.cg, lt.cb) / d2;
                    f3 contrib = ((beta * spectrum) * Li) / (P * 1.0f);
                    l0 = make_float4(0.0f + contrib.x, 0.0f + contrib.y, 0.0f + contrib.z, 0.0f);
                }
            }
            BSample bs;
            if (1 < L.max_bounces && bsdf_sample<MODE>(seed, sf.albedo, sf.roughness, conductor, sf.wo, bs)) {
                emit_next = continue_path(sf, bs, beta, o, d, 1, L.max_bounces);
                if (!kBetaQ) stqs(W.beta + path, make_float4(beta.x, beta.y, beta.z, __uint_as_float(seed)));
            }
        }
        if (valid) stqs(W.L + path, l0);  // every path of the batch, hit or miss
        const int qi = PT_SORT_EXT ? block_append_sorted<kWaves, kSortKeys>(cnt(W, 1, kQueue), emit_next ? octant(d) : -1, lds_q)
                                   : block_append<kWaves>(cnt(W, 1, kQueue), emit_next, lds_q);
        if (emit_next) {
            stqs(no + qi, make_float4(o.x, o.y, o.z, __int_as_float(path)));
            stqs(nd + qi, make_float4(d.x, d.y, d.z, 0.0f));
            if (kBetaQ) stqs(queue_beta(W, 1) + qi, make_float4(beta.x, beta.y, beta.z, __uint_as_float(seed)));
        }
    }
}

// Fused modes: the shadow rays of bounce b and the extension rays of bounce b + 1 start at
// the same hit points and are independent, so one launch traces both queues (one SIMT tail
// and one launch instead of two).  Items [0, n_ext) are extension rays (closest hit ->
// hit records), items [n_ext, n_ext + n_sh) shadow rays (any hit -> deferred NEE add).
template <bool STATS, bool TEX, int BLK = kBlockTrace>
__global__ __launch_bounds__(BLK, wf_waves(TEX)) void k_trace_pair(DevScene S, WFState W, int b,
                                                                      unsigned long long* counters) {
#if PT_TAIL_PROBE
    unsigned long long tp0;
    tail_probe_begin(tp0);
#endif
    const int n_ext = *cnt(W, b + 1, kQueue);
    const int n_sh = *cnt(W, b, kShadowQ);
    const float4* ro = W.ray_o[(b + 1) & 1];
    const float4* rd = W.ray_d[(b + 1) & 1];
    TravStats ts;
    auto fetch = [&](int i, TravState& st) {
        if (i < n_ext) {
            const float4 a = ldq_pair(ro + i), c = ldq_pair(rd + i);
            trav_init(st, mk(a.x, a.y, a.z), mk(c.x, c.y, c.z), 0.0f, 100.0f);
            st.path = __float_as_int(a.w);
        } else {
            const int j = i - n_ext;
            const float4 c = ldq_pair(W.sh_d + j), k = ldq_pair(W.sh_c + j);
            // origin | path: the shadow ray's own record, or (Lambert) the continuation ray of the
            // same path, which starts at the same point (k_shade_fused)
            const int q = __float_as_int(k.w);
            const float4 a = ldq_pair(q >= 0 ? ro + q : W.sh_o + j);
            trav_init(st, mk(a.x, a.y, a.z), mk(c.x, c.y, c.z), 0.0f, c.w);
            st.any = true;
            // an any-hit traversal only writes h.tri: the record's other fields carry the path
            // and the contribution to finish()
            st.h.orig = __float_as_int(a.w);
            st.h.t = k.x;
            st.h.u = k.y;
            st.h.v = k.z;
        }
    };
#if PT_SPLIT_FINISH
    // the deferred NEE add as load (finish, before the refill's record loads) + store (commit,
    // after them): the lane does not wait for the radiance line before the refill
    struct NeeAdd {
        float4* p;
        float4 v;
        float x, y, z;
    };
    auto finish = [&](int i, const TravState& st) -> NeeAdd {
        NeeAdd a{nullptr, make_float4(0.0f, 0.0f, 0.0f, 0.0f), 0.0f, 0.0f, 0.0f};
        const Hit& h = st.h;
        // the hit-record stores first: a store issued after the radiance load would wait for it
        if (i < n_ext) stq_pair(W.hit + i, hit_record(h, st.path));
        __builtin_amdgcn_sched_barrier(0);
        if (STATS && i >= n_ext && h.tri < 0) ts.unocc++;
        if (PT_NEE_MODE == 2 && !PT_PROBE_NO_NEE_ADD && i >= n_ext)  // k_nee_add adds
            reinterpret_cast<int*>(W.sh_c + (i - n_ext))[3] = h.tri < 0 ? h.orig : -1;
        if (PT_NEE_MODE != 2 && !PT_PROBE_NO_NEE_ADD && i >= n_ext && h.tri < 0) {  // unoccluded: add the deferred NEE contribution
            a.p = W.L + h.orig;
            if (PT_NEE_MODE == 0) a.v = *a.p;
            a.x = h.t;
            a.y = h.u;
            a.z = h.v;
        }
        return a;
    };
    auto commit = [&](const NeeAdd& a) {
        if (PT_NEE_MODE == 1 && a.p) {
            float* f = reinterpret_cast<float*>(a.p);
            __hip_atomic_fetch_add(f + 0, a.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(f + 1, a.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(f + 2, a.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (a.p) {
            *a.p = make_float4(a.v.x + a.x, a.v.y + a.y, a.v.z + a.z, 0.0f);
        }
    };
#else
    auto finish = [&](int i, const TravState& st) {
        const Hit& h = st.h;
        if (i < n_ext) {
            W.hit[i] = hit_record(h, st.path);
        } else if (h.tri < 0) {  // unoccluded: add the deferred NEE contribution
            const float4 l = W.L[h.orig];
            W.L[h.orig] = make_float4(l.x + h.t, l.y + h.u, l.z + h.v, 0.0f);
        }
    };
    auto commit = NoCommit{};
#endif
    // The queue is [extension rays | shadow rays] in contiguous wave slices, so all but one wave
    // trace a single ray kind; a mixed-kind loop serves both (per-kind loops in one kernel and
    // per-wave shares of both kinds were slower).
    int first, end;
    const int n_all = n_ext + n_sh;
    RayPool pool;
    if (PT_TRACE_POOL > 0 && pool_pays(n_all)) {
        pool.ctr = cnt(W, b, kPool);
        pool.end = n_all;
        pool.begin = n_all - (int)((long long)n_all * PT_TRACE_POOL / 100);
    } else {
        pool.begin = pool.end = n_all;
    }
    wave_slice(pool.begin, first, end);
    trace_queue<kRayMixed, STATS, TEX, BLK>(S, first, end, ts, W, fetch, finish, commit, pool);
#if PT_TAIL_PROBE
    tail_probe_end(b);
#endif
    if (blockIdx.x == 0 && threadIdx.x == 0 && counters) {
        atomicAdd(&counters[0], (unsigned long long)n_ext);           // path segments
        atomicAdd(&counters[5], (unsigned long long)n_sh);            // shadow rays
        atomicAdd(&counters[6], (unsigned long long)(n_ext + n_sh));  // rays of timed trace kernels
        atomicAdd(&counters[7], 48ull * (unsigned long long)(n_ext + n_sh));  // their queue bytes
        atomicAdd(&counters[16], (unsigned long long)(n_ext + n_sh));         // the same, k_trace_pair alone
        atomicAdd(&counters[17], 48ull * (unsigned long long)(n_ext + n_sh));
        atomicAdd(&counters[19], (unsigned long long)n_sh);
    }
    flush_trav_stats<STATS>(counters, ts);
}

// First half of a Default / Layered bounce: surface, metallic coin and light pick (the draws
// GlossyDiffuse::f must follow, devicePrograms.cu:400-445), then the item is queued for the
// later phases, by bucket (shade_bucket): the BSDF-sample queue for every hit that continues,
// and either a shadow ray (visibility still unknown; the ray carries item | bucket << 28) or,
// at bounce 0 with the (pixel, light) visibility table, the NEE queue directly.
template <int MODE, bool TEX>
__global__ __launch_bounds__(kBlockShA) void k_shade_a(DevScene S, DevLaunch L, WFState W, int b, int vis0) {
    const int n = *cnt(W, b, kQueue);
    const float4* rd = W.ray_d[b & 1];
    __shared__ int lds_sh[kWavesShA + 1];
    __shared__ int lds_nee[kNeeBuckets * (kWavesShA + 1)], lds_smp[kSmpBuckets * (kWavesShA + 1)];
    if ((int)(blockIdx.x * kBlockShA) >= n) return;  // block-uniform
    const int i = (int)(blockIdx.x * kBlockShA + threadIdx.x);
    bool emit = false;
    int nee_bucket = -1, smp_bucket = -1, code = 0;
    f3 so, sdir;
    float stmax = 0.0f;
    if (i < n && !wf_cancelled(W)) {  // a cancelled wave still joins the appends
        const float4 hv = W.hit[i];
        const float4 c = rd[i];  // beside the hit record (as k_shade_fused)
        const int path = __float_as_int(hv.x);
        const Hit h = decode_hit(hv);
        if (h.tri >= 0) {
            SurfaceHit sf;
            reconstruct<TEX>(S, h, mk(c.x, c.y, c.z), sf);
            float4 bv = W.beta[path];
            uint32_t seed = __float_as_uint(bv.w);
            if (path == debug_path_id(L)) {  // pt_set_debug_pixel (devicePrograms.cu:637-644)
                const float4 l = W.L[path];
                debug_record(L, b + 1, __float_as_int(S.isect[3 * h.tri].w), sf, mk(bv.x, bv.y, bv.z),
                             mk(l.x, l.y, l.z));
            }
            const bool conductor = rnd(seed) < sf.metallic;
            int li;
            const float P = pick_light(L, seed, li);
            W.beta[path] = make_float4(bv.x, bv.y, bv.z, __uint_as_float(seed));
            W.aux[path] = (li << 1) | (conductor ? 1 : 0);
            const int bk = shade_bucket<MODE>(conductor, sf.roughness);
            // the last bounce's sampled direction is never traced (SamplePath :646): no sample item
            if (b + 1 < L.max_bounces) {
                smp_bucket = bk;
                if (kSmpDark && (MODE == kModeLayered || !conductor) &&
                    fmaxf(fmaxf(sf.albedo.x, sf.albedo.y), sf.albedo.z) < PT_SMP_DARK)
                    smp_bucket = kSmpDark0 + bk - 1;
            }
            if (P > 0.0f) {
                const DevLight lt = L.lights[li];
                f3 ldir = mk(lt.px, lt.py, lt.pz) - sf.pos;
                const f3 ln = normalize(ldir);  // k_shade_nee's light direction, the same bits
                int nb = 0;  // conductor
                if (MODE == kModeLayered || !conductor)
                    nb = PT_NEE_CROSS && !same_hemisphere(sf.wo, to_local(sf.fr, ln)) ? kNeeCross
                                                                                     : nee_layered_bucket(bk, sf.albedo);
                if (vis0) {
                    if (W.vis[vis0_index(L, path, li)]) nee_bucket = nb;
                } else {
                    so = sf.pos + 1e-3f * sf.ng;
                    sdir = ln;
                    stmax = length(ldir);
                    code = i | (nb << kItemBits);
                    emit = true;
                }
            }
        }
    }
    const int si = block_append<kWavesShA>(cnt(W, b, kShadowQ), emit, lds_sh);
    if (emit) {
        W.sh_o[si] = make_float4(so.x, so.y, so.z, __int_as_float(code));
        W.sh_d[si] = make_float4(sdir.x, sdir.y, sdir.z, stmax);
    }
    const int ni = block_append_k<kWavesShA, kNeeBuckets>(cnt(W, b, kNee0), nee_bucket, lds_nee);
    if (nee_bucket >= 0) W.nq[nee_index(W, nee_bucket, ni)] = i;
    const int mi = block_append_k<kWavesShA, kSmpBuckets>(cnt(W, b, kSmp0), smp_bucket, lds_smp);
    if (smp_bucket >= 0) W.sq[smp_index(W, smp_bucket, mi)] = i;
}

// Any-hit visibility of the shadow queue of bounce b.  table = 1: the bounce-0 (pixel, light)
// table (k_shadow0_setup), vis[j] = 1 if unoccluded; table = 0: vis[j] = the ray's item code
// if unoccluded, else -1 (k_nee_compact reads it).
template <bool TEX, int BLK = kBlockTrace>
__global__ __launch_bounds__(BLK, wf_waves(false)) void k_shadow_vis(DevScene S, WFState W, int b, int table,
                                                                      unsigned long long* counters) {
    const int n = *cnt(W, b, kShadowQ);
    if (blockIdx.x == 0 && threadIdx.x == 0 && counters) atomicAdd(&counters[5], (unsigned long long)n);
    TravStats ts;
    trace_slice<kRayAny, false, TEX, BLK>(
        S, n, ts, W,
        [&](int j, TravState& st) {
            const float4 a = ldq_x(W.sh_o + j), c = ldq_x(W.sh_d + j);
            trav_init(st, mk(a.x, a.y, a.z), mk(c.x, c.y, c.z), 0.0f, c.w);
            st.path = __float_as_int(a.w);
        },
        [&](int j, const TravState& st) {
            const bool occluded = st.h.tri >= 0;
            W.vis[j] = table ? (occluded ? 0 : 1) : (occluded ? -1 : st.path);
        }, cnt(W, b, kPoolSh));
}

// PT_NEE_MODE 2: the unoccluded shadow rays of k_trace_pair(b) add their contributions to the
// path radiance in shadow-queue order (sh_c[j] = contribution | path, or -1 when occluded).
__global__ __launch_bounds__(kBlockWF) void k_nee_add(WFState W, int b) {
    const int n = *cnt(W, b, kShadowQ);
    if (wf_cancelled(W)) return;
    for (int j = (int)(blockIdx.x * kBlockWF + threadIdx.x); j < n; j += (int)(gridDim.x * kBlockWF)) {
        const float4 k = ldqs(W.sh_c + j);
        const int p = __float_as_int(k.w);
        if (p >= 0) {
            const float4 l = W.L[p];
            W.L[p] = make_float4(l.x + k.x, l.y + k.y, l.z + k.z, 0.0f);
        }
    }
}

// Visible shadow rays of bounce b -> the NEE bucket queues (vis[j] = item | bucket << 28, or -1).
// kCompactPer consecutive entries per thread, so a block appends 8192 entries with one atomic
// per bucket.
constexpr int kCompactPer = 8;
__global__ __launch_bounds__(kBlockSh) void k_nee_compact(WFState W, int b) {
    const int n = *cnt(W, b, kShadowQ);
    const int base = (int)(blockIdx.x * kBlockSh * kCompactPer);
    if (base >= n) return;  // block-uniform
    __shared__ int lds[kNeeBuckets * (kWavesSh + 1)];
    const int j0 = base + (int)threadIdx.x * kCompactPer;
    const bool cx = wf_cancelled(W);  // a cancelled wave compacts nothing but joins the barriers
    int v[kCompactPer];
    int c[kNeeBuckets] = {};
#pragma unroll
    for (int k = 0; k < kCompactPer; ++k) {
        v[k] = j0 + k < n && !cx ? W.vis[j0 + k] : -1;
#pragma unroll
        for (int q = 0; q < kNeeBuckets; ++q) c[q] += (v[k] >= 0 && (v[k] >> kItemBits) == q) ? 1 : 0;
    }
    // block-exclusive prefix of every bucket's count: wave scan, then the wave totals in LDS
    const int lane = lane_id(), wave = threadIdx.x >> 6;
    int incl[kNeeBuckets];
#pragma unroll
    for (int q = 0; q < kNeeBuckets; ++q) {
        int x = c[q];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        incl[q] = x;
        if (lane == 63) lds[q * kWavesSh + wave] = x;
    }
    __syncthreads();
    if ((int)threadIdx.x < kNeeBuckets) {
        const int q = threadIdx.x;
        int tot = 0;
        for (int w = 0; w < kWavesSh; ++w) {
            const int t = lds[q * kWavesSh + w];
            lds[q * kWavesSh + w] = tot;
            tot += t;
        }
        lds[kNeeBuckets * kWavesSh + q] = tot > 0 ? atomicAdd(cnt(W, b, kNee0 + q), tot) : 0;
    }
    __syncthreads();
    int off[kNeeBuckets];
#pragma unroll
    for (int q = 0; q < kNeeBuckets; ++q)
        off[q] = lds[kNeeBuckets * kWavesSh + q] + lds[q * kWavesSh + wave] + incl[q] - c[q];
#pragma unroll
    for (int k = 0; k < kCompactPer; ++k) {
        if (v[k] < 0) continue;
        const int q = v[k] >> kItemBits;
        int slot = off[0];
#pragma unroll
        for (int r = 1; r < kNeeBuckets; ++r) slot = q == r ? off[r] : slot;
#pragma unroll
        for (int r = 0; r < kNeeBuckets; ++r) off[r] += q == r ? 1 : 0;
        W.nq[nee_index(W, q, slot)] = v[k] & ((1 << kItemBits) - 1);
    }
}

// Entry idx of the NEE / sample queue (bucket q: slots nee_index / smp_index, length
// *cnt(W, b, c0 + q)), or -1 past the total.  Buckets are taken in order, so all but a few waves
// hold one bucket.
__device__ __forceinline__ int nee_entry(const WFState& W, int b, int idx) {
    int base = 0;
#pragma unroll
    for (int q = 0; q < kNeeBuckets; ++q) {
        const int n = *cnt(W, b, kNee0 + q);
        if (idx < base + n) return W.nq[nee_index(W, q, idx - base)];
        base += n;
    }
    return -1;
}
__device__ __forceinline__ int smp_entry(const WFState& W, int b, int idx) {
    int base = 0;
#pragma unroll
    for (int q = 0; q < kSmpBuckets; ++q) {
        const int n = *cnt(W, b, kSmp0 + q);
        if (idx < base + n) return W.sq[smp_index(W, q, idx - base)];
        base += n;
    }
    return -1;
}
__device__ __forceinline__ int smp_total(const WFState& W, int b) {
    int n = 0;
#pragma unroll
    for (int q = 0; q < kSmpBuckets; ++q) n += *cnt(W, b, kSmp0 + q);
    return n;
}
__device__ __forceinline__ int nee_total(const WFState& W, int b) {
    int n = 0;
#pragma unroll
    for (int q = 0; q < kNeeBuckets; ++q) n += *cnt(W, b, kNee0 + q);
    return n;
}

// NEE of a Default / Layered bounce over the items whose light is visible (devicePrograms.cu:
// 446-472).  The stochastic GlossyDiffuse eval dominates (≈10^4 instructions per call, DESIGN.md
// §5) and a wave pays for its slowest lane: the items come from the bucketed NEE queue, so every
// wave but the last of each bucket is full and runs one BSDF code path.  Every path sees the
// same operations and random numbers in the same order (the eval writes the advanced seed back
// to W.beta before k_shade_smp reads it).
template <int MODE, bool TEX>
__global__ __launch_bounds__(kBlockShB, PT_SHB_WAVES) void k_shade_nee(DevScene S, DevLaunch L, WFState W, int b) {
    if (blockIdx.x == 0 && threadIdx.x == 0 && L.counters)
        atomicAdd(&L.counters[15], (unsigned long long)nee_total(W, b));
    if ((int)(blockIdx.x * kBlockShB) >= nee_total(W, b)) return;  // block-uniform
    if (wf_cancelled(W)) return;  // no barrier below
    const int j = nee_entry(W, b, (int)(blockIdx.x * kBlockShB + threadIdx.x));
    if (j < 0) return;
    const float4 hv = W.hit[j], c = W.ray_d[b & 1][j];
    const int path = __float_as_int(hv.x);
    const Hit h = decode_hit(hv);
    SurfaceHit sf;
    reconstruct<TEX>(S, h, mk(c.x, c.y, c.z), sf);
#if PT_NEE_LEAN
    // only the path, the light index, |cos| and the squared distance stay live across the layered
    // walk; the throughput and the light are loaded again after it (the same values and
    // operations as below, so the same bits)
    const int aux = W.aux[path];
    const int li = aux >> 1;
    uint32_t seed = __float_as_uint(W.beta[path].w);
    f3 lds;
    float d2;
    {
        const DevLight lt = L.lights[li];
        const f3 lpos = mk(lt.px, lt.py, lt.pz);
        lds = to_local(sf.fr, normalize(lpos - sf.pos));
        const f3 dd = sf.pos - lpos;
        d2 = dd.x * dd.x + dd.y * dd.y + dd.z * dd.z;
    }
    const float cosl = abs_dot(lds, mk(0.0f, 0.0f, 1.0f));
#if PT_NEE_PROBE
    // probe build only (tools/nee_probe.py): waves of the layered walk, those of them on its run-time
    // path (some lane has the light across the shading plane) and those with both top kinds
    if (L.counters) {
        const bool lay = MODE == kModeLayered || !(aux & 1);
        const unsigned long long any = __builtin_amdgcn_ballot_w64(lay);
        const unsigned long long cross = __builtin_amdgcn_ballot_w64(lay && !same_hemisphere(sf.wo, lds));
        const unsigned long long spec = __builtin_amdgcn_ballot_w64(lay && sqr(sf.roughness) < 1e-3f);
        const unsigned long long act = __builtin_amdgcn_ballot_w64(true);
        if (lane_id() == __ffsll((long long)act) - 1 && any) {
            atomicAdd(&L.counters[21], 1ull);
            if (cross) atomicAdd(&L.counters[20], 1ull);
            if (spec && spec != any) atomicAdd(&L.counters[22], 1ull);
            atomicAdd(&L.counters[23], (unsigned long long)__popcll(cross));
            atomicAdd(&L.counters[24], (unsigned long long)__popcll(any));
        }
    }
#endif
    f3 f = bsdf_f<MODE, true>(seed, sf.albedo, sf.roughness, aux & 1, sf.wo, lds);
    f3 spectrum = f * cosl;
    const float4 bv = W.beta[path];
    const f3 beta = mk(bv.x, bv.y, bv.z);
    if (!is_zero(spectrum)) {
        const float P = L.n_lights == 1 ? 1.0f : 1.0f / (float)L.n_lights;
        const DevLight lt = L.lights[li];
        f3 Li = mk(lt.cr, lt.cg, lt.cb) / d2;
        f3 add = ((beta * spectrum) * Li) / (P * 1.0f);
        float4 l = W.L[path];
        W.L[path] = make_float4(l.x + add.x, l.y + add.y, l.z + add.z, 0.0f);
    }
#else
    const float4 bv = W.beta[path];
    uint32_t seed = __float_as_uint(bv.w);
    const f3 beta = mk(bv.x, bv.y, bv.z);
    const int aux = W.aux[path];
    const int li = aux >> 1;
    const float P = L.n_lights == 1 ? 1.0f : 1.0f / (float)L.n_lights;
    const DevLight lt = L.lights[li];
    f3 lpos = mk(lt.px, lt.py, lt.pz);
    f3 lds = to_local(sf.fr, normalize(lpos - sf.pos));
    f3 f = bsdf_f<MODE>(seed, sf.albedo, sf.roughness, aux & 1, sf.wo, lds);
    f3 spectrum = f * abs_dot(lds, mk(0.0f, 0.0f, 1.0f));
    if (!is_zero(spectrum)) {
        f3 dd = sf.pos - lpos;
        float d2 = dd.x * dd.x + dd.y * dd.y + dd.z * dd.z;
        f3 Li = mk(lt.cr, lt.cg, lt.cb) / d2;
        f3 add = ((beta * spectrum) * Li) / (P * 1.0f);
        float4 l = W.L[path];
        W.L[path] = make_float4(l.x + add.x, l.y + add.y, l.z + add.z, 0.0f);
    }
#endif
    W.beta[path] = make_float4(bv.x, bv.y, bv.z, __uint_as_float(seed));  // f may draw
}

// BSDF sample + continuation of a Default / Layered bounce (devicePrograms.cu:474-509) over the
// bucketed sample queue; continuation rays are appended to queue b + 1.
template <int MODE, bool TEX>
__global__ __launch_bounds__(kBlockShB, PT_SMP_WAVES) void k_shade_smp(DevScene S, DevLaunch L, WFState W, int b) {
    constexpr int kW = kBlockShB / 64;
    __shared__ int lds_q[kW + 1];
    if ((int)(blockIdx.x * kBlockShB) >= smp_total(W, b)) return;  // block-uniform
    const int j = smp_entry(W, b, (int)(blockIdx.x * kBlockShB + threadIdx.x));
    bool emit_next = false;
    f3 o, d;
    int path = 0;
    if (j >= 0 && !wf_cancelled(W)) {  // a cancelled wave still joins the appends
        const float4 hv = W.hit[j], c = W.ray_d[b & 1][j];
        path = __float_as_int(hv.x);
        const Hit h = decode_hit(hv);
        d = mk(c.x, c.y, c.z);
        SurfaceHit sf;
        reconstruct<TEX>(S, h, d, sf);
        const float4 bv = W.beta[path];
        uint32_t seed = __float_as_uint(bv.w);
        f3 beta = mk(bv.x, bv.y, bv.z);
        BSample bs;
        if (bsdf_sample<MODE, true>(seed, sf.albedo, sf.roughness, W.aux[path] & 1, sf.wo, bs)) {
            emit_next = continue_path(sf, bs, beta, o, d, b + 1, L.max_bounces);
            W.beta[path] = make_float4(beta.x, beta.y, beta.z, __uint_as_float(seed));
        }
    }
    float4* no = W.ray_o[(b + 1) & 1];
    float4* nd = W.ray_d[(b + 1) & 1];
    const int qi = block_append<kW>(cnt(W, b + 1, kQueue), emit_next, lds_q);
    if (emit_next) {
        no[qi] = make_float4(o.x, o.y, o.z, __int_as_float(path));
        nd[qi] = make_float4(d.x, d.y, d.z, 0.0f);
    }
}

__global__ __launch_bounds__(kBlockWF) void k_accum(WFState W, DevLaunch L, int nf) {
    const int P = L.width * L.height;
    for (int p = blockIdx.x * blockDim.x + threadIdx.x; p < P; p += gridDim.x * blockDim.x) {
        const size_t idx = (size_t)p * 3;
        if (L.frame_stride) {  // render-ahead: each frame its own 1-spp image, a one-frame sum into zeros
            for (int f = 0; f < nf; ++f) {
                const float4 l = W.L[(size_t)f * P + p];
                float* o = L.accum + (size_t)f * L.frame_stride + idx;
                o[0] = 0.0f + l.x;
                o[1] = 0.0f + l.y;
                o[2] = 0.0f + l.z;
            }
            continue;
        }
        if (L.accum64) {  // pt_set_accum_fp64: the frames' fp32 radiance summed in fp64
            double sx = L.accum64[idx], sy = L.accum64[idx + 1], sz = L.accum64[idx + 2];
            for (int f = 0; f < nf; ++f) {
                const float4 l = W.L[(size_t)f * P + p];
                sx += (double)l.x;
                sy += (double)l.y;
                sz += (double)l.z;
            }
            L.accum64[idx] = sx;
            L.accum64[idx + 1] = sy;
            L.accum64[idx + 2] = sz;
            L.accum[idx] = (float)sx;
            L.accum[idx + 1] = (float)sy;
            L.accum[idx + 2] = (float)sz;
            continue;
        }
        float sx = L.accum[idx], sy = L.accum[idx + 1], sz = L.accum[idx + 2];
        for (int f = 0; f < nf; ++f) {  // frames in order: the sequential accumulation
            const float4 l = W.L[(size_t)f * P + p];
            sx += l.x;
            sy += l.y;
            sz += l.z;
        }
        L.accum[idx] = sx;
        L.accum[idx + 1] = sy;
        L.accum[idx + 2] = sz;
    }
}

__global__ __launch_bounds__(kBlockWF) void k_f64_to_f32(const double* __restrict__ a, float* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        b[i] = (float)a[i];
}

inline bool fused_mode(int mode) { return mode == kModeLambert || mode == kModeConductor || mode == kModeDielectric; }

// Grid covering `items` slots, one per thread.
inline dim3 item_grid(int items, int block) { return dim3((unsigned)std::max(1, (items + block - 1) / block)); }

// Exactly the blocks that are resident at once (occupancy query, cached) — the lane-
// refilling trace kernels, whose waves each own a static queue slice.
template <typename K>
dim3 occupancy_grid(K kernel, int cus, int block = kBlockTrace) {
    static std::unordered_map<const void*, int> cache;
    const void* key = reinterpret_cast<const void*>(kernel);
    auto it = cache.find(key);
    int per_cu = 0;
    if (it == cache.end()) {
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0) != hipSuccess || per_cu < 1)
            per_cu = 1;
        cache[key] = per_cu;
    } else {
        per_cu = it->second;
    }
// (2x / 4x oversubscribed trace grids with the two wavefront streams: Lambert +0.2 / +0.5 %,
// Dielectric +1.7 / +1.4 %, Layered -0.4 %: noise-level)
#ifndef PT_TRACE_OVERSUB
#define PT_TRACE_OVERSUB 1
#endif
    return dim3((unsigned)(PT_TRACE_OVERSUB * per_cu * std::max(1, cus)));
}

// phase (Default / Layered): 0 = k_shade_a, 1 = k_shade_nee, 2 = k_shade_smp
template <int MODE, bool TEX>
hipError_t launch_shade_t(bool fused, const DevScene& S, const DevLaunch& L, const WFState& W, int b, int items,
                          hipStream_t stream, int phase, int vis0, int shade0) {
    if (fused) {
        if constexpr (MODE == kModeLambert || MODE == kModeConductor || MODE == kModeDielectric)
        {
            if (shade0)
                hipLaunchKernelGGL((k_shade_fused<MODE, TEX, true>), item_grid(items, shf_block(MODE)), dim3(shf_block(MODE)), 0,
                                   stream, S, L, W, b, vis0);
            else
                hipLaunchKernelGGL((k_shade_fused<MODE, TEX, false>), item_grid(items, shf_block(MODE)), dim3(shf_block(MODE)), 0,
                                   stream, S, L, W, b, vis0);
        }
    } else if (phase == 0) {
        hipLaunchKernelGGL((k_shade_a<MODE, TEX>), item_grid(items, kBlockShA), dim3(kBlockShA), 0, stream, S, L, W, b,
                           vis0);
    } else if (phase == 1) {
        hipLaunchKernelGGL((k_shade_nee<MODE, TEX>), item_grid(items, kBlockShB), dim3(kBlockShB), 0, stream, S, L,
                           W, b);
    } else {
        hipLaunchKernelGGL((k_shade_smp<MODE, TEX>), item_grid(items, kBlockShB), dim3(kBlockShB), 0, stream, S, L,
                           W, b);
    }
    return hipGetLastError();
}

template <int MODE>
hipError_t launch_shade(bool fused, const DevScene& S, const DevLaunch& L, const WFState& W, int b, int items,
                        hipStream_t stream, int phase, int vis0, int shade0) {
    return S.texinfo ? launch_shade_t<MODE, true>(fused, S, L, W, b, items, stream, phase, vis0, shade0)
                     : launch_shade_t<MODE, false>(fused, S, L, W, b, items, stream, phase, vis0, shade0);
}

template <int MODE>
hipError_t launch_shade0_pixel_t(const DevScene& S, const DevLaunch& L, const WFState& W, int nf, hipStream_t stream) {
    constexpr int block = shf_block(MODE);
    const dim3 grid = item_grid(L.width * L.height, block);
    if (S.texinfo)
        hipLaunchKernelGGL((k_shade0_pixel<MODE, true>), grid, dim3(block), 0, stream, S, L, W, nf);
    else
        hipLaunchKernelGGL((k_shade0_pixel<MODE, false>), grid, dim3(block), 0, stream, S, L, W,
                           nf);
    return hipGetLastError();
}
hipError_t launch_shade0_pixel(int mode, const DevScene& S, const DevLaunch& L, const WFState& W, int nf,
                               hipStream_t stream) {
    switch (mode) {
        case kModeLambert: return launch_shade0_pixel_t<kModeLambert>(S, L, W, nf, stream);
        case kModeConductor: return launch_shade0_pixel_t<kModeConductor>(S, L, W, nf, stream);
        default: return launch_shade0_pixel_t<kModeDielectric>(S, L, W, nf, stream);
    }
}

// vis0: n_lights when the bounce-0 (pixel, light) visibility table is used at this bounce, else 0
hipError_t launch_shade_mode(int mode, bool fused, const DevScene& S, const DevLaunch& L, const WFState& W, int b,
                             int items, hipStream_t stream, int phase, int vis0, int shade0 = 0) {
    switch (mode) {
        case kModeLambert: return launch_shade<kModeLambert>(fused, S, L, W, b, items, stream, phase, vis0, shade0);
        case kModeConductor: return launch_shade<kModeConductor>(fused, S, L, W, b, items, stream, phase, vis0, shade0);
        case kModeDielectric: return launch_shade<kModeDielectric>(fused, S, L, W, b, items, stream, phase, vis0, shade0);
        case kModeLayered: return launch_shade<kModeLayered>(fused, S, L, W, b, items, stream, phase, vis0, shade0);
        default: return launch_shade<kModeDefault>(fused, S, L, W, b, items, stream, phase, vis0, shade0);
    }
}

}  // namespace

hipError_t accum_f64_to_f32(const double* sum64, float* sum32, size_t n, hipStream_t stream) {
    const unsigned blocks = (unsigned)std::min<size_t>((n + kBlockWF - 1) / kBlockWF, 8192);
    hipLaunchKernelGGL(k_f64_to_f32, dim3(std::max(1u, blocks)), dim3(kBlockWF), 0, stream, sum64, sum32, n);
    return hipGetLastError();
}

size_t wavefront_bytes(int paths, int max_bounces) {
    size_t P = (size_t)paths;
    return P * sizeof(float4) * (4 /*rays x2 queues*/ + 1 /*hit*/ + 3 /*beta x2, L*/ + 3 /*shadow*/) +
           P * (2 + kNeeRegions + kShadeBuckets) * sizeof(int) + count_bytes(max_bounces);
}

hipError_t wavefront_alloc(WFState& W, int paths, int max_bounces) {
    size_t P = (size_t)paths;
    hipError_t e = hipSuccess;
    auto al = [&](void** p, size_t bytes) {
        if (e == hipSuccess) e = hipMalloc(p, bytes > 0 ? bytes : 16);
    };
    al((void**)&W.ray_o[0], P * sizeof(float4));
    al((void**)&W.ray_o[1], P * sizeof(float4));
    al((void**)&W.ray_d[0], P * sizeof(float4));
    al((void**)&W.ray_d[1], P * sizeof(float4));
    al((void**)&W.hit, P * sizeof(float4));
    al((void**)&W.beta, P * sizeof(float4));
    al((void**)&W.beta_q, P * sizeof(float4));
    al((void**)&W.L, P * sizeof(float4));
    al((void**)&W.sh_o, P * sizeof(float4));
    al((void**)&W.sh_d, P * sizeof(float4));
    al((void**)&W.sh_c, P * sizeof(float4));
    al((void**)&W.aux, P * sizeof(int));
    al((void**)&W.vis, P * sizeof(int));
    al((void**)&W.nq, P * kNeeRegions * sizeof(int));
    al((void**)&W.sq, P * kShadeBuckets * sizeof(int));
    al((void**)&W.count, count_bytes(max_bounces));
    if (e != hipSuccess) {
        // no partial queue set survives a failed allocation: paths stays 0, so the next
        // launch_frames allocates again instead of launching on null queues
        wavefront_free(W);
        (void)hipGetLastError();
        return e;
    }
    W.paths = paths;
    W.max_bounces = max_bounces;
    return e;
}

void wavefront_free(WFState& W) {
    void* ps[] = {W.ray_o[0], W.ray_o[1], W.ray_d[0], W.ray_d[1], W.hit, W.beta, W.beta_q, W.L, W.sh_o, W.sh_d, W.sh_c,
                  W.aux, W.vis, W.nq, W.sq, W.count};
    for (void* p : ps)
        if (p) (void)hipFree(p);
    W = WFState{};
}

hipError_t launch_wavefront_frame(int mode, bool stats, const DevScene& S, const DevLaunch& L, const WFState& W,
                                  uint32_t frame, int nf, bool primary_dedup, int cus, hipStream_t stream,
                                  const hipEvent_t* trace_events, int* n_timed, hipEvent_t accum_wait,
                                  hipEvent_t accum_done, const hipEvent_t* shade_events, int* n_shade_timed,
                                  bool wide_trace) {
    const int P = L.width * L.height * nf;  // paths in flight
    const int maxb = L.max_bounces;
    hipError_t e = hipSuccess;
    if (W.cancel_seen && W.hold_release) {  // pt_set_debug_hold: the batch waits in k_hold first
        hipLaunchKernelGGL(k_hold, dim3(1), dim3(64), 0, stream, W);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    e = hipMemsetAsync(W.count, 0, count_bytes(maxb), stream);
    if (e != hipSuccess) return e;
    // fused modes with the primary dedup: frame 0's camera rays only (k_camera `lean`, shade0)
    const bool lean = fused_mode(mode) && primary_dedup && nf > 1 && maxb > 0;
    hipLaunchKernelGGL(k_camera, item_grid(lean ? L.width * L.height : P, kBlockWF), dim3(kBlockWF), 0, stream, W, L,
                       frame, nf, lean ? 1 : 0);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    const bool fused = fused_mode(mode);
    const bool tex = S.texinfo != nullptr;  // textured scene: kernels with texture sampling
    int timed = 0;                          // trace launches bracketed by trace_events
    int stimed = 0;                         // shading launches bracketed by shade_events
    // the timed shading kernel of a bounce: k_shade_fused / k_shade0_pixel (fused modes), k_shade_nee
    // (Default / Layered: the stochastic layered eval, 53-60 % of their frame)
    auto shade_timed = [&](auto launch) -> hipError_t {
        hipError_t r;
        if (shade_events && (r = hipEventRecord(shade_events[2 * stimed], stream)) != hipSuccess) return r;
        if ((r = launch()) != hipSuccess) return r;
        if (shade_events && (r = hipEventRecord(shade_events[2 * stimed + 1], stream)) != hipSuccess) return r;
        ++stimed;
        return hipSuccess;
    };
    // the untextured trace kernels of a one-stream call take the wide workgroups (kBlockTraceWide)
    const bool wide = wide_trace && (!tex || PT_WIDE_TEX);
#define PT_TRACE_LAUNCH(KERN, BLK, ...) \
    hipLaunchKernelGGL((KERN), occupancy_grid(KERN, cus, BLK), dim3(BLK), 0, stream, __VA_ARGS__)
    auto extend = [&](int b, int dup, int copies) -> hipError_t {
        hipError_t r;
        if (trace_events && (r = hipEventRecord(trace_events[2 * timed], stream)) != hipSuccess) return r;
        if (tex && wide && PT_WIDE_TEX) {
            if (stats)
                PT_TRACE_LAUNCH((k_extend<true, true, kBlockTraceWide>), kBlockTraceWide, S, W, b, dup, copies, L.counters);
            else
                PT_TRACE_LAUNCH((k_extend<false, true, kBlockTraceWide>), kBlockTraceWide, S, W, b, dup, copies, L.counters);
        } else if (tex) {
            if (stats)
                PT_TRACE_LAUNCH((k_extend<true, true>), kBlockTrace, S, W, b, dup, copies, L.counters);
            else
                PT_TRACE_LAUNCH((k_extend<false, true>), kBlockTrace, S, W, b, dup, copies, L.counters);
        } else if (wide) {
            if (stats)
                PT_TRACE_LAUNCH((k_extend<true, false, kBlockTraceWide>), kBlockTraceWide, S, W, b, dup, copies, L.counters);
            else
                PT_TRACE_LAUNCH((k_extend<false, false, kBlockTraceWide>), kBlockTraceWide, S, W, b, dup, copies, L.counters);
        } else if (stats) {
            PT_TRACE_LAUNCH((k_extend<true, false>), kBlockTrace, S, W, b, dup, copies, L.counters);
        } else {
            PT_TRACE_LAUNCH((k_extend<false, false>), kBlockTrace, S, W, b, dup, copies, L.counters);
        }
        if (trace_events && (r = hipEventRecord(trace_events[2 * timed + 1], stream)) != hipSuccess) return r;
        ++timed;
        return hipGetLastError();
    };
    auto pair = [&](int b) -> hipError_t {
        hipError_t r;
        if (trace_events && (r = hipEventRecord(trace_events[2 * timed], stream)) != hipSuccess) return r;
        if (tex && wide && PT_WIDE_TEX) {
            if (stats)
                PT_TRACE_LAUNCH((k_trace_pair<true, true, kBlockTraceWide>), kBlockTraceWide, S, W, b, L.counters);
            else
                PT_TRACE_LAUNCH((k_trace_pair<false, true, kBlockTraceWide>), kBlockTraceWide, S, W, b, L.counters);
        } else if (tex) {
            if (stats)
                PT_TRACE_LAUNCH((k_trace_pair<true, true>), kBlockTrace, S, W, b, L.counters);
            else
                PT_TRACE_LAUNCH((k_trace_pair<false, true>), kBlockTrace, S, W, b, L.counters);
        } else if (wide) {
            if (stats)
                PT_TRACE_LAUNCH((k_trace_pair<true, false, kBlockTraceWide>), kBlockTraceWide, S, W, b, L.counters);
            else
                PT_TRACE_LAUNCH((k_trace_pair<false, false, kBlockTraceWide>), kBlockTraceWide, S, W, b, L.counters);
        } else if (stats) {
            PT_TRACE_LAUNCH((k_trace_pair<true, false>), kBlockTrace, S, W, b, L.counters);
        } else {
            PT_TRACE_LAUNCH((k_trace_pair<false, false>), kBlockTrace, S, W, b, L.counters);
        }
        if (trace_events && (r = hipEventRecord(trace_events[2 * timed + 1], stream)) != hipSuccess) return r;
        ++timed;
        if (PT_NEE_MODE == 2 && !PT_PROBE_NO_NEE_ADD)
            hipLaunchKernelGGL(k_nee_add, dim3(8 * cus), dim3(kBlockWF), 0, stream, W, b);
        return hipGetLastError();
    };
    auto shadow_vis = [&](int b, int table) -> hipError_t {
        if (tex && wide && PT_WIDE_TEX)
            PT_TRACE_LAUNCH((k_shadow_vis<true, kBlockTraceWide>), kBlockTraceWide, S, W, b, table, L.counters);
        else if (tex)
            PT_TRACE_LAUNCH((k_shadow_vis<true>), kBlockTrace, S, W, b, table, L.counters);
        else if (wide)
            PT_TRACE_LAUNCH((k_shadow_vis<false, kBlockTraceWide>), kBlockTraceWide, S, W, b, table, L.counters);
        else
            PT_TRACE_LAUNCH((k_shadow_vis<false>), kBlockTrace, S, W, b, table, L.counters);
        if (!table) hipLaunchKernelGGL(k_nee_compact, item_grid(P, kBlockSh * kCompactPer), dim3(kBlockSh), 0, stream, W, b);
        return hipGetLastError();
    };
    // bounce-0 shadow dedup: one shadow ray per (pixel, light) instead of one per path; pays
    // off while the batch has at least as many frames as there are lights
    const int P1 = L.width * L.height;
    const int vis0 = (primary_dedup && nf > 1 && L.n_lights >= 1 && L.n_lights <= nf) ? L.n_lights : 0;
    auto shadow0 = [&]() -> hipError_t {
        if (!vis0) return hipSuccess;
        if (tex)
            hipLaunchKernelGGL(k_shadow0_setup<true>, item_grid(P1 * vis0, kBlockWF), dim3(kBlockWF),
                               0, stream, S, L,
                               W);
        else
            hipLaunchKernelGGL(k_shadow0_setup<false>, item_grid(P1 * vis0, kBlockWF), dim3(kBlockWF),
                               0, stream, S,
                               L, W);
        hipError_t r = hipGetLastError();
        if (r != hipSuccess || (r = shadow_vis(0, 1)) != hipSuccess) return r;
        // the table's rays must not be traced again as bounce-0 shadow rays
        return hipMemsetAsync(W.count + kShadowQ * kCntStride, 0, sizeof(int), stream);
    };
    if (maxb <= 0) {
        // SamplePath's loop never runs (devicePrograms.cu:646): black frames, no segments
    } else if (fused) {
        // extend(0); then per bounce: shade(b) -> [shadow rays of b + extension rays of b+1]
        // lean bounce 0 with the visibility table: one hit record and one surface per pixel
        const bool pixel0 = lean && vis0;
        if ((e = extend(0, primary_dedup ? nf : 1, pixel0 ? 1 : (primary_dedup ? nf : 1))) != hipSuccess) return e;
        if ((e = shadow0()) != hipSuccess) return e;
        for (int b = 0; b < maxb; ++b) {
            if (b == 0 && pixel0) {
                if ((e = shade_timed([&] { return launch_shade0_pixel(mode, S, L, W, nf, stream); })) != hipSuccess)
                    return e;
            } else if ((e = shade_timed([&] {
                            return launch_shade_mode(mode, true, S, L, W, b, P, stream, 0, b == 0 ? vis0 : 0,
                                                     b == 0 && lean);
                        })) != hipSuccess) {
                return e;
            }
            if ((e = pair(b)) != hipSuccess) return e;
        }
    } else {
        for (int b = 0; b < maxb; ++b) {
            const int dup = b == 0 && primary_dedup ? nf : 1;
            if ((e = extend(b, dup, dup)) != hipSuccess) return e;
            const int v0 = b == 0 ? vis0 : 0;
            if (v0 && (e = shadow0()) != hipSuccess) return e;
            // k_shade_a queues the bounce's items by bucket; the visible ones (the bounce-0 table,
            // or k_shadow_vis + k_nee_compact) get the NEE eval, the continuing ones the sample
            if ((e = launch_shade_mode(mode, false, S, L, W, b, P, stream, 0, v0)) != hipSuccess) return e;
            if (!v0 && (e = shadow_vis(b, 0)) != hipSuccess) return e;
            if ((e = shade_timed([&] { return launch_shade_mode(mode, false, S, L, W, b, P, stream, 1, v0); })) !=
                hipSuccess)
                return e;
            if (b + 1 < maxb && (e = launch_shade_mode(mode, false, S, L, W, b, P, stream, 2, v0)) != hipSuccess)
                return e;
        }
    }
#undef PT_TRACE_LAUNCH
    if (accum_wait && (e = hipStreamWaitEvent(stream, accum_wait, 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_accum, item_grid(L.width * L.height, kBlockWF), dim3(kBlockWF), 0, stream, W, L, nf);
    if (accum_done && (e = hipEventRecord(accum_done, stream)) != hipSuccess) return e;
    if (n_timed) *n_timed = timed;  // fused modes: max_bounces + 1; Default / Layered: max_bounces
    if (n_shade_timed) *n_shade_timed = stimed;  // max_bounces
    return hipGetLastError();
}

}  // namespace pt
