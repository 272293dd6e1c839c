// pt_capi.cpp — the C ABI of libptamd.so (include/ptamd.h): host driver for the gfx950
// path tracer.  Replaces Renderer/OptiX/OptixRenderer.{h,cpp} of Damo12320/OptixPathtracer
// (context/module/pipeline/SBT setup collapse into: upload scene -> LBVH build -> launch).
//
// There is no CPU fallback: every render and trace call runs the HIP kernels or fails
// with a negative status.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ptamd.h"
#include "pt_internal.h"

using namespace pt;

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string& msg) {
    g_last_error = msg;
    return code;
}
// Device allocations that fail for lack of memory report PT_ERR_NOMEM (the caller can retry
// with fewer frames per launch); every other HIP failure is PT_ERR_HIP.
int hip_fail(hipError_t e, const char* where) {
    g_last_error = std::string(where) + ": " + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? PT_ERR_NOMEM : PT_ERR_HIP;
}

#define PT_HIP(call, where)                              \
    do {                                                 \
        hipError_t e__ = (call);                         \
        if (e__ != hipSuccess) return hip_fail(e__, where); \
    } while (0)

// glm mat4 * vec4 for the host-side pre-transform (GetVertices, devicePrograms.cu:77-81)
void xform4(const float* m, const float v[4], float out[4]) { mat4_mul_vec4(m, v, out); }

// Reusable HIP event pairs, one pair per timed launch; summed once the launches retire.
struct EventPool {
    std::vector<hipEvent_t> start, stop;
    size_t used = 0;
    hipError_t next(hipEvent_t* a, hipEvent_t* b) {
        if (used == start.size()) {
            hipEvent_t e0 = nullptr, e1 = nullptr;
            hipError_t e = hipEventCreate(&e0);
            if (e == hipSuccess) e = hipEventCreate(&e1);
            if (e != hipSuccess) return e;
            start.push_back(e0);
            stop.push_back(e1);
        }
        *a = start[used];
        *b = stop[used];
        used++;
        return hipSuccess;
    }
    void give_back(size_t k) { used -= std::min(k, used); }  // the last k pairs went unrecorded
    hipError_t collect(double* ms_sum, size_t* n) {
        *ms_sum = 0.0;
        *n = used;
        if (used == 0) return hipSuccess;
        hipError_t e = hipEventSynchronize(stop[used - 1]);
        for (size_t i = 0; i < used && e == hipSuccess; ++i) {
            float ms = 0.0f;
            e = hipEventElapsedTime(&ms, start[i], stop[i]);
            *ms_sum += ms;
        }
        used = 0;
        return e;
    }
    void destroy() {
        for (hipEvent_t e : start) (void)hipEventDestroy(e);
        for (hipEvent_t e : stop) (void)hipEventDestroy(e);
        start.clear();
        stop.clear();
        used = 0;
    }
};

// Device counters: [0] segments [1] nodes visited [2] triangle tests [3] rays [4] stack
// overflows [5] shadow rays [6] timed trace-kernel rays [7] their bytes [8] strict re-traces
// [9..13] wave schedule of the trace kernels (pt_stats wave_*) [14] node visits served from LDS
// [15] items of the timed shading kernel (pt_stats shade_kernel_items) [16] [17] rays and
// algorithmic bytes of the k_trace_pair launches alone (pt_stats pair_kernel_*).
constexpr int kCounters = 28;  // [20..26]: trace coherence histogram (pt_get_trace_coherence)
// event pairs held by one renderer before launch_frames retires them (EventPool)
constexpr size_t kMaxPendingEvents = 4096;
// the smallest traversal stack of any kernel (pt_device.h stack_capacity: 71 entries for the
// wavefront's 11 LDS entries and 64 spill slots in chunks of 5)
constexpr int kMinTraversalStack = std::min(stack_capacity(PT_WF_STACK), stack_capacity(PT_MK_STACK));

}  // namespace

struct pt_renderer {
    int device = 0;
    hipStream_t stream = nullptr;
    // wavefront batches alternate between two streams, each with its own queues, so one batch's
    // kernels overlap the other's (pt_set_wavefront_streams; 1 = everything on `stream`)
    static constexpr int kMaxWFStreams = 4;
    int wf_streams = 0;  // 0 = auto (launch_frames): two for Conductor and Dielectric, one otherwise
    hipStream_t xstream[kMaxWFStreams] = {};  // [0] unused: stream 0 is `stream`
    WFState xwf[kMaxWFStreams];               // [0] unused: stream 0's queues are `wf`
    hipEvent_t ev_fork = nullptr, ev_join[kMaxWFStreams] = {}, ev_accum[2] = {nullptr, nullptr};
    hipStream_t wf_stream(int k) const { return k ? xstream[k] : stream; }
    // scene
    BNode4* d_nodes = nullptr;
    float4* d_isect = nullptr;
    float4* d_shade = nullptr;
    int bvh_nodes = 0, bvh_depth = 0;
    bool trav_stats = false;
    WFState wf;
    float4* d_mats = nullptr;
    int ntri = 0;
    int nmesh = 0;
    // launch state (LaunchParams.h:9-28)
    int width = 0, height = 0;
    float cam_pos[3] = {0, 0, 0};
    float inv_view[16] = {0};
    float inv_proj[16] = {0};
    DevLight* d_lights = nullptr;
    int n_lights = 0;
    int lights_cap = 0;
    int max_bounces = 0;
    int material_mode = PT_MAT_DEFAULT;
    int kernel = PT_KERNEL_MEGA;
    uint32_t frame_id = 0;
    // buffers
    float4* d_tuv = nullptr;       // per-triangle texcoords (leaf order), textured scenes only
    uint32_t* d_texels = nullptr;  // RGBA8 texel pool
    int4* d_texinfo = nullptr;     // per texture: offset, width, height
    float* d_frame = nullptr;   // 1-spp frame (pt_render)
    // render-ahead (pt_set_render_ahead): while nothing that changes the image changes between
    // pt_render calls, a miss renders the next k frames in one wavefront batch into a ring of
    // 1-spp images (k doubling per sequential miss up to render_ahead), and the calls for those
    // frame ids download them from the ring
    struct RenderKey {
        int w = 0, h = 0, n_lights = 0, max_bounces = 0, mode = 0, kernel = 0, debug_pixel = -1;
        uint32_t lights_version = 0, debug_frame = 0, debug_version = 0;
        const void* lights = nullptr;
        float cam[3 + 16 + 16] = {};
        bool operator==(const RenderKey& o) const {
            return w == o.w && h == o.h && n_lights == o.n_lights && max_bounces == o.max_bounces && mode == o.mode &&
                   kernel == o.kernel && debug_pixel == o.debug_pixel && lights_version == o.lights_version &&
                   debug_frame == o.debug_frame && debug_version == o.debug_version && lights == o.lights &&
                   std::memcmp(cam, o.cam, sizeof cam) == 0;
        }
    };
    int render_ahead = 64;
    // A render-ahead batch is also bounded by memory and by time (ahead_frames): its queues and
    // the two ring slots take at most a quarter of the device memory (and only what is free), and
    // its estimated duration stays within ahead_budget_ms (pt_set_render_ahead_budget), so a
    // call that changes the state waits for at most about that much work already enqueued.
    double ahead_budget_ms = 50.0;
    double frame_ms_est = 0.0;  // ms per frame of the last measured ring batch (0: none yet)
    int ahead_oom_cap = 1 << 30;  // largest batch since an allocation failed (reset per sequence)
    // Two ring slots: once the ramp reaches its length, pt_render enqueues the next batch into
    // the other slot while the caller downloads this one's frames (on dl_stream, after the
    // slot's `ready` event), so rendering and the device-to-host copies overlap.
    struct RingSlot {
        float* d = nullptr;
        int cap = 0;
        uint32_t first = 0, n = 0;
        RenderKey key;
        hipEvent_t start = nullptr, ready = nullptr;  // recorded on `stream` around the slot's batch
        bool measured = true;                         // its duration is in frame_ms_est
        bool speculative = false;                     // a cancellable look-ahead batch (cancel_look_ahead)
        // a speculative batch a call has taken a frame from (render_frame_image): no longer
        // cancellable, and a cancel of a later batch waits for it first
        bool served = false;
    };
    RingSlot ring[2];
    int ring_k = 1, ring_last = 0;  // ramp length, slot rendered last
    bool spec_pending = false;      // a look-ahead batch was enqueued since the last collect
    hipStream_t dl_stream = nullptr;
    hipEvent_t ev_frame = nullptr;  // after the d_frame render (no ring)
    // a one-frame call in row bands (pt_set_band_split): band 0 holds the first band0_rows rows
    // (0: the last one-frame call was not banded); ev_band0 follows its k_accum, so pt_render can
    // download them while band 1 still renders
    int band0_rows = 0;
    hipEvent_t ev_band0 = nullptr;
    uint32_t lights_version = 0;
    uint32_t debug_version = 0;  // bumped by pt_set_debug_pixel (the records are rewritten)
    float* d_display = nullptr;  // progressive view buffer (pt_display_*)
    int display_max = -1;
    int display_samples = 0;
    bool display_ready = false;
    float* d_accum = nullptr;   // internal sum buffer
    float* user_accum = nullptr;
    unsigned long long* d_counters = nullptr;
    // stats: one HIP event pair per kernel launch, on the library stream
    EventPool ev;
    uint64_t launches = 0;
    // optional per-launch timing of the wavefront's closest-hit trace kernel (k_extend)
    bool kernel_timing = false;
    bool primary_dedup = true;  // pt_set_primary_dedup
    bool band_split = true;     // pt_set_band_split: one-frame calls render two row bands on two streams
    bool wide_trace = true;     // one-stream calls: wide trace workgroups (PT_WIDE_TRACE env 0 turns it off)
    EventPool tev;
    std::vector<hipEvent_t> tev_frame;  // 2 * (max_bounces + 1) events handed to one frame
    double trace_ms = 0.0;
    uint64_t trace_launches = 0;
    // the k_trace_pair launches among them (fused modes: every timed trace launch after a batch's
    // k_extend), in a pool of their own so their time is reported per kernel (pt_stats pair_kernel_*)
    EventPool pev;
    double pair_ms = 0.0;
    uint64_t pair_launches = 0;
    // the same for the dominant shading kernel of a bounce (pt_stats shade_kernel_*)
    EventPool sev;
    std::vector<hipEvent_t> sev_frame;
    double shade_ms = 0.0;
    uint64_t shade_launches = 0;
    // render-ahead frames rendered into the ring and calls served from it (pt_stats)
    uint64_t ahead_rendered = 0, ahead_served = 0;
    // Look-ahead cancellation (cancel_look_ahead, pt_wavefront.hip wf_cancel_poll): the newest
    // cancel epoch in pinned host memory, which the kernels of a speculative batch read over PCIe
    // (d_cancel_host) and relay through a device word (d_cancel_seen); cancel_epoch is the epoch
    // the next speculative batch is enqueued under.
    unsigned* h_cancel = nullptr;
    unsigned* d_cancel_host = nullptr;
    unsigned* d_cancel_seen = nullptr;
    unsigned cancel_epoch = 0;
    uint64_t ahead_cancelled = 0;  // look-ahead batches cancelled (pt_stats)
    // pt_set_debug_hold (tests): the next speculative batches start with k_hold, which waits until
    // the batch is cancelled, the pinned release word is set, or 10 s pass
    bool debug_hold = false;
    unsigned* h_hold_release = nullptr;
    unsigned* d_hold_release = nullptr;
    uint64_t ahead_held = 0;  // speculative batches enqueued behind a hold (pt_stats)
    bool pending = false;
    uint64_t samples = 0;
    double last_ms = 0.0, total_ms = 0.0;
    uint64_t calls = 0;
    double bvh_ms = 0.0;
    int frames_per_launch = 128;  // 56 GB of queues at 1080p (16 -> 64 frames +5 % Lambert,
                                  // 64 -> 128 with the ray pools +0.7 to +2.5 %)
    int nf_fit = 0;  // > 0: the largest batch whose queues fitted after an out-of-memory halving
                     // (launch_frames); cleared by pt_set_frames_per_launch and pt_resize, and once
                     // the free memory would hold the full batch again
    // pt_set_queue_budget: the most bytes all wavefront streams' queues may hold together
    // (0 = default, a quarter of the device memory; < 0 = no budget, only the 2^28-path cap)
    int64_t queue_budget = 0;
    int last_streams = 0, last_batch = 0;  // streams and frames per batch of the last wavefront call
    // multi-device (pt_options.n_devices >= 1): this renderer is device 0 of the list; peers are
    // single-device renderers of the other devices; comms[g] is device g's RCCL communicator
    std::vector<pt_renderer*> peers;
    std::vector<ncclComm_t> comms;
    float* d_part = nullptr;  // device 0's own partial sum (the total is accum())
    // pt_set_accum_fp64: the sum is kept in fp64 (d_accum64; device 0 of a multi-device renderer
    // also d_part64), accum() holds its fp32 rounding
    bool accum64 = false;
    double* d_accum64 = nullptr;
    double* d_part64 = nullptr;
    // debug path (pt_set_debug_pixel): pixel W*y+x (-1 = off), frame id, per-bounce records
    int debug_pixel = -1;
    uint32_t debug_frame = 0;
    float* d_debug = nullptr;

    DevScene scene() const {
        DevScene S;
        S.nodes = d_nodes;
        S.isect = d_isect;
        S.shade = d_shade;
        S.mats = d_mats;
        S.tuv = d_tuv;
        S.texels = d_texels;
        S.texinfo = d_texinfo;
        S.ntri = ntri;
        S.n_nodes = bvh_nodes;
        S.lds_nodes = nullptr;
        S.n_lds = 0;
        return S;
    }
    float* accum() const { return user_accum ? user_accum : d_accum; }
};

namespace {

int collect_pending(pt_renderer* r) {
    if (!r->pending) return PT_OK;
    double sum = 0.0, tsum = 0.0, ssum = 0.0;
    size_t n = 0, tn = 0, sn = 0;
    PT_HIP(r->ev.collect(&sum, &n), "frame events");
    PT_HIP(r->tev.collect(&tsum, &tn), "trace-kernel events");
    double psum = 0.0;
    size_t pn = 0;
    PT_HIP(r->pev.collect(&psum, &pn), "pair-kernel events");
    tsum += psum;  // trace_kernel_* cover k_extend and k_trace_pair together, as before
    tn += pn;
    r->pair_ms += psum;
    r->pair_launches += pn;
    PT_HIP(r->sev.collect(&ssum, &sn), "shading-kernel events");
    r->spec_pending = false;  // ev.collect waited for every enqueued batch
    r->launches += n;
    r->last_ms = sum;
    r->total_ms += sum;
    r->trace_ms += tsum;
    r->trace_launches += tn;
    r->shade_ms += ssum;
    r->shade_launches += sn;
    r->pending = false;
    return PT_OK;
}

int next_event_pair(pt_renderer* r, hipEvent_t* a, hipEvent_t* b) {
    PT_HIP(r->ev.next(a, b), "hipEventCreate");
    return PT_OK;
}

DevLaunch make_launch(const pt_renderer* r, float* accum, uint32_t frame_base, uint32_t n_frames,
                      double* accum64 = nullptr, size_t frame_stride = 0) {
    DevLaunch L;
    L.width = r->width;
    L.height = r->height;
    L.row0 = 0;
    L.image_height = r->height;
    std::memcpy(L.cam_pos, r->cam_pos, sizeof L.cam_pos);
    std::memcpy(L.inv_view, r->inv_view, sizeof L.inv_view);
    std::memcpy(L.inv_proj, r->inv_proj, sizeof L.inv_proj);
    L.lights = r->d_lights;
    L.n_lights = r->n_lights;
    L.max_bounces = r->max_bounces;
    L.frame_base = frame_base;
    L.n_frames = n_frames;
    L.accum = accum;
    L.accum64 = accum64;
    L.frame_stride = frame_stride;
    L.counters = r->d_counters;
    L.debug_pixel = r->d_debug ? r->debug_pixel : -1;
    L.debug_frame = r->debug_frame;
    L.debug = r->d_debug;
    return L;
}

// Bytes the wavefront queues of all streams hold now.
size_t queue_bytes_held(const pt_renderer* r) {
    size_t b = r->wf.paths > 0 ? wavefront_bytes(r->wf.paths, r->wf.max_bounces) : 0;
    for (int k = 1; k < pt_renderer::kMaxWFStreams; ++k)
        if (r->xwf[k].paths > 0) b += wavefront_bytes(r->xwf[k].paths, r->xwf[k].max_bounces);
    return b;
}

// The most bytes all streams' queues may hold together (pt_set_queue_budget): the caller's
// figure, or by default a quarter of the device memory -- 72 GB on an MI355X, above the 56 GB the
// 128-frame 1080p batch takes on one stream, so the Lambert, Default and Layered modes keep it,
// while two-stream Conductor / Dielectric calls take 82-frame batches.  SIZE_MAX:
// no budget.
size_t queue_budget_bytes(const pt_renderer* r) {
    if (r->queue_budget < 0) return SIZE_MAX;
    if (r->queue_budget > 0) return (size_t)r->queue_budget;
    size_t total = 0;
    if (hipDeviceTotalMem(&total, r->device) != hipSuccess || total == 0) {
        (void)hipGetLastError();
        return SIZE_MAX;
    }
    return total / 4;
}

// Launch frames [first, first+n) in chunks, adding into accum; brackets with events.  Does not
// wait for earlier work: the event pairs of every launch since the last synchronisation point
// are summed at the next pt_synchronize / pt_get_stats / download (collect_pending).
// frame_stride > 0 (wavefront only): frame first + j is written alone to accum + j * frame_stride.
int launch_frames(pt_renderer* r, float* accum, uint32_t first, uint32_t n, double* accum64 = nullptr,
                  size_t frame_stride = 0, bool speculative = false) {
    int rc = PT_OK;
    // callers that never synchronise through the library (pt_stream interop, device sum buffers,
    // loops over pt_launch / pt_display_add_frame) would grow the event pools without bound:
    // past kMaxPendingEvents pairs, retire them first (this waits for the enqueued work)
    if (r->ev.used + r->tev.used + r->pev.used + r->sev.used > kMaxPendingEvents && (rc = collect_pending(r)) != PT_OK)
        return rc;
    const DevScene S = r->scene();
    uint32_t done = 0;
    const uint32_t chunk = (uint32_t)std::max(1, r->frames_per_launch);
    r->pending = true;
    r->band0_rows = 0;  // set below when this call renders its frame in row bands
    // AUTO = wavefront: it beats the megakernel in every material mode (1080p
    // depth 8, 16 frames per launch, Msamples/s wavefront / megakernel: Lambert 725 / 414,
    // Dielectric 1239 / 758, Default 255 / 104).
    int kernel = r->kernel;
    if (kernel == PT_KERNEL_AUTO) kernel = PT_KERNEL_WAVEFRONT;
    // Lambert / Conductor / Dielectric: k_extend at bounce 0, then k_trace_pair per bounce
    const bool fused = r->material_mode == PT_MAT_LAMBERT || r->material_mode == PT_MAT_CONDUCTOR ||
                       r->material_mode == PT_MAT_DIELECTRIC;
    if (accum64 && kernel != PT_KERNEL_WAVEFRONT)
        return fail(PT_ERR_INVALID, "fp64 accumulation (pt_set_accum_fp64) runs with the wavefront kernel");
    if (frame_stride && kernel != PT_KERNEL_WAVEFRONT)
        return fail(PT_ERR_INVALID, "per-frame images (render-ahead) run with the wavefront kernel");
    if (kernel == PT_KERNEL_WAVEFRONT) {
        // Frames per wavefront launch chain: the queues hold nf frames' paths (208 B each), at most
        // kMaxWFPaths of them.  Batching amortises launch gaps and the per-kernel SIMT tail:
        // Lambert 1080p 545 / 648 / 664 Msamples/s at 1 / 8 / 16 frames.
        constexpr int kMaxWFPaths = 1 << 28;  // 56 GB of queues at 208 B per path
        const int P = r->width * r->height;
        const int maxb = std::max(1, r->max_bounces);
        const int nf_full = std::max(1, std::min({r->frames_per_launch, (int)std::min<uint32_t>(n, 1u << 20),
                                                  kMaxWFPaths / std::max(1, P)}));
        // a batch size that fitted after an out-of-memory halving is kept until the free memory
        // (plus what the queues hold now) would take the full batch again
        if (r->nf_fit > 0 && r->nf_fit < nf_full) {
            size_t free_b = 0, total_b = 0;
            if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
                if (free_b + queue_bytes_held(r) >= wavefront_bytes(P * nf_full, maxb)) r->nf_fit = 0;
            } else {
                (void)hipGetLastError();
            }
        }
        int nf_cap = std::min(nf_full, r->nf_fit > 0 ? r->nf_fit : (1 << 30));
        // two batches or more: alternate them between two streams with their own queues, so one
        // batch's kernels run beside the other's (the memory-bound shading of one beside the
        // VALU-bound tracing of the other, and each kernel's SIMT tail filled); k_accum still adds
        // the batches in frame order (accum_wait / accum_done)
        const int nbatch = (int)((n + (uint32_t)nf_cap - 1) / (uint32_t)nf_cap);
        // One frame (pt_render / pt_display_add_frame without render-ahead, the path a viewer that
        // moves the camera every frame gets): its rows split into two bands, one per stream, so
        // each band's kernels fill the other's SIMT tails.  Every pixel's path depends only on its
        // pixel and frame id, so the image is the same bit for bit.
        const bool bands = n == 1 && r->band_split && r->height >= 16;  // both bands non-empty
        // auto: a second stream pays where one batch's shading fills the other's trace tails
        // (Conductor +0.6 %, Dielectric +4 % at 128 frames); Lambert, Default and Layered run as
        // fast on one stream with half the queue memory
        const bool two = r->material_mode == PT_MAT_CONDUCTOR || r->material_mode == PT_MAT_DIELECTRIC;
        const int want = r->wf_streams > 0 ? r->wf_streams : (bands || two ? 2 : 1);
        int ns = std::max(1, std::min(want, bands ? 2 : nbatch));
        // the queue budget (pt_set_queue_budget): the ns streams' queues
        // together stay within it, by smaller batches (every batch size gives the same image);
        // queues that streams beyond ns still hold are freed when they would overrun it
        const size_t budget = queue_budget_bytes(r);
        if (budget != SIZE_MAX) {
            const size_t per_frame = wavefront_bytes(P, maxb);
            const int nf_b = (int)std::max<size_t>(1, budget / ((size_t)ns * per_frame));
            nf_cap = std::min(nf_cap, nf_b);
            size_t used = (size_t)ns * wavefront_bytes(P * nf_cap, maxb);
            for (int k = ns; k < pt_renderer::kMaxWFStreams; ++k) {
                if (r->xwf[k].paths == 0) continue;
                const size_t held = wavefront_bytes(r->xwf[k].paths, r->xwf[k].max_bounces);
                if (used + held <= budget) {
                    used += held;
                    continue;
                }
                PT_HIP(hipStreamSynchronize(r->xstream[k]), "hipStreamSynchronize");
                wavefront_free(r->xwf[k]);
            }
        }
        for (int k = 0; k < ns; ++k) {
            WFState& w = k ? r->xwf[k] : r->wf;
            // queues larger than the budget's share (a lowered budget) are allocated again, smaller
            // (a budget below one frame's queues still allows one frame: no reallocation per call)
            const bool over = budget != SIZE_MAX && w.paths > P &&
                              (size_t)ns * wavefront_bytes(w.paths, w.max_bounces) > budget;
            if (w.paths < P * nf_cap || w.max_bounces < r->max_bounces || over) {
                for (int j = 0; j < pt_renderer::kMaxWFStreams; ++j)
                    if (r->wf_stream(j)) PT_HIP(hipStreamSynchronize(r->wf_stream(j)), "hipStreamSynchronize");
                wavefront_free(w);
                hipError_t ae = wavefront_alloc(w, P * nf_cap, maxb);
                if (ae == hipErrorOutOfMemory && k == 0) {
                    // queues of the other streams (an earlier call's, or a mode with more
                    // streams) go first, then the full batch again
                    bool freed = false;
                    for (int j = 1; j < pt_renderer::kMaxWFStreams; ++j)
                        if (r->xwf[j].paths > 0) {
                            wavefront_free(r->xwf[j]);
                            freed = true;
                        }
                    if (freed) ae = wavefront_alloc(w, P * nf_cap, maxb);
                }
                // the first stream's queues: halve the batch until they fit (every batch size gives
                // the same image), PT_ERR_NOMEM only when one frame does not; the size that fitted
                // stays the cap until the memory would take the full batch (above),
                // pt_set_frames_per_launch or pt_resize
                while (ae == hipErrorOutOfMemory && k == 0 && nf_cap > 1) {
                    nf_cap = (nf_cap + 1) / 2;
                    r->nf_fit = nf_cap;
                    ae = wavefront_alloc(w, P * nf_cap, maxb);
                }
                // the extra streams only overlap batches: when their queues do not fit, render on
                // the k streams that do (the image is the same, added in frame order either way)
                if (ae == hipErrorOutOfMemory && k > 0) {
                    ns = k;
                    break;
                }
                PT_HIP(ae, "wavefront_alloc");
            }
        }
        r->last_streams = ns;
        r->last_batch = nf_cap;
        const bool dual = ns > 1;
        if (dual && !r->ev_fork) {
            PT_HIP(hipEventCreateWithFlags(&r->ev_fork, hipEventDisableTiming), "hipEventCreate");
            for (hipEvent_t& e : r->ev_accum) PT_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
        }
        for (int k = 1; k < ns; ++k)
            if (!r->xstream[k]) {
                PT_HIP(hipStreamCreateWithFlags(&r->xstream[k], hipStreamNonBlocking), "hipStreamCreate");
                PT_HIP(hipEventCreateWithFlags(&r->ev_join[k], hipEventDisableTiming), "hipEventCreate");
            }
        int dev_cus = 256;
        (void)hipDeviceGetAttribute(&dev_cus, hipDeviceAttributeMultiprocessorCount, r->device);
        hipEvent_t a = nullptr, b = nullptr;  // dual: one event pair around the whole call
        if (dual) {
            rc = next_event_pair(r, &a, &b);
            if (rc) return rc;
            PT_HIP(hipEventRecord(a, r->stream), "hipEventRecord");
            PT_HIP(hipEventRecord(r->ev_fork, r->stream), "hipEventRecord");
            for (int k = 1; k < ns; ++k) PT_HIP(hipStreamWaitEvent(r->xstream[k], r->ev_fork, 0), "hipStreamWaitEvent");
        }
        const int nband = bands && ns > 1 ? 2 : 1;  // row bands of a one-frame call
        // band 0 is the smaller one (7/16 of the rows), so it finishes first and pt_render's
        // download of its rows overlaps the rest of band 1
        const int rows0 = r->height * 7 / 16;
        r->band0_rows = nband > 1 ? rows0 : 0;
        if (nband > 1 && !r->ev_band0) PT_HIP(hipEventCreateWithFlags(&r->ev_band0, hipEventDisableTiming), "hipEventCreate");
        int batch = 0;
        for (uint32_t f = 0; f < n; ++batch) {  // one event pair per batch (the batch's kernel chain)
            const int nf = (int)std::min<uint32_t>((uint32_t)nf_cap, n - f);
            DevLaunch L = make_launch(r, frame_stride ? accum + (size_t)f * frame_stride : accum, first + f,
                                      (uint32_t)nf, accum64, frame_stride);
            const int band = nband > 1 ? batch : 0;
            if (nband > 1) {  // rows [row0, row0 + height) of the frame; the sum buffers at the band
                L.row0 = band == 0 ? 0 : rows0;
                L.height = band == 0 ? rows0 : r->height - rows0;
                const size_t off = 3 * (size_t)r->width * (size_t)L.row0;
                L.accum += off;
                if (L.accum64) L.accum64 += off;
            }
            const int sk = batch % ns;  // stream of this batch
            hipStream_t st = r->wf_stream(sk);
            if (!dual) {
                rc = next_event_pair(r, &a, &b);
                if (rc) return rc;
            }
            const hipEvent_t* tev = nullptr;
            const hipEvent_t* sev = nullptr;
            if (r->kernel_timing) {
                r->tev_frame.resize(2 * (size_t)(r->max_bounces + 1));  // <= max_bounces + 1 trace launches
                // launch 0 is the batch's k_extend; in the fused modes the others are k_trace_pair
                for (int k = 0; k <= r->max_bounces; ++k)
                    PT_HIP((k > 0 && fused ? r->pev : r->tev).next(&r->tev_frame[2 * k], &r->tev_frame[2 * k + 1]),
                           "hipEventCreate");
                tev = r->tev_frame.data();
                r->sev_frame.resize(2 * (size_t)(r->max_bounces + 1));  // <= max_bounces shading launches
                for (int k = 0; k <= r->max_bounces; ++k)
                    PT_HIP(r->sev.next(&r->sev_frame[2 * k], &r->sev_frame[2 * k + 1]), "hipEventCreate");
                sev = r->sev_frame.data();
            }
            if (!dual) PT_HIP(hipEventRecord(a, r->stream), "hipEventRecord");
            int n_timed = 0, n_stimed = 0;
            WFState wq = sk ? r->xwf[sk] : r->wf;
            if (speculative && r->d_cancel_seen) {  // a look-ahead batch: its kernels poll the cancel words
                wq.cancel_host = r->d_cancel_host;
                wq.cancel_seen = r->d_cancel_seen;
                wq.cancel_epoch = r->cancel_epoch;
                if (r->debug_hold && r->d_hold_release && batch == 0) {  // pt_set_debug_hold: k_hold first
                    wq.hold_release = r->d_hold_release;
                    r->ahead_held++;
                }
            }
            PT_HIP(launch_wavefront_frame(r->material_mode, r->trav_stats, S, L, wq, first + f,
                                          nf, r->primary_dedup, dev_cus, st, tev, &n_timed,
                                          // batches add into the sum in frame order; bands touch disjoint pixels
                                          dual && batch > 0 && nband == 1 ? r->ev_accum[(batch - 1) & 1] : nullptr,
                                          dual && nband == 1 ? r->ev_accum[batch & 1] : nullptr, sev, &n_stimed,
                                          ns == 1 && r->wide_trace),
                   "wavefront launch");
            if (tev) {  // pairs never recorded (the last ones handed out)
                const int unused = r->max_bounces + 1 - n_timed;
                const int unused_pair = fused ? std::min(unused, r->max_bounces) : 0;
                r->pev.give_back((size_t)unused_pair);
                r->tev.give_back((size_t)(unused - unused_pair));
            }
            if (sev) r->sev.give_back((size_t)(r->max_bounces + 1 - n_stimed));
            if (!dual) PT_HIP(hipEventRecord(b, r->stream), "hipEventRecord");
            if (nband > 1 && band == 0) PT_HIP(hipEventRecord(r->ev_band0, st), "hipEventRecord");
            if (band + 1 == nband) f += (uint32_t)nf;
        }
        if (dual) {
            for (int k = 1; k < ns; ++k) {
                PT_HIP(hipEventRecord(r->ev_join[k], r->xstream[k]), "hipEventRecord");
                PT_HIP(hipStreamWaitEvent(r->stream, r->ev_join[k], 0), "hipStreamWaitEvent");
            }
            PT_HIP(hipEventRecord(b, r->stream), "hipEventRecord");
        }
        done = n;
    }
    while (done < n) {
        uint32_t k = std::min(chunk, n - done);
        DevLaunch L = make_launch(r, accum, first + done, k);
        hipEvent_t a, b;
        rc = next_event_pair(r, &a, &b);
        if (rc) return rc;
        PT_HIP(hipEventRecord(a, r->stream), "hipEventRecord");
        PT_HIP(launch_render(kernel, r->material_mode, r->trav_stats, S, L, r->stream), "render launch");
        PT_HIP(hipEventRecord(b, r->stream), "hipEventRecord");
        done += k;
    }
    r->samples += (uint64_t)n * (uint64_t)r->width * (uint64_t)r->height;
    r->calls++;
    return PT_OK;
}

bool valid_mode(int m) { return m >= PT_MAT_DEFAULT && m <= PT_MAT_LAYERED; }

// Everything a 1-spp image depends on besides its frame id (the scene is fixed at pt_create).
pt_renderer::RenderKey render_key(const pt_renderer* r) {
    pt_renderer::RenderKey k;
    k.w = r->width;
    k.h = r->height;
    k.n_lights = r->n_lights;
    k.max_bounces = r->max_bounces;
    k.mode = r->material_mode;
    k.kernel = r->kernel;
    k.debug_pixel = r->d_debug ? r->debug_pixel : -1;
    k.debug_frame = r->debug_frame;
    k.lights_version = r->lights_version;
    k.debug_version = r->debug_version;
    k.lights = r->d_lights;
    std::memcpy(k.cam, r->cam_pos, sizeof r->cam_pos);
    std::memcpy(k.cam + 3, r->inv_view, sizeof r->inv_view);
    std::memcpy(k.cam + 19, r->inv_proj, sizeof r->inv_proj);
    return k;
}

void ring_free(pt_renderer* r) {
    for (pt_renderer::RingSlot& s : r->ring) {
        if (s.d) (void)hipFree(s.d);  // hipFree waits for the work that may still read it
        s.d = nullptr;
        s.cap = 0;
        s.n = 0;
        s.measured = true;
        s.speculative = false;
        s.served = false;
    }
    r->ring_k = 1;
    r->ahead_oom_cap = 1 << 30;
}

// Frames one render-ahead batch may hold now.  Memory: the batch's wavefront queues (one stream)
// and both ring slots take at most a quarter of the device memory, and no more than is free
// besides what the renderer already holds for them (render-ahead sized its queues
// like pt_render_frames, 28 GB at 1080p).  Time: the batch's estimated duration stays within
// ahead_budget_ms, from the per-frame time of the last measured ring batch (a call that changes
// the state waits behind at most the batch in flight).  Always >= 1.
int ahead_frames(pt_renderer* r, size_t n3, bool by_time) {
    int k = std::min(r->render_ahead, r->ahead_oom_cap);
    const size_t P = n3 / 3;
    const size_t per_frame = wavefront_bytes((int)P, std::max(1, r->max_bounces)) + 2 * sizeof(float) * n3;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && total_b > 0) {
        size_t held = 2 * sizeof(float) * n3 * (size_t)std::max(r->ring[0].cap, r->ring[1].cap);
        if (r->wf.paths > 0) held += wavefront_bytes(r->wf.paths, r->wf.max_bounces);
        const size_t avail = std::min(total_b / 4, free_b + held);
        k = std::min<size_t>((size_t)k, std::max<size_t>(1, avail / per_frame));
    } else {
        (void)hipGetLastError();
    }
    if (by_time && r->ahead_budget_ms > 0.0 && r->frame_ms_est > 0.0)
        k = std::min(k, std::max(1, (int)(r->ahead_budget_ms / r->frame_ms_est)));
    return std::max(1, k);
}

// A finished ring batch's duration per frame -> frame_ms_est (no wait: only batches done by now).
void ring_measure(pt_renderer* r) {
    for (pt_renderer::RingSlot& sl : r->ring) {
        if (sl.measured || sl.n == 0 || hipEventQuery(sl.ready) != hipSuccess) continue;
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, sl.start, sl.ready) == hipSuccess && ms > 0.0f) r->frame_ms_est = ms / sl.n;
        (void)hipGetLastError();
        sl.measured = true;
    }
}

// Slot s of the ring with room for `cap` frames and its events.
int ring_reserve(pt_renderer* r, int s, int cap, size_t n3) {
    pt_renderer::RingSlot& sl = r->ring[s];
    if (!sl.ready) PT_HIP(hipEventCreate(&sl.ready), "hipEventCreate");
    if (!sl.start) PT_HIP(hipEventCreate(&sl.start), "hipEventCreate");
    if (cap <= sl.cap) return PT_OK;
    if (sl.d) {
        PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
        (void)hipFree(sl.d);
        sl.d = nullptr;
        sl.cap = 0;
    }
    const hipError_t e = hipMalloc(&sl.d, sizeof(float) * n3 * (size_t)cap);
    if (e != hipSuccess) {
        (void)hipGetLastError();  // a later launch's hipGetLastError must not see this failure
        return hip_fail(e, "hipMalloc render-ahead ring");
    }
    sl.cap = cap;
    return PT_OK;
}

// The cancel words of the look-ahead batches (allocated at the first one; false if they cannot
// be, and the batch is then enqueued without them).
bool cancel_words(pt_renderer* r) {
    if (r->d_cancel_seen) return true;
    unsigned* h = nullptr;
    unsigned* d = nullptr;
    if (hipHostMalloc((void**)&h, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    *h = 0;
    void* hd = nullptr;
    if (hipHostGetDevicePointer(&hd, h, 0) != hipSuccess || hipMalloc((void**)&d, sizeof(unsigned)) != hipSuccess ||
        hipMemsetAsync(d, 0, sizeof(unsigned), r->stream) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipHostFree(h);
        if (d) (void)hipFree(d);
        return false;
    }
    r->h_cancel = h;
    r->d_cancel_host = static_cast<unsigned*>(hd);
    r->d_cancel_seen = d;
    r->cancel_epoch = 0;
    return true;
}

// Render frames [first, first + n) into ring slot s (room for `cap` frames) as 1-spp images and
// record its events.  `speculative`: the look-ahead batch, which cancel_look_ahead can stop.
int ring_fill(pt_renderer* r, int s, const pt_renderer::RenderKey& k, uint32_t first, int n, int cap, size_t n3,
              bool speculative = false) {
    pt_renderer::RingSlot& sl = r->ring[s];
    sl.n = 0;
    sl.measured = true;
    sl.served = false;
    sl.speculative = speculative && cancel_words(r);
    int rc = ring_reserve(r, s, std::max(n, cap), n3);
    if (rc == PT_OK) PT_HIP(hipEventRecord(sl.start, r->stream), "hipEventRecord");
    if (rc == PT_OK) rc = launch_frames(r, sl.d, first, (uint32_t)n, nullptr, n3, sl.speculative);
    if (rc != PT_OK) return rc;
    PT_HIP(hipEventRecord(sl.ready, r->stream), "hipEventRecord");
    sl.key = k;
    sl.first = first;
    sl.n = (uint32_t)n;
    sl.measured = false;
    r->ahead_rendered += (uint64_t)n;
    return PT_OK;
}

// Cancel the look-ahead batch in flight.  The reference renders one
// frame per Render() call (OptixRenderer.cpp:617-647) and its viewer moves the camera between
// calls (OptixView.cpp:133-139); frames pt_render rendered ahead under the old state are then
// useless, and the next call would wait behind up to ahead_budget_ms of them.  When the state
// no longer matches the speculative slot (or `force`: the caller is about to change it, and
// waits on the library stream first), a newer epoch is published in the pinned host word: the
// batch's kernels see it within about a trace kernel's poll interval and stop
// (pt_wavefront.hip wf_cancel_poll), the rest of its launches drain as no-ops, and the slot
// is discarded.  A batch that already finished is kept.
void cancel_look_ahead(pt_renderer* r, bool force = false) {
    if (!r->spec_pending || !r->h_cancel) return;
    pt_renderer::RingSlot& sl = r->ring[r->ring_last];
    if (sl.n == 0 || !sl.speculative) return;  // not speculative: also a batch a call took a frame from
    if (!force && sl.key == render_key(r)) return;
    if (hipEventQuery(sl.ready) == hipSuccess) return;  // done: its frames stay valid for their state
    (void)hipGetLastError();                            // hipErrorNotReady
    // The epoch stops every batch enqueued under an older one: a served batch still in flight
    // (the other slot, enqueued earlier on the same stream) finishes first
    pt_renderer::RingSlot& other = r->ring[r->ring_last ^ 1];
    if (other.served && other.n > 0 && hipEventQuery(other.ready) != hipSuccess) {
        (void)hipGetLastError();
        (void)hipEventSynchronize(other.ready);
    }
    ++r->cancel_epoch;
    __atomic_store_n(r->h_cancel, r->cancel_epoch, __ATOMIC_SEQ_CST);
    sl.n = 0;
    sl.speculative = false;
    r->ahead_cancelled++;
}

// The 1-spp image of frame r->frame_id for pt_render / pt_display_add_frame (OptixRenderer::Render,
// OptixRenderer.cpp:617-647), enqueued on r->stream; *ready (if given) is an event after which the
// image may be read from another stream.  With render-ahead (wavefront kernel), a frame a ring
// slot holds under the same render state is taken from it; a miss renders the next k frames as one
// batch into a slot, k doubling on every miss that continues the ring's frame sequence under the
// same state (up to ahead_frames: render_ahead, the memory cap and the time budget) and 1
// otherwise, so an interactive caller that changes the camera every frame pays for one frame per
// call.  With `look_ahead` (pt_render, whose downloads run on dl_stream), the first call served
// from a slot of the full ramp length also enqueues the following frames into the other slot,
// which the GPU renders while the caller downloads this slot's frames.  Each ring image is the
// one-frame sum into zeros that the plain path computes, bit for bit.  The debug pixel's records
// belong to the call that renders its frame, so with a debug pixel set every call renders its
// own frame.
int render_frame_image(pt_renderer* r, const float** img, hipEvent_t* ready = nullptr, bool look_ahead = false,
                       hipEvent_t* part_ready = nullptr, size_t* part_floats = nullptr) {
    const size_t n3 = 3 * (size_t)r->width * (size_t)r->height;
    const int kernel = r->kernel == PT_KERNEL_AUTO ? PT_KERNEL_WAVEFRONT : r->kernel;
    const uint32_t f = r->frame_id;
    const bool debug = r->d_debug && r->debug_pixel >= 0;
    cancel_look_ahead(r);  // a state change since the look-ahead batch: stop it (also with render-ahead now off)
    if (r->render_ahead > 1 && kernel == PT_KERNEL_WAVEFRONT && !debug) {
        ring_measure(r);
        const pt_renderer::RenderKey k = render_key(r);
        int s = -1;
        bool seq = false;
        for (int i = 0; i < 2; ++i) {
            const pt_renderer::RingSlot& sl = r->ring[i];
            if (sl.n == 0 || !(k == sl.key)) continue;
            if (f - sl.first < sl.n) s = i;  // unsigned: also false for f < first
            if (i == r->ring_last && f == sl.first + sl.n) seq = true;
        }
        int rc = PT_OK;
        if (s < 0) {  // miss: the next k frames into the slot not rendered last
            if (!seq) r->ahead_oom_cap = 1 << 30;  // a new sequence tries the full length again
            const int kmax = ahead_frames(r, n3, false);
            const int kf = seq ? std::min(2 * r->ring_k, ahead_frames(r, n3, true)) : 1;
            s = r->ring_last ^ 1;
            rc = ring_fill(r, s, k, f, kf, kf == 1 ? 1 : kmax, n3);
            if (rc == PT_OK) {
                r->ring_k = kf;
                r->ring_last = s;
            } else if (rc == PT_ERR_NOMEM) {
                // no room for this batch: later batches of the sequence stay below it, and this
                // call renders its own frame alone (below)
                r->ahead_oom_cap = std::max(1, kf / 2);
                r->ring[s].n = 0;
            }
        }
        if (rc == PT_OK) {
            pt_renderer::RingSlot& sl = r->ring[s];
            // A frame handed out of a speculative batch may be read by work the caller has
            // already queued behind it (pt_display_add_frame's blend does not wait for the
            // batch): the batch is no longer cancellable
            if (sl.speculative) {
                sl.speculative = false;
                sl.served = true;
            }
            *img = sl.d + (size_t)(f - sl.first) * n3;
            if (ready) *ready = sl.ready;
            r->ahead_served++;
            const int o = s ^ 1;
            const uint32_t next = sl.first + sl.n;
            // the ramp is done once doubling this slot's length would pass the target length (the
            // length, a device-memory query, only for a call that may enqueue: ADVICE round 4)
            const bool may_look = look_ahead && f == sl.first && sl.n > 1 &&
                                  !(r->ring[o].n > 0 && r->ring[o].key == k && r->ring[o].first == next);
            const int kl = may_look ? ahead_frames(r, n3, true) : 0;  // the full ramp length now
            if (may_look && 2 * (int)sl.n > kl) {
                const int lrc = ring_fill(r, o, k, next, kl, ahead_frames(r, n3, false), n3, true);
                if (lrc == PT_OK) {
                    r->ring_k = kl;
                    r->ring_last = o;
                    r->spec_pending = true;
                } else if (lrc != PT_ERR_NOMEM) {
                    return lrc;
                } else {
                    r->ring[o].n = 0;
                }  // no room for the second slot: this call's frame is served all the same
            }
            return PT_OK;
        }
        if (rc != PT_ERR_NOMEM) return rc;
    }
    PT_HIP(hipMemsetAsync(r->d_frame, 0, sizeof(float) * n3, r->stream), "hipMemset frame");
    const int rc = launch_frames(r, r->d_frame, f, 1);
    if (rc) return rc;
    *img = r->d_frame;
    if (part_ready && r->band0_rows > 0) {  // the first band's rows are final once ev_band0 passes
        *part_ready = r->ev_band0;
        *part_floats = 3 * (size_t)r->width * (size_t)r->band0_rows;
    }
    if (ready) {
        if (!r->ev_frame) PT_HIP(hipEventCreateWithFlags(&r->ev_frame, hipEventDisableTiming), "hipEventCreate");
        PT_HIP(hipEventRecord(r->ev_frame, r->stream), "hipEventRecord");
        *ready = r->ev_frame;
    }
    return PT_OK;
}

// Multi-device pt_render_frames: frame ids first .. first+n-1 split into contiguous blocks
// (device g renders first + g*n/N .. , the same split as optixpathtracer_amd/sharding.py), each
// device adding its block in frame order into its own fp32 sum; then one ncclReduce (sum) of
// the N sums onto device 0's accum().  Every sample keeps its (pixel, frame id) seed, so the
// image equals the single-device one up to the fp32 order of the N-way sum.  Each device's work
// and its reduce are enqueued on that device's stream; nothing waits here.
int render_frames_multi(pt_renderer* r, uint32_t first, uint32_t n) {
    const int N = (int)r->comms.size();
    const size_t count = 3 * (size_t)r->width * (size_t)r->height;
    uint32_t f = first;
    for (int g = 0; g < N; ++g) {
        const uint32_t per = n / (uint32_t)N, extra = n % (uint32_t)N;
        const uint32_t ng = per + ((uint32_t)g < extra ? 1u : 0u);
        pt_renderer* d = g == 0 ? r : r->peers[(size_t)g - 1];
        if (ng > 0) {
            PT_HIP(hipSetDevice(d->device), "hipSetDevice");
            const int rc = launch_frames(d, g == 0 ? r->d_part : d->accum(), f, ng,
                                         r->accum64 ? (g == 0 ? r->d_part64 : d->d_accum64) : nullptr);
            if (rc) return rc;
        }
        f += ng;
    }
    ncclResult_t nr = ncclGroupStart();
    for (int g = 0; g < N && nr == ncclSuccess; ++g) {
        pt_renderer* d = g == 0 ? r : r->peers[(size_t)g - 1];
        if (r->accum64) {  // fp64 partial sums -> fp64 total on device 0
            const double* send = g == 0 ? r->d_part64 : d->d_accum64;
            double* recv = g == 0 ? r->d_accum64 : d->d_accum64;  // significant on the root only
            nr = ncclReduce(send, recv, count, ncclFloat64, ncclSum, 0, r->comms[(size_t)g], d->stream);
        } else {
            const float* send = g == 0 ? r->d_part : d->accum();
            float* recv = g == 0 ? r->accum() : d->accum();  // significant on the root only
            nr = ncclReduce(send, recv, count, ncclFloat32, ncclSum, 0, r->comms[(size_t)g], d->stream);
        }
    }
    const ncclResult_t ne = ncclGroupEnd();
    (void)hipSetDevice(r->device);
    if (nr != ncclSuccess || ne != ncclSuccess)
        return fail(PT_ERR_HIP, std::string("ncclReduce: ") + ncclGetErrorString(nr != ncclSuccess ? nr : ne));
    if (r->accum64) PT_HIP(accum_f64_to_f32(r->d_accum64, r->accum(), count, r->stream), "fp64 -> fp32 sum");
    return PT_OK;
}

// fp64 sum buffers (pt_set_accum_fp64) of one device for a W x H image, zeroed
int alloc_accum64(pt_renderer* r, int width, int height) {
    const size_t bytes = sizeof(double) * 3 * (size_t)width * (size_t)height;
    if (r->d_accum64) (void)hipFree(r->d_accum64);
    if (r->d_part64) (void)hipFree(r->d_part64);
    r->d_accum64 = r->d_part64 = nullptr;
    PT_HIP(hipMalloc(&r->d_accum64, bytes), "hipMalloc fp64 accum");
    PT_HIP(hipMemsetAsync(r->d_accum64, 0, bytes, r->stream), "hipMemset fp64 accum");
    if (!r->comms.empty()) {
        PT_HIP(hipMalloc(&r->d_part64, bytes), "hipMalloc fp64 partial sum");
        PT_HIP(hipMemsetAsync(r->d_part64, 0, bytes, r->stream), "hipMemset fp64 partial sum");
    }
    return PT_OK;
}

}  // namespace

extern "C" {

const char* pt_last_error(void) { return g_last_error.c_str(); }
const char* pt_version(void) { return "ptamd 0.1.0 gfx950"; }

int pt_create(const pt_scene* scene, const pt_options* options, pt_renderer** out) {
    if (!out) return fail(PT_ERR_INVALID, "pt_create: out is NULL");
    *out = nullptr;
    if (!scene || scene->n_meshes < 0 || (scene->n_meshes > 0 && !scene->meshes))
        return fail(PT_ERR_INVALID, "pt_create: invalid scene");
    pt_options opt{};
    if (options) opt = *options;
    // multi-device: validate the list, build device 0 here and the others as peers below
    std::vector<int> devlist;
    if (opt.n_devices < 0) return fail(PT_ERR_INVALID, "pt_create: negative n_devices");
    for (int g = 0; g < opt.n_devices; ++g) devlist.push_back(opt.device_list ? opt.device_list[g] : opt.device + g);
    if (!devlist.empty()) opt.device = devlist[0];
    if (!valid_mode(opt.material_mode)) return fail(PT_ERR_INVALID, "pt_create: invalid material_mode");
    if (opt.bvh_builder != PT_BVH_AUTO && opt.bvh_builder != PT_BVH_PLOC && opt.bvh_builder != PT_BVH_LBVH &&
        opt.bvh_builder != PT_BVH_SAH && opt.bvh_builder != PT_BVH_SAH_GPU)
        return fail(PT_ERR_INVALID, "pt_create: invalid bvh_builder");
    if (opt.kernel != PT_KERNEL_MEGA && opt.kernel != PT_KERNEL_WAVEFRONT && opt.kernel != PT_KERNEL_AUTO)
        return fail(PT_ERR_INVALID, "pt_create: invalid kernel");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev <= 0) return fail(PT_ERR_HIP, "pt_create: no HIP device available");
    if (opt.device < 0 || opt.device >= ndev) return fail(PT_ERR_INVALID, "pt_create: device out of range");
    for (size_t g = 0; g < devlist.size(); ++g) {
        if (devlist[g] < 0 || devlist[g] >= ndev) return fail(PT_ERR_INVALID, "pt_create: device_list entry out of range");
        for (size_t h = 0; h < g; ++h)
            if (devlist[h] == devlist[g]) return fail(PT_ERR_INVALID, "pt_create: device_list repeats a device");
    }
    PT_HIP(hipSetDevice(opt.device), "hipSetDevice");

    // ---- host: world-space triangle soup in original (mesh-concatenated) order ----
    size_t ntri = 0;
    for (int m = 0; m < scene->n_meshes; ++m) {
        const pt_mesh& me = scene->meshes[m];
        if (me.n_triangles < 0 || me.n_vertices < 0) return fail(PT_ERR_INVALID, "pt_create: negative counts");
        if (me.n_triangles > 0 && (!me.vertices || !me.indices))
            return fail(PT_ERR_INVALID, "pt_create: mesh without vertices/indices");
        ntri += (size_t)me.n_triangles;
    }
    if (ntri > (size_t)0x3fffffff) return fail(PT_ERR_INVALID, "pt_create: too many triangles");
    // textures (CreateTextures, OptixRenderer.cpp:562-612): one RGBA8 texel pool + (offset, w, h)
    const int ntex = scene->n_textures;
    if (ntex < 0 || (ntex > 0 && !scene->textures)) return fail(PT_ERR_INVALID, "pt_create: invalid textures");
    std::vector<int4> texinfo((size_t)std::max(1, ntex));
    size_t ntexel = 0;
    for (int k = 0; k < ntex; ++k) {
        const pt_texture& tx = scene->textures[k];
        if (tx.width <= 0 || tx.height <= 0 || !tx.rgba8) return fail(PT_ERR_INVALID, "pt_create: invalid texture");
        texinfo[(size_t)k] = make_int4((int)ntexel, tx.width, tx.height, 0);
        ntexel += (size_t)tx.width * (size_t)tx.height;
    }
    if (ntexel > (size_t)0x7fffffff) return fail(PT_ERR_INVALID, "pt_create: textures too large");
    bool any_tex = false;
    for (int m = 0; m < scene->n_meshes; ++m) {
        const pt_mesh& me = scene->meshes[m];
        for (int id : {me.albedo_tex, me.normal_tex, me.metal_rough_tex}) {
            if (id < -1 || id >= ntex) return fail(PT_ERR_INVALID, "pt_create: texture id out of range");
            any_tex = any_tex || id >= 0;
        }
    }
    std::vector<float4> tri(3 * ntri), nrm(3 * ntri), uvs(any_tex ? 2 * ntri : 0);
    std::vector<float4> mats((size_t)kMatStride * (size_t)std::max(1, scene->n_meshes));
    float cmin[3] = {INFINITY, INFINITY, INFINITY}, cmax[3] = {-INFINITY, -INFINITY, -INFINITY};
    size_t t = 0;
    for (int m = 0; m < scene->n_meshes; ++m) {
        const pt_mesh& me = scene->meshes[m];
        auto ibits = [](int v) {
            float f;
            std::memcpy(&f, &v, 4);
            return f;
        };
        const bool textured = me.albedo_tex >= 0 || me.normal_tex >= 0 || me.metal_rough_tex >= 0;
        mats[kMatStride * m] = make_float4(me.albedo[0], me.albedo[1], me.albedo[2], me.metallic);
        mats[kMatStride * m + 1] =
            make_float4(me.roughness, me.normals ? 1.0f : 0.0f, ibits(me.albedo_tex), ibits(me.normal_tex));
        mats[kMatStride * m + 2] = make_float4(ibits(me.metal_rough_tex), textured ? 1.0f : 0.0f, 0.0f, 0.0f);
        // world-space vertices (modelMatrix * vec4(v,1)); normals pre-transformed with w = 0
        std::vector<float> wv(3 * (size_t)me.n_vertices), wn(3 * (size_t)me.n_vertices, 0.0f);
        for (int v = 0; v < me.n_vertices; ++v) {
            float in4[4] = {me.vertices[3 * v], me.vertices[3 * v + 1], me.vertices[3 * v + 2], 1.0f}, o4[4];
            xform4(me.model_matrix, in4, o4);
            wv[3 * v] = o4[0];
            wv[3 * v + 1] = o4[1];
            wv[3 * v + 2] = o4[2];
            if (me.normals) {
                float n4[4] = {me.normals[3 * v], me.normals[3 * v + 1], me.normals[3 * v + 2], 0.0f};
                xform4(me.model_matrix, n4, o4);
                wn[3 * v] = o4[0];
                wn[3 * v + 1] = o4[1];
                wn[3 * v + 2] = o4[2];
            }
        }
        for (int i = 0; i < me.n_triangles; ++i, ++t) {
            float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
            float uv[6] = {0, 0, 0, 0, 0, 0};  // Mesh::texCoord, zeros when absent (Mesh.cpp:50-53)
            for (int k = 0; k < 3; ++k) {
                int vi = me.indices[3 * i + k];
                if (vi < 0 || vi >= me.n_vertices) return fail(PT_ERR_INVALID, "pt_create: index out of range");
                if (me.texcoords) {
                    uv[2 * k] = me.texcoords[2 * vi];
                    uv[2 * k + 1] = me.texcoords[2 * vi + 1];
                }
                float wbits;
                // w tags: v0 = original triangle index, v1 = mesh, v2 = alpha cut-out flag
                int tag = (k == 0) ? (int)t : (k == 1 ? m : (me.albedo_tex >= 0 ? 1 : 0));
                std::memcpy(&wbits, &tag, 4);
                tri[3 * t + k] = make_float4(wv[3 * vi], wv[3 * vi + 1], wv[3 * vi + 2], wbits);
                nrm[3 * t + k] = make_float4(wn[3 * vi], wn[3 * vi + 1], wn[3 * vi + 2], 0.0f);
                for (int a = 0; a < 3; ++a) {
                    lo[a] = std::min(lo[a], wv[3 * vi + a]);
                    hi[a] = std::max(hi[a], wv[3 * vi + a]);
                }
            }
            for (int a = 0; a < 3; ++a) {
                float c = 0.5f * (lo[a] + hi[a]);
                cmin[a] = std::min(cmin[a], c);
                cmax[a] = std::max(cmax[a], c);
            }
            if (any_tex) {
                uvs[2 * t] = make_float4(uv[0], uv[1], uv[2], uv[3]);
                uvs[2 * t + 1] = make_float4(uv[4], uv[5], 0.0f, 0.0f);
            }
        }
    }

    pt_renderer* r = new pt_renderer();
    // A/B switch for the wide trace workgroups (tools/ab.sh runs one library with and without)
    if (const char* e = std::getenv("PTAMD_WIDE_TRACE")) r->wide_trace = std::atoi(e) != 0;
    r->device = opt.device;
    r->material_mode = opt.material_mode;
    r->kernel = opt.kernel;
    r->ntri = (int)ntri;
    r->nmesh = scene->n_meshes;
    auto cleanup_fail = [&](int code) {
        pt_destroy(r);
        return code;
    };
#define PT_HIPC(call, where)                                         \
    do {                                                             \
        hipError_t e__ = (call);                                     \
        if (e__ != hipSuccess) return cleanup_fail(hip_fail(e__, where)); \
    } while (0)
    PT_HIPC(hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking), "hipStreamCreate");
    // The download stream and the second wavefront stream right after the library stream: HIP
    // spreads streams over GPU_MAX_HW_QUEUES (4) hardware queues in creation order, and two streams
    // that land on one queue run in sequence.  Created lazily (first pt_render, first two-batch
    // render) they could share a queue with r->stream after other streams had been created in
    // between; then a pt_render download waited for the look-ahead batch behind it on that queue.
    PT_HIPC(hipStreamCreateWithFlags(&r->dl_stream, hipStreamNonBlocking), "hipStreamCreate");
    PT_HIPC(hipStreamCreateWithFlags(&r->xstream[1], hipStreamNonBlocking), "hipStreamCreate");
    PT_HIPC(hipEventCreateWithFlags(&r->ev_join[1], hipEventDisableTiming), "hipEventCreate");
    PT_HIPC(hipMalloc(&r->d_counters, kCounters * sizeof(unsigned long long)), "hipMalloc counters");
    PT_HIPC(hipMemsetAsync(r->d_counters, 0, kCounters * sizeof(unsigned long long), r->stream), "hipMemset");
    PT_HIPC(hipMalloc(&r->d_mats, sizeof(float4) * mats.size()), "hipMalloc mats");
    PT_HIPC(hipMemcpyAsync(r->d_mats, mats.data(), sizeof(float4) * mats.size(), hipMemcpyHostToDevice, r->stream),
            "upload mats");
    if (ntex > 0) {
        PT_HIPC(hipMalloc(&r->d_texinfo, sizeof(int4) * (size_t)ntex), "hipMalloc texinfo");
        PT_HIPC(hipMemcpyAsync(r->d_texinfo, texinfo.data(), sizeof(int4) * (size_t)ntex, hipMemcpyHostToDevice,
                               r->stream),
                "upload texinfo");
        PT_HIPC(hipMalloc(&r->d_texels, sizeof(uint32_t) * ntexel), "hipMalloc texels");
        for (int k = 0; k < ntex; ++k) {
            const pt_texture& tx = scene->textures[k];
            PT_HIPC(hipMemcpy(r->d_texels + texinfo[(size_t)k].x, tx.rgba8,
                              sizeof(uint32_t) * (size_t)tx.width * (size_t)tx.height, hipMemcpyHostToDevice),
                    "upload texels");
        }
    }
    if (ntri > 0) {
        float4 *d_tri_orig = nullptr, *d_nrm_orig = nullptr, *d_uv_orig = nullptr;
        if (any_tex) {
            PT_HIPC(hipMalloc(&r->d_tuv, sizeof(float4) * 2 * ntri), "hipMalloc tuv");
            PT_HIPC(hipMalloc(&d_uv_orig, sizeof(float4) * 2 * ntri), "hipMalloc uv_orig");
            PT_HIPC(hipMemcpyAsync(d_uv_orig, uvs.data(), sizeof(float4) * 2 * ntri, hipMemcpyHostToDevice,
                                   r->stream),
                    "upload uv");
        }
        PT_HIPC(hipMalloc(&r->d_isect, sizeof(float4) * 3 * ntri), "hipMalloc isect");
        PT_HIPC(hipMalloc(&r->d_shade, sizeof(float4) * 4 * ntri), "hipMalloc shade");
        PT_HIPC(hipMalloc(&r->d_nodes, sizeof(BNode4) * std::max<size_t>(1, ntri)), "hipMalloc nodes");
        PT_HIPC(hipMalloc(&d_tri_orig, sizeof(float4) * 3 * ntri), "hipMalloc tri_orig");
        PT_HIPC(hipMalloc(&d_nrm_orig, sizeof(float4) * 3 * ntri), "hipMalloc nrm_orig");
        PT_HIPC(hipMemcpyAsync(d_tri_orig, tri.data(), sizeof(float4) * 3 * ntri, hipMemcpyHostToDevice, r->stream),
                "upload tri");
        PT_HIPC(hipMemcpyAsync(d_nrm_orig, nrm.data(), sizeof(float4) * 3 * ntri, hipMemcpyHostToDevice, r->stream),
                "upload nrm");
        BuildInput in;
        in.tri_orig = d_tri_orig;
        in.nrm_orig = d_nrm_orig;
        in.uv_orig = d_uv_orig;
        in.n = (int)ntri;
        // AUTO: the binned-SAH tree (fewest node visits of the builders), built on the
        // GPU; every peer of a multi-device renderer builds its own on its own device
        in.builder = opt.bvh_builder == PT_BVH_LBVH   ? kBuilderLBVH
                     : opt.bvh_builder == PT_BVH_PLOC ? kBuilderPLOC
                     : opt.bvh_builder == PT_BVH_SAH  ? kBuilderSAH
                                                      : kBuilderSAHGPU;
        in.tri_host = tri.data();
        for (int a = 0; a < 3; ++a) {
            in.cmin[a] = cmin[a];
            in.cmax[a] = cmax[a];
        }
        BuildOutput bo;
        bo.nodes = r->d_nodes;
        bo.isect = r->d_isect;
        bo.shade = r->d_shade;
        bo.tuv = r->d_tuv;
        float ms = 0.0f;
        hipError_t be = lbvh_build(in, bo, r->stream, &ms);
        (void)hipStreamSynchronize(r->stream);
        (void)hipFree(d_tri_orig);
        (void)hipFree(d_nrm_orig);
        if (d_uv_orig) (void)hipFree(d_uv_orig);
        if (be != hipSuccess) return cleanup_fail(hip_fail(be, "lbvh_build"));
        r->bvh_ms = ms;
        r->bvh_nodes = bo.n_nodes;
        r->bvh_depth = bo.depth;
        // a traversal holds at most 3 stack entries per BVH4 level; the smallest traversal stack
        // (kMinTraversalStack) must hold them, or rays could lose subtrees
        if (3 * bo.depth > kMinTraversalStack)
            return cleanup_fail(fail(PT_ERR_INVALID, "pt_create: BVH too deep for the traversal stack (depth " +
                                                         std::to_string(bo.depth) + ")"));
    }
    PT_HIPC(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
#undef PT_HIPC
    if (!devlist.empty()) {
        // one single-device renderer per further device (own stream, scene copy, BVH build --
        // the build is deterministic, so every device traces the same BVH), and one RCCL
        // communicator over the list (ncclCommInitAll: a clique in this process)
        for (size_t g = 1; g < devlist.size(); ++g) {
            pt_options po = opt;
            po.device = devlist[g];
            po.n_devices = 0;
            po.device_list = nullptr;
            pt_renderer* p = nullptr;
            int rc = pt_create(scene, &po, &p);
            if (rc) {
                const std::string msg = g_last_error;
                pt_destroy(r);
                return fail(rc, "pt_create (device " + std::to_string(devlist[g]) + "): " + msg);
            }
            r->peers.push_back(p);
        }
        r->comms.assign(devlist.size(), nullptr);
        const ncclResult_t nr = ncclCommInitAll(r->comms.data(), (int)devlist.size(), devlist.data());
        if (nr != ncclSuccess) {
            r->comms.clear();
            pt_destroy(r);
            return fail(PT_ERR_HIP, std::string("pt_create: ncclCommInitAll: ") + ncclGetErrorString(nr));
        }
        (void)hipSetDevice(r->device);
    }
    *out = r;
    return PT_OK;
}

int pt_destroy(pt_renderer* r) {
    if (!r) return PT_OK;
    if (r->h_hold_release) __atomic_store_n(r->h_hold_release, 1u, __ATOMIC_SEQ_CST);  // a held batch ends now
    for (pt_renderer* p : r->peers) (void)hipSetDevice(p->device), (void)hipStreamSynchronize(p->stream);
    (void)hipSetDevice(r->device);
    if (r->stream) (void)hipStreamSynchronize(r->stream);
    for (ncclComm_t c : r->comms)
        if (c) (void)ncclCommDestroy(c);
    for (pt_renderer* p : r->peers) pt_destroy(p);
    (void)hipSetDevice(r->device);
    if (r->d_part) (void)hipFree(r->d_part);
    if (r->d_part64) (void)hipFree(r->d_part64);
    if (r->d_accum64) (void)hipFree(r->d_accum64);
    (void)hipSetDevice(r->device);
    if (r->d_nodes) (void)hipFree(r->d_nodes);
    if (r->d_isect) (void)hipFree(r->d_isect);
    if (r->d_shade) (void)hipFree(r->d_shade);
    if (r->d_mats) (void)hipFree(r->d_mats);
    if (r->d_tuv) (void)hipFree(r->d_tuv);
    if (r->d_texels) (void)hipFree(r->d_texels);
    if (r->d_texinfo) (void)hipFree(r->d_texinfo);
    if (r->d_lights) (void)hipFree(r->d_lights);
    if (r->d_frame) (void)hipFree(r->d_frame);
    ring_free(r);
    if (r->d_accum) (void)hipFree(r->d_accum);
    if (r->d_display) (void)hipFree(r->d_display);
    if (r->d_counters) (void)hipFree(r->d_counters);
    if (r->d_debug) (void)hipFree(r->d_debug);
    if (r->d_cancel_seen) (void)hipFree(r->d_cancel_seen);
    if (r->h_cancel) (void)hipHostFree(r->h_cancel);
    if (r->h_hold_release) (void)hipHostFree(r->h_hold_release);
    wavefront_free(r->wf);
    for (int k = 1; k < pt_renderer::kMaxWFStreams; ++k) {
        wavefront_free(r->xwf[k]);
        if (r->xstream[k]) (void)hipStreamDestroy(r->xstream[k]);
        if (r->ev_join[k]) (void)hipEventDestroy(r->ev_join[k]);
    }
    for (hipEvent_t e : {r->ev_fork, r->ev_accum[0], r->ev_accum[1], r->ev_band0, r->ring[0].ready, r->ring[1].ready,
                         r->ring[0].start, r->ring[1].start, r->ev_frame})
        if (e) (void)hipEventDestroy(e);
    if (r->dl_stream) (void)hipStreamDestroy(r->dl_stream);
    r->ev.destroy();
    r->tev.destroy();
    r->pev.destroy();
    r->sev.destroy();
    if (r->stream) (void)hipStreamDestroy(r->stream);
    delete r;
    return PT_OK;
}

int pt_resize(pt_renderer* r, int32_t width, int32_t height) {
    if (!r) return fail(PT_ERR_INVALID, "pt_resize: NULL renderer");
    if (width < 0 || height < 0) return fail(PT_ERR_INVALID, "pt_resize: negative size");
    if (width == 0 || height == 0) return PT_OK;  // minimised window: no-op (OptixRenderer.cpp:651)
    for (pt_renderer* p : r->peers) {
        const int rc = pt_resize(p, width, height);
        if (rc) return rc;
    }
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    cancel_look_ahead(r, true);  // the wait below must not sit behind speculative frames
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    size_t bytes = sizeof(float) * 3 * (size_t)width * (size_t)height;
    if (r->d_frame) (void)hipFree(r->d_frame);
    ring_free(r);
    if (r->d_accum) (void)hipFree(r->d_accum);
    if (r->d_display) (void)hipFree(r->d_display);
    if (r->d_part) (void)hipFree(r->d_part);
    if (r->d_accum64) (void)hipFree(r->d_accum64);
    if (r->d_part64) (void)hipFree(r->d_part64);
    r->d_frame = r->d_accum = r->d_display = r->d_part = nullptr;
    r->d_accum64 = r->d_part64 = nullptr;
    r->display_ready = false;
    // the size is committed only once every buffer exists (a failed allocation leaves an
    // unsized renderer, on which the render calls return PT_ERR_STATE)
    r->width = r->height = 0;
    r->user_accum = nullptr;
    r->nf_fit = 0;  // a new size: the queues may fit the full batch again
    PT_HIP(hipMalloc(&r->d_frame, bytes), "hipMalloc frame");
    PT_HIP(hipMalloc(&r->d_accum, bytes), "hipMalloc accum");
    PT_HIP(hipMemsetAsync(r->d_accum, 0, bytes, r->stream), "hipMemset accum");
    if (!r->comms.empty()) {
        PT_HIP(hipMalloc(&r->d_part, bytes), "hipMalloc partial sum");
        PT_HIP(hipMemsetAsync(r->d_part, 0, bytes, r->stream), "hipMemset partial sum");
    }
    if (r->accum64) {
        const int rc = alloc_accum64(r, width, height);
        if (rc) return rc;
    }
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    r->width = width;
    r->height = height;
    return PT_OK;
}

int pt_set_camera(pt_renderer* r, const float position[3], const float inverse_view[16],
                  const float inverse_projection[16]) {
    if (!r || !position || !inverse_view || !inverse_projection) return fail(PT_ERR_INVALID, "pt_set_camera: NULL");
    std::memcpy(r->cam_pos, position, sizeof r->cam_pos);
    std::memcpy(r->inv_view, inverse_view, sizeof r->inv_view);
    std::memcpy(r->inv_proj, inverse_projection, sizeof r->inv_proj);
    for (pt_renderer* p : r->peers) (void)pt_set_camera(p, position, inverse_view, inverse_projection);
    cancel_look_ahead(r);  // a moved camera: the look-ahead frames in flight are stale
    return PT_OK;
}

int pt_set_lights(pt_renderer* r, const pt_point_light* lights, int32_t count) {
    if (!r || count < 0 || (count > 0 && !lights)) return fail(PT_ERR_INVALID, "pt_set_lights: invalid");
    for (pt_renderer* p : r->peers) {
        const int rc = pt_set_lights(p, lights, count);
        if (rc) return rc;
    }
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    cancel_look_ahead(r, true);  // new lights: the upload below must not wait behind speculative frames
    if (count > r->lights_cap) {
        PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
        if (r->d_lights) (void)hipFree(r->d_lights);
        // no lights until the new array exists (a failed allocation must not leave a stale
        // count over a NULL array)
        r->d_lights = nullptr;
        r->n_lights = 0;
        r->lights_cap = 0;
        PT_HIP(hipMalloc(&r->d_lights, sizeof(DevLight) * (size_t)count), "hipMalloc lights");
        r->lights_cap = count;
    }
    if (count > 0) {
        std::vector<DevLight> h((size_t)count);
        for (int i = 0; i < count; ++i)
            h[i] = DevLight{lights[i].position[0], lights[i].position[1], lights[i].position[2],
                            lights[i].color[0],    lights[i].color[1],    lights[i].color[2]};
        PT_HIP(hipMemcpyAsync(r->d_lights, h.data(), sizeof(DevLight) * (size_t)count, hipMemcpyHostToDevice,
                              r->stream),
               "upload lights");
        PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    }
    r->n_lights = count;
    r->lights_version++;  // new contents, possibly in the same array: the render-ahead ring is stale
    return PT_OK;
}

int pt_set_max_bounces(pt_renderer* r, int32_t max_bounces) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_max_bounces: NULL");
    // SetMaxBounces (OptixRenderer.cpp:677-679) takes any int; a negative count would never
    // enter SamplePath's loop, like 0, so it is rejected here rather than silently renamed
    if (max_bounces < 0) return fail(PT_ERR_INVALID, "pt_set_max_bounces: negative count");
    r->max_bounces = max_bounces;
    for (pt_renderer* p : r->peers) p->max_bounces = max_bounces;
    cancel_look_ahead(r);
    return PT_OK;
}

int pt_set_material_mode(pt_renderer* r, int32_t mode) {
    if (!r || !valid_mode(mode)) return fail(PT_ERR_INVALID, "pt_set_material_mode: invalid");
    r->material_mode = mode;
    for (pt_renderer* p : r->peers) p->material_mode = mode;
    cancel_look_ahead(r);
    return PT_OK;
}

int pt_set_kernel(pt_renderer* r, int32_t kernel) {
    if (!r || (kernel != PT_KERNEL_MEGA && kernel != PT_KERNEL_WAVEFRONT && kernel != PT_KERNEL_AUTO))
        return fail(PT_ERR_INVALID, "pt_set_kernel: invalid");
    r->kernel = kernel;
    for (pt_renderer* p : r->peers) p->kernel = kernel;
    cancel_look_ahead(r);
    return PT_OK;
}

int pt_render(pt_renderer* r, float* host_rgb) {
    if (!r) return fail(PT_ERR_INVALID, "pt_render: NULL renderer");
    if (r->width == 0) return PT_OK;  // OptixRenderer.cpp:621
    if (!host_rgb) return fail(PT_ERR_INVALID, "pt_render: NULL output");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    r->frame_id++;  // :623
    size_t bytes = sizeof(float) * 3 * (size_t)r->width * (size_t)r->height;
    const float* img = nullptr;
    hipEvent_t ready = nullptr, part = nullptr;
    size_t part_floats = 0;
    int rc = render_frame_image(r, &img, &ready, true, &part, &part_floats);
    if (rc) return rc;
    // the download runs on its own stream after the image's event, so a look-ahead batch that
    // render_frame_image enqueued on r->stream keeps rendering while this frame is copied
    if (!r->dl_stream) PT_HIP(hipStreamCreateWithFlags(&r->dl_stream, hipStreamNonBlocking), "hipStreamCreate");
    if (part) {  // a banded frame: its first band's rows while the second band renders
        PT_HIP(hipStreamWaitEvent(r->dl_stream, part, 0), "hipStreamWaitEvent");
        PT_HIP(hipMemcpyAsync(host_rgb, img, sizeof(float) * part_floats, hipMemcpyDeviceToHost, r->dl_stream),
               "download frame");
        host_rgb += part_floats;
        img += part_floats;
        bytes -= sizeof(float) * part_floats;
    }
    PT_HIP(hipStreamWaitEvent(r->dl_stream, ready, 0), "hipStreamWaitEvent");
    PT_HIP(hipMemcpyAsync(host_rgb, img, bytes, hipMemcpyDeviceToHost, r->dl_stream), "download frame");
    PT_HIP(hipStreamSynchronize(r->dl_stream), "hipStreamSynchronize");
    // with a look-ahead batch in flight the launch events are retired later (pt_get_stats, a
    // synchronising call, or launch_frames' kMaxPendingEvents bound), not by waiting for it here
    return r->spec_pending ? PT_OK : collect_pending(r);
}

int pt_launch(pt_renderer* r, const pt_launch_params* lp) {
    static_assert(sizeof(pt_point_light) == sizeof(DevLight), "pt_point_light is read as DevLight on the device");
    if (!r || !lp) return fail(PT_ERR_INVALID, "pt_launch: NULL");
    const int w = lp->frame.size[0], h = lp->frame.size[1];
    if (w < 0 || h < 0 || lp->point_light_count < 0 || lp->max_bounces < 0)
        return fail(PT_ERR_INVALID, "pt_launch: negative size, light count or max bounces");
    if (w == 0 || h == 0) return PT_OK;  // an empty launch grid
    if (!lp->frame.color_buffer || (lp->point_light_count > 0 && !lp->point_lights))
        return fail(PT_ERR_INVALID, "pt_launch: NULL color buffer or lights");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    // this launch's state replaces the renderer's for the duration of the enqueue only
    const int ow = r->width, oh = r->height, on = r->n_lights, ob = r->max_bounces;
    float opos[3], oview[16], oproj[16];
    std::memcpy(opos, r->cam_pos, sizeof opos);
    std::memcpy(oview, r->inv_view, sizeof oview);
    std::memcpy(oproj, r->inv_proj, sizeof oproj);
    DevLight* olights = r->d_lights;
    r->width = w;
    r->height = h;
    std::memcpy(r->cam_pos, lp->camera.position, sizeof r->cam_pos);
    std::memcpy(r->inv_view, lp->camera.inverse_view_matrix, sizeof r->inv_view);
    std::memcpy(r->inv_proj, lp->camera.inverse_projection_matrix, sizeof r->inv_proj);
    r->d_lights = reinterpret_cast<DevLight*>(const_cast<pt_point_light*>(lp->point_lights));
    r->n_lights = lp->point_light_count;
    r->max_bounces = lp->max_bounces;
    // colorBuffer[fbIndex] = pathRadiance (devicePrograms.cu:705): a one-frame sum into zeros
    hipError_t e = hipMemsetAsync(lp->frame.color_buffer, 0, sizeof(float) * 3 * (size_t)w * (size_t)h, r->stream);
    int rc = e == hipSuccess ? launch_frames(r, lp->frame.color_buffer, lp->frame.id, 1)
                             : fail(PT_ERR_HIP, std::string("pt_launch: hipMemsetAsync: ") + hipGetErrorString(e));
    r->width = ow;
    r->height = oh;
    std::memcpy(r->cam_pos, opos, sizeof opos);
    std::memcpy(r->inv_view, oview, sizeof oview);
    std::memcpy(r->inv_proj, oproj, sizeof oproj);
    r->d_lights = olights;
    r->n_lights = on;
    r->max_bounces = ob;
    return rc;
}

int pt_display_reset(pt_renderer* r, int32_t max_samples) {
    if (!r) return fail(PT_ERR_INVALID, "pt_display_reset: NULL");
    if (r->width == 0) return fail(PT_ERR_STATE, "pt_display_reset: call pt_resize first");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    const size_t n = 3 * (size_t)r->width * (size_t)r->height;
    if (!r->d_display) PT_HIP(hipMalloc(&r->d_display, sizeof(float) * n), "hipMalloc display");
    PT_HIP(display_fill(r->d_display, n, 1.0f, r->stream), "display clear");  // glClearColor(1,1,1,1)
    r->display_max = max_samples;
    r->display_samples = 0;
    r->display_ready = true;
    return PT_OK;
}

int pt_display_add_frame(pt_renderer* r, int32_t* samples) {
    if (!r) return fail(PT_ERR_INVALID, "pt_display_add_frame: NULL");
    if (!r->display_ready) return fail(PT_ERR_STATE, "pt_display_add_frame: call pt_display_reset first");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    r->frame_id++;  // Render: OptixRenderer.cpp:623
    const size_t n = 3 * (size_t)r->width * (size_t)r->height;
    const float* img = nullptr;
    int rc = render_frame_image(r, &img);
    if (rc) return rc;
    r->display_samples++;  // OptixView.cpp:239-248
    const bool continuous = r->display_max < 0;
    const float w = continuous ? 1.0f / (float)r->display_samples : 1.0f / (float)r->display_max;
    PT_HIP(display_blend(r->d_display, img, n, w, continuous, r->stream), "display blend");
    if (samples) *samples = r->display_samples;
    return PT_OK;
}

int pt_display_download(pt_renderer* r, float* host_rgb) {
    if (!r || !host_rgb) return fail(PT_ERR_INVALID, "pt_display_download: NULL");
    if (!r->display_ready) return fail(PT_ERR_STATE, "pt_display_download: call pt_display_reset first");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    const size_t bytes = sizeof(float) * 3 * (size_t)r->width * (size_t)r->height;
    PT_HIP(hipMemcpyAsync(host_rgb, r->d_display, bytes, hipMemcpyDeviceToHost, r->stream), "download display");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    return collect_pending(r);
}

int pt_accum_clear(pt_renderer* r) {
    if (!r) return fail(PT_ERR_INVALID, "pt_accum_clear: NULL");
    if (r->width == 0) return fail(PT_ERR_STATE, "pt_accum_clear: call pt_resize first");
    for (pt_renderer* p : r->peers) {
        const int rc = pt_accum_clear(p);
        if (rc) return rc;
    }
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    size_t bytes = sizeof(float) * 3 * (size_t)r->width * (size_t)r->height;
    PT_HIP(hipMemsetAsync(r->accum(), 0, bytes, r->stream), "hipMemset accum");
    if (r->d_part) PT_HIP(hipMemsetAsync(r->d_part, 0, bytes, r->stream), "hipMemset partial sum");
    if (r->d_accum64) PT_HIP(hipMemsetAsync(r->d_accum64, 0, 2 * bytes, r->stream), "hipMemset fp64 accum");
    if (r->d_part64) PT_HIP(hipMemsetAsync(r->d_part64, 0, 2 * bytes, r->stream), "hipMemset fp64 partial sum");
    return PT_OK;
}

int pt_render_frames(pt_renderer* r, uint32_t first_frame_id, uint32_t n_frames) {
    if (!r) return fail(PT_ERR_INVALID, "pt_render_frames: NULL");
    if (r->width == 0) return fail(PT_ERR_STATE, "pt_render_frames: call pt_resize first");
    if (n_frames == 0) return PT_OK;
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    if (r->comms.empty())
        return launch_frames(r, r->accum(), first_frame_id, n_frames, r->accum64 ? r->d_accum64 : nullptr);
    return render_frames_multi(r, first_frame_id, n_frames);
}

int pt_render_accumulate(pt_renderer* r, uint32_t spp, uint32_t first_frame_id, float* host_rgb_mean) {
    if (!r) return fail(PT_ERR_INVALID, "pt_render_accumulate: NULL");
    if (r->width == 0) return fail(PT_ERR_STATE, "pt_render_accumulate: call pt_resize first");
    if (spp == 0) return fail(PT_ERR_INVALID, "pt_render_accumulate: spp must be > 0");
    int rc = pt_accum_clear(r);
    if (rc) return rc;
    rc = pt_render_frames(r, first_frame_id, spp);
    if (rc) return rc;
    if (host_rgb_mean) return pt_accum_download(r, host_rgb_mean, 1.0f / (float)spp);
    return pt_synchronize(r);
}

int pt_set_accum_device_buffer(pt_renderer* r, float* device_sum_rgb) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_accum_device_buffer: NULL");
    r->user_accum = device_sum_rgb;
    return PT_OK;
}

float* pt_accum_device_ptr(pt_renderer* r) { return r ? r->accum() : nullptr; }

int pt_set_accum_fp64(pt_renderer* r, int32_t on) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_accum_fp64: NULL");
    for (pt_renderer* p : r->peers) {
        const int rc = pt_set_accum_fp64(p, on);
        if (rc) return rc;
    }
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    r->accum64 = on != 0;
    if (r->accum64 && r->width > 0) {
        // start from the current fp32 sum (device 0 of a multi-device renderer: its own partial
        // sum, which the next reduce adds to the others'), so a switch keeps what is there
        const int rc = alloc_accum64(r, r->width, r->height);
        if (rc) return rc;
        const size_t n = 3 * (size_t)r->width * (size_t)r->height;
        std::vector<float> h32(n);
        std::vector<double> h64(n);
        const float* src = r->comms.empty() ? r->accum() : r->d_part;
        double* dst = r->comms.empty() ? r->d_accum64 : r->d_part64;
        // on the library stream, after alloc_accum64's zeroing: a null-stream hipMemcpy would not
        // wait for the non-blocking stream, and the memset could land on the seeded sum
        PT_HIP(hipMemcpyAsync(h32.data(), src, n * sizeof(float), hipMemcpyDeviceToHost, r->stream), "download accum");
        PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
        for (size_t i = 0; i < n; ++i) h64[i] = (double)h32[i];
        PT_HIP(hipMemcpyAsync(dst, h64.data(), n * sizeof(double), hipMemcpyHostToDevice, r->stream),
               "upload fp64 accum");
        PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    } else if (!r->accum64) {
        if (r->d_accum64) (void)hipFree(r->d_accum64);
        if (r->d_part64) (void)hipFree(r->d_part64);
        r->d_accum64 = r->d_part64 = nullptr;
    }
    return PT_OK;
}

double* pt_accum_device_ptr64(pt_renderer* r) { return r ? r->d_accum64 : nullptr; }

int pt_accum_download64(pt_renderer* r, double* host_rgb) {
    if (!r || !host_rgb) return fail(PT_ERR_INVALID, "pt_accum_download64: NULL");
    if (r->width == 0) return fail(PT_ERR_STATE, "pt_accum_download64: call pt_resize first");
    if (!r->d_accum64) return fail(PT_ERR_STATE, "pt_accum_download64: fp64 accumulation is off (pt_set_accum_fp64)");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    size_t n = 3 * (size_t)r->width * (size_t)r->height;
    PT_HIP(hipMemcpyAsync(host_rgb, r->d_accum64, n * sizeof(double), hipMemcpyDeviceToHost, r->stream),
           "download fp64 accum");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    return collect_pending(r);
}

int pt_accum_download(pt_renderer* r, float* host_rgb, float scale) {
    if (!r || !host_rgb) return fail(PT_ERR_INVALID, "pt_accum_download: NULL");
    if (r->width == 0) return fail(PT_ERR_STATE, "pt_accum_download: call pt_resize first");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    size_t n = 3 * (size_t)r->width * (size_t)r->height;
    PT_HIP(hipMemcpyAsync(host_rgb, r->accum(), n * sizeof(float), hipMemcpyDeviceToHost, r->stream), "download accum");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    if (scale != 1.0f)
        for (size_t i = 0; i < n; ++i) host_rgb[i] *= scale;
    return collect_pending(r);
}

int pt_synchronize(pt_renderer* r) {
    if (!r) return fail(PT_ERR_INVALID, "pt_synchronize: NULL");
    for (pt_renderer* p : r->peers) {
        const int rc = pt_synchronize(p);
        if (rc) return rc;
    }
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    return collect_pending(r);
}

void* pt_stream(pt_renderer* r) { return r ? (void*)r->stream : nullptr; }
int32_t pt_device_count(const pt_renderer* r) { return r ? (int32_t)(1 + r->peers.size()) : 0; }
int pt_devices(const pt_renderer* r, int32_t* devices, int32_t max) {
    if (!r || max < 0 || (max > 0 && !devices)) return fail(PT_ERR_INVALID, "pt_devices: invalid");
    for (int32_t g = 0; g < max && g < pt_device_count(r); ++g) devices[g] = g == 0 ? r->device : r->peers[g - 1]->device;
    return PT_OK;
}
uint32_t pt_frame_id(const pt_renderer* r) { return r ? r->frame_id : 0u; }
int pt_set_frame_id(pt_renderer* r, uint32_t frame_id) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_frame_id: NULL");
    r->frame_id = frame_id;
    return PT_OK;
}

int pt_get_stats(pt_renderer* r, pt_stats* out) {
    if (!r || !out) return fail(PT_ERR_INVALID, "pt_get_stats: NULL");
    int rc = pt_synchronize(r);
    if (rc) return rc;
    unsigned long long c[kCounters];
    PT_HIP(hipMemcpy(c, r->d_counters, sizeof c, hipMemcpyDeviceToHost), "download counters");
    std::memset(out, 0, sizeof *out);
    out->segments = c[0];
    out->samples = r->samples;
    out->last_render_ms = r->last_ms;
    out->total_render_ms = r->total_ms;
    out->render_calls = r->calls;
    out->kernel_launches = r->launches;
    out->frames_per_launch = r->frames_per_launch;
    out->bvh_build_ms = r->bvh_ms;
    out->bvh_nodes = r->bvh_nodes;
    out->bvh_depth = r->bvh_depth;
    out->nodes_visited = c[1];
    out->tri_tests = c[2];
    out->rays = c[3];
    out->stack_overflows = c[4];
    out->triangles = r->ntri;
    out->trace_kernel_ms = r->trace_ms;
    out->trace_kernel_launches = r->trace_launches;
    out->pair_kernel_ms = r->pair_ms;
    out->pair_kernel_launches = r->pair_launches;
    out->shadow_rays = c[5];
    out->trace_kernel_rays = c[6];
    out->trace_kernel_bytes = c[7];
    out->strict_retraces = c[8];
    out->wave_steps = c[9];
    out->wave_active_lanes = c[10];
    out->wave_node_steps = c[11];
    out->wave_tri_steps = c[12];
    out->wave_refills = c[13];
    out->lds_nodes_visited = c[14];
    out->shade_kernel_ms = r->shade_ms;
    out->shade_kernel_launches = r->shade_launches;
    out->shade_kernel_items = c[15];
    out->frames_rendered_ahead = r->ahead_rendered;
    out->frames_served_ahead = r->ahead_served;
    out->look_ahead_cancelled = r->ahead_cancelled;
    out->pair_kernel_rays = c[16];
    out->pair_kernel_bytes = c[17];
    out->pair_kernel_shadow_rays = c[19];
    out->nee_unoccluded = c[18];
    out->queue_bytes = queue_bytes_held(r);
    const size_t qb = queue_budget_bytes(r);
    out->queue_budget = qb == SIZE_MAX ? 0 : qb;
    out->last_streams = r->last_streams;
    out->last_batch_frames = r->last_batch;
    out->look_ahead_held = r->ahead_held;
    // a multi-device renderer reports the work of all its devices (times are device 0's)
    for (pt_renderer* p : r->peers) {
        pt_stats ps;
        rc = pt_get_stats(p, &ps);
        if (rc) return rc;
        out->segments += ps.segments;
        out->samples += ps.samples;
        out->nodes_visited += ps.nodes_visited;
        out->tri_tests += ps.tri_tests;
        out->rays += ps.rays;
        out->stack_overflows += ps.stack_overflows;
        out->wave_steps += ps.wave_steps;
        out->wave_active_lanes += ps.wave_active_lanes;
        out->wave_node_steps += ps.wave_node_steps;
        out->wave_tri_steps += ps.wave_tri_steps;
        out->wave_refills += ps.wave_refills;
        out->lds_nodes_visited += ps.lds_nodes_visited;
        out->shade_kernel_items += ps.shade_kernel_items;
        out->shadow_rays += ps.shadow_rays;
        out->trace_kernel_rays += ps.trace_kernel_rays;
        out->trace_kernel_bytes += ps.trace_kernel_bytes;
        out->strict_retraces += ps.strict_retraces;
        out->nee_unoccluded += ps.nee_unoccluded;
        // the per-kernel ray and byte counts of every device, like trace_kernel_*
        out->pair_kernel_rays += ps.pair_kernel_rays;
        out->pair_kernel_bytes += ps.pair_kernel_bytes;
        out->pair_kernel_shadow_rays += ps.pair_kernel_shadow_rays;
        out->queue_bytes += ps.queue_bytes;
    }
    return PT_OK;
}

int pt_stats_reset(pt_renderer* r) {
    if (!r) return fail(PT_ERR_INVALID, "pt_stats_reset: NULL");
    int rc = pt_synchronize(r);
    if (rc) return rc;
    for (pt_renderer* p : r->peers) {
        if ((rc = pt_stats_reset(p)) != PT_OK) return rc;
    }
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    PT_HIP(hipMemset(r->d_counters, 0, kCounters * sizeof(unsigned long long)), "hipMemset counters");
    r->samples = 0;
    r->last_ms = r->total_ms = 0.0;
    r->calls = 0;
    r->launches = 0;
    r->trace_ms = 0.0;
    r->trace_launches = 0;
    r->pair_ms = 0.0;
    r->pair_launches = 0;
    r->shade_ms = 0.0;
    r->shade_launches = 0;
    r->ahead_rendered = r->ahead_served = 0;
    r->ahead_cancelled = 0;
    r->ahead_held = 0;
    return PT_OK;
}

int pt_set_render_ahead(pt_renderer* r, int32_t frames) {
    if (!r || frames < 1 || frames > 1024) return fail(PT_ERR_INVALID, "pt_set_render_ahead: frames must be 1..1024");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    ring_free(r);
    r->render_ahead = frames;
    return PT_OK;
}

int pt_set_render_ahead_budget(pt_renderer* r, float max_ms) {
    if (!r || !(max_ms >= 0.0f)) return fail(PT_ERR_INVALID, "pt_set_render_ahead_budget: max_ms must be >= 0");
    r->ahead_budget_ms = max_ms;
    return PT_OK;
}

int pt_set_frames_per_launch(pt_renderer* r, int32_t frames) {
    if (!r || frames < 1) return fail(PT_ERR_INVALID, "pt_set_frames_per_launch: invalid");
    r->frames_per_launch = frames;
    r->nf_fit = 0;
    for (pt_renderer* p : r->peers) {
        p->frames_per_launch = frames;
        p->nf_fit = 0;
    }
    return PT_OK;
}

int pt_get_trace_coherence(pt_renderer* r, uint64_t hist[8]) {
    if (!r || !hist) return fail(PT_ERR_INVALID, "pt_get_trace_coherence: NULL");
    int rc = pt_synchronize(r);
    if (rc) return rc;
    unsigned long long c[kCounters];
    PT_HIP(hipMemcpy(c, r->d_counters, sizeof c, hipMemcpyDeviceToHost), "download counters");
    uint64_t steps = 0;
    for (int k = 0; k < 6; ++k) {
        hist[k] = c[20 + k];
        steps += c[20 + k];
    }
    hist[6] = steps;
    hist[7] = c[26];
    for (pt_renderer* p : r->peers) {  // a multi-device renderer: every device's steps
        uint64_t ph[8];
        if ((rc = pt_get_trace_coherence(p, ph)) != PT_OK) return rc;
        for (int k = 0; k < 8; ++k) hist[k] += ph[k];
    }
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    return PT_OK;
}

int pt_set_queue_budget(pt_renderer* r, int64_t bytes) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_queue_budget: NULL");
    r->queue_budget = bytes;
    for (pt_renderer* p : r->peers) p->queue_budget = bytes;
    return PT_OK;
}

int pt_set_debug_hold(pt_renderer* r, int32_t on) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_debug_hold: NULL");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    if (!r->h_hold_release) {
        unsigned* h = nullptr;
        void* d = nullptr;
        PT_HIP(hipHostMalloc((void**)&h, sizeof(unsigned), hipHostMallocMapped | hipHostMallocCoherent),
               "hipHostMalloc hold word");
        *h = 1u;
        const hipError_t e = hipHostGetDevicePointer(&d, h, 0);
        if (e != hipSuccess) {
            (void)hipHostFree(h);
            return hip_fail(e, "hipHostGetDevicePointer hold word");
        }
        r->h_hold_release = h;
        r->d_hold_release = static_cast<unsigned*>(d);
    }
    // on: later speculative batches wait in k_hold; off: a batch waiting there goes on now
    __atomic_store_n(r->h_hold_release, on ? 0u : 1u, __ATOMIC_SEQ_CST);
    r->debug_hold = on != 0;
    return PT_OK;
}

int pt_camera_from_blender(const float bp[3], const float br[3], float fov_deg, int32_t W, int32_t H, float pos[3],
                           float inv_view[16], float inv_proj[16]) {
    if (!bp || !br || !pos || !inv_view || !inv_proj || W <= 0 || H <= 0)
        return fail(PT_ERR_INVALID, "pt_camera_from_blender: invalid");
    const float deg2rad = 0.01745329251994329576923690768489f;  // glm::radians
    f3 p = mk(bp[0], bp[2], -bp[1]);                             // GlmHelperMethods.cpp:4-6
    f3 rot = mk(90.0f - br[0], 180.0f + br[2], br[1]);           // GlmHelperMethods.cpp:8-10
    f3 rr = mk(rot.x * deg2rad, rot.y * deg2rad, rot.z * deg2rad);
    float x = sinf(rr.y);  // Camera::GetForward, Camera.cpp:37-49
    x *= cosf(rr.x);
    float y = -sinf(rr.x);
    float z = cosf(rr.x);
    z *= cosf(rr.y);
    f3 fwd = normalize(mk(x, y, z));
    // glm::lookAtRH(pos, pos + fwd, (0,1,0)) — Camera.cpp:64-66
    f3 center = p + fwd;
    f3 f = normalize(center - p);
    f3 s = normalize(cross(f, mk(0.0f, 1.0f, 0.0f)));
    f3 u = cross(s, f);
    float V[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    V[0] = s.x; V[4] = s.y; V[8] = s.z;
    V[1] = u.x; V[5] = u.y; V[9] = u.z;
    V[2] = -f.x; V[6] = -f.y; V[10] = -f.z;
    V[12] = -dot(s, p); V[13] = -dot(u, p); V[14] = dot(f, p);
    // glm::perspectiveRH_NO(fovy, aspect, 0.1, 100) — Camera.cpp:68-70, OptixRenderer.cpp:663
    float fovy = fov_deg * deg2rad;
    float aspect = (float)W / (float)H;
    const float zn = 0.1f, zf = 100.0f;
    float th = tanf(fovy / 2.0f);
    float P[16] = {0};
    P[0] = 1.0f / (aspect * th);
    P[5] = 1.0f / th;
    P[10] = -(zf + zn) / (zf - zn);
    P[11] = -1.0f;
    P[14] = -(2.0f * zf * zn) / (zf - zn);
    // glm::inverse (detail/func_matrix.inl compute_inverse<4,4>)
    auto inverse = [](const float* m, float* out) {
        auto M = [&](int c, int r) { return m[c * 4 + r]; };
        float C00 = M(2, 2) * M(3, 3) - M(3, 2) * M(2, 3), C02 = M(1, 2) * M(3, 3) - M(3, 2) * M(1, 3);
        float C03 = M(1, 2) * M(2, 3) - M(2, 2) * M(1, 3), C04 = M(2, 1) * M(3, 3) - M(3, 1) * M(2, 3);
        float C06 = M(1, 1) * M(3, 3) - M(3, 1) * M(1, 3), C07 = M(1, 1) * M(2, 3) - M(2, 1) * M(1, 3);
        float C08 = M(2, 1) * M(3, 2) - M(3, 1) * M(2, 2), C10 = M(1, 1) * M(3, 2) - M(3, 1) * M(1, 2);
        float C11 = M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2), C12 = M(2, 0) * M(3, 3) - M(3, 0) * M(2, 3);
        float C14 = M(1, 0) * M(3, 3) - M(3, 0) * M(1, 3), C15 = M(1, 0) * M(2, 3) - M(2, 0) * M(1, 3);
        float C16 = M(2, 0) * M(3, 2) - M(3, 0) * M(2, 2), C18 = M(1, 0) * M(3, 2) - M(3, 0) * M(1, 2);
        float C19 = M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2), C20 = M(2, 0) * M(3, 1) - M(3, 0) * M(2, 1);
        float C22 = M(1, 0) * M(3, 1) - M(3, 0) * M(1, 1), C23 = M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1);
        const float F0[4] = {C00, C00, C02, C03}, F1[4] = {C04, C04, C06, C07}, F2[4] = {C08, C08, C10, C11};
        const float F3[4] = {C12, C12, C14, C15}, F4[4] = {C16, C16, C18, C19}, F5[4] = {C20, C20, C22, C23};
        const float V0[4] = {M(1, 0), M(0, 0), M(0, 0), M(0, 0)}, V1[4] = {M(1, 1), M(0, 1), M(0, 1), M(0, 1)};
        const float V2[4] = {M(1, 2), M(0, 2), M(0, 2), M(0, 2)}, V3[4] = {M(1, 3), M(0, 3), M(0, 3), M(0, 3)};
        const float SA[4] = {+1, -1, +1, -1}, SB[4] = {-1, +1, -1, +1};
        float I0[4], I1[4], I2[4], I3[4];
        for (int i = 0; i < 4; ++i) {
            I0[i] = (V1[i] * F0[i] - V2[i] * F1[i] + V3[i] * F2[i]) * SA[i];
            I1[i] = (V0[i] * F0[i] - V2[i] * F3[i] + V3[i] * F4[i]) * SB[i];
            I2[i] = (V0[i] * F1[i] - V1[i] * F3[i] + V3[i] * F5[i]) * SA[i];
            I3[i] = (V0[i] * F2[i] - V1[i] * F4[i] + V2[i] * F5[i]) * SB[i];
        }
        float d0 = M(0, 0) * I0[0], d1 = M(0, 1) * I1[0], d2 = M(0, 2) * I2[0], d3 = M(0, 3) * I3[0];
        float one = 1.0f / ((d0 + d1) + (d2 + d3));
        for (int i = 0; i < 4; ++i) {
            out[i] = I0[i] * one;
            out[4 + i] = I1[i] * one;
            out[8 + i] = I2[i] * one;
            out[12 + i] = I3[i] * one;
        }
    };
    pos[0] = p.x;
    pos[1] = p.y;
    pos[2] = p.z;
    inverse(V, inv_view);
    inverse(P, inv_proj);
    return PT_OK;
}

int pt_trace_rays(pt_renderer* r, const float* host_rays, int32_t n, int32_t* prim, float* t, float* u, float* v,
                  int32_t* backface, int32_t any_hit) {
    if (!r || n < 0 || (n > 0 && (!host_rays || !prim || !t || !u || !v || !backface)))
        return fail(PT_ERR_INVALID, "pt_trace_rays: invalid");
    if (n == 0) return PT_OK;
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    float *d_rays = nullptr, *d_t = nullptr, *d_u = nullptr, *d_v = nullptr;
    int *d_p = nullptr, *d_b = nullptr;
    size_t nn = (size_t)n;
    hipError_t e = hipMalloc(&d_rays, 8 * nn * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_t, nn * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_u, nn * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_v, nn * sizeof(float));
    if (e == hipSuccess) e = hipMalloc(&d_p, nn * sizeof(int));
    if (e == hipSuccess) e = hipMalloc(&d_b, nn * sizeof(int));
    if (e == hipSuccess) e = hipMemcpyAsync(d_rays, host_rays, 8 * nn * sizeof(float), hipMemcpyHostToDevice, r->stream);
    if (e == hipSuccess) e = launch_trace(r->scene(), d_rays, n, d_p, d_t, d_u, d_v, d_b, any_hit, r->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(prim, d_p, nn * sizeof(int), hipMemcpyDeviceToHost, r->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(t, d_t, nn * sizeof(float), hipMemcpyDeviceToHost, r->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(u, d_u, nn * sizeof(float), hipMemcpyDeviceToHost, r->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(v, d_v, nn * sizeof(float), hipMemcpyDeviceToHost, r->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(backface, d_b, nn * sizeof(int), hipMemcpyDeviceToHost, r->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(r->stream);
    (void)hipFree(d_rays);
    (void)hipFree(d_t);
    (void)hipFree(d_u);
    (void)hipFree(d_v);
    (void)hipFree(d_p);
    (void)hipFree(d_b);
    if (e != hipSuccess) return hip_fail(e, "pt_trace_rays");
    return PT_OK;
}

}  // extern "C"

extern "C" int pt_bvh_download(pt_renderer* r, void* nodes, int64_t node_bytes, void* triangles,
                               int64_t triangle_bytes) {
    if (!r || node_bytes < 0 || triangle_bytes < 0 || (node_bytes > 0 && !nodes) ||
        (triangle_bytes > 0 && !triangles))
        return fail(PT_ERR_INVALID, "pt_bvh_download: invalid");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    const int64_t nb = std::min<int64_t>(node_bytes, (int64_t)sizeof(BNode4) * r->bvh_nodes);
    const int64_t tb = std::min<int64_t>(triangle_bytes, (int64_t)sizeof(float4) * 3 * r->ntri);
    if (nb > 0) PT_HIP(hipMemcpy(nodes, r->d_nodes, (size_t)nb, hipMemcpyDeviceToHost), "download nodes");
    if (tb > 0) PT_HIP(hipMemcpy(triangles, r->d_isect, (size_t)tb, hipMemcpyDeviceToHost), "download triangles");
    return PT_OK;
}

extern "C" int pt_set_debug_pixel(pt_renderer* r, int32_t x, int32_t y, uint32_t frame_id) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_debug_pixel: NULL");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    if (x < 0 || y < 0) {  // off
        r->debug_pixel = -1;
        return PT_OK;
    }
    if (r->width == 0 || x >= r->width || y >= r->height)
        return fail(PT_ERR_INVALID, "pt_set_debug_pixel: pixel outside the frame (call pt_resize first)");
    const size_t bytes = sizeof(float) * kDebugRecordFloats * kDebugMaxBounces;
    if (!r->d_debug) PT_HIP(hipMalloc(&r->d_debug, bytes), "hipMalloc debug records");
    PT_HIP(hipMemset(r->d_debug, 0, bytes), "hipMemset debug records");
    r->debug_pixel = r->width * y + x;
    r->debug_frame = frame_id;
    r->debug_version++;  // records cleared: no ring image rendered before stands for this state
    return PT_OK;
}

extern "C" int pt_get_debug_path(pt_renderer* r, pt_debug_bounce* out, int32_t max, int32_t* n_bounces) {
    static_assert(sizeof(pt_debug_bounce) == sizeof(float) * kDebugRecordFloats, "pt_debug_bounce layout");
    if (!r || max < 0 || (max > 0 && !out) || !n_bounces) return fail(PT_ERR_INVALID, "pt_get_debug_path: invalid");
    *n_bounces = 0;
    if (!r->d_debug) return fail(PT_ERR_STATE, "pt_get_debug_path: call pt_set_debug_pixel first");
    PT_HIP(hipSetDevice(r->device), "hipSetDevice");
    PT_HIP(hipStreamSynchronize(r->stream), "hipStreamSynchronize");
    std::vector<pt_debug_bounce> rec(kDebugMaxBounces);
    PT_HIP(hipMemcpy(rec.data(), r->d_debug, sizeof(pt_debug_bounce) * rec.size(), hipMemcpyDeviceToHost),
           "download debug records");
    int n = 0;
    while (n < kDebugMaxBounces && rec[(size_t)n].bounce == n + 1) ++n;
    *n_bounces = n;
    for (int k = 0; k < n && k < max; ++k) out[k] = rec[(size_t)k];
    return PT_OK;
}

extern "C" int pt_set_traversal_stats(pt_renderer* r, int32_t enable) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_traversal_stats: NULL");
    r->trav_stats = enable != 0;
    for (pt_renderer* p : r->peers) p->trav_stats = enable != 0;
    return PT_OK;
}

extern "C" int pt_set_wavefront_streams(pt_renderer* r, int32_t streams) {
    if (!r || streams < 0 || streams > pt_renderer::kMaxWFStreams)
        return fail(PT_ERR_INVALID, "pt_set_wavefront_streams: 0 (auto) or 1 to 4");
    int rc = collect_pending(r);
    if (rc != PT_OK) return rc;
    r->wf_streams = streams;
    for (pt_renderer* p : r->peers)
        if ((rc = pt_set_wavefront_streams(p, streams)) != PT_OK) return rc;
    return PT_OK;
}

extern "C" int pt_set_primary_dedup(pt_renderer* r, int32_t enable) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_primary_dedup: NULL");
    int rc = collect_pending(r);
    if (rc) return rc;
    r->primary_dedup = enable != 0;
    for (pt_renderer* p : r->peers) {
        if ((rc = pt_set_primary_dedup(p, enable)) != PT_OK) return rc;
    }
    return PT_OK;
}

extern "C" int pt_set_band_split(pt_renderer* r, int32_t enable) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_band_split: NULL");
    int rc = collect_pending(r);
    if (rc) return rc;
    r->band_split = enable != 0;
    for (pt_renderer* p : r->peers) {
        if ((rc = pt_set_band_split(p, enable)) != PT_OK) return rc;
    }
    return PT_OK;
}

extern "C" int pt_set_kernel_timing(pt_renderer* r, int32_t enable) {
    if (!r) return fail(PT_ERR_INVALID, "pt_set_kernel_timing: NULL");
    int rc = collect_pending(r);
    if (rc) return rc;
    r->kernel_timing = enable != 0;
    for (pt_renderer* p : r->peers) {
        if ((rc = pt_set_kernel_timing(p, enable)) != PT_OK) return rc;
    }
    return PT_OK;
}
