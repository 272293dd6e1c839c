// hbm_calib.hip — what rocprofv3's FETCH_SIZE / WRITE_SIZE report on gfx950 for the access
// patterns of this repo's trace and shading kernels, against byte counts known by
// construction.  Each kernel below moves exactly `items` x 16 B of one kind (plus a 4-B result
// per workgroup), over a 4-GiB buffer (16x the 256-MiB Infinity Cache, so repeated runs do not
// hit it).  Run each counter in its own pass (MI355X_MICROARCH.md), e.g.
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d out/fetch -o run -- ./hbm_calib
//   rocprofv3 --pmc WRITE_SIZE --output-format csv -d out/write -o run -- ./hbm_calib
// and read the per-dispatch counters against the bytes the program prints (tools/hbm_calib.py).
//
// Patterns:
//   read_stream    16 B per lane, consecutive lanes -> consecutive records (queue reads)
//   read_gather    16 B per lane at hashed positions over 4 GiB (path-order gathers)
//   read_chunks    runs of 24 consecutive records per wave at scattered chunk bases (the trace
//                  kernels' refill: idle lanes take the next records of the wave's slice)
//   write_stream   16 B per lane, consecutive (queue appends)
//   write_window   a wave writes the 512 records of its slice window in a lane-shuffled order
//                  over 8 iterations (trace kernels: rays finish out of order within a slice)
//   write_scatter  16 B per lane at bijectively permuted positions over 4 GiB (W.L adds)
//   rmw_scatter    read + write of 16 B at permuted positions (the read counts as fetch)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                       \
    do {                                                                            \
        hipError_t e_ = (x);                                                        \
        if (e_ != hipSuccess) {                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
            std::exit(1);                                                           \
        }                                                                           \
    } while (0)

constexpr unsigned long long kRecords = 1ull << 28;  // 4 GiB of float4
constexpr unsigned kMask = (unsigned)(kRecords - 1);

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}
// bijection on [0, 2^28): odd multiplier mod 2^28
__device__ __forceinline__ unsigned perm(unsigned i) { return (i * 2654435761u) & kMask; }

__device__ __forceinline__ void sink(float v, float* out) {
    // one 4-B store per workgroup keeps the loads alive
    __shared__ float s;
    if (threadIdx.x == 0) s = 0.0f;
    __syncthreads();
    atomicAdd(&s, v);
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = s;
}

__global__ void read_stream(const float4* __restrict__ a, unsigned items, float* out) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = 0.0f;
    if (i < items) {
        const float4 x = a[i];
        v = x.x + x.y + x.z + x.w;
    }
    sink(v, out);
}
__global__ void read_gather(const float4* __restrict__ a, unsigned items, float* out) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = 0.0f;
    if (i < items) {
        const float4 x = a[hash32(i) & kMask];
        v = x.x + x.y + x.z + x.w;
    }
    sink(v, out);
}
__global__ void read_chunks(const float4* __restrict__ a, unsigned items, float* out) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    float v = 0.0f;
    if (i < items) {
        const unsigned chunk = i / 24, k = i - chunk * 24;
        const float4 x = a[(hash32(chunk) % (unsigned)(kRecords / 24 - 1)) * 24u + k];
        v = x.x + x.y + x.z + x.w;
    }
    sink(v, out);
}
__global__ void write_stream(float4* __restrict__ a, unsigned items) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < items) a[i] = make_float4((float)i, 1.0f, 2.0f, 3.0f);
}
__global__ void write_window(float4* __restrict__ a, unsigned items) {
    // wave w owns records [512 w, 512 w + 512); iteration k writes record 512 w + (lane * 8 + k)
    // permuted within the window (hash), so every line of the window fills over 8 iterations
    const unsigned wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, lane = threadIdx.x & 63;
    const unsigned base = wave * 512u;
    if (base >= items) return;
    for (unsigned k = 0; k < 8; ++k) {
        const unsigned j = (lane * 8u + k) * 173u & 511u;  // 173 odd: a bijection on [0, 512)
        a[base + j] = make_float4((float)j, 1.0f, 2.0f, 3.0f);
    }
}
__global__ void write_scatter(float4* __restrict__ a, unsigned items) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < items) a[perm(i)] = make_float4((float)i, 1.0f, 2.0f, 3.0f);
}
__global__ void rmw_scatter(float4* __restrict__ a, unsigned items) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < items) {
        const unsigned j = perm(i);
        const float4 x = a[j];
        a[j] = make_float4(x.x + 1.0f, x.y, x.z, x.w);
    }
}

int main() {
    const unsigned items = 1u << 26;  // 1 GiB of records per pattern
    float4* a = nullptr;
    float* out = nullptr;
    CK(hipMalloc(&a, kRecords * sizeof(float4)));
    CK(hipMalloc(&out, (items / 256) * sizeof(float)));
    CK(hipMemset(a, 0, kRecords * sizeof(float4)));
    CK(hipDeviceSynchronize());
    const dim3 blk(256), grd(items / 256);
    const double gib = (double)items * 16.0;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const char* name, auto launch, double rd, double wr) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.0f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        std::printf("{\"kernel\": \"%s\", \"read_bytes\": %.0f, \"write_bytes\": %.0f, \"ms\": %.4f}\n", name, rd,
                    wr, ms);
    };
    const double sink_b = (double)(items / 256) * 4.0;
    run("read_stream", [&] { hipLaunchKernelGGL(read_stream, grd, blk, 0, 0, a, items, out); }, gib, sink_b);
    run("read_gather", [&] { hipLaunchKernelGGL(read_gather, grd, blk, 0, 0, a, items, out); }, gib, sink_b);
    run("read_chunks", [&] { hipLaunchKernelGGL(read_chunks, grd, blk, 0, 0, a, items, out); }, gib, sink_b);
    run("write_stream", [&] { hipLaunchKernelGGL(write_stream, grd, blk, 0, 0, a, items); }, 0.0, gib);
    run("write_window", [&] { hipLaunchKernelGGL(write_window, dim3(items / 512 / 4), blk, 0, 0, a, items); }, 0.0,
        gib);
    run("write_scatter", [&] { hipLaunchKernelGGL(write_scatter, grd, blk, 0, 0, a, items); }, 0.0, gib);
    run("rmw_scatter", [&] { hipLaunchKernelGGL(rmw_scatter, grd, blk, 0, 0, a, items); }, gib, gib);
    CK(hipDeviceSynchronize());
    CK(hipFree(a));
    CK(hipFree(out));
    return 0;
}
