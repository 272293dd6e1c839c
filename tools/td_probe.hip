// Vector-memory data-path probe (TA/TD cost of a 16-B-per-lane load by address pattern).
//
// The trace kernels keep the per-CU texture address/data units 81 % / 94 % busy
// (TA_TA_BUSY_sum, TD_TD_BUSY_sum over 256 units and GRBM_GUI_ACTIVE / 8), so the
// cost of one `global_load_dwordx4` by how many distinct cache lines its lanes touch and how many
// lanes are active decides which node layouts pay.  Every pattern reads an L1/L2-resident 64-KB
// window per workgroup; all CUs run 8 waves per SIMD; time / loads gives CU cycles per wave-load.
//   hipcc --offload-arch=gfx950 -O3 tools/td_probe.hip -o tools/td_probe && tools/td_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

constexpr int kBlock = 256, kIters = 4096;

// pattern: lanes per 128-B line (64 = all lanes one line, 8 = contiguous, 1 = every lane its own
// line); active: lanes that load (the rest are exec-masked off)
__global__ __launch_bounds__(kBlock) void k_probe(const float4* __restrict__ buf, float* out, int lanes_per_line,
                                                  int active, int stride_lines) {
    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    // 64-KB window per workgroup (512 lines); each wave walks it with its own phase
    const float4* base = buf + (size_t)(blockIdx.x & 255) * 4096;
    const int line = lane / lanes_per_line;            // line of this lane within the group
    const int chunk = (lane % lanes_per_line) & 7;      // 16-B chunk within the line
    float acc = 0.0f;
    int off = wave * 37;
    if (lane < active) {
        for (int i = 0; i < kIters; ++i) {
            const int l = (off + line * stride_lines) & 511;
            const float4 v = base[l * 8 + chunk];
            acc += (v.x + v.y) + (v.z + v.w);
            off += 11;
        }
    }
    if (acc == 12345.0f) out[blockIdx.x] = acc;
}

int main() {
    hipDeviceProp_t p;
    hipGetDeviceProperties(&p, 0);
    const int cus = p.multiProcessorCount;
    const size_t n = (size_t)256 * 4096;
    float4* buf;
    float* out;
    hipMalloc(&buf, n * sizeof(float4));
    hipMalloc(&out, 65536 * sizeof(float));
    hipMemset(buf, 0, n * sizeof(float4));
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int grid = cus * 8;  // 8 workgroups of 4 waves per CU = 8 waves per SIMD
    struct P {
        int lpl, active, stride;
        const char* name;
    } ps[] = {{64, 64, 1, "all 64 lanes one line"},
              {8, 64, 1, "8 lanes per line (coalesced 1 KB)"},
              {4, 64, 1, "4 lanes per line"},
              {2, 64, 1, "2 lanes per line"},
              {1, 64, 1, "1 lane per line (64 lines)"},
              {1, 32, 1, "1 lane per line, 32 lanes active"},
              {1, 16, 1, "1 lane per line, 16 lanes active"},
              {8, 32, 1, "8 lanes per line, 32 lanes active"}};
    hipLaunchKernelGGL(k_probe, dim3(grid), dim3(kBlock), 0, 0, buf, out, 8, 64, 1);
    hipDeviceSynchronize();
    printf("{\"cus\": %d, \"clock_mhz\": %d, \"patterns\": [\n", cus, p.clockRate / 1000);
    for (size_t k = 0; k < sizeof(ps) / sizeof(ps[0]); ++k) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_probe, dim3(grid), dim3(kBlock), 0, 0, buf, out, ps[k].lpl, ps[k].active, ps[k].stride);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        // wave-loads per CU: 8 workgroups x 4 waves x kIters
        const double loads = 8.0 * 4 * kIters;
        const double cyc = ms * 1e-3 * (p.clockRate * 1e3) / loads;
        printf("  {\"pattern\": \"%s\", \"ms\": %.3f, \"cu_cycles_per_wave_load\": %.2f}%s\n", ps[k].name, ms, cyc,
               k + 1 < sizeof(ps) / sizeof(ps[0]) ? "," : "");
    }
    printf("]}\n");
    return 0;
}
