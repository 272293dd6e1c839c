// pt_display.hip — device-side progressive view buffer.
//
// Restates the GL accumulation of the reference's viewer on the device, so a headless caller
// gets the same displayed image without a per-spp PCIe download and GL blend:
//   OptixView::AddNewFrameToBuffer (Renderer/OptixView.cpp:226-255) + AddPathtracedFrame.frag
//   :18-24: continuous (maxSamples < 0): fb = mix(fb, new, 1/n); otherwise fb += new * (1/max).
//   The framebuffer starts from glClearColor(1,1,1,1) (OptixView.cpp:145-149).
// GLSL mix(x, y, a) = x * (1 - a) + y * a, evaluated here without contraction (-ffp-contract=off).
#include "pt_internal.h"

namespace pt {

namespace {

__global__ void k_fill(float* p, size_t n, float v) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = v;
}

__global__ void k_blend(float* fb, const float* frame, size_t n, float w, int continuous) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float a = fb[i], b = frame[i];
        fb[i] = continuous ? a * (1.0f - w) + b * w : a + b * w;
    }
}

inline dim3 grid_for(size_t n) { return dim3((unsigned)std::min<size_t>((n + 255) / 256, 65535)); }

}  // namespace

hipError_t display_fill(float* p, size_t n, float v, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_fill, grid_for(n), dim3(256), 0, stream, p, n, v);
    return hipGetLastError();
}

hipError_t display_blend(float* fb, const float* frame, size_t n, float w, bool continuous, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_blend, grid_for(n), dim3(256), 0, stream, fb, frame, n, w, continuous ? 1 : 0);
    return hipGetLastError();
}

}  // namespace pt
