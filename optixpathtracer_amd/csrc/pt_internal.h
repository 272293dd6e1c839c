// pt_internal.h — host-side declarations shared by the C-ABI (pt_capi.cpp) and the kernel
// translation units (pt_build.hip, pt_render.hip).  Not part of the public ABI.
#pragma once
#include <hip/hip_runtime.h>

#include "pt_device.h"

namespace pt {

// Scene triangle soup in ORIGINAL order (meshes concatenated), world space.
struct BuildInput {
    const float4* tri_orig;  // 3 per triangle: v0|orig idx bits, v1|material bits, v2|0
    const float4* nrm_orig;  // 3 per triangle
    int n;
    float cmin[3], cmax[3];  // centroid bounds (Morton quantisation range)
};

// LBVH in leaf order.
struct BuildOutput {
    BNode* nodes;  // n-1
    float4* tri;   // 3n
    float4* nrm;   // 3n
};

// GPU LBVH build (Morton codes -> radix sort -> Karras 2012 hierarchy -> AABBs from a sparse
// table over the sorted leaves).  Replaces optixAccelBuild (OptixRenderer.cpp:306-456).
// Returns hipSuccess or the first error; *ms = device time of the build.
hipError_t lbvh_build(const BuildInput& in, BuildOutput& out, hipStream_t stream, float* ms);

// Render launches.
hipError_t launch_render(int kernel, int mode, const DevScene& S, const DevLaunch& L, hipStream_t stream);
hipError_t launch_trace(const DevScene& S, const float* d_rays, int n, int* d_prim, float* d_thit, float* d_u,
                        float* d_v, int* d_back, int any_hit, hipStream_t stream);

}  // namespace pt
