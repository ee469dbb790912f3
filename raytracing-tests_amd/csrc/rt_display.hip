// Display pass: the stage's fullscreen-quad blit of the compute output into the
// RGBA8 framebuffer -- In-Next-Week/01_BoundingVolumeHierarchy/BVH.cpp:6-43 (colour, or the
// depth image as grey when u_UseDpthTexture) and the IOW-03 pass materials.cpp:154-161.  The
// quad covers the viewport texel for texel, so the blit is a per-pixel conversion: GL's
// float -> unorm8 store (clamp to [0, 1], round to nearest; NaN -> 0).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_kernels.hpp"

namespace rtk {
namespace {

__device__ __forceinline__ uint8_t unorm8(float f) {
    if (!(f > 0.0f)) return 0;  // also NaN
    if (f >= 1.0f) return 255;
    return (uint8_t)__builtin_floorf(f * 255.0f + 0.5f);
}

__global__ __launch_bounds__(256) void k_display(const float4 *rgba, const float *depth, uint32_t n, int use_depth,
                                                 uchar4 *out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;  // no cross-lane work in this kernel
    float4 c;
    if (use_depth) {
        const float d = depth[i];
        c = make_float4(d, d, d, 1.0f);
    } else {
        c = rgba[i];
    }
    out[i] = make_uchar4(unorm8(c.x), unorm8(c.y), unorm8(c.z), unorm8(c.w));
}

}  // namespace

hipError_t display_rgba8(const float *rgba, const float *depth, uint32_t n, int use_depth, uint8_t *out,
                         hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_display, dim3((n + 255) / 256), dim3(256), 0, s, reinterpret_cast<const float4 *>(rgba),
                       depth, n, use_depth, reinterpret_cast<uchar4 *>(out));
    return hipGetLastError();
}

}  // namespace rtk
