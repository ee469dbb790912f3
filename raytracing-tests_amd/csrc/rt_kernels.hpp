// rt_kernels.hpp -- launch-side declarations shared by rt_kernels.hip and rt_capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtk {

// Per-launch uniforms, computed on the host exactly as the reference host + shader
// prologue would (camera vectors are derived on the device with the contract's ops).
struct Frame {
    int W, H, spp, max_bounces, show_normal;
    // pixel mapping: rect mode (tiles == nullptr) or tile-list mode
    int x0, y0, tw, th;
    const int *tiles;
    int n_tiles, tile_size;
    float *out_rgba;    // full image (rect mode) or packed tiles (tile mode)
    float *out_depth;   // may be null
    unsigned long long *counters;  // 6 x u64
    float pos[3], dir[3];
    float aperture, focus, screen_dist, inv_spp;
    float sphere[4];    // IOW-01 only
};

// IOW-03 device scene: "hot" records walked by the linear loop + "cold" hit attributes.
constexpr int kIowHot = 20;   // pos3 type M9 scale3 inv_scale3 pad
constexpr int kIowCold = 8;   // color3 material3 scat2
// INW device scene
constexpr int kInwHot = 28;   // pos3 R9 scale3 delta3 type extra inv_scale3 inv_s2_3 ri_acc pad
constexpr int kInwCold = 8;   // refr refl srfr srfl color3 ri

constexpr int kIowBvhStack = 32;  // deepest IOW BVH the kernel walks; deeper trees use the linear loop
struct IowScene {
    const float *hot, *cold;
    uint32_t n;
    const float4 *nodes;     // conservative BVH over the objects ((2n-1)*2 float4) or null = linear loop
    const float *sunflower;  // spp*2
    const float *fib;        // spp*4 (xyz + pad)
    const int *ring;         // spp*2
};
struct InwScene {
    const float4 *hot;       // n * 7 float4
    const float4 *cold;      // n * 2 float4
    const float4 *nodes;     // (2n-1) * 2 float4
    const float *lights;     // L * 7
    uint32_t n, n_lights;
    int layout;
    const float *sunflower;  // spp*2
};

hipError_t launch_iow01(const Frame &f, hipStream_t s);
// Persistent work-queue launches: `counter` (one u32, device) is zeroed on `s` before the
// kernel; at most `blocks_cap` blocks are launched (they pull pixels until none are left).
hipError_t launch_iow03(const Frame &f, const IowScene &sc, unsigned *counter, int s_stop, int blocks_cap,
                        hipStream_t s);
hipError_t launch_inw(const Frame &f, const InwScene &sc, unsigned *counter, int blocks_cap, hipStream_t s);

}  // namespace rtk
