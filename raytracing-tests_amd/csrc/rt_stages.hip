// The reference's simple In-One-Weekend stages, one thread per pixel:
//   IOW-00  In-One-Weekend/base.cpp:7-28 -- the base stage's default compute shader, a UV
//           gradient (00_Image/image.cpp:46-53 dispatches it W x H);
//   IOW-02  In-One-Weekend/02_Groups/computeShaderSrc.glsl -- cuboids / ellipsoids, mirror
//           bounces weighted pow(0.4, i), front / back culling (groups.cpp:56-84).
// Same numerics contract as every other kernel (rt_math.hpp); pow(0.4, i) is a host table.
#include <hip/hip_runtime.h>

#include "rt_kernels.hpp"
#include "rt_math.hpp"

namespace rtk {
namespace {

__global__ __launch_bounds__(256) void k_iow00(int W, int H, float4 *out) {
    const int x = (int)(blockIdx.x * 16 + (threadIdx.x & 15)), y = (int)(blockIdx.y * 16 + (threadIdx.x >> 4));
    if (x >= W || y >= H) return;  // no cross-lane work in this kernel
    const float r = (float)x * rcp((float)W - 1.0f), g = (float)y * rcp((float)H - 1.0f);  // base.cpp:13-14
    out[(size_t)y * W + x] = make_float4(r, g, 0.25f, 1.0f);
}

// t_RayXObj 02.glsl:37-94 with the u_Cull_Front / u_Cull_Back modes (CUBOID = 1, ELLIPSOID = 2)
__device__ __forceinline__ float t_obj_cull(f3 o, f3 d, int type, f3 s, bool cf, bool cb) {
    float t = -1.0f;
    if (type == 2) {
        const f3 a2 = f3{o.x * rcp(s.x), o.y * rcp(s.y), o.z * rcp(s.z)};
        const f3 a3 = f3{d.x * rcp(s.x), d.y * rcp(s.y), d.z * rcp(s.z)};
        const float hb = dot(a2, a3), a = dot(a3, a3), c = dot(a2, a2) - 1.0f;
        const float det = hb * hb - a * c;
        if (det > 0.0f) {
            const float t0 = (-hb - __builtin_sqrtf(det)) * rcp(a), t1 = (-hb + __builtin_sqrtf(det)) * rcp(a);
            if (!cb && !cf) t = (t0 > t1 || t0 < 0.0f) ? t1 : t0;
            else if (!cf) t = fminf(t0, t1);
            else if (!cb) t = fmaxf(t0, t1);
        }
    } else if (type == 1) {
        const f3 bmin = (-s) * 0.5f, bmax = s * 0.5f;
        float t1 = (bmin.x - o.x) * rcp(d.x), t2 = (bmax.x - o.x) * rcp(d.x);
        float tmin = fminf(t1, t2), tmax = fmaxf(t1, t2);
        t1 = (bmin.y - o.y) * rcp(d.y); t2 = (bmax.y - o.y) * rcp(d.y);
        tmin = fmaxf(tmin, fminf(fminf(t1, t2), tmax));
        tmax = fminf(tmax, fmaxf(fmaxf(t1, t2), tmin));
        t1 = (bmin.z - o.z) * rcp(d.z); t2 = (bmax.z - o.z) * rcp(d.z);
        tmin = fmaxf(tmin, fminf(fminf(t1, t2), tmax));
        tmax = fminf(tmax, fmaxf(fmaxf(t1, t2), tmin));
        if (tmax > fmaxf(tmin, 0.0f)) {
            if (!cb && !cf) t = tmin > 0.0f ? tmin : tmax;
            else if (!cf) t = tmin;
            else if (!cb) t = tmax;
        }
    }
    return t > 0.0f ? t : -1.0f;
}

// out_Pixel 02.glsl:129-222 for pixel (x, y) of the frame
__global__ __launch_bounds__(256) void k_iow02(Frame f, const float *types, const float *rec, uint32_t n,
                                               const int *ring, const float *pw, int cull_front, int cull_back) {
    const int lx = (int)(blockIdx.x * 16 + (threadIdx.x & 15)), ly = (int)(blockIdx.y * 16 + (threadIdx.x >> 4));
    if (lx >= f.tw || ly >= f.th) return;  // no cross-lane work in this kernel
    const int x = f.x0 + lx, y = f.y0 + ly, W = f.W, H = f.H;
    if (x < 0 || y < 0 || x >= W || y >= H) return;
    const bool cf = cull_front != 0, cb = cull_back != 0;
    const f3 D = mk(f.dir[0], f.dir[1], f.dir[2]), P = mk(f.pos[0], f.pos[1], f.pos[2]);
    const float aspect = (float)W * rcp((float)H);
    const f3 up = f3{0, 1, 0};
    float sx = ((float)x * 2.0f - (float)W) * rcp(2.0f * (float)W);
    sx *= aspect;
    const float sy = ((float)y * 2.0f - (float)H) * rcp(2.0f * (float)H);
    int grid = 1;
    while (grid * grid < f.spp) grid++;
    f3 fc = f3{0, 0, 0};
    int s = 0;
    bool early = false;
    unsigned long long seg = 0;
    for (; s < f.spp; s++) {
        f3 ro = P, rd;
        {
            const f3 cr = cross(D, up), cu = cross(cr, D);
            const int ix = ring[2 * s], iy = ring[2 * s + 1];
            if (ix < 0) { early = true; break; }  // 02.glsl:156
            const float dx = aspect * rcp((float)(W * grid)), dy = 1.0f * rcp((float)(H * grid));
            rd = normalize((D * f.focus + cr * (sx + dx * (float)ix)) + cu * (sy + dy * (float)iy));
        }
        float min_t = 32000.0f;
        f3 nrm = D, fsc = f3{0, 0, 0};
        for (int i = 0; i < f.max_bounces; i++) {
            f3 sc = background(rd, false);
            m3 hm = m3{f3{0, 0, 0}, f3{0, 0, 0}, f3{0, 0, 0}};
            seg++;
            for (uint32_t j = 0; j < n; j++) {
                const float *r = rec + (size_t)j * 18;
                const int type = (int)types[j];
                const f3 pos = mk(r[0], r[1], r[2]);
                const m3 M = m3{mk(r[3], r[4], r[5]), mk(r[6], r[7], r[8]), mk(r[9], r[10], r[11])};
                const f3 scale = mk(r[12], r[13], r[14]);
                const f3 to = mul(M, ro - pos), td = normalize(mul(M, rd));  // 02.glsl:194-198
                const float t = t_obj_cull(to, td, type, scale, cf, cb);
                if (min_t > t && t > 0.0f) {
                    const f3 h = to + td * t;  // SurfaceNormal 02.glsl:95-127
                    nrm = type == 2 ? f3{h.x * rcp(scale.x) * scale.x, h.y * rcp(scale.y) * scale.y,
                                         h.z * rcp(scale.z) * scale.z}
                                    : (type == 1 ? cuboid_normal(h, scale) : f3{0, 0, 0});
                    sc = mk(r[15], r[16], r[17]);
                    hm = M;
                    min_t = t;
                }
            }
            fsc = fsc + sc * pw[i];  // pow(0.4, i), 02.glsl:206
            if (f.show_normal) { fsc = nrm; break; }
            if (min_t > 30000.0f) break;
            ro = ro + rd * (min_t - 0.00005f);  // 02.glsl:215
            rd = reflect(rd, normalize(mul(inverse(hm), nrm)));
            nrm = f3{0, 0, 0};
            min_t = 32000.0f;
        }
        fc = fc + fsc;
    }
    const f3 o = fc * rcp((float)(early ? s : f.spp));
    reinterpret_cast<float4 *>(f.out_rgba)[(size_t)y * W + x] = make_float4(o.x, o.y, o.z, 1.0f);
    if (f.counters) {
        atomicAdd(f.counters + 0, seg);
        atomicAdd(f.counters + 2, seg * n);
    }
}

}  // namespace

hipError_t launch_iow00(int W, int H, float *out, hipStream_t s) {
    hipLaunchKernelGGL(k_iow00, dim3((unsigned)((W + 15) / 16), (unsigned)((H + 15) / 16)), dim3(256), 0, s, W, H,
                       reinterpret_cast<float4 *>(out));
    return hipGetLastError();
}
hipError_t launch_iow02(const Frame &f, const float *types, const float *rec, uint32_t n, const int *ring,
                        const float *pw, int cull_front, int cull_back, hipStream_t s) {
    hipLaunchKernelGGL(k_iow02, dim3((unsigned)((f.tw + 15) / 16), (unsigned)((f.th + 15) / 16)), dim3(256), 0, s, f,
                       types, rec, n, ring, pw, cull_front, cull_back);
    return hipGetLastError();
}

}  // namespace rtk
