// rt_math.hpp -- device vector math under the numerics contract:
//   IEEE binary32, GLSL evaluation order, no contraction (built with -ffp-contract=off),
//   GLSL a/b == a * RN(1/b) (correctly rounded reciprocal, -fhip-fp32-correctly-rounded-divide-sqrt),
//   correctly rounded sqrt, normalize(v) == v * RN(1/sqrt(dot(v,v))), min/max == fminf/fmaxf.
// Under this contract every operation has exactly one IEEE result, so the GPU reproduces
// the CPU oracle bit for bit; the GLSL builtins are restated from the GLSL 4.40 spec.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtk {

struct f3 { float x, y, z; };

__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return f3{a.x + b.x, a.y + b.y, a.z + b.z}; }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return f3{a.x - b.x, a.y - b.y, a.z - b.z}; }
__device__ __forceinline__ f3 operator-(f3 a) { return f3{-a.x, -a.y, -a.z}; }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return f3{a.x * s, a.y * s, a.z * s}; }
// component-wise select (an aggregate ?: can lower to a private-memory copy)
__device__ __forceinline__ f3 sel(bool c, f3 a, f3 b) { return f3{c ? a.x : b.x, c ? a.y : b.y, c ? a.z : b.z}; }
__device__ __forceinline__ f3 mulv(f3 a, f3 b) { return f3{a.x * b.x, a.y * b.y, a.z * b.z}; }
__device__ __forceinline__ float dot(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 cross(f3 a, f3 b) {
    return f3{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ float rcp(float b) { return 1.0f / b; }
// RN(1/s) for s = RN(sqrt(x)) of a float x, i.e. s in [2^-75, 2^64] or 0, +inf, NaN.  The
// compiler's correctly rounded 1.0f / s is div_scale x2, rcp, five fma, div_fmas and div_fixup;
// the div_scale steps only rescale operands whose reciprocal could leave the normal range (not
// the case on this domain), where div_fmas is a plain fma.  This is the same arithmetic without
// them; rt_debug_check_fastmath(0) compares it with 1.0f / sqrt(x) for all 2^32 x on the device
// (tests/test_gpu_fastmath.py).  Outside the domain (denormal or huge s) it is not exact.
__device__ __forceinline__ float rcp_sqrt_domain(float s) {
    const float r0 = __builtin_amdgcn_rcpf(s);
    const float r = __builtin_fmaf(__builtin_fmaf(-s, r0, 1.0f), r0, r0);
    const float q1 = __builtin_fmaf(__builtin_fmaf(-s, r, 1.0f), r, r);
    const float q2 = __builtin_fmaf(__builtin_fmaf(-s, q1, 1.0f), r, q1);
    return __builtin_amdgcn_div_fixupf(q2, s, 1.0f);
}
__device__ __forceinline__ float len(f3 v) { return __builtin_sqrtf(dot(v, v)); }
__device__ __forceinline__ f3 normalize(f3 v) { return v * rcp_sqrt_domain(__builtin_sqrtf(dot(v, v))); }
__device__ __forceinline__ float get(f3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }

// column-major 3x3 (GLSL mat3 / glm::mat3), c0..c2 columns
struct m3 { f3 c0, c1, c2; };
__device__ __forceinline__ f3 mul(const m3 &m, f3 v) { return (m.c0 * v.x + m.c1 * v.y) + m.c2 * v.z; }
__device__ __forceinline__ f3 tmul(const m3 &m, f3 v) { return f3{dot(m.c0, v), dot(m.c1, v), dot(m.c2, v)}; }

__device__ __forceinline__ f3 reflect(f3 I, f3 N) { return I - N * (2.0f * dot(N, I)); }
__device__ __forceinline__ f3 refract(f3 I, f3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return f3{0.0f, 0.0f, 0.0f};
    return I * eta - N * (eta * d + __builtin_sqrtf(k));
}

// glm::inverse / GLSL inverse of a mat3 (adjugate over determinant)
__device__ __forceinline__ m3 inverse(const m3 &m) {
    const float a00 = m.c0.x, a01 = m.c0.y, a02 = m.c0.z;  // a[c][r]
    const float a10 = m.c1.x, a11 = m.c1.y, a12 = m.c1.z;
    const float a20 = m.c2.x, a21 = m.c2.y, a22 = m.c2.z;
    float det = +a00 * (a11 * a22 - a21 * a12) - a10 * (a01 * a22 - a21 * a02) + a20 * (a01 * a12 - a11 * a02);
    float o = 1.0f / det;
    m3 r;
    r.c0.x = +(a11 * a22 - a21 * a12) * o;
    r.c1.x = -(a10 * a22 - a20 * a12) * o;
    r.c2.x = +(a10 * a21 - a20 * a11) * o;
    r.c0.y = -(a01 * a22 - a21 * a02) * o;
    r.c1.y = +(a00 * a22 - a20 * a02) * o;
    r.c2.y = -(a00 * a21 - a20 * a01) * o;
    r.c0.z = +(a01 * a12 - a11 * a02) * o;
    r.c1.z = -(a00 * a12 - a10 * a02) * o;
    r.c2.z = +(a00 * a11 - a10 * a01) * o;
    return r;
}

// Background_Color (03...glsl:123-126, 01_BVH...glsl:9-12; black ends: 04...glsl:23-30)
__device__ __forceinline__ f3 background(f3 d, bool black) {
    const f3 lo = black ? f3{0, 0, 0} : f3{1.0f, 1.0f, 1.0f};
    const f3 hi = black ? f3{0, 0, 0} : f3{0.3f, 0.4f, 1.0f};
    float t = (d.y + 1.0f) * 0.5f;
    return lo * (1.0f - t) + hi * t;
}

// cuboid face normal (03...glsl:101-119, 01_BVH...glsl:165-182)
__device__ __forceinline__ f3 cuboid_normal(f3 h, f3 s) {
    float md = fabsf(h.x - s.x * 0.5f);
    int index = 0;
    float dist = fabsf(h.x + s.x * 0.5f);
    if (md > dist) { md = dist; index = 1; }
    dist = fabsf(h.y - s.y * 0.5f); if (md > dist) { md = dist; index = 2; }
    dist = fabsf(h.y + s.y * 0.5f); if (md > dist) { md = dist; index = 3; }
    dist = fabsf(h.z - s.z * 0.5f); if (md > dist) { md = dist; index = 4; }
    dist = fabsf(h.z + s.z * 0.5f); if (md > dist) { md = dist; index = 5; }
    const float sg = (index & 1) ? -1.0f : 1.0f;
    const int ax = index >> 1;
    return f3{ax == 0 ? sg : 0.0f, ax == 1 ? sg : 0.0f, ax == 2 ? sg : 0.0f};
}

// unit ellipsoid / cuboid ray test in the object's local frame (t_RayXObj 03...glsl:55-95,
// t_RayXGeom 01_BVH...glsl:112-155).  is = per-object RN(1/scale).
__device__ __forceinline__ float t_ellipsoid(f3 o, f3 d, f3 is) {
    f3 a2 = mulv(o, is), a3 = mulv(d, is);
    float hb = dot(a2, a3), a = dot(a3, a3), c = dot(a2, a2) - 1.0f;
    float det = hb * hb - a * c;
    float t = -1.0f;
    if (det > 0.0f) {
        float ia = rcp(a), sq = __builtin_sqrtf(det);
        float t0 = (-hb - sq) * ia, t1 = (-hb + sq) * ia;
        t = (t0 > t1 || t0 < 0.0f) ? t1 : t0;
    }
    return t > 0.0f ? t : -1.0f;
}
// t_cuboid with the reciprocals of d given (id = 1/d, correctly rounded as rcp computes them)
__device__ __forceinline__ float t_cuboid_rcp(f3 o, f3 id3, f3 s) {
    f3 bmin = (-s) * 0.5f, bmax = s * 0.5f;
    float id = id3.x;
    float t1 = (bmin.x - o.x) * id, t2 = (bmax.x - o.x) * id;
    float tmin = fminf(t1, t2), tmax = fmaxf(t1, t2);
    id = id3.y;
    t1 = (bmin.y - o.y) * id; t2 = (bmax.y - o.y) * id;
    tmin = fmaxf(tmin, fminf(fminf(t1, t2), tmax));
    tmax = fminf(tmax, fmaxf(fmaxf(t1, t2), tmin));
    id = id3.z;
    t1 = (bmin.z - o.z) * id; t2 = (bmax.z - o.z) * id;
    tmin = fmaxf(tmin, fminf(fminf(t1, t2), tmax));
    tmax = fminf(tmax, fmaxf(fmaxf(t1, t2), tmin));
    float t = tmax > tmin ? (tmin > 0.0f ? tmin : tmax) : -1.0f;
    return t > 0.0f ? t : -1.0f;
}
__device__ __forceinline__ float t_cuboid(f3 o, f3 d, f3 s) {
    f3 bmin = (-s) * 0.5f, bmax = s * 0.5f;
    float id = rcp(d.x);
    float t1 = (bmin.x - o.x) * id, t2 = (bmax.x - o.x) * id;
    float tmin = fminf(t1, t2), tmax = fmaxf(t1, t2);
    id = rcp(d.y);
    t1 = (bmin.y - o.y) * id; t2 = (bmax.y - o.y) * id;
    tmin = fmaxf(tmin, fminf(fminf(t1, t2), tmax));
    tmax = fminf(tmax, fmaxf(fmaxf(t1, t2), tmin));
    id = rcp(d.z);
    t1 = (bmin.z - o.z) * id; t2 = (bmax.z - o.z) * id;
    tmin = fmaxf(tmin, fminf(fminf(t1, t2), tmax));
    tmax = fminf(tmax, fmaxf(fmaxf(t1, t2), tmin));
    float t = tmax > tmin ? (tmin > 0.0f ? tmin : tmax) : -1.0f;
    return t > 0.0f ? t : -1.0f;
}

// wave-level uint64 sum (64 lanes) for the counters
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}

}  // namespace rtk
