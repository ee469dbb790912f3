// Texture producers of SURVEY 8f2 on the GPU (the texture SAMPLING lives in the INW kernel,
// rt_kernels.hip inw_tex_color):
//   - noise textures: Helper::Noise::MakeTexture<glm::vec3> (Utilities/utility.h:69-192) with
//     Snoise2 / Fbm2 / Turbulance (Utilities/utility.cpp:609-769);
//   - the Mercator <-> cubic re-projection of TEXTURE_2D::LoadFromDiskToGPU
//     (Utilities/utility.cpp:266-463).
// Both are host C++ in the reference (4 std::async column batches); here every texel is one
// thread.  The numerics are the reference's C++ ones (true division, the double-precision
// sub-expressions it has, float -> uint8 truncation), restated operation for operation from
// the CPU oracle's definition (oracle/rt_oracle_tex.c), so the bytes are identical.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "rt_kernels.hpp"

namespace rtk {
namespace {

constexpr int kTB = 256;

// ------------------------------------------------------------------ noise (utility.cpp:609-769)
__constant__ uint8_t kPerm[256] = {
    151, 160, 137, 91, 90, 15, 131, 13, 201, 95, 96, 53, 194, 233, 7, 225, 140, 36, 103, 30, 69, 142, 8, 99, 37,
    240, 21, 10, 23, 190, 6, 148, 247, 120, 234, 75, 0, 26, 197, 62, 94, 252, 219, 203, 117, 35, 11, 32, 57, 177,
    33, 88, 237, 149, 56, 87, 174, 20, 125, 136, 171, 168, 68, 175, 74, 165, 71, 134, 139, 48, 27, 166, 77, 146,
    158, 231, 83, 111, 229, 122, 60, 211, 133, 230, 220, 105, 92, 41, 55, 46, 245, 40, 244, 102, 143, 54, 65, 25,
    63, 161, 1, 216, 80, 73, 209, 76, 132, 187, 208, 89, 18, 169, 200, 196, 135, 130, 116, 188, 159, 86, 164, 100,
    109, 198, 173, 186, 3, 64, 52, 217, 226, 250, 124, 123, 5, 202, 38, 147, 118, 126, 255, 82, 85, 212, 207, 206,
    59, 227, 47, 16, 58, 17, 182, 189, 28, 42, 223, 183, 170, 213, 119, 248, 152, 2, 44, 154, 163, 70, 221, 153,
    101, 155, 167, 43, 172, 9, 129, 22, 39, 253, 19, 98, 108, 110, 79, 113, 224, 232, 178, 185, 112, 104, 218,
    246, 97, 228, 251, 34, 242, 193, 238, 210, 144, 12, 191, 179, 162, 241, 81, 51, 145, 235, 249, 14, 239, 107,
    49, 192, 214, 31, 181, 199, 106, 157, 184, 84, 204, 176, 115, 121, 50, 45, 127, 4, 150, 254, 138, 236, 205,
    93, 222, 114, 67, 29, 24, 72, 243, 141, 128, 195, 78, 66, 215, 61, 156, 180};

// fastFloor (utility.cpp:611): int(x) - 1 for integral x, as in the reference
__device__ __forceinline__ int fast_floor(float x) { return ((float)(int)x < x) ? (int)x : (int)x - 1; }

// grad2 (utility.cpp:636-653); both sign tests read bit 0 (`h&2 != 0` parses as h & 1)
__device__ __forceinline__ float grad2(uint32_t hash, float x, float y) {
    const uint32_t h = hash & 7u;
    float u = h < 4 ? x : y, v = h < 4 ? 2.0f * y : 2.0f * x;
    if (h & 1u) { u = -u; v = -v; }
    return u + v;
}

// one corner of Snoise2: (0.5 - x*x - y*y) in double, stored to float
__device__ __forceinline__ float corner(float x, float y, uint32_t hash) {
    float t = (float)(0.5 - (double)(x * x) - (double)(y * y));
    if (t < 0.0f) return 0.0f;
    t *= t;
    return t * t * grad2(kPerm[hash], x, y);
}

// Snoise2 (utility.cpp:657-737)
__device__ float snoise2(float x, float y) {
    const float F2 = 0.366025403f, G2 = 0.211324865f;
    const float s = (x + y) * F2;
    const int i = fast_floor(x + s), j = fast_floor(y + s);
    const float t = (float)(i + j) * G2;
    const float x0 = x - ((float)i - t), y0 = y - ((float)j - t);
    const uint32_t i1 = x0 > y0 ? 1u : 0u, j1 = 1u - i1;
    const float x1 = x0 - (float)i1 + G2, y1 = y0 - (float)j1 + G2;
    const float x2 = (float)((double)x0 - 1.0 + 2.0 * (double)G2);
    const float y2 = (float)((double)y0 - 1.0 + 2.0 * (double)G2);
    const uint32_t ii = (uint32_t)i & 255u, jj = (uint32_t)j & 255u;
    const float n0 = corner(x0, y0, (ii + kPerm[jj]) & 255u);
    const float n1 = corner(x1, y1, (ii + i1 + kPerm[(jj + j1) & 255u]) & 255u);
    const float n2 = corner(x2, y2, (ii + 1u + kPerm[(jj + 1u) & 255u]) & 255u);
    return n0 + n1 + n2;
}

// Snoise2 at (x*freq, y*freq), or the Fbm2 (:758-767) / Turbulance (:741-755) octave sum
__device__ float noise_at(int type, float x, float y, float freq, float lac, float gain, int octaves) {
    if (type == 0) return snoise2(x * freq, y * freq);
    float sum = 0.0f, amp = 1.0f;
    for (int o = 0; o < octaves; o++) {
        float f = snoise2(x * freq, y * freq) * amp;
        if (type == 2 && f < 0) f = -f;
        sum += f;
        freq *= lac;
        amp *= gain;
    }
    return sum;
}

// order-preserving float <-> uint for atomicMin / atomicMax
__device__ __forceinline__ uint32_t ord(float f) {
    const uint32_t b = __float_as_uint(f);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float unord(uint32_t u) {
    return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u);
}

struct NoiseArgs {
    int type, octaves, n_grad;
    float freq, lac, gain;
    float grad[3 * 66];
};
// workspace: [0] ord(min) [1] ord(max) [2] status, then W*H floats of noise
__global__ void k_noise_init(uint32_t *ws) {
    ws[0] = ord(1.0f);  // each of the reference's batches starts from min 1, max 0 (utility.h:103)
    ws[1] = ord(0.0f);
    ws[2] = 0u;
}

__global__ __launch_bounds__(kTB) void k_noise_eval(int W, int H, NoiseArgs a, uint32_t *ws) {
    const uint32_t idx = blockIdx.x * kTB + threadIdx.x;
    float *noise = reinterpret_cast<float *>(ws + 4);
    float v = 0.0f;
    const bool ok = idx < (uint32_t)W * (uint32_t)H;
    if (ok) {
        const uint32_t X = idx % (uint32_t)W, Y = idx / (uint32_t)W;
        v = noise_at(a.type, (float)X, (float)Y, a.freq, a.lac, a.gain, a.octaves);
        noise[idx] = v;
    }
    // min / max over the block, then one atomic each (NaN-free values: any order gives the
    // reference's MIN / MAX result up to the sign of a zero, which no output byte depends on)
    uint32_t lo = ok ? ord(v) : 0xffffffffu, hi = ok ? ord(v) : 0u;
    for (int d = 32; d > 0; d >>= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, d, 64));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, d, 64));
    }
    __shared__ uint32_t s_lo[kTB / 64], s_hi[kTB / 64];
    if ((threadIdx.x & 63) == 0) { s_lo[threadIdx.x >> 6] = lo; s_hi[threadIdx.x >> 6] = hi; }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kTB / 64; w++) { lo = min(lo, s_lo[w]); hi = max(hi, s_hi[w]); }
        atomicMin(ws, lo);
        atomicMax(ws + 1, hi);
    }
}

// double -> uint8_t of `pixel = 255.999*color` (x86-64: truncate to int32, keep the low byte)
__device__ __forceinline__ uint8_t to_u8(double v) {
    if (!(v > -2147483648.0 && v < 2147483648.0)) return 0;
    return (uint8_t)(uint32_t)(int32_t)v;
}

// func2 (utility.h:151-180): normalise by the range, map through the gradient
__global__ __launch_bounds__(kTB) void k_noise_color(int W, int H, NoiseArgs a, uint32_t *ws, uint8_t *rgb) {
    const uint32_t idx = blockIdx.x * kTB + threadIdx.x;
    if (idx >= (uint32_t)W * (uint32_t)H) return;  // no cross-lane work in this kernel
    const float mn = unord(ws[0]), mx = unord(ws[1]);
    const float *noise = reinterpret_cast<const float *>(ws + 4);
    const int G = a.n_grad;
    if (!(mx - mn != 0.0f)) {  // degenerate range: the reference divides by zero
        rgb[3 * (size_t)idx] = rgb[3 * (size_t)idx + 1] = rgb[3 * (size_t)idx + 2] = 0;
        if (idx == 0) ws[2] = 1u;
        return;
    }
    const float gdw = (float)(1.0 / (double)(G - 1));
    float factor = (noise[idx] - mn) / (mx - mn);
    uint32_t region = (uint32_t)(factor * (float)(G - 1));
    if (region > (uint32_t)(G - 2)) region = (uint32_t)(G - 2);
    factor = (factor - (float)(int)(factor / gdw) * gdw) * (float)(G - 1);  // MOD (utility.h:13)
    for (int c = 0; c < 3; c++) {
        const float g0 = a.grad[3 * region + c], d = a.grad[3 * (region + 1) + c] - g0;
        rgb[3 * (size_t)idx + c] = to_u8(255.999 * (double)(g0 + d * factor));
    }
}

// ------------------------------------------------- double-precision transcendentals
// The oracle's dm_* routines (oracle/rt_oracle_tex.c), the same operations in the same order.
constexpr double kPio2_1 = 0x1.921fb544p+0, kPio2_1t = 0x1.0b4611a626331p-34;
constexpr double kPi = 0x1.921fb54442d18p+1, kPiLo = 0x1.1a62633145c07p-53;
constexpr double kPio2 = 0x1.921fb54442d18p+0, kPio2Lo = 0x1.1a62633145c07p-54;
constexpr double kPio6 = 0x1.0c152382d7365p-1, kSqrt3 = 0x1.bb67ae8584caap+0;
constexpr double kTanPi12 = 0x1.126145e9ecd58p-2, k2OverPi = 0x1.45f306dc9c883p-1;

__device__ double dm_atan_pos(double x) {
    bool inv = false;
    double base = 0.0;
    if (x > 1.0) { x = 1.0 / x; inv = true; }
    if (x > kTanPi12) { x = (x * kSqrt3 - 1.0) / (kSqrt3 + x); base = kPio6; }
    const double x2 = x * x;
    double p = 0.0;
    for (int k = 17; k >= 0; k--) p = p * x2 + ((k & 1) ? -1.0 : 1.0) / (double)(2 * k + 1);
    double r = base + x * p;
    if (inv) r = (kPio2 - r) + kPio2Lo;
    return r;
}
__device__ double dm_atan2(double y, double x) {
    if (y != y || x != x) return x + y;
    if (y == 0.0) {
        if (x > 0.0 || (x == 0.0 && !__builtin_signbit(x))) return y;
        return __builtin_signbit(y) ? -(kPi + kPiLo) : kPi + kPiLo;
    }
    if (x == 0.0) return y > 0.0 ? kPio2 + kPio2Lo : -(kPio2 + kPio2Lo);
    double a = dm_atan_pos(__builtin_fabs(y) / __builtin_fabs(x));
    if (x < 0.0) a = (kPi - a) + kPiLo;
    return y < 0.0 ? -a : a;
}
__device__ double dm_acos(double x) { return dm_atan2(__builtin_sqrt((1.0 - x) * (1.0 + x)), x); }
__device__ void dm_sincos(double x, double &s_out, double &c_out) {
    const double kf = __builtin_floor(x * k2OverPi + 0.5);
    const double r = (x - kf * kPio2_1) - kf * kPio2_1t, r2 = r * r;
    double s = 1.0, c = 1.0;
    for (int n = 22; n >= 2; n -= 2) {
        s = 1.0 - r2 / (double)(n * (n + 1)) * s;
        c = 1.0 - r2 / (double)((n - 1) * n) * c;
    }
    s = r * s;
    const long long q = ((long long)kf % 4 + 4) % 4;
    s_out = q == 0 ? s : (q == 1 ? c : (q == 2 ? -s : -c));
    c_out = q == 0 ? c : (q == 1 ? -s : (q == 2 ? -c : s));
}
__device__ __forceinline__ float f_sin(float x) { double s, c; dm_sincos((double)x, s, c); return (float)s; }
__device__ __forceinline__ float f_cos(float x) { double s, c; dm_sincos((double)x, s, c); return (float)c; }

// ------------------------------------------------------------------ re-projection
__device__ __forceinline__ uint32_t u32_of(float v) {
    return v <= 0.0f ? 0u : (v >= 4294967040.0f ? 0xffffffffu : (uint32_t)v);
}

// XYtoUVCoord (utility.cpp:306-349)
__device__ void xy_to_uv(float X, float Y, float &U, float &V) {
    const float x = X - (float)(int)X;
    const float omx = (float)(1.0 - (double)x), omy = (float)(1.0 - (double)Y);
    float fx, fy, fz;
    switch ((int)X) {
        case 0: fx = x; fz = omy; fy = 1.0f; break;
        case 1: fy = omx; fz = omy; fx = 1.0f; break;
        case 2: fx = x; fy = Y; fz = 1.0f; break;
        case 3: fz = x; fy = Y; fx = 0.0f; break;
        case 4: fy = omx; fx = omy; fz = 0.0f; break;
        default: fz = x; fx = omy; fy = 0.0f; break;
    }
    fx -= 0.5f; fy -= 0.5f; fz -= 0.5f;
    const float inv = 1.0f / __builtin_sqrtf(fx * fx + fy * fy + fz * fz);  // glm::normalize
    fx *= inv; fy *= inv; fz *= inv;
    V = (float)dm_acos((double)-fy) / 3.14159274f;             // acosf / glm::pi<float>()
    U = (float)dm_atan2((double)fz, (double)fx) / 6.28318548f;  // atan2f / float(2*pi)
    if (U < 0) U = (float)((double)U + 1.0);
}

// UVtoXYCoord (utility.cpp:370-422)
__device__ void uv_to_xy(float U, float V, float &X, float &Y) {
    const float rad = (float)0.01745329251994329576923690768489;  // glm::radians
    const float pitch = (V * 180.0f - 90.0f) * rad, yaw = (U * 360.0f) * rad;
    const float cp = f_cos(pitch);
    float f0 = f_cos(yaw) * cp, f1 = f_sin(pitch), f2 = f_sin(yaw) * cp;
    float mx = f0;
    uint32_t face = mx > 0 ? 1u : 3u;
    const float s0 = (float)(mx > 0 ? 1 : -1);
    float d0 = 1.0f * s0, d1 = 0.0f * s0, d2 = 0.0f * s0;
    if (__builtin_fabsf(mx) < __builtin_fabsf(f1)) {
        mx = f1;
        face = mx > 0 ? 0u : 5u;
        const float s1 = (float)(mx > 0 ? 1 : -1);
        d0 = 0.0f * s1; d1 = 1.0f * s1; d2 = 0.0f * s1;
    }
    if (__builtin_fabsf(mx) < __builtin_fabsf(f2)) {
        mx = f2;
        face = mx > 0 ? 2u : 4u;
        const float s2 = (float)(mx > 0 ? 1 : -1);
        d0 = 0.0f * s2; d1 = 0.0f * s2; d2 = 1.0f * s2;
    }
    const float d = f0 * d0 + f1 * d1 + f2 * d2;
    f0 = (f0 / d) * 0.5f + 0.5f;
    f1 = (f1 / d) * 0.5f + 0.5f;
    f2 = (f2 / d) * 0.5f + 0.5f;
    float tx, ty;
    switch (face) {
        case 0: tx = f0; ty = (float)(1.0 - (double)f2); break;
        case 1: tx = (float)(1.0 - (double)f1); ty = (float)(1.0 - (double)f2); break;
        case 2: tx = f0; ty = f1; break;
        case 3: tx = f2; ty = f1; break;
        case 4: tx = (float)(1.0 - (double)f1); ty = (float)(1.0 - (double)f0); break;
        default: tx = f2; ty = (float)(1.0 - (double)f0); break;
    }
    X = (float)face + tx;
    Y = ty;
}

// One loop position of MercatorToCubic (:350-372) / CubicToMercator (:423-446): the flat
// texel it loads from and the one it stores to (~0 when the store falls outside).
struct RemapPos { size_t load, store; uint32_t key; };
__device__ RemapPos remap_pos(uint32_t col, uint32_t py, uint32_t W, uint32_t H, int load_as) {
    const uint32_t wid0 = W / 4 + 1;
    const uint32_t b = min(col / wid0, 3u), px = col - b * wid0;
    float lx, ly, sx, sy;
    if (load_as == 0) {
        const float y = (float)((double)py / (double)H);
        float x = (float)((double)(6u * col) / (double)W);
        xy_to_uv(x, y, lx, ly);
        x = (float)((double)x / 6.0);
        sx = x; sy = y;
    } else {
        const float V = (float)py / (float)H, U = (float)col / (float)W;
        float x, y;
        uv_to_xy(U, V, x, y);
        x /= 6.0f;
        lx = x; ly = y;
        sx = U; sy = V;
    }
    const size_t n = (size_t)W * H;
    RemapPos r;
    r.load = (size_t)u32_of(lx * (float)W) + (size_t)u32_of(ly * (float)H) * W;
    if (r.load >= n) r.load = n - 1;
    r.store = (size_t)u32_of(sx * (float)W) + (size_t)u32_of(sy * (float)H) * W;
    if (r.store >= n) r.store = ~(size_t)0;
    r.key = (b * H + py) * wid0 + px + 1u;  // sequential loop order (batch, row, column)
    return r;
}

__global__ __launch_bounds__(kTB) void k_remap_claim(uint32_t W, uint32_t H, int load_as, uint32_t *claim) {
    const uint32_t i = blockIdx.x * kTB + threadIdx.x;
    if (i >= W * H) return;  // no cross-lane work in this kernel
    const RemapPos r = remap_pos(i % W, i / W, W, H, load_as);
    if (r.store != ~(size_t)0) atomicMax(claim + r.store, r.key);
}

__global__ __launch_bounds__(kTB) void k_remap_write(uint32_t W, uint32_t H, int C, int load_as,
                                                     const uint32_t *claim, const uint8_t *in, uint8_t *out) {
    const uint32_t i = blockIdx.x * kTB + threadIdx.x;
    if (i >= W * H) return;  // no cross-lane work in this kernel
    const RemapPos r = remap_pos(i % W, i / W, W, H, load_as);
    if (r.store == ~(size_t)0 || claim[r.store] != r.key) return;
    for (int c = 0; c < C; c++) {
        const float v = (float)in[r.load * C + c] / 255.0f;  // pixelLoad :285
        out[r.store * C + c] = to_u8((double)v * 255.9999);  // pixelStore :299
    }
}

}  // namespace

bool noise_batches_exact(uint32_t W) {
    if (W == 0) return false;
    const uint32_t wid = W / 4 + 1;
    const long long last = (long long)wid - (long long)((4ull * wid) % W);
    return last >= 0 && 3 * (long long)wid + last == (long long)W;
}

size_t noise_workspace_bytes(int W, int H) { return 16 + (size_t)W * (size_t)H * sizeof(float); }

hipError_t noise_texture(int W, int H, int type, const float *grad, int n_grad, float freq, float lac, float gain,
                         int octaves, uint8_t *d_rgb, void *d_ws, hipStream_t s) {
    NoiseArgs a{};
    a.type = type; a.octaves = octaves; a.freq = freq; a.lac = lac; a.gain = gain;
    // a short gradient list gets 0 in front, then 1 at the end (utility.h:72-77)
    int G = 0;
    if (n_grad < 2) { a.grad[0] = a.grad[1] = a.grad[2] = 0.0f; G = 1; }
    for (int k = 0; k < 3 * n_grad; k++) a.grad[3 * G + k] = grad[k];
    G += n_grad;
    if (G < 2) { a.grad[3] = a.grad[4] = a.grad[5] = 1.0f; G = 2; }
    a.n_grad = G;
    uint32_t *ws = static_cast<uint32_t *>(d_ws);
    const unsigned blocks = unsigned(((size_t)W * H + kTB - 1) / kTB);
    hipLaunchKernelGGL(k_noise_init, dim3(1), dim3(1), 0, s, ws);
    hipLaunchKernelGGL(k_noise_eval, dim3(blocks), dim3(kTB), 0, s, W, H, a, ws);
    hipLaunchKernelGGL(k_noise_color, dim3(blocks), dim3(kTB), 0, s, W, H, a, ws, d_rgb);
    return hipGetLastError();
}

size_t remap_workspace_bytes(int W, int H) { return (size_t)W * (size_t)H * sizeof(uint32_t); }

hipError_t texture_remap(const uint8_t *d_in, int W, int H, int C, int load_as, uint8_t *d_out, void *d_ws,
                         hipStream_t s) {
    const size_t n = (size_t)W * H;
    hipError_t e = hipMemsetAsync(d_ws, 0, n * sizeof(uint32_t), s);
    if (e == hipSuccess) e = hipMemsetAsync(d_out, 0, n * (size_t)C, s);
    if (e != hipSuccess) return e;
    const unsigned blocks = unsigned((n + kTB - 1) / kTB);
    uint32_t *claim = static_cast<uint32_t *>(d_ws);
    hipLaunchKernelGGL(k_remap_claim, dim3(blocks), dim3(kTB), 0, s, (uint32_t)W, (uint32_t)H, load_as, claim);
    hipLaunchKernelGGL(k_remap_write, dim3(blocks), dim3(kTB), 0, s, (uint32_t)W, (uint32_t)H, C, load_as,
                       (const uint32_t *)claim, d_in, d_out);
    return hipGetLastError();
}

}  // namespace rtk
