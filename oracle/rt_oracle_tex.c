/*
 * rt_oracle_tex.c -- CPU ORACLE for the texture producers of SURVEY 8f2.  TEST
 * INFRASTRUCTURE ONLY (see rt_oracle.h).
 *
 *   orc_noise_texture  <- Helper::Noise::MakeTexture<glm::vec3>   Utilities/utility.h:69-192
 *                         Snoise2 / Fbm2 / Turbulance, perm[]      Utilities/utility.cpp:609-769
 *   orc_texture_remap  <- TEXTURE_2D::LoadFromDiskToGPU(loc, loadAs, mapTo)  utility.cpp:266-463
 *
 * These are host C++ in the reference, so the numerics are C's, not GLSL's: a/b is a true
 * division, `x - 1.0 + 2.0*G2` is evaluated in double, float -> uint8 truncates.  The only
 * transcendentals (the remap's acosf / atan2f / cosf / sinf) are evaluated as
 * RN_float(f(double)) with the double-precision routines below: parity with the
 * reference's libm is unpinned (its last-ulp behaviour is the platform's), the GPU kernels
 * restate the same routines operation for operation.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "rt_oracle.h"

/* ---------------------------------------------------------------- noise (utility.cpp:609-769) */
static const uint8_t kPerm[256] = {
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

/* fastFloor utility.cpp:611 -- note int(x) - 1 for integral x (kept) */
static int fast_floor(float x) { return ((float)(int)x < x) ? (int)x : (int)x - 1; }

/* grad2 utility.cpp:636-653.  `h & 1 != 0` and `h&2 != 0` both parse as h & (1): the second
 * test is bit 0 as well (kept). */
static float grad2(uint8_t hash, float x, float y) {
    const uint8_t h = hash & 7;
    float u = y, v = 2 * x;
    if (h < 4) { u = x; v = 2 * y; }
    if (h & 1) u = -u;
    if (h & 1) v = -v;
    return u + v;
}

/* Snoise2 utility.cpp:657-737 */
static float snoise2(float x, float y) {
    const float F2 = 0.366025403f, G2 = 0.211324865f;
    float n0, n1, n2;
    const float s = (x + y) * F2;
    const float xs = x + s, ys = y + s;
    const int i = fast_floor(xs), j = fast_floor(ys);
    const float t = (float)(i + j) * G2;
    const float X0 = (float)i - t, Y0 = (float)j - t;
    const float x0 = x - X0, y0 = y - Y0;
    uint8_t i1, j1;
    if (x0 > y0) { i1 = 1; j1 = 0; } else { i1 = 0; j1 = 1; }
    const float x1 = x0 - (float)i1 + G2, y1 = y0 - (float)j1 + G2;
    const float x2 = (float)((double)x0 - 1.0 + 2.0 * (double)G2);
    const float y2 = (float)((double)y0 - 1.0 + 2.0 * (double)G2);
    const uint8_t ii = (uint8_t)i, jj = (uint8_t)j;
    float t0 = (float)(0.5 - (double)(x0 * x0) - (double)(y0 * y0));
    if (t0 < 0.0f) n0 = 0.0f;
    else {
        t0 *= t0;
        uint8_t tmp = jj;
        tmp = (uint8_t)(ii + kPerm[tmp]);
        n0 = t0 * t0 * grad2(kPerm[tmp], x0, y0);
    }
    float t1 = (float)(0.5 - (double)(x1 * x1) - (double)(y1 * y1));
    if (t1 < 0.0f) n1 = 0.0f;
    else {
        t1 *= t1;
        uint8_t tmp = (uint8_t)(jj + j1);
        tmp = (uint8_t)(ii + i1 + kPerm[tmp]);
        n1 = t1 * t1 * grad2(kPerm[tmp], x1, y1);
    }
    float t2 = (float)(0.5 - (double)(x2 * x2) - (double)(y2 * y2));
    if (t2 < 0.0f) n2 = 0.0f;
    else {
        t2 *= t2;
        uint8_t tmp = (uint8_t)(jj + 1);
        tmp = (uint8_t)(ii + 1 + kPerm[tmp]);
        n2 = t2 * t2 * grad2(kPerm[tmp], x2, y2);
    }
    return n0 + n1 + n2;
}

/* Turbulance utility.cpp:741-755, Fbm2 :758-767 */
static float noise_at(int type, float x, float y, float freq, float lac, float gain, int octaves) {
    if (type == 0) return snoise2(x * freq, y * freq);
    float sum = 0, amp = 1.0f;
    for (int i = 0; i < octaves; i++) {
        float f = snoise2(x * freq, y * freq) * amp;
        if (type == 2 && f < 0) f = -f;
        sum += f;
        freq *= lac;
        amp *= gain;
    }
    return sum;
}

/* the reference's column batches (utility.h:96-101) tile [0, width) exactly only for some
 * widths (600 does); others index out of bounds there, and are rejected here */
static int noise_batches_exact(uint32_t W) {
    const uint32_t wid = W / 4 + 1;
    const long long last = (long long)wid - (long long)((4 * wid) % W);
    return last >= 0 && 3 * (long long)wid + last == (long long)W;
}

/* double -> uint8_t of the reference's `pixel = 255.999*color` (x86-64: truncate to int32,
 * keep the low byte) */
static uint8_t to_u8(double v) {
    if (!(v > -2147483648.0 && v < 2147483648.0)) return 0;
    return (uint8_t)(uint32_t)(int32_t)v;
}

int orc_noise_texture(int width, int height, int type, const float *gradient, int n_grad, float freq,
                      float lac, float gain, int octaves, uint8_t *rgb_out) {
    if (width <= 0 || height <= 0 || type < 0 || type > 2 || octaves < 0 || !rgb_out || n_grad < 0 || n_grad > 64)
        return -1;
    if (n_grad > 0 && !gradient) return -1;
    if (!noise_batches_exact((uint32_t)width)) return -1;
    /* a short gradient list gets 0 in front, then 1 at the end (utility.h:72-77) */
    float g[3 * 66];
    int G = 0;
    if (n_grad < 2) { g[0] = g[1] = g[2] = 0.0f; G = 1; }
    memcpy(g + 3 * G, gradient ? gradient : g, sizeof(float) * 3 * (size_t)n_grad);
    G += n_grad;
    if (G < 2) { g[3] = g[4] = g[5] = 1.0f; G = 2; }
    const uint32_t W = (uint32_t)width, H = (uint32_t)height;
    float *noise = (float *)malloc(sizeof(float) * (size_t)W * H);
    if (!noise) return -1;
    /* the four column batches of `func` (utility.h:94-131); each starts from (1, 0) */
    float mn = 0, mx = 0;
    for (uint32_t b = 0; b < 4; b++) {
        uint32_t wid = W / 4 + 1;
        const uint32_t off = b * wid;
        if (b == 3) wid -= (4 * wid) % W;
        float bmn = 1.0f, bmx = 0.0f;
        for (uint32_t Y = 0; Y < H; Y++)
            for (uint32_t X = 0; X < wid; X++) {
                const uint32_t idx = off + X + Y * W;
                const float v = noise_at(type, (float)(X + off), (float)Y, freq, lac, gain, octaves);
                bmn = bmn > v ? v : bmn;  /* MIN(x,y) utility.h:10 */
                bmx = bmx > v ? bmx : v;  /* MAX(x,y) utility.h:11 */
                noise[idx] = v;
            }
        if (b == 0) { mn = bmn; mx = bmx; }
        else { mn = mn > bmn ? bmn : mn; mx = mx > bmx ? mx : bmx; }
    }
    if (!(mx - mn != 0.0f)) { free(noise); return -1; } /* degenerate range: the reference divides by 0 */
    /* func2 utility.h:151-180 */
    const float gdw = (float)(1.0 / (double)(G - 1));
    for (size_t k = 0; k < (size_t)W * H; k++) {
        float factor = (noise[k] - mn) / (mx - mn);
        uint32_t region = (uint32_t)(factor * (float)(G - 1));
        if (region > (uint32_t)(G - 2)) region = (uint32_t)(G - 2);
        factor = (factor - (float)(int)(factor / gdw) * gdw) * (float)(G - 1); /* MOD utility.h:13 */
        for (int c = 0; c < 3; c++) {
            const float a = g[3 * region + c], d = g[3 * (region + 1) + c] - a;
            const float col = a + d * factor;
            rgb_out[k * 3 + c] = to_u8(255.999 * (double)col);
        }
    }
    free(noise);
    return 0;
}

/* ------------------------------------------------- double-precision transcendentals
 * Written with +, -, *, / and sqrt only, in a fixed order, so that the GPU kernels
 * (rt_texture.hip) reproduce them bit for bit; accurate to a few double ulps
 * (tests/test_textures.py checks them against libm), hence RN_float(f(double)) is the
 * correctly rounded float result except in double-rounding corner cases. */
static const double kPio2_1 = 0x1.921fb544p+0, kPio2_1t = 0x1.0b4611a626331p-34;  /* Cody-Waite pi/2 */
static const double kPi = 0x1.921fb54442d18p+1, kPiLo = 0x1.1a62633145c07p-53;
static const double kPio2 = 0x1.921fb54442d18p+0, kPio2Lo = 0x1.1a62633145c07p-54;
static const double kPio6 = 0x1.0c152382d7365p-1, kSqrt3 = 0x1.bb67ae8584caap+0;
static const double kTanPi12 = 0x1.126145e9ecd58p-2, k2OverPi = 0x1.45f306dc9c883p-1;

/* atan(x), x >= 0: atan(x) = pi/2 - atan(1/x) above 1, pi/6 + atan((x*sqrt3 - 1)/(sqrt3 + x))
 * above tan(pi/12), then the odd Taylor series to x^35 */
static double dm_atan_pos(double x) {
    int inv = 0;
    double base = 0.0;
    if (x > 1.0) { x = 1.0 / x; inv = 1; }
    if (x > kTanPi12) { x = (x * kSqrt3 - 1.0) / (kSqrt3 + x); base = kPio6; }
    const double x2 = x * x;
    double p = 0.0;
    for (int k = 17; k >= 0; k--) p = p * x2 + ((k & 1) ? -1.0 : 1.0) / (double)(2 * k + 1);
    double r = base + x * p;
    if (inv) r = (kPio2 - r) + kPio2Lo;
    return r;
}
static double dm_atan2(double y, double x) {
    if (y != y || x != x) return x + y;
    if (y == 0.0) {
        if (x > 0.0 || (x == 0.0 && !signbit(x))) return y;
        return signbit(y) ? -(kPi + kPiLo) : kPi + kPiLo;
    }
    if (x == 0.0) return y > 0.0 ? kPio2 + kPio2Lo : -(kPio2 + kPio2Lo);
    double a = dm_atan_pos(fabs(y) / fabs(x));
    if (x < 0.0) a = (kPi - a) + kPiLo;
    return y < 0.0 ? -a : a;
}
static double dm_acos(double x) { return dm_atan2(sqrt((1.0 - x) * (1.0 + x)), x); }
/* sin and cos: k = round(x * 2/pi), r = (x - k*pio2_1) - k*pio2_1t, nested Taylor products
 * to r^23 / r^22, quadrant swap */
static void dm_sincos(double x, double *s_out, double *c_out) {
    const double kf = floor(x * k2OverPi + 0.5);
    const double r = (x - kf * kPio2_1) - kf * kPio2_1t, r2 = r * r;
    double s = 1.0, c = 1.0;
    for (int n = 22; n >= 2; n -= 2) {
        s = 1.0 - r2 / (double)(n * (n + 1)) * s;
        c = 1.0 - r2 / (double)((n - 1) * n) * c;
    }
    s = r * s;
    const long long q = ((long long)kf % 4 + 4) % 4;
    double so = s, co = c;
    if (q == 1) { so = c; co = -s; }
    else if (q == 2) { so = -s; co = -c; }
    else if (q == 3) { so = -c; co = s; }
    *s_out = so; *c_out = co;
}
static float f_acos(float x) { return (float)dm_acos((double)x); }
static float f_atan2(float y, float x) { return (float)dm_atan2((double)y, (double)x); }
static float f_sin(float x) { double s, c; dm_sincos((double)x, &s, &c); return (float)s; }
static float f_cos(float x) { double s, c; dm_sincos((double)x, &s, &c); return (float)c; }

/* exported for the accuracy tests only */
double orc_dm_atan2(double y, double x) { return dm_atan2(y, x); }
double orc_dm_acos(double x) { return dm_acos(x); }
void orc_dm_sincos(double x, double *s, double *c) { dm_sincos(x, s, c); }

/* ----------------------------------------------------------------- re-projection
 * utility.cpp:266-463.  Both directions loop over destination-side coordinates in the
 * four column batches, read the source texel at the mapped position (pixelLoad :273-287)
 * and write the destination texel at the loop position (pixelStore :289-302).  Defined
 * here where the reference is undefined:
 *   - the destination starts zeroed (the reference's buffer is uninitialised, and its
 *     store position can skip a texel when float rounding maps two loop columns to one);
 *   - when two loop positions store to one texel, the later one in sequential loop order
 *     (batch, row, column) wins (the reference races four threads);
 *   - a load past the last texel reads the last texel; a store past it is dropped. */
static uint32_t u32_of(float v) { return v <= 0.0f ? 0u : (v >= 4294967040.0f ? 0xffffffffu : (uint32_t)v); }

/* XYtoUVCoord utility.cpp:306-349 (MERCATOR -> CUBIC) */
static void xy_to_uv(float X, float Y, float *U, float *V) {
    const float x = X - (float)(int)X;
    float fx = 0, fy = 0, fz = 0;
    switch ((int)X) {
        case 0: fx = x; fz = (float)(1.0 - (double)Y); fy = 1.0f; break;
        case 1: fy = (float)(1.0 - (double)x); fz = (float)(1.0 - (double)Y); fx = 1.0f; break;
        case 2: fx = x; fy = Y; fz = 1.0f; break;
        case 3: fz = x; fy = Y; fx = 0.0f; break;
        case 4: fy = (float)(1.0 - (double)x); fx = (float)(1.0 - (double)Y); fz = 0.0f; break;
        default: fz = x; fx = (float)(1.0 - (double)Y); fy = 0.0f; break;
    }
    fx -= 0.5f; fy -= 0.5f; fz -= 0.5f;
    const float inv = 1.0f / sqrtf(fx * fx + fy * fy + fz * fz); /* glm::normalize */
    fx *= inv; fy *= inv; fz *= inv;
    *V = f_acos(-fy) / 3.14159274f;        /* glm::pi<float>() */
    *U = f_atan2(fz, fx) / 6.28318548f;    /* float(2*glm::pi<double>()) */
    if (*U < 0) *U = (float)((double)*U + 1.0);
}

/* UVtoXYCoord utility.cpp:370-422 (CUBIC -> MERCATOR) */
static void uv_to_xy(float U, float V, float *X, float *Y) {
    const float rad = (float)0.01745329251994329576923690768489; /* glm::radians */
    const float pitch = (V * 180.0f - 90.0f) * rad;
    const float yaw = (U * 360.0f) * rad;
    float f[3];
    f[0] = f_cos(yaw) * f_cos(pitch);
    f[1] = f_sin(pitch);
    f[2] = f_sin(yaw) * f_cos(pitch);
    float mx = f[0];
    uint32_t face = mx > 0 ? 1u : 3u;
    float fd[3] = {1.0f, 0.0f, 0.0f};
    for (int k = 0; k < 3; k++) fd[k] *= (float)(mx > 0 ? 1 : -1);
    for (int i = 1; i < 3; i++) {
        if (fabsf(mx) < fabsf(f[i])) {
            mx = f[i];
            face = mx > 0 ? (i == 1 ? 0u : 2u) : (i == 1 ? 5u : 4u);
            fd[0] = 0.0f; fd[1] = (float)(i == 1); fd[2] = (float)(i == 2);
            for (int k = 0; k < 3; k++) fd[k] *= (float)(mx > 0 ? 1 : -1);
        }
    }
    const float d = f[0] * fd[0] + f[1] * fd[1] + f[2] * fd[2];
    for (int k = 0; k < 3; k++) { f[k] /= d; f[k] *= 0.5f; f[k] += 0.5f; }
    float tx, ty;
    switch (face) {
        case 0: tx = f[0]; ty = (float)(1.0 - (double)f[2]); break;
        case 1: tx = (float)(1.0 - (double)f[1]); ty = (float)(1.0 - (double)f[2]); break;
        case 2: tx = f[0]; ty = f[1]; break;
        case 3: tx = f[2]; ty = f[1]; break;
        case 4: tx = (float)(1.0 - (double)f[1]); ty = (float)(1.0 - (double)f[0]); break;
        default: tx = f[2]; ty = (float)(1.0 - (double)f[0]); break;
    }
    *X = (float)face + tx;
    *Y = ty;
}

int orc_texture_remap(const uint8_t *in, int width, int height, int channels, int load_as, int map_to,
                      uint8_t *out) {
    if (!in || !out || width <= 0 || height <= 0 || (channels != 3 && channels != 4)) return -1;
    if (load_as < 0 || load_as > 1 || map_to < 0 || map_to > 1) return -1;
    const uint32_t W = (uint32_t)width, H = (uint32_t)height, C = (uint32_t)channels;
    const size_t n = (size_t)W * H;
    if (load_as == map_to) { memcpy(out, in, n * C); return 0; }
    if (!noise_batches_exact(W)) return -1;
    memset(out, 0, n * C);
    for (uint32_t b = 0; b < 4; b++) {
        uint32_t wid = W / 4 + 1;
        const uint32_t off = b * wid;
        if (b == 3) wid -= (4 * wid) % W;
        for (uint32_t py = 0; py < H; py++)
            for (uint32_t px = 0; px < wid; px++) {
                float lx, ly, sx, sy;  /* load position, store position (both in [0,1]^2) */
                if (load_as == 0) {    /* MERCATOR -> CUBIC, MercatorToCubic :350-372 */
                    const float y = (float)((double)py / (double)H);
                    float x = (float)((double)(6 * (px + off)) / (double)W);
                    xy_to_uv(x, y, &lx, &ly);
                    x = (float)((double)x / 6.0);
                    sx = x; sy = y;
                } else {               /* CUBIC -> MERCATOR, CubicToMercator :423-446 */
                    const float V = (float)py / (float)H, U = (float)(px + off) / (float)W;
                    float x, y;
                    uv_to_xy(U, V, &x, &y);
                    x /= 6.0f;
                    lx = x; ly = y;
                    sx = U; sy = V;
                }
                size_t li = (size_t)u32_of(lx * (float)W) + (size_t)u32_of(ly * (float)H) * W;
                if (li >= n) li = n - 1;
                const size_t si = (size_t)u32_of(sx * (float)W) + (size_t)u32_of(sy * (float)H) * W;
                if (si >= n) continue;
                for (uint32_t c = 0; c < C; c++) {
                    const float v = (float)in[li * C + c] / 255.0f;
                    out[si * C + c] = to_u8((double)v * 255.9999);
                }
            }
    }
    return 0;
}
