/*
 * rt_oracle_common.h -- GLSL 4.40 builtins restated under the numerics contract
 * (see rt_oracle.h).  TEST INFRASTRUCTURE ONLY.
 *
 * Every helper follows the GLSL definition (GLSL 4.40 spec sec. 8) with GLSL's left-to-
 * right evaluation order; the translation unit is compiled with -ffp-contract=off so no
 * multiply-add is ever fused.
 */
#ifndef RT_ORACLE_COMMON_H
#define RT_ORACLE_COMMON_H
#include <math.h>
#include <stdint.h>

typedef struct { float x, y, z; } v3;
typedef struct { v3 c[3]; } m3; /* column-major, c[col], as GLSL mat3 / glm::mat3 */

static inline v3 V3(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline float v3get(v3 v, int i) { return i == 0 ? v.x : (i == 1 ? v.y : v.z); }
static inline void v3set(v3 *v, int i, float f) { if (i == 0) v->x = f; else if (i == 1) v->y = f; else v->z = f; }
static inline v3 add(v3 a, v3 b) { return V3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return V3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 neg(v3 a) { return V3(-a.x, -a.y, -a.z); }
/* vec3 * float and float * vec3 (IEEE multiplication is commutative) */
static inline v3 mul(v3 a, float s) { return V3(a.x * s, a.y * s, a.z * s); }
static inline v3 mulv(v3 a, v3 b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
/* GLSL dot: ((a.x*b.x + a.y*b.y) + a.z*b.z) */
static inline float dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static inline v3 cross(v3 a, v3 b) {
    return V3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* contract: a/b == a * RN(1/b) */
static inline float rcp(float b) { return 1.0f / b; }
static inline float length(v3 v) { return sqrtf(dot(v, v)); }
static inline v3 normalize(v3 v) { return mul(v, 1.0f / sqrtf(dot(v, v))); }
/* GLSL mat3 * vec3: m[0]*v.x + m[1]*v.y + m[2]*v.z */
static inline v3 m3mul(m3 m, v3 v) { return add(add(mul(m.c[0], v.x), mul(m.c[1], v.y)), mul(m.c[2], v.z)); }
/* transpose(m) * v: component r = dot(m[r], v) */
static inline v3 m3tmul(m3 m, v3 v) { return V3(dot(m.c[0], v), dot(m.c[1], v), dot(m.c[2], v)); }
/* GLSL reflect(I, N) = I - 2.0 * dot(N, I) * N */
static inline v3 reflect3(v3 I, v3 N) { return sub(I, mul(N, 2.0f * dot(N, I))); }
/* GLSL refract(I, N, eta) */
static inline v3 refract3(v3 I, v3 N, float eta) {
    float d = dot(N, I);
    float k = 1.0f - eta * eta * (1.0f - d * d);
    if (k < 0.0f) return V3(0.0f, 0.0f, 0.0f);
    return sub(mul(I, eta), mul(N, eta * d + sqrtf(k)));
}
static inline float fmin_(float a, float b) { return fminf(a, b); }
static inline float fmax_(float a, float b) { return fmaxf(a, b); }
/* float -> uint as the contract defines it (negative -> 0) */
static inline uint32_t f2u(float f) { return f <= 0.0f ? 0u : (uint32_t)f; }

/* GLSL inverse(mat3) / glm::inverse, adjugate form (glm func_matrix.inl compute_inverse) */
static inline m3 m3inverse(m3 m) {
#define M(cc_, rr_) v3get(m.c[cc_], rr_)
    float det = +M(0, 0) * (M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2))
                - M(1, 0) * (M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2))
                + M(2, 0) * (M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2));
    float o = 1.0f / det;
    m3 r;
    r.c[0].x = +(M(1, 1) * M(2, 2) - M(2, 1) * M(1, 2)) * o;
    r.c[1].x = -(M(1, 0) * M(2, 2) - M(2, 0) * M(1, 2)) * o;
    r.c[2].x = +(M(1, 0) * M(2, 1) - M(2, 0) * M(1, 1)) * o;
    r.c[0].y = -(M(0, 1) * M(2, 2) - M(2, 1) * M(0, 2)) * o;
    r.c[1].y = +(M(0, 0) * M(2, 2) - M(2, 0) * M(0, 2)) * o;
    r.c[2].y = -(M(0, 0) * M(2, 1) - M(2, 0) * M(0, 1)) * o;
    r.c[0].z = +(M(0, 1) * M(1, 2) - M(1, 1) * M(0, 2)) * o;
    r.c[1].z = -(M(0, 0) * M(1, 2) - M(1, 0) * M(0, 2)) * o;
    r.c[2].z = +(M(0, 0) * M(1, 1) - M(1, 0) * M(0, 1)) * o;
#undef M
    return r;
}

/* Background_Color, identical in IOW-03 (03...glsl:123-126) and INW-01 (01_BVH...glsl:9-12);
 * INW-04 replaces both gradient ends by 0 when lights exist (04...glsl:23-30). */
static inline v3 background(v3 d, int black) {
    v3 lo = black ? V3(0, 0, 0) : V3(1.0f, 1.0f, 1.0f);
    v3 hi = black ? V3(0, 0, 0) : V3(0.3f, 0.4f, 1.0f);
    float t = (d.y + 1.0f) * 0.5f;
    return add(mul(lo, 1.0f - t), mul(hi, t));
}
#endif
