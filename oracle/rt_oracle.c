/*
 * rt_oracle.c -- CPU ORACLE (test infrastructure only; see rt_oracle.h for the rules,
 * the parity status and the numerics contract).
 *
 * Paths below are relative to /root/reference/Raytracing-Sandbox/Src/.
 *   "03.glsl"  = In-One-Weekend/03_Shadows_and_Materials/computeShaderSrc.glsl
 *   "01.glsl"  = In-One-Weekend/01_Adding_Sphere/computeShaderSrc.glsl
 *   "BVH.glsl" = In-Next-Week/01_BoundingVolumeHierarchy/computeShaderSrc.glsl
 *   "04.glsl"  = In-Next-Week/04_Lights_Camera_And_Action/computeShaderSrc.glsl
 *   "02.glsl"  = In-One-Weekend/02_Groups/computeShaderSrc.glsl
 *   "base.cpp" = In-One-Weekend/base.cpp (the default compute shader, IOW-00)
 */
#include "rt_oracle.h"
#include "rt_oracle_common.h"

#include <stdlib.h>
#include <string.h>
#include <time.h>
#ifdef _OPENMP
#include <omp.h>
#endif

static int g_threads = 0;
int orc_num_threads(void) {
#ifdef _OPENMP
    return g_threads > 0 ? g_threads : omp_get_max_threads();
#else
    return 1;
#endif
}
void orc_set_threads(int n) { g_threads = n; }

static double now_ms(void) {
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec * 1e3 + ts.tv_nsec * 1e-6;
}

typedef struct { uint64_t seg, nodes, prims, shadow, drops, nans; } ctr;
static void ctr_add(orc_stats *st, const ctr *c) {
    st->segments += c->seg; st->node_visits += c->nodes; st->prim_tests += c->prims;
    st->shadow_queries += c->shadow; st->stack_drops += c->drops; st->nan_drops += c->nans;
}

/* ===================================================================================
 * Sample tables.  The shaders evaluate cos/sin of the golden angle per sample; under the
 * contract they are evaluated once in double precision and rounded to float.
 * =================================================================================== */
#define SHADER_PI 3.1415926538 /* #define PI 3.1415926538 (03.glsl:26, BVH.glsl:13) */

int orc_sample_tables(int spp, float *sunflower, float *fib, int *ring) {
    if (spp < 1) return -1;
    const double PHI = SHADER_PI * (3.0 - sqrt(5.0)); /* 03.glsl:27, BVH.glsl:14 */
    const double b = floor(2.0 * sqrt((double)spp) + 0.5); /* round(2*sqrt(max_pt)) */
    for (int i = 0; i < spp; i++) {
        double th = PHI * (double)i;
        if (sunflower) {
            /* sunflower_distr 03.glsl:153-163 / SunflowerDistribution BVH.glsl:15-27 with
             * aperture factored out: r = 1 (outer ring) or sqrt((i-0.5)/(n-(b+1)/2)). */
            if (i == 0) { sunflower[0] = 0.0f; sunflower[1] = 0.0f; }
            else {
                double rho = ((double)i > (double)spp - b) ? 1.0
                             : sqrt(((double)i - 0.5) / ((double)spp - (b + 1.0) / 2.0));
                sunflower[2 * i + 0] = (float)(rho * cos(th));
                sunflower[2 * i + 1] = (float)(rho * sin(th));
            }
        }
        if (fib) {
            /* fibonacciHemiSpherePtDirn 03.glsl:164-172 before the scatteritivity scaling */
            double y = 1.0 - ((double)i / (double)(spp - 1));
            double radius = sqrt(1.0 - y * y);
            fib[3 * i + 0] = (float)(cos(th) * radius);
            fib[3 * i + 1] = (float)y;
            fib[3 * i + 2] = (float)(sin(th) * radius);
        }
    }
    if (ring) {
        /* 03.glsl:366-368 and 383-397: ring-ordered stratified sub-pixel indices */
        int grid = 1;
        while (grid * grid < spp) grid++;
        int focus = 0, x = 0, y = 0;
        for (int s = 0; s < spp; s++) {
            if (focus < grid) {
                if (x == 0 && y == 0) { focus++; x = focus; y = focus; ring[2 * s] = focus; ring[2 * s + 1] = focus; }
                else if (x < y) { y--; ring[2 * s] = focus; ring[2 * s + 1] = y; }
                else { x--; ring[2 * s] = x; ring[2 * s + 1] = focus; }
            } else { ring[2 * s] = -1; ring[2 * s + 1] = -1; } /* early-return marker */
        }
    }
    return 0;
}

/* ===================================================================================
 * IOW-01: 01.glsl:98-146
 * =================================================================================== */
int orc_render_iow01(const orc_camera *cam, const float sphere[4], const orc_params *p,
                     float *rgba, orc_stats *st) {
    if (!cam || !sphere || !p || !rgba || p->width <= 0 || p->height <= 0) return -1;
    double t0 = now_ms();
    const int W = p->width, H = p->height;
    int x0 = p->tile_x0, y0 = p->tile_y0, tw = p->tile_w, th = p->tile_h;
    if (tw <= 0 || th <= 0) { x0 = 0; y0 = 0; tw = W; th = H; }
    const v3 D = V3(cam->dir[0], cam->dir[1], cam->dir[2]);
    const v3 P = V3(cam->pos[0], cam->pos[1], cam->pos[2]);
    const v3 C = V3(sphere[0], sphere[1], sphere[2]);
    const float R = sphere[3];
#pragma omp parallel for schedule(dynamic, 1) num_threads(orc_num_threads())
    for (int yy = y0; yy < y0 + th; yy++) {
        for (int xx = x0; xx < x0 + tw; xx++) {
            if (xx < 0 || yy < 0 || xx >= W || yy >= H) continue;
            float aspect = (float)W * rcp((float)H);                       /* :101 */
            v3 up = V3(0, 1, 0);
            v3 cr = cross(D, up), cu = cross(cr, D);                       /* :103-104 */
            float sx = ((float)xx * 2.0f - (float)W) * rcp(2.0f * (float)W); /* :105 */
            sx *= aspect;
            float sy = ((float)yy * 2.0f - (float)H) * rcp(2.0f * (float)H); /* :107 */
            v3 pis = add(add(add(P, mul(D, cam->focus_dist)), mul(cr, sx)), mul(cu, sy)); /* :109 */
            /* CreatePlane((0,-2,0),(0,-2,1),(1,-2,0)) :39-45,112 */
            v3 p1 = V3(0, -2, 0), p2 = V3(0, -2, 1), p3 = V3(1, -2, 0);
            v3 pn = normalize(cross(sub(p2, p1), sub(p3, p1)));
            float pw = -(pn.x * p1.x + pn.y * p1.y + pn.z * p1.z);
            v3 ro = P, rd = normalize(sub(pis, P));                          /* CreateRay :35-38 */
            v3 color = background(rd, 0);                                    /* RayColor :92-96 */
            float min_depth = 10000.0f;
            { /* plane :121-125, t_RayXPlane :65-70 */
                float t = -(pn.x * ro.x + pn.y * ro.y + pn.z * ro.z + pw)
                          * rcp(pn.x * rd.x + pn.y * rd.y + pn.z * rd.z);
                if (min_depth > t && t > 0) { color = V3(0.8f, 0.1f, 0.7f); min_depth = t; }
            }
            { /* sphere :127-132, t_RayXSphere :76-86 */
                v3 rs = sub(ro, C);
                float hb = dot(rd, rs), a = dot(rd, rd), c = dot(rs, rs) - R * R;
                float det = hb * hb - a * c;
                float t = (det > 0 && hb < 0) ? ((-hb - sqrtf(det)) * rcp(a)) : -1.0f;
                if (min_depth > t && t > 0) {
                    v3 ip = add(ro, mul(rd, t));
                    color = p->show_normal ? normalize(sub(ip, C)) : V3(1, 0, 0);
                    min_depth = t;
                }
            }
            float *o = rgba + ((size_t)yy * W + xx) * 4;
            o[0] = color.x; o[1] = color.y; o[2] = color.z; o[3] = 1.0f;
        }
    }
    if (st) { memset(st, 0, sizeof(*st)); st->segments = (uint64_t)tw * th; st->ms = now_ms() - t0; }
    return 0;
}

/* ===================================================================================
 * IOW-03: 03.glsl
 * =================================================================================== */
#define IOW_CUBOID 1    /* 03.glsl:24 */
#define IOW_ELLIPSOID 2 /* 03.glsl:25 */

typedef struct { v3 o, d; } ray_t;

/* t_RayXObj 03.glsl:55-95 (identical to t_RayXGeom BVH.glsl:112-155) */
static float t_ray_obj(ray_t r, int type, v3 s) {
    float t = -1.0f;
    if (type == 2 /* ellipsoid, caller maps codes */) {
        v3 is = V3(rcp(s.x), rcp(s.y), rcp(s.z));
        v3 a2 = mulv(r.o, is), a3 = mulv(r.d, is);
        float hb = dot(a2, a3), a = dot(a3, a3), c = dot(a2, a2) - 1.0f;
        float det = hb * hb - a * c;
        if (det > 0) {
            float ia = rcp(a), sq = sqrtf(det);
            float t0 = (-hb - sq) * ia, t1 = (-hb + sq) * ia;
            t = (t0 > t1 || t0 < 0) ? t1 : t0;
        }
    } else if (type == 1 /* cuboid */) {
        v3 bmin = mul(neg(s), 0.5f), bmax = mul(s, 0.5f);
        float t1 = (bmin.x - r.o.x) * rcp(r.d.x), t2 = (bmax.x - r.o.x) * rcp(r.d.x);
        float tmin = fmin_(t1, t2), tmax = fmax_(t1, t2);
        for (int i = 1; i < 3; ++i) {
            float id = rcp(v3get(r.d, i));
            t1 = (v3get(bmin, i) - v3get(r.o, i)) * id;
            t2 = (v3get(bmax, i) - v3get(r.o, i)) * id;
            tmin = fmax_(tmin, fmin_(fmin_(t1, t2), tmax));
            tmax = fmin_(tmax, fmax_(fmax_(t1, t2), tmin));
        }
        t = tmax > tmin ? (tmin > 0 ? tmin : tmax) : -1.0f;
    }
    return t > 0 ? t : -1.0f;
}

/* cuboid face normal, shared by 03.glsl:101-119 and BVH.glsl:165-182 */
static v3 cuboid_normal(v3 h, v3 s) {
    float md = fabsf(h.x - s.x * 0.5f);
    int index = 0;
    float dist = fabsf(h.x + s.x * 0.5f);
    if (md > dist) { md = dist; index = 1; }
    for (int i = 1; i < 3; ++i) {
        dist = fabsf(v3get(h, i) - v3get(s, i) * 0.5f);
        if (md > dist) { md = dist; index = i * 2; }
        dist = fabsf(v3get(h, i) + v3get(s, i) * 0.5f);
        if (md > dist) { md = dist; index = i * 2 + 1; }
    }
    v3 r = V3(0, 0, 0);
    v3set(&r, index / 2, index % 2 == 0 ? 1.0f : -1.0f);
    return r;
}

/* SurfaceNormal 03.glsl:96-122 (IOW ellipsoid "normal" is h/s*s, not h/s^2) */
static v3 iow_normal(float t, ray_t r, int type, v3 s) {
    v3 h = add(r.o, mul(r.d, t));
    if (type == 2) return V3(h.x * rcp(s.x) * s.x, h.y * rcp(s.y) * s.y, h.z * rcp(s.z) * s.z);
    if (type == 1) return cuboid_normal(h, s);
    return V3(0, 0, 0);
}

typedef struct {
    v3 point, normal, reflected, material, color;
    float scat[2];
} rrd_t; /* RayReturnData 03.glsl:38-47 */

typedef struct {
    const float *types, *rec;
    uint32_t n;
    const float *sf, *fib;
    const int *ring;
    int spp, max_bounces;
} iow_scene;

static m3 rec_m3(const float *r) {
    m3 m;
    m.c[0] = V3(r[0], r[1], r[2]); m.c[1] = V3(r[3], r[4], r[5]); m.c[2] = V3(r[6], r[7], r[8]);
    return m;
}

/* LaunchRay 03.glsl:196-256 */
static rrd_t launch_ray(const iow_scene *S, v3 go, v3 gd, float max_t, float contrib, ctr *c) {
    float min_t = max_t;
    m3 rot_hit = {{{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}};
    rrd_t data;
    memset(&data, 0, sizeof(data));
    v3 final_td = V3(0, 0, 0);
    c->seg++;
    for (uint32_t j = 0; j < S->n; j++) {
        c->prims++;
        int type = (int)S->types[j];                       /* :203 */
        const float *R = S->rec + (size_t)j * 24;
        v3 pos = V3(R[0], R[1], R[2]);                     /* :204 */
        m3 M = rec_m3(R + 3);                              /* :205-207 */
        v3 scale = V3(R[12], R[13], R[14]);                /* :208 */
        v3 to = m3mul(M, sub(go, pos));                    /* :210 */
        v3 td = m3mul(M, gd);                              /* :211 */
        ray_t tr = {to, normalize(td)};                    /* :212 */
        int t3 = type == IOW_ELLIPSOID ? 2 : (type == IOW_CUBOID ? 1 : 0);
        float t = t_ray_obj(tr, t3, scale);                /* :213 */
        if (min_t > t && t > 0) {                          /* :216-226 */
            data.normal = iow_normal(t, tr, t3, scale);
            data.color = V3(R[15], R[16], R[17]);
            data.material = V3(R[18], R[19], R[20]);
            data.scat[0] = R[21]; data.scat[1] = R[22];
            final_td = td;
            rot_hit = M;
            min_t = t;
        }
    }
    if (min_t < max_t) {                                   /* :228-253 */
        int inside = dot(data.normal, final_td) > 0;
        v3 n_ = inside ? neg(data.normal) : data.normal;
        data.reflected = reflect3(final_td, n_);
        if (!inside) {
            v3 nir = normalize(cross(n_, final_td));
            v3 nn = normalize(cross(nir, n_));
            float s = inside ? data.scat[0] : data.scat[1];
            float k = 1.0f / sqrtf(1.0f + s * s);
            v3 max_reflect = add(mul(n_, s * k), mul(nn, k));
            data.reflected = (dot(data.reflected, n_) > dot(max_reflect, n_)) ? data.reflected : max_reflect;
        }
        m3 inv = m3inverse(rot_hit);                       /* :248 */
        data.point = add(go, mul(gd, min_t));              /* :250 */
        data.normal = normalize(m3mul(inv, data.normal));
        data.reflected = normalize(m3mul(inv, data.reflected));
        data.color = mul(data.color, contrib);
    } else {
        data.point = V3(0, 0, 0); data.normal = V3(0, 0, 0);
    }
    return data;
}

/* fibonacciHemiSpherePtDirn 03.glsl:164-184 (table part precomputed) */
static v3 fib_dir(const iow_scene *S, int idx, float s, v3 focus) {
    float x = S->fib[3 * idx + 0], y = S->fib[3 * idx + 1], z = S->fib[3 * idx + 2];
    x *= s; y *= s; z *= s;
    v3 yc = focus;
    v3 zc = normalize(cross(V3(0, 1.0f, 0), yc));
    v3 xc = normalize(cross(yc, zc));
    v3 pt = add(focus, add(add(mul(xc, x), mul(yc, y)), mul(zc, z)));
    return normalize(pt);
}

static float schlick(float cosine, float ri) { /* 03.glsl:185-190 */
    float r0 = (1.0f - ri) * rcp(1.0f + ri);
    r0 = r0 * r0;
    float q = 1.0f - cosine;
    float q5 = q * q * q * q * q;
    return r0 + (1.0f - r0) * q5;
}

#define IOW_STACK 4 /* stack_capacity 03.glsl:258 */
typedef struct {
    ray_t ray[IOW_STACK];
    float contrib[IOW_STACK], ri[IOW_STACK];
    int bounce[IOW_STACK];
    int size;
} iow_stack; /* per-invocation globals 03.glsl:260-264, persist across samples of a pixel */

static void iow_push(iow_stack *k, ray_t r, float c, float ri, int b, ctr *cc) {
    if (k->size < IOW_STACK) {
        k->ray[k->size] = r; k->contrib[k->size] = c; k->ri[k->size] = ri; k->bounce[k->size] = b;
        k->size++;
    } else cc->drops++;
}

/* LaunchRays 03.glsl:285-358 */
static v3 launch_rays(const iow_scene *S, iow_stack *K, v3 ro, v3 rd, int sidx, ctr *c) {
    ray_t r0 = {ro, rd};
    iow_push(K, r0, 1.0f, 1.0f, 0, c);
    v3 sample = V3(0, 0, 0);
    int skip = 0;
    while (K->size > 0) {
        K->size--;
        float contribution = K->contrib[K->size], ri = K->ri[K->size];
        int bounced = K->bounce[K->size];
        ray_t cur = K->ray[K->size];
        rrd_t data = launch_ray(S, cur.o, cur.d, 32000.0f, contribution, c);
        int hit = dot(data.normal, data.normal) > 0.9f;
        sample = add(sample, mul(hit ? data.color : background(cur.d, 0), contribution));
        if (bounced < S->max_bounces && hit) {
            bounced++;
            int spawnRefl = 0, spawnRefr = 0;
            v3 refr_dir = V3(0, 0, 0), refl_dir = V3(0, 0, 0); /* uninitialised -> 0 */
            float cos_t = dot(data.normal, cur.d);
            float sin_t = sqrtf(1.0f - cos_t * cos_t);
            float target_ri;
            {
                int pi = K->size - 1 - skip;
                float parent = (pi < 0) ? 1.0f : (pi < IOW_STACK ? K->ri[pi] : 0.0f);
                target_ri = cos_t > 0 ? parent : data.material.z;
            }
            float rr = (ri * rcp(target_ri)) * sin_t;
            float refr_c = data.material.x, refl_c = data.material.y;
            v3 n_ = cos_t > 0 ? data.normal : neg(data.normal);
            if (cos_t < 0) {
                refl_dir = fib_dir(S, sidx, data.scat[1], data.reflected); spawnRefl = 1;
                float inc = refr_c * schlick(-cos_t, ri * rcp(target_ri));
                refr_c -= inc; refl_c += inc;
            } else if (rr > 1.0f) {
                refr_dir = data.reflected; spawnRefl = 1; refl_c = 1.0f; /* sic: 03.glsl:332 */
            }
            if (rr <= 1.0f) {
                v3 yc = mul(n_, cos_t), xc = sub(cur.d, yc);
                spawnRefr = 1;
                refr_dir = add(mul(n_, rr), mul(xc, sqrtf(1.0f - rr * rr)));
                refr_dir = fib_dir(S, sidx, data.scat[0], refr_dir);
            }
            skip = (spawnRefl && spawnRefr) ? skip - 1 : (spawnRefl ? skip : (spawnRefr ? skip + 1 : 0));
            if (spawnRefl) {
                ray_t nr = {sub(data.point, mul(n_, 0.000015f)), refl_dir};
                if (isnan(dot(refl_dir, refl_dir))) c->nans++;
                iow_push(K, nr, contribution * refl_c, ri, bounced, c);
            }
            if (spawnRefr) {
                ray_t nr = {add(data.point, mul(n_, 0.000015f)), refr_dir};
                if (isnan(dot(refr_dir, refr_dir))) c->nans++;
                iow_push(K, nr, contribution * refr_c, target_ri, bounced, c);
            }
        } else skip = 0;
    }
    return sample;
}

int orc_render_iow03(const float *types, const float *records, uint32_t n,
                     const orc_camera *cam, const orc_params *p, float *rgba, orc_stats *st) {
    if (!types || !records || !cam || !p || !rgba || p->width <= 0 || p->height <= 0 || p->spp < 1)
        return -1;
    double t0 = now_ms();
    const int W = p->width, H = p->height, spp = p->spp;
    int x0 = p->tile_x0, y0 = p->tile_y0, tw = p->tile_w, th = p->tile_h;
    if (tw <= 0 || th <= 0) { x0 = 0; y0 = 0; tw = W; th = H; }
    float *sf = (float *)malloc(sizeof(float) * 2 * spp);
    float *fb = (float *)malloc(sizeof(float) * 3 * spp);
    int *ring = (int *)malloc(sizeof(int) * 2 * spp);
    orc_sample_tables(spp, sf, fb, ring);
    iow_scene S = {types, records, n, sf, fb, ring, spp, p->max_bounces};
    const v3 D = V3(cam->dir[0], cam->dir[1], cam->dir[2]);
    const v3 P = V3(cam->pos[0], cam->pos[1], cam->pos[2]);
    const float sd = 1.0f / (2.0f * (float)tan((double)(cam->fov_y_rad * 0.5f))); /* :377 */
    int grid = 1;
    while (grid * grid < spp) grid++;                                            /* :366-368 */
    ctr total = {0, 0, 0, 0, 0, 0};
#pragma omp parallel num_threads(orc_num_threads())
    {
        ctr c = {0, 0, 0, 0, 0, 0};
#pragma omp for schedule(dynamic, 1)
        for (int yy = y0; yy < y0 + th; yy++) {
            for (int xx = x0; xx < x0 + tw; xx++) {
                if (xx < 0 || yy < 0 || xx >= W || yy >= H) continue;
                iow_stack K;
                memset(&K, 0, sizeof(K));
                /* out_Pixel 03.glsl:362-418 */
                float aspect = (float)W * rcp((float)H);
                float sx = (aspect * ((float)xx * 2.0f - (float)W)) * rcp(2.0f * (float)W);
                float sy = ((float)yy * 2.0f - (float)H) * rcp(2.0f * (float)H);
                float dsx = aspect * rcp((float)(W * grid));
                float dsy = 1.0f * rcp((float)(H * grid));
                v3 fc = V3(0, 0, 0);
                v3 look_at = add(P, mul(D, cam->focus_dist));
                v3 up = V3(0, 1, 0);
                v3 cr = cross(D, up), cu = cross(cr, D);
                int done = 0;
                for (int s = 0; s < spp && !done; s++) {
                    int ix = ring[2 * s], iy = ring[2 * s + 1];
                    if (ix < 0) { /* :396 early return */
                        fc = mul(fc, rcp((float)s));
                        done = 1;
                        break;
                    }
                    float rx = (sf[2 * s] * cam->aperture) * 0.5f, ry = (sf[2 * s + 1] * cam->aperture) * 0.5f;
                    v3 ro = add(add(P, mul(cr, rx)), mul(cu, ry));
                    v3 ld = normalize(sub(look_at, ro));
                    v3 r_ = cross(ld, up), u_ = cross(cr, ld);
                    v3 rd = normalize(add(add(mul(ld, sd), mul(r_, sx + dsx * (float)ix)),
                                          mul(u_, sy + dsy * (float)iy)));
                    if (!p->show_normal) fc = add(fc, launch_rays(&S, &K, ro, rd, s, &c));
                    else fc = add(fc, launch_ray(&S, ro, rd, 32000.0f, 1.0f, &c).normal);
                }
                if (!done) fc = mul(fc, rcp((float)spp));
                float *o = rgba + ((size_t)yy * W + xx) * 4;
                o[0] = fc.x; o[1] = fc.y; o[2] = fc.z; o[3] = 1.0f;
            }
        }
#pragma omp critical
        {
            total.seg += c.seg; total.nodes += c.nodes; total.prims += c.prims;
            total.shadow += c.shadow; total.drops += c.drops; total.nans += c.nans;
        }
    }
    free(sf); free(fb); free(ring);
    if (st) { memset(st, 0, sizeof(*st)); ctr_add(st, &total); st->ms = now_ms() - t0; }
    return 0;
}

/* ===================================================================================
 * INW-01 / INW-04: BVH.glsl, 04.glsl
 * =================================================================================== */
#define INW_ELLIPSOID 1 /* BVH.glsl:109 */
#define INW_CUBOID 2    /* BVH.glsl:110 */
#define FSTACK 40       /* stack_capacity BVH.glsl:80 */
#define MAX_T_DEPTH 32000.0f

typedef struct { float data[FSTACK]; uint32_t size; } fstack; /* FLT_STACK BVH.glsl:81-85 */

static inline void stk_push(fstack *k, float v, ctr *c) { /* STK_PUSH :86 */
    if (k->size < FSTACK) { k->data[k->size] = v; k->size++; } else c->drops++;
}
static inline void stk_push_ray(fstack *k, ray_t r, float contrib, float bounced, ctr *c) { /* :88-97 */
    if (k->size < (FSTACK - 7)) {
        float *d = k->data + k->size;
        d[0] = r.o.x; d[1] = r.o.y; d[2] = r.o.z; d[3] = r.d.x; d[4] = r.d.y; d[5] = r.d.z;
        d[6] = contrib; d[7] = bounced;
        k->size += 8;
    } else c->drops++;
}

typedef struct {
    const float *geom, *nodes, *lights;
    uint32_t n, n_lights;
    int layout, spp, max_bounces;
    const float *sf;
    v3 camdir;
    const orc_texture *tex; /* u_MaterialTextures[u_NumOfTexture2D] (04.glsl:10) */
    uint32_t n_tex;
    int n_focus;            /* MULTIFOCUS (BVH.glsl:388-404, 425-427, 479-481, 505-536, 544-549): 0 = off */
    float focus[9];         /* u_Camera.FocusDist[u_NumOfFocusDist] (BVH.glsl:220,226; base.h:458-473) */
} inw_scene;

typedef struct { v3 pos, scale, delta; m3 R; int type; float extra; } xform_t;

/* the five texel fetches of IntersectRay BVH.glsl:232-253 / 04.glsl:244-267 */
static xform_t fetch_xform(const inw_scene *S, int g) {
    const float *f = S->geom + (size_t)g * 28;
    xform_t x;
    x.pos = V3(f[0], f[1], f[2]);
    x.R.c[0] = V3(f[3], f[4], f[5]); x.R.c[1] = V3(f[6], f[7], f[8]); x.R.c[2] = V3(f[9], f[10], f[11]);
    x.scale = V3(f[12], f[13], f[14]);
    x.delta = V3(f[15], f[16], f[17]);
    x.type = (int)f2u(f[18] + 0.1f);
    x.extra = f[19];
    return x;
}

/* IntersectRay BVH.glsl:230-269 / 04.glsl:281-322 (normal may be NULL: IntersectRayMinimal) */
static int intersect_ray(const inw_scene *S, ray_t ray, int g, float ratio, float *tlim, v3 *normal,
                         float *extra) {
    xform_t x = fetch_xform(S, g);
    /* transform.Rotation_Matrix = transpose(R); M*(...) == transpose(R)*(...) */
    v3 ov = add(sub(ray.o, x.pos), mul(x.delta, 1.0f - ratio));
    ray_t tr = {m3tmul(x.R, ov), m3tmul(x.R, ray.d)};
    int t3 = x.type == INW_ELLIPSOID ? 2 : (x.type == INW_CUBOID ? 1 : 0);
    float t = t_ray_obj(tr, t3, x.scale);
    if (t > 0 && t < *tlim) {
        *tlim = t;
        if (normal) {
            v3 h = add(tr.o, mul(tr.d, t)), nl;
            if (t3 == 2) {
                v3 s = x.scale;
                nl = normalize(V3(h.x * rcp(s.x * s.x), h.y * rcp(s.y * s.y), h.z * rcp(s.z * s.z)));
            } else if (t3 == 1) nl = cuboid_normal(h, x.scale);
            else nl = V3(0, 0, 0);
            *normal = m3mul(x.R, nl);
        }
        if (extra) *extra = x.extra;
        return 1;
    }
    return 0;
}

/* TestIntersectAABB BVH.glsl:187-208 */
static int test_aabb(v3 mn, v3 mx, ray_t r, float tlim) {
    float id0 = rcp(r.d.x);
    float t1 = (mn.x - r.o.x) * id0, t2 = (mx.x - r.o.x) * id0;
    float tmin = fmin_(t1, t2), tmax = fmax_(t1, t2);
    for (int i = 0; i < 3; i++) {
        float id = rcp(v3get(r.d, i));
        float a = (v3get(mn, i) - v3get(r.o, i)) * id;
        float b = (v3get(mx, i) - v3get(r.o, i)) * id;
        t1 = fmin_(a, b); t2 = fmax_(a, b);
        tmin = fmax_(t1, tmin); tmax = fmin_(t2, tmax);
        if (tmax <= tmin) return 0;
    }
    return tlim > 0.0f ? tlim > tmin : 1;
}

/* closest-hit LBVH DFS, BVH.glsl:431-473 / 04.glsl:524-563 / shadow 04.glsl:620-657 */
static float traverse(const inw_scene *S, fstack *K, ray_t ray, float ratio, float *tlim, v3 *normal,
                      float *extra, float init_geom, int minimal, ctr *c) {
    float final_geom = init_geom;
    uint32_t I = K->size;
    stk_push(K, 0.0f, c);
    const int invert = dot(S->camdir, V3(1, 1, 1)) > 0;
    for (;;) {
        float geom = -1.0f;
        while (K->size > I) {
            K->size--;
            float node = K->data[K->size];
            const float *nd = S->nodes + (size_t)node * 8;
            v3 mn = V3(nd[0], nd[1], nd[2]), mx = V3(nd[3], nd[4], nd[5]);
            float left = nd[6];
            c->nodes++;
            if (test_aabb(mn, mx, ray, *tlim)) {
                if (left > 0.1f) {
                    float right = left + 1.0f;
                    stk_push(K, invert ? right : left, c);
                    stk_push(K, invert ? left : right, c);
                } else { geom = -left; break; }
            }
        }
        if (geom > -0.9f) {
            c->prims++;
            int hit = intersect_ray(S, ray, (int)geom, ratio, tlim, minimal ? NULL : normal, extra);
            if (hit) final_geom = geom;
        } else break;
    }
    K->size = I;
    return final_geom;
}

/* Surrounding RI: BVH.glsl:486-502 + IfInsideAABBAndLeaf_TryAccumulateRI :272-345 */
static float surrounding_ri(const inw_scene *S, fstack *K, v3 hp, float ratio, ctr *c) {
    float acc = 0.0f;
    uint32_t cnt = 0;
    uint32_t I = K->size;
    stk_push(K, 0.0f, c);
    while (K->size > I) {
        K->size--;
        float node = K->data[K->size];
        const float *nd = S->nodes + (size_t)node * 8;
        c->nodes++;
        v3 mn = V3(nd[0], nd[1], nd[2]), mx = V3(nd[3], nd[4], nd[5]);
        float left = nd[6];
        if (hp.x <= mx.x && hp.y <= mx.y && hp.z <= mx.z && hp.x >= mn.x && hp.y >= mn.y && hp.z >= mn.z) {
            if (left < 0.1f) {
                c->prims++;
                int g = (int)(-left);
                xform_t x = fetch_xform(S, g);
                v3 v = add(sub(hp, x.pos), mul(x.delta, 1.0f - ratio));
                v = m3tmul(x.R, v);
                v.x *= rcp(x.scale.x); v.y *= rcp(x.scale.y); v.z *= rcp(x.scale.z);
                int type = (int)(S->geom[(size_t)g * 28 + 18] + 0.1f);
                int inside;
                if (type == INW_ELLIPSOID) inside = dot(v, v) <= 1.0f;
                else if (type == INW_CUBOID) inside = fabsf(v.x) <= 0.5f && fabsf(v.y) <= 0.5f && fabsf(v.z) <= 0.5f;
                else inside = 0;
                if (inside) {
                    /* RI: texel 5.x (layout 1, BVH.glsl:336) or texel 4.w (layout 4, 04.glsl:369) */
                    acc += S->layout == 4 ? S->geom[(size_t)g * 28 + 19] : S->geom[(size_t)g * 28 + 20];
                    cnt++;
                }
            } else {
                stk_push(K, left, c);
                stk_push(K, left + 1.0f, c);
            }
        }
    }
    if (acc > 1.0f) acc *= rcp((float)cnt);
    else acc = 1.0f;
    return acc;
}

static int is_lit_geom(const inw_scene *S, uint32_t in) { /* 04.glsl:468-474 */
    int r = 0;
    for (uint32_t i = 0; i < S->n_lights && !r; i++) {
        uint32_t idx;
        memcpy(&idx, S->lights + (size_t)i * 7 + 6, 4);
        r = in == idx;
    }
    return r;
}

/* texture(u_MaterialTextures[k], st) of a compute shader: no derivatives, so lambda = 0 and
 * the magnification filter applies -- GL_NEAREST (utility.cpp:182 Upload(..., GL_LINEAR,
 * GL_NEAREST)) -- with GL_REPEAT wrapping (utility.cpp:191-192): texel (floor(s*w) mod w,
 * floor(t*h) mod h) of an RGB8 / RGBA8 image, each channel c/255 (unorm8 -> float).
 * The texel address is computed in binary32 (the driver's fixed-point addressing is not
 * observable here: parity unpinned). */
static int tex_wrap(float u, int size) {
    float f = floorf(u);
    if (!(f == f) || f > 2147483520.0f || f < -2147483520.0f) return 0; /* NaN / inf -> texel 0 */
    long long i = (long long)f % size;
    return (int)(i < 0 ? i + size : i);
}
static v3 tex_fetch(const orc_texture *t, float s, float tt) {
    const int i = tex_wrap(s * (float)t->width, t->width), j = tex_wrap(tt * (float)t->height, t->height);
    const uint8_t *px = t->texels + ((size_t)j * t->width + i) * (size_t)t->channels;
    return V3((float)px[0] / 255.0f, (float)px[1] / 255.0f, (float)px[2] / 255.0f);
}

/* FillHitMaterialData 04.glsl:416-464, the TextureIndex > 0 branch: cube-projection UV of the
 * object-space hit position, colour *= texel */
static v3 tex_color(const orc_texture *t, v3 lp) {
    lp = normalize(lp);
    float mx = lp.x;
    uint32_t face = mx > 0 ? 1u : 3u;
    v3 fd = mul(V3(1, 0, 0), mx > 0 ? 1.0f : -1.0f);
    for (int i = 1; i < 3; i++) {
        const float li = v3get(lp, i);
        if (fabsf(mx) < fabsf(li)) {
            mx = li;
            face = mx > 0 ? (i == 1 ? 0u : 2u) : (i == 1 ? 5u : 4u);
            fd = mul(V3((float)(i == 0), (float)(i == 1), (float)(i == 2)), mx > 0 ? 1.0f : -1.0f);
        }
    }
    lp = mul(lp, rcp(dot(lp, fd)));
    lp = mul(lp, 0.5f);
    lp = add(lp, V3(0.5f, 0.5f, 0.5f));
    float u = 0, v = 0;
    switch (face) {
        case 0: u = lp.x; v = 1.0f - lp.z; break;
        case 1: u = 1.0f - lp.y; v = 1.0f - lp.z; break;
        case 2: u = lp.x; v = lp.y; break;
        case 3: u = lp.z; v = lp.y; break;
        case 4: u = 1.0f - lp.y; v = 1.0f - lp.x; break;
        default: u = lp.z; v = 1.0f - lp.x; break;
    }
    return tex_fetch(t, (float)face * 0.16666f + u * 0.16666f, v);
}

/* deviateWithLinmit90deg BVH.glsl:28-46 (power == 1) */
static v3 deviate(const inw_scene *S, v3 dir, float tan_theta, int s) {
    float ap = (2.0f * tan_theta) * 0.5f;
    float nx = S->sf[2 * s] * ap, ny = S->sf[2 * s + 1] * ap; /* pow(x, 1) == x */
    v3 right = cross(dir, V3(0, 1, 0));
    v3 up = cross(right, dir);
    return normalize(add(dir, mul(add(mul(right, nx), mul(up, ny)), 0.1f)));
}

/* out_Pixel BVH.glsl:364-599 / 04.glsl:476-715 for one sample s (one invocation) */
static void inw_sample(const inw_scene *S, int px, int py, int W, int H, float sd, v3 campos,
                       float fov_unused, float aperture, float focus, int s, v3 *out_color,
                       float *out_depth, ctr *c) {
    (void)fov_unused;
    fstack K;
    K.size = 0;
    K.data[0] = 0; /* prepare() */
    v3 color = V3(0, 0, 0);
    float depth = 0.0f; /* uninitialised out -> 0 */
    const v3 D = S->camdir;
    const float ratio = (float)s * rcp((float)S->spp);
    {
        float aspect = (float)W * rcp((float)H);
        float srx = (float)px * rcp((float)W) - 0.5f;
        float sry = (float)py * rcp((float)H) - 0.5f;
        srx *= aspect;
        v3 up = V3(0, 1, 0);
        v3 cr = cross(D, up), cu = cross(cr, D);
        ray_t cam;
        cam.o = campos;
        cam.d = normalize(add(add(mul(D, sd), mul(cr, srx)), mul(cu, sry)));
        float ox = S->sf[2 * s] * (aperture * 0.5f), oy = S->sf[2 * s + 1] * (aperture * 0.5f);
        v3 rr = cross(cam.d, up), ru = cross(rr, cam.d);
        if (S->n_focus > 0) { /* MULTIFOCUS lens set-up, BVH.glsl:388-400 */
            float first_limit = S->focus[0] * 0.5f;
            v3 nd = normalize(add(add(mul(cam.d, first_limit), mul(rr, ox)), mul(ru, oy)));
            v3 rn = normalize(sub(mul(neg(rr), ox), mul(ru, oy)));
            float mult = 1.0f / dot(cam.d, nd);
            cam.d = nd;
            stk_push(&K, rn.x, c); stk_push(&K, rn.y, c); stk_push(&K, rn.z, c); /* 0..2 */
            stk_push(&K, mult, c);                                              /* 3 */
            stk_push(&K, first_limit, c);                                       /* 4 */
            stk_push(&K, 0.0f, c);                                              /* 5 crossedLens */
        } else {
            v3 tip = add(add(add(cam.o, cam.d), mul(rr, ox)), mul(ru, oy));
            v3 la = normalize(sub(add(cam.o, mul(cam.d, focus)), tip));
            cam.o = sub(tip, la);
            cam.d = la;
        }
        stk_push_ray(&K, cam, 1.0f, 0.0f, c);
    }
    const int L4 = S->layout == 4;
    while (K.size > 0) {
        v3 normal = V3(0, 0, 0), hitpoint;
        float contribution, bounced, surr = 0.0f;
        float m_ri = 0, m_refr = 0, m_refl = 0, m_srfr = 0, m_srfl = 0;
        v3 m_color = V3(0, 0, 0);
        v3 incoming;
        ray_t cur;
        {   /* STK_POP_RAY_DATA_TO: size >= 8 here, (size-7) > 0 always holds */
            K.size -= 8;
            float *d = K.data + K.size;
            cur.o = V3(d[0], d[1], d[2]); cur.d = V3(d[3], d[4], d[5]);
            contribution = d[6]; bounced = (float)(int)d[7];
        }
        c->seg++;
        /* SET LIMIT BVH.glsl:424-428: the primary ray of a MULTIFOCUS sample stops at the lens */
        const int mf0 = S->n_focus > 0 && (int)(bounced + 0.1f) == 0;
        const float tlim0 = mf0 ? K.data[4] : MAX_T_DEPTH;
        float tlim = tlim0;
        float extra = 0.0f;
        float fg = traverse(S, &K, cur, ratio, &tlim, &normal, &extra, L4 ? -1.0f : 0.0f, 0, c);
        incoming = cur.d;
        hitpoint = add(cur.o, mul(cur.d, tlim));
        if (tlim < tlim0) {
            const float *f = S->geom + (size_t)fg * 28;
            if (!L4) { /* FillHitData BVH.glsl:349-361 */
                m_ri = f[20]; m_refr = f[21]; m_refl = f[22]; m_srfr = f[23]; m_srfl = f[24];
                m_color = V3(f[25], f[26], f[27]);
            } else {   /* FillHitMaterialData 04.glsl:403-415 (TextureIndex == 0 path) */
                m_ri = extra; m_refr = f[20]; m_refl = f[21]; m_srfr = f[22]; m_srfl = f[23];
                m_color = V3(f[24], f[25], f[26]);
                const uint32_t ti = f2u(f[27] + 0.1f);
                if (ti > 0 && ti <= S->n_tex) { /* :416; local posn :569 (Position without motion) */
                    const xform_t x = fetch_xform(S, (int)fg);
                    m_color = mulv(m_color, tex_color(S->tex + (ti - 1), m3tmul(x.R, sub(hitpoint, x.pos))));
                }
            }
            surr = surrounding_ri(S, &K, add(hitpoint, mul(normal, 0.001f)), ratio, c);
        } else if (mf0 && (int)(K.data[5] + 0.1f) < S->n_focus) {
            /* move to the next focal lens, BVH.glsl:506-528 */
            v3 rn = V3(K.data[0], K.data[1], K.data[2]);
            K.data[0] = -K.data[0]; K.data[1] = -K.data[1]; K.data[2] = -K.data[2];
            float mult = K.data[3], dist = K.data[4];
            cur.o = add(cur.o, mul(cur.d, mult * dist));
            cur.d = reflect3(cur.d, rn);
            int lens = (int)(K.data[5] + 0.1f);
            if (lens < S->n_focus - 1)
                K.data[4] = (S->focus[lens + 1] - S->focus[lens]) * 0.5f +
                            (S->focus[lens] - (lens > 0 ? S->focus[lens - 1 > 0 ? lens - 1 : 0] : 0.0f)) * 0.5f;
            else K.data[4] = MAX_T_DEPTH - mult * K.data[4];
            K.data[5] += 1.0f;
            K.size = 6;
            stk_push_ray(&K, cur, 1.0f, 0.0f, c);
            continue;
        } else {
            color = add(color, mul(background(cur.d, L4 && S->n_lights > 0), contribution));
            depth = tlim;
            if (mf0) K.size = 0; /* BVH.glsl:531-535 */
            continue;
        }
        if (mf0) K.size = 0;     /* BVH.glsl:544-549: the lens record is dropped after a primary hit */
        if (L4) { /* 04.glsl:604-665 */
            uint32_t is_lit = S->n_lights > 0 ? 0u : (uint32_t)is_lit_geom(S, f2u(fg + 0.1f));
            if (is_lit == 0) {
                for (uint32_t i = 0; i < S->n_lights; i++) {
                    const float *lt = S->lights + (size_t)i * 7;
                    v3 bmin = V3(lt[0], lt[1], lt[2]), bmax = V3(lt[3], lt[4], lt[5]);
                    ray_t sr;
                    sr.o = add(hitpoint, mul(normal, 0.0001f));
                    float sl = length(sub(mul(add(bmax, bmin), 0.5f), sr.o)) + length(sub(bmax, bmin));
                    sr.d = normalize(sub(add(bmin, mul(sub(bmax, bmin), ratio)), sr.o));
                    c->shadow++;
                    float sg = traverse(S, &K, sr, ratio, &sl, NULL, NULL, -1.0f, 1, c);
                    is_lit += (uint32_t)is_lit_geom(S, f2u(sg + 0.1f));
                }
                uint32_t nl = S->n_lights > 1 ? S->n_lights : 1u;
                contribution *= (float)is_lit * rcp((float)nl);
            } else {
                color = V3(1, 1, 1);
                K.size = 0;
                break;
            }
        }
        int bounce_ok;
        if (!L4) { bounced += 1.0f; bounce_ok = bounced < (float)S->max_bounces; } /* BVH.glsl:552-554 */
        else bounce_ok = bounced < (float)S->max_bounces;                        /* 04.glsl:669 */
        if ((m_refl > 0.002f || m_refr > 0.002f) && contribution > 0.01f && bounce_ok) {
            if (L4) bounced += 1.0f;                                             /* 04.glsl:670 */
            v3 refl = V3(0, 0, 0), refr = V3(0, 0, 0);
            int inner = dot(normal, incoming) > 0;
            if (!inner) {
                if (m_refl > 0.002f) {
                    refl = normalize(reflect3(incoming, normal));
                    if (m_srfl > 0.001f) refl = deviate(S, refl, m_srfl, s);
                }
                if (m_refr > 0.002f) {
                    refr = normalize(refract3(incoming, normal, surr * rcp(m_ri)));
                    if (m_srfr > 0.001f) refr = deviate(S, refr, m_srfr, s);
                }
            } else {
                normal = mul(normal, -1.0f);
                refr = refract3(incoming, normal, m_ri * rcp(surr));
                if (dot(refr, refr) < 0.1f) refl = reflect3(incoming, normal);
            }
            float carried = 0.0f;
            float rr2 = dot(refr, refr);
            if (isnan(rr2)) c->nans++;
            if (rr2 > 0.1f) {
                ray_t nr = {sub(hitpoint, mul(normal, 0.0001f)), refr};
                carried += m_refr;
                stk_push_ray(&K, nr, contribution * m_refr, bounced, c);
            }
            if (dot(refl, refl) > 0.1f) {
                ray_t nr = {add(hitpoint, mul(normal, 0.0001f)), refl};
                carried += m_refl;
                stk_push_ray(&K, nr, contribution * m_refl, bounced, c);
            }
            contribution *= (1.0f - 0.5f * carried);
        }
        color = add(color, mul(m_color, contribution));
    }
    *out_color = color;
    *out_depth = depth;
}

/* MULTIFOCUS focus list of the next orc_render_inw_tex call (set by orc_render_inw_mf only) */
static _Thread_local int g_mf_n = 0;
static _Thread_local float g_mf_focus[9];

int orc_render_inw(const float *geom, uint32_t n, int layout, const float *nodes,
                   const float *lights, uint32_t n_lights, const orc_camera *cam,
                   const orc_params *p, float *rgba, float *depth, orc_stats *st) {
    return orc_render_inw_tex(geom, n, layout, nodes, lights, n_lights, NULL, 0, cam, p, rgba, depth, st);
}

/* INW-01 with the MULTIFOCUS branch compiled in (BVH.glsl:388-404 etc.; the reference ships
 * it as "#if MULTIFOCUS", never defined): n_focus in 1..9 focus distances. */
int orc_render_inw_mf(const float *geom, uint32_t n, const float *nodes, const orc_camera *cam,
                      const float *focus, int n_focus, const orc_params *p, float *rgba, float *depth,
                      orc_stats *st) {
    if (!focus || n_focus < 1 || n_focus > 9) return -1;
    g_mf_n = n_focus;
    memcpy(g_mf_focus, focus, sizeof(float) * (size_t)n_focus);
    int rc = orc_render_inw_tex(geom, n, 1, nodes, NULL, 0, NULL, 0, cam, p, rgba, depth, st);
    g_mf_n = 0;
    return rc;
}

int orc_render_inw_tex(const float *geom, uint32_t n, int layout, const float *nodes,
                       const float *lights, uint32_t n_lights, const orc_texture *tex, uint32_t n_tex,
                       const orc_camera *cam, const orc_params *p, float *rgba, float *depth, orc_stats *st) {
    if (!geom || !nodes || !cam || !p || !rgba || n == 0 || p->width <= 0 || p->height <= 0 || p->spp < 1)
        return -1;
    if (layout != 1 && layout != 4) return -1;
    if (n_lights > 0 && !lights) return -1;
    if (n_tex > 0 && !tex) return -1;
    for (uint32_t k = 0; k < n_tex; k++)
        if (!tex[k].texels || tex[k].width <= 0 || tex[k].height <= 0 || (tex[k].channels != 3 && tex[k].channels != 4))
            return -1;
    if (layout == 4 && n_tex == 0)
        for (uint32_t g = 0; g < n; g++)
            if (f2u(geom[(size_t)g * 28 + 27] + 0.1f) > 0) return -4; /* textured objects need textures */
    double t0 = now_ms();
    const int W = p->width, H = p->height, spp = p->spp;
    int x0 = p->tile_x0, y0 = p->tile_y0, tw = p->tile_w, th = p->tile_h;
    if (tw <= 0 || th <= 0) { x0 = 0; y0 = 0; tw = W; th = H; }
    float *sf = (float *)malloc(sizeof(float) * 2 * spp);
    orc_sample_tables(spp, sf, NULL, NULL);
    inw_scene S;
    S.geom = geom; S.nodes = nodes; S.lights = lights; S.n = n; S.n_lights = layout == 4 ? n_lights : 0;
    S.layout = layout; S.spp = spp; S.max_bounces = p->max_bounces; S.sf = sf;
    S.camdir = V3(cam->dir[0], cam->dir[1], cam->dir[2]);
    S.tex = layout == 4 ? tex : NULL;
    S.n_tex = layout == 4 ? n_tex : 0;
    S.n_focus = 0;
    if (g_mf_n > 0 && layout == 1) {
        S.n_focus = g_mf_n;
        memcpy(S.focus, g_mf_focus, sizeof(float) * (size_t)g_mf_n);
    }
    const float sd = 1.0f / (2.0f * (float)tan((double)(cam->fov_y_rad * 0.5f)));
    const v3 P = V3(cam->pos[0], cam->pos[1], cam->pos[2]);
    ctr total = {0, 0, 0, 0, 0, 0};
#pragma omp parallel num_threads(orc_num_threads())
    {
        ctr c = {0, 0, 0, 0, 0, 0};
#pragma omp for schedule(dynamic, 1)
        for (int yy = y0; yy < y0 + th; yy++) {
            for (int xx = x0; xx < x0 + tw; xx++) {
                if (xx < 0 || yy < 0 || xx >= W || yy >= H) continue;
                v3 acc = V3(0, 0, 0);
                float dmid = 0.0f;
                for (int s = 0; s < spp; s++) {
                    v3 col; float dep;
                    inw_sample(&S, xx, yy, W, H, sd, P, cam->fov_y_rad, cam->aperture, cam->focus_dist, s,
                               &col, &dep, &c);
                    v3 g = V3(sqrtf(col.x), sqrtf(col.y), sqrtf(col.z)); /* BVH.glsl:670 */
                    acc = (s == 0) ? g : add(acc, g);                     /* End() :644-651 */
                    if (s == spp / 2) dmid = dep;                          /* :667-668 */
                }
                acc = mul(acc, rcp((float)spp));
                float *o = rgba + ((size_t)yy * W + xx) * 4;
                o[0] = acc.x; o[1] = acc.y; o[2] = acc.z; o[3] = 1.0f;
                if (depth) depth[(size_t)yy * W + xx] = dmid;
            }
        }
#pragma omp critical
        {
            total.seg += c.seg; total.nodes += c.nodes; total.prims += c.prims;
            total.shadow += c.shadow; total.drops += c.drops; total.nans += c.nans;
        }
    }
    free(sf);
    if (st) { memset(st, 0, sizeof(*st)); ctr_add(st, &total); st->ms = now_ms() - t0; }
    return 0;
}

/* ===================================================================================
 * IOW-00: the base stage's default compute shader (base.cpp:7-28): a UV gradient
 * =================================================================================== */
int orc_render_iow00(const orc_params *p, float *rgba) {
    if (!p || !rgba || p->width <= 0 || p->height <= 0) return -1;
    const int W = p->width, H = p->height;
    for (int y = 0; y < H; y++)
        for (int x = 0; x < W; x++) {
            float *o = rgba + ((size_t)y * W + x) * 4;
            o[0] = (float)x * rcp((float)W - 1.0f); /* pixel_coords.x / (imageSize.x - 1.0) :13 */
            o[1] = (float)y * rcp((float)H - 1.0f); /* :14 */
            o[2] = 0.25f;
            o[3] = 1.0f;
        }
    return 0;
}

/* ===================================================================================
 * IOW-02: 02.glsl (groups.h:11-17 record: position, inverse rotation mat3, scale, colour)
 * =================================================================================== */
/* t_RayXObj 02.glsl:37-94, with the u_Cull_Front / u_Cull_Back modes */
static float t_ray_obj_cull(ray_t r, int type, v3 s, int cull_front, int cull_back) {
    float t = -1.0f;
    if (type == IOW_ELLIPSOID) {
        v3 a2 = V3(r.o.x * rcp(s.x), r.o.y * rcp(s.y), r.o.z * rcp(s.z));
        v3 a3 = V3(r.d.x * rcp(s.x), r.d.y * rcp(s.y), r.d.z * rcp(s.z));
        float hb = dot(a2, a3), a = dot(a3, a3), c = dot(a2, a2) - 1.0f;
        float det = hb * hb - a * c;
        if (det > 0) {
            float t0 = (-hb - sqrtf(det)) * rcp(a), t1 = (-hb + sqrtf(det)) * rcp(a);
            if (!cull_back && !cull_front) t = (t0 > t1 || t0 < 0) ? t1 : t0;
            else if (!cull_front) t = fmin_(t0, t1);
            else if (!cull_back) t = fmax_(t0, t1);
        }
    } else if (type == IOW_CUBOID) {
        v3 bmin = mul(neg(s), 0.5f), bmax = mul(s, 0.5f);
        float t1 = (bmin.x - r.o.x) * rcp(r.d.x), t2 = (bmax.x - r.o.x) * rcp(r.d.x);
        float tmin = fmin_(t1, t2), tmax = fmax_(t1, t2);
        for (int i = 1; i < 3; ++i) {
            t1 = (v3get(bmin, i) - v3get(r.o, i)) * rcp(v3get(r.d, i));
            t2 = (v3get(bmax, i) - v3get(r.o, i)) * rcp(v3get(r.d, i));
            tmin = fmax_(tmin, fmin_(fmin_(t1, t2), tmax));
            tmax = fmin_(tmax, fmax_(fmax_(t1, t2), tmin));
        }
        if (tmax > fmax_(tmin, 0.0f)) {
            if (!cull_back && !cull_front) t = tmin > 0 ? tmin : tmax;
            else if (!cull_front) t = tmin;
            else if (!cull_back) t = tmax;
        }
    }
    return t > 0 ? t : -1.0f;
}

int orc_render_iow02(const float *types, const float *records, uint32_t n, const orc_camera *cam,
                     const orc_params *p, int cull_front, int cull_back, float *rgba, orc_stats *st) {
    if ((n > 0 && (!types || !records)) || !cam || !p || !rgba || p->width <= 0 || p->height <= 0 || p->spp < 1 ||
        p->max_bounces < 0)
        return -1;
    double t0 = now_ms();
    const int W = p->width, H = p->height, spp = p->spp, nb = p->max_bounces;
    int x0 = p->tile_x0, y0 = p->tile_y0, tw = p->tile_w, th = p->tile_h;
    if (tw <= 0 || th <= 0) { x0 = 0; y0 = 0; tw = W; th = H; }
    int *ring = (int *)malloc(sizeof(int) * 2 * (size_t)spp);
    float *pw = (float *)malloc(sizeof(float) * (size_t)(nb > 0 ? nb : 1));
    orc_sample_tables(spp, NULL, NULL, ring);
    for (int i = 0; i < nb; i++) pw[i] = (float)pow((double)0.4f, (double)i); /* pow(0.4, i) :206 */
    const v3 D = V3(cam->dir[0], cam->dir[1], cam->dir[2]);
    const v3 P = V3(cam->pos[0], cam->pos[1], cam->pos[2]);
    int grid = 1;
    while (grid * grid < spp) grid++;
    uint64_t seg_total = 0;
#pragma omp parallel for schedule(dynamic, 1) num_threads(orc_num_threads()) reduction(+ : seg_total)
    for (int yy = y0; yy < y0 + th; yy++) {
        for (int xx = x0; xx < x0 + tw; xx++) {
            if (xx < 0 || yy < 0 || xx >= W || yy >= H) continue;
            float aspect = (float)W * rcp((float)H);                          /* :133 */
            const v3 up = V3(0, 1, 0);
            float sx = ((float)xx * 2.0f - (float)W) * rcp(2.0f * (float)W);  /* :135 */
            sx *= aspect;
            float sy = ((float)yy * 2.0f - (float)H) * rcp(2.0f * (float)H);  /* :137 */
            v3 fc = V3(0, 0, 0);
            int s = 0, early = 0;
            for (; s < spp; s++) {
                v3 ro = P, rd;
                {
                    v3 cr = cross(D, up), cu = cross(cr, D);
                    if (ring[2 * s] < 0) { early = 1; break; } /* :156: return final_color/samples_processed */
                    float dx = aspect * rcp((float)(W * grid));
                    float dy = 1.0f * rcp((float)(H * grid));
                    rd = normalize(add(add(mul(D, cam->focus_dist), mul(cr, sx + dx * (float)ring[2 * s])),
                                       mul(cu, sy + dy * (float)ring[2 * s + 1])));
                }
                float min_t = 32000.0f;
                v3 nrm = D;
                v3 fsc = V3(0, 0, 0);
                for (int i = 0; i < nb; i++) {
                    v3 sc = background(rd, 0);                                /* :172-175 */
                    m3 hit_m = {{{0, 0, 0}, {0, 0, 0}, {0, 0, 0}}};
                    seg_total++;
                    for (uint32_t j = 0; j < n; j++) {
                        const float *r = records + (size_t)j * 18;
                        int type = (int)types[j];
                        v3 pos = V3(r[0], r[1], r[2]);
                        m3 M = rec_m3(r + 3);
                        v3 scale = V3(r[12], r[13], r[14]), col = V3(r[15], r[16], r[17]);
                        ray_t tr = {m3mul(M, sub(ro, pos)), normalize(m3mul(M, rd))}; /* :194-198 */
                        float t = t_ray_obj_cull(tr, type, scale, cull_front, cull_back);
                        if (min_t > t && t > 0) {
                            nrm = iow_normal(t, tr, type, scale);
                            sc = col;
                            hit_m = M;
                            min_t = t;
                        }
                    }
                    fsc = add(fsc, mul(sc, pw[i]));                           /* :206 */
                    if (p->show_normal) { fsc = nrm; break; }
                    if (min_t > 30000.0f) break;
                    ro = add(ro, mul(rd, min_t - 0.00005f));                  /* :215 */
                    v3 tn = normalize(m3mul(m3inverse(hit_m), nrm));
                    rd = reflect3(rd, tn);
                    nrm = V3(0, 0, 0);
                    min_t = 32000.0f;
                }
                fc = add(fc, fsc);
            }
            v3 out = early ? mul(fc, rcp((float)s)) : mul(fc, rcp((float)spp));
            float *o = rgba + ((size_t)yy * W + xx) * 4;
            o[0] = out.x; o[1] = out.y; o[2] = out.z; o[3] = 1.0f;
        }
    }
    free(ring);
    free(pw);
    if (st) {
        memset(st, 0, sizeof(*st));
        st->segments = seg_total;
        st->prim_tests = seg_total * n;
        st->ms = now_ms() - t0;
    }
    return 0;
}
