/*
 * rt_oracle_host.c -- CPU ORACLE, host half (test infrastructure only; rules in rt_oracle.h).
 *
 * Restates the reference's host code that produces the bytes the shaders consume:
 *   utility.cpp:489-516        Helper::MATH::MakeRotation{X,Y,Z} (glm column-major ctor)
 *   materials.h:48-86          IOW-03 Geometry::FillBuffer / ResetInvRotationMatrix
 *   In-Next-Week/base.h:24-71  Transform_Data::CalculateBBMinMax / FillTransformBuff
 *   BVH.h:47-58                INW-01 GeometryData::FillBuffer
 *   lights.h:40-141            INW-04 GeometryData_04::CalculateBBMinMax / FillBuffer
 *   lights.cpp:255-271         light SSBO records
 *   LBVH/lbvh.h:11-269         LBVH::ConstructLBVH / ConstructLBVH_Buff
 * (paths relative to /root/reference/Raytracing-Sandbox/Src/)
 *
 * glm is an un-vendored, unpinned submodule (.gitmodules); its mat3 product / inverse are
 * restated from glm's published func_matrix.inl forms -- PARITY UNPINNED at that boundary.
 * std::sort leaves the order of equal keys unspecified (the reference was built with MSVC);
 * the contract breaks Morton+diagonal ties by ObjectID ascending -- PARITY UNPINNED for ties.
 */
#include "rt_oracle.h"
#include "rt_oracle_common.h"
#include <stdlib.h>
#include <string.h>

#define RMIN(x, y) ((x) > (y) ? (y) : (x)) /* utility.h:10 */
#define RMAX(x, y) ((x) > (y) ? (x) : (y)) /* utility.h:11 */

static float radians_f(float deg) { return deg * (float)0.01745329251994329576923690768489; }

static m3 m3cols(float a, float b, float c, float d, float e, float f, float g, float h, float i) {
    m3 m; /* glm::mat3(x0,y0,z0, x1,y1,z1, x2,y2,z2): columns */
    m.c[0] = V3(a, b, c); m.c[1] = V3(d, e, f); m.c[2] = V3(g, h, i);
    return m;
}
static m3 rotx(float r) { float c = cosf(r), s = sinf(r); return m3cols(1, 0, 0, 0, c, -s, 0, s, c); }
static m3 roty(float r) { float c = cosf(r), s = sinf(r); return m3cols(c, 0, s, 0, 1, 0, -s, 0, c); }
static m3 rotz(float r) { float c = cosf(r), s = sinf(r); return m3cols(c, -s, 0, s, c, 0, 0, 0, 1); }
/* glm mat3*mat3: Result[j] = A[0]*B[j][0] + A[1]*B[j][1] + A[2]*B[j][2] */
static m3 m3mm(m3 a, m3 b) {
    m3 r;
    for (int j = 0; j < 3; j++)
        r.c[j] = add(add(mul(a.c[0], b.c[j].x), mul(a.c[1], b.c[j].y)), mul(a.c[2], b.c[j].z));
    return r;
}
static m3 rot_zxy(const float deg[3]) {
    return m3mm(m3mm(rotz(radians_f(deg[2])), rotx(radians_f(deg[0]))), roty(radians_f(deg[1])));
}
static float m3at(m3 m, int c, int r) { return v3get(m.c[c], r); }

/* Transform_Data::CalculateBBMinMax base.h:24-42 (ellipsoid-style bound) */
static void bb_transform(const orc_geom_desc *g, float out[6]) {
    m3 m = rot_zxy(g->rotation_deg);
    m = m3mm(m, m3cols(g->scale[0], 0, 0, 0, g->scale[1], 0, 0, 0, g->scale[2]));
    float x = sqrtf(m3at(m, 0, 0) * m3at(m, 0, 0) + m3at(m, 1, 0) * m3at(m, 1, 0) + m3at(m, 2, 0) * m3at(m, 2, 0));
    float y = sqrtf(m3at(m, 0, 1) * m3at(m, 0, 1) + m3at(m, 1, 1) * m3at(m, 1, 1) + m3at(m, 2, 1) * m3at(m, 2, 1));
    float z = sqrtf(m3at(m, 0, 2) * m3at(m, 0, 2) + m3at(m, 1, 2) * m3at(m, 1, 2) + m3at(m, 2, 2) * m3at(m, 2, 2));
    const float *p = g->position, *l = g->last_position;
    out[0] = -x + RMIN(p[0], l[0]); out[1] = -y + RMIN(p[1], l[1]); out[2] = -z + RMIN(p[2], l[2]);
    out[3] = x + RMAX(p[0], l[0]);  out[4] = y + RMAX(p[1], l[1]);  out[5] = z + RMAX(p[2], l[2]);
}

/* GeometryData_04::CalculateBBMinMax lights.h:40-84 */
static void bb_04(const orc_geom_desc *g, float out[6]) {
    if (g->type == 1) { bb_transform(g, out); return; } /* Ellipsoid: same formula */
    if (g->type == 2) {
        m3 m = rot_zxy(g->rotation_deg);
        float bmin[3] = {0, 0, 0}, bmax[3] = {0, 0, 0};
        for (int i = 0; i < 8; i++) {
            float co[3];
            int bit = 1;
            for (int a = 0; a < 3; a++) { co[a] = (i & bit) ? 0.5f * g->scale[a] : -0.5f * g->scale[a]; bit <<= 1; }
            v3 v = m3mul(m, V3(co[0], co[1], co[2]));
            for (int a = 0; a < 3; a++) { bmin[a] = RMIN(v3get(v, a), bmin[a]); bmax[a] = RMAX(v3get(v, a), bmax[a]); }
        }
        const float *p = g->position, *l = g->last_position;
        for (int a = 0; a < 3; a++) { out[a] = bmin[a] + RMIN(p[a], l[a]); out[3 + a] = bmax[a] + RMAX(p[a], l[a]); }
        return;
    }
    for (int a = 0; a < 6; a++) out[a] = 0.0f;
}

int orc_pack_iow03(const orc_geom_desc *g, uint32_t n, float *types, float *records) {
    if (!g || !types || !records) return -1;
    for (uint32_t k = 0; k < n; k++) {
        const orc_geom_desc *d = g + k;
        float *r = records + (size_t)k * 24;
        m3 inv = m3cols(1, 0, 0, 0, 1, 0, 0, 0, 1); /* glm::mat3(1.0f) default, materials.h:97 */
        if (d->rotation_deg[0] != 0 || d->rotation_deg[1] != 0 || d->rotation_deg[2] != 0)
            inv = m3inverse(rot_zxy(d->rotation_deg)); /* ResetInvRotationMatrix :77-86 */
        r[0] = d->position[0]; r[1] = d->position[1]; r[2] = d->position[2];
        for (int i = 0; i < 9; i++) r[3 + i] = m3at(inv, i / 3, i % 3);
        r[12] = d->scale[0]; r[13] = d->scale[1]; r[14] = d->scale[2];
        r[15] = d->color[0]; r[16] = d->color[1]; r[17] = d->color[2];
        r[18] = d->refractivity; r[19] = d->reflectivity; r[20] = d->refractive_index;
        r[21] = d->scat_refract; r[22] = d->scat_reflect; r[23] = 0.0f;
        types[k] = (float)d->type; /* CopyObjBuffer materials.cpp:339-342 */
    }
    return 0;
}

int orc_pack_inw(const orc_geom_desc *g, uint32_t n, int layout, float *geom, float *aabbs,
                 float *lights, uint32_t *n_lights) {
    if (!g || (layout != 1 && layout != 4)) return -1;
    uint32_t nl = 0;
    for (uint32_t k = 0; k < n; k++) {
        const orc_geom_desc *d = g + k;
        if (geom) {
            float *b = geom + (size_t)k * 28;
            memset(b, 0, 28 * sizeof(float));
            /* FillTransformBuff base.h:56-71 */
            for (int i = 0; i < 3; i++) { b[i] = d->position[i]; b[15 + i] = d->position[i] - d->last_position[i]; }
            m3 m = rot_zxy(d->rotation_deg);
            for (int i = 0; i < 9; i++) b[3 + i] = m3at(m, i / 3, i % 3);
            for (int i = 0; i < 3; i++) b[12 + i] = d->scale[i];
            b[18] = (float)d->type;
            if (layout == 1) { /* BVH.h:47-58 */
                b[19] = 0.0f;
                b[20] = d->refractive_index; b[21] = d->refractivity; b[22] = d->reflectivity;
                b[23] = d->scat_refract; b[24] = d->scat_reflect;
                b[25] = d->color[0]; b[26] = d->color[1]; b[27] = d->color[2];
            } else { /* lights.h:115-141 */
                b[27] = (float)d->texture_index;
                if (!d->emissive) {
                    b[24] = d->color[0]; b[25] = d->color[1]; b[26] = d->color[2];
                    b[19] = d->refractive_index; b[21] = d->reflectivity; b[20] = d->refractivity;
                } else {
                    b[24] = 1.0f; b[25] = 1.0f; b[26] = 1.0f;
                    b[19] = 1.0f; b[21] = 0.0f; b[20] = 0.0f;
                }
                b[22] = d->scat_refract; b[23] = d->scat_reflect;
            }
        }
        float bb[6];
        if (layout == 1) bb_transform(d, bb); else bb_04(d, bb);
        if (aabbs) memcpy(aabbs + (size_t)k * 6, bb, sizeof(bb));
        if (layout == 4 && d->emissive) { /* Lights::FillBuffer lights.cpp:261-264 */
            if (lights) {
                float *L = lights + (size_t)nl * 7;
                memcpy(L, bb, sizeof(bb));
                uint32_t idx = k;
                memcpy(L + 6, &idx, 4);
            }
            nl++;
        }
    }
    if (n_lights) *n_lights = nl;
    return 0;
}

/* ---------------------------------------------------------------------------- LBVH */
static uint32_t expand_bits(uint32_t v) { /* lbvh.h:11-18 */
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
static uint32_t morton_code(float x, float y, float z) { /* lbvh.h:21-30 */
    const float res = 1024.0f;
    x = fminf(fmaxf(x * res, 0.0f), res - 1.0f);
    y = fminf(fmaxf(y * res, 0.0f), res - 1.0f);
    z = fminf(fmaxf(z * res, 0.0f), res - 1.0f);
    return expand_bits((uint32_t)x) * 4 + expand_bits((uint32_t)y) * 2 + expand_bits((uint32_t)z);
}

typedef struct { uint32_t code, id; float diag2; } key_t_;
static int key_cmp(const void *pa, const void *pb) { /* lbvh.h:112-120 + ObjectID tie-break */
    const key_t_ *a = (const key_t_ *)pa, *b = (const key_t_ *)pb;
    if (a->code != b->code) return a->code < b->code ? -1 : 1;
    if (a->diag2 < b->diag2) return -1;
    if (b->diag2 < a->diag2) return 1;
    return a->id < b->id ? -1 : (a->id > b->id ? 1 : 0);
}

typedef struct { int parent, left, right; uint32_t obj; float mn[3], mx[3]; } lnode;

int orc_lbvh_build(const float *aabbs, uint32_t n, float *out) {
    if (!aabbs || !out || n == 0) return -1;
    if (n == 1) { /* lbvh.h:61-68, then ConstructLBVH_Buff of a single leaf */
        memcpy(out, aabbs, 6 * sizeof(float));
        out[6] = -(float)0u; out[7] = 0.0f;
        return 0;
    }
    float smin[3], smax[3];
    for (int a = 0; a < 3; a++) { smin[a] = aabbs[a]; smax[a] = aabbs[3 + a]; }
    for (uint32_t i = 1; i < n; i++)
        for (int a = 0; a < 3; a++) {
            smin[a] = RMIN(smin[a], aabbs[i * 6 + a]);
            smax[a] = RMAX(smax[a], aabbs[i * 6 + 3 + a]);
        }
    key_t_ *keys = (key_t_ *)malloc(sizeof(key_t_) * n);
    for (uint32_t i = 0; i < n; i++) {
        const float *b = aabbs + (size_t)i * 6;
        float p[3];
        for (int a = 0; a < 3; a++) {
            p[a] = (b[a] + b[3 + a]) * 0.5f;
            p[a] -= smin[a];
            p[a] /= (smax[a] - smin[a]); /* host C++ division (lbvh.h:102-104) */
        }
        keys[i].code = morton_code(p[0], p[1], p[2]);
        keys[i].id = i;
        float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
        keys[i].diag2 = dx * dx + dy * dy + dz * dz; /* glm::dot */
    }
    qsort(keys, n, sizeof(key_t_), key_cmp);
    uint8_t *ub = (uint8_t *)malloc(n);
    for (uint32_t i = 1; i < n; i++) { /* lbvh.h:124-130 */
        uint32_t x = keys[i - 1].code ^ keys[i].code;
        uint8_t h = 0;
        while (x > 0) { x >>= 1; h++; }
        ub[i - 1] = h;
    }
    const uint32_t total = 2 * n - 1;
    lnode *nd = (lnode *)calloc(total, sizeof(lnode));
    for (uint32_t i = 0; i < n; i++) { /* leaves :135-150 */
        nd[i].parent = nd[i].left = nd[i].right = -1;
        nd[i].obj = keys[i].id;
        memcpy(nd[i].mn, aabbs + (size_t)keys[i].id * 6, 3 * sizeof(float));
        memcpy(nd[i].mx, aabbs + (size_t)keys[i].id * 6 + 3, 3 * sizeof(float));
    }
    /* internal nodes :152-210; queue of internal indices (node n+i has idx i) */
    uint32_t *q = (uint32_t *)malloc(sizeof(uint32_t) * (n - 1) * 2 + 8);
    uint32_t qh = 0, qt = 0, qcap = (n - 1) * 2 + 2;
    for (uint32_t i = 0; i < n - 1; i++) {
        nd[n + i].parent = nd[n + i].left = nd[n + i].right = -1;
        q[qt++] = i;
    }
    uint32_t level = ub[0];
    for (uint32_t i = 0; i < n - 1; i++) level = RMIN((uint32_t)ub[i], level);
    uint32_t nxt = 0, init_q = n - 1;
    while (qh != qt) {
        uint32_t idx = q[qh % qcap];
        qh++;
        init_q--;
        int solved = 0;
        lnode *cur = &nd[n + idx];
        if (ub[idx] <= level) {
            int L = (int)idx; while (nd[L].parent >= 0) L = nd[L].parent;
            int R = (int)idx + 1; while (nd[R].parent >= 0) R = nd[R].parent;
            cur->left = L; cur->right = R;
            nd[L].parent = (int)(n + idx); nd[R].parent = (int)(n + idx);
            for (int a = 0; a < 3; a++) {
                cur->mn[a] = RMIN(nd[L].mn[a], nd[R].mn[a]);
                cur->mx[a] = RMAX(nd[L].mx[a], nd[R].mx[a]);
            }
            solved = 1;
        } else {
            if (nxt == 0 || nxt > ub[idx]) nxt = ub[idx];
        }
        if (!solved) { q[qt % qcap] = idx; qt++; }
        if (init_q == 0) { level = nxt; nxt = 0; init_q = qt - qh; }
    }
    /* ConstructLBVH_Buff :216-268: BFS from the root */
    int root = (int)total - 1;
    while (nd[root].parent >= 0) root = nd[root].parent;
    uint32_t *bq = (uint32_t *)malloc(sizeof(uint32_t) * total * 2);
    uint32_t bh = 0, bt = 0, index = 0;
    bq[bt++] = (uint32_t)root; bq[bt++] = 0;
    while (bh != bt) {
        uint32_t cn = bq[bh++], parent = bq[bh++];
        uint32_t L = 0, R = 0;
        if (nd[cn].left >= 0) { bq[bt++] = (uint32_t)nd[cn].left; bq[bt++] = index; L = index + (bt - bh) / 2; }
        if (nd[cn].right >= 0) { bq[bt++] = (uint32_t)nd[cn].right; bq[bt++] = index; R = index + (bt - bh) / 2; }
        float *o = out + (size_t)index * 8;
        memcpy(o, nd[cn].mn, 3 * sizeof(float));
        memcpy(o + 3, nd[cn].mx, 3 * sizeof(float));
        (void)R;
        o[6] = (L == 0) ? -(float)nd[cn].obj : (float)L;
        o[7] = (float)parent;
        index++;
    }
    free(bq); free(q); free(nd); free(ub); free(keys);
    return 0;
}
