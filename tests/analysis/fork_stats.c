/*
 * fork_stats.c -- offline analysis (not product, not a test): what would it cost to run every
 * IOW-03 sample as a function of the stale RI entries it inherits, instead of speculating on
 * them?
 *
 * IOW-03 keeps its 4-deep ray stack across the samples of a pixel (03.glsl:260-264). The
 * parent-RI lookup (03.glsl:316-319) can read entries 1..3 above the stack top before the
 * sample wrote them. Those entries hold values from V = {0, 1, every material RI} (pushes carry
 * 1.0, an inherited RI, material.z or another read of the stack). So a sample is a function of
 * (entries 1..3 it reads before writing) -> (colour, counters, written entries). "Fork on read"
 * evaluates that function for every value of V at each such read, sharing the prefix.
 *
 * For sampled pixels of a scene this prints, per sample: segments on the exact path, segments
 * over all branches (prefix shared), branches, and the longest branch.
 *
 * Lives under tests/ because it builds on the CPU oracle (test infrastructure); it is an offline
 * study, not a test.  Driven by tests/analysis/fork_stats.py, which compiles it to /tmp.
 */
#include "../../oracle/rt_oracle.c"

#define MAXV 8
typedef struct {
    float val[MAXV];
    int nv;
} vset;

/* one execution of sample `sidx` from stack state K (entries 1..3 given by `assume`, where
 * known bit e set means the value is assumed), stopping at the first read of an unassumed,
 * unwritten entry.  Returns 1 when complete, 0 when it needs entry *need (after *seg_at
 * segments). */
typedef struct {
    int complete, need;
    uint64_t seg;
    int reads;      /* entries read before written (incoming reads) on this path */
    int written;    /* entries written */
    float out_ri[IOW_STACK];
} run_t;

static run_t run_sample(const iow_scene *S, const iow_stack *K0, int known0, v3 ro, v3 rd, int sidx) {
    iow_stack Kv = *K0, *K = &Kv;
    int known = known0 | 1; /* entry 0 is written by the first push */
    int written = 0, reads = 0;
    ctr c = {0, 0, 0, 0, 0, 0};
    run_t out;
    memset(&out, 0, sizeof(out));
    ray_t r0 = {ro, rd};
    if (K->size < IOW_STACK) written |= 1 << K->size;
    iow_push(K, r0, 1.0f, 1.0f, 0, &c);
    int skip = 0;
    while (K->size > 0) {
        K->size--;
        float contribution = K->contrib[K->size], ri = K->ri[K->size];
        int bounced = K->bounce[K->size];
        ray_t cur = K->ray[K->size];
        rrd_t data = launch_ray(S, cur.o, cur.d, 32000.0f, contribution, &c);
        int hit = dot(data.normal, data.normal) > 0.9f;
        if (bounced < S->max_bounces && hit) {
            bounced++;
            int spawnRefl = 0, spawnRefr = 0;
            v3 refr_dir = V3(0, 0, 0), refl_dir = V3(0, 0, 0);
            float cos_t = dot(data.normal, cur.d);
            float sin_t = sqrtf(1.0f - cos_t * cos_t);
            float target_ri;
            {
                int pi = K->size - 1 - skip;
                if (cos_t > 0 && pi >= 0 && pi < IOW_STACK) {
                    if (!(written & (1 << pi))) {
                        reads |= 1 << pi;
                        if (!(known & (1 << pi))) {
                            out.complete = 0; out.need = pi; out.seg = c.seg;
                            return out;
                        }
                    }
                }
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
                refr_dir = data.reflected; spawnRefl = 1; refl_c = 1.0f;
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
                if (K->size < IOW_STACK) written |= 1 << K->size;
                iow_push(K, nr, contribution * refl_c, ri, bounced, &c);
            }
            if (spawnRefr) {
                ray_t nr = {add(data.point, mul(n_, 0.000015f)), refr_dir};
                if (K->size < IOW_STACK) written |= 1 << K->size;
                iow_push(K, nr, contribution * refr_c, target_ri, bounced, &c);
            }
        } else skip = 0;
    }
    out.complete = 1; out.seg = c.seg; out.reads = reads; out.written = written;
    memcpy(out.out_ri, K->ri, sizeof(out.out_ri));
    return out;
}

/* total segments over all branches (prefix shared), leaves, longest branch */
static void fork_work(const iow_scene *S, iow_stack *K, int known, const vset *V, v3 ro, v3 rd, int sidx,
                      uint64_t *work, uint64_t *leaves, uint64_t *longest, int depth) {
    run_t r = run_sample(S, K, known, ro, rd, sidx);
    if (r.complete || depth > 6) {
        *work += r.seg; *leaves += 1;
        if (r.seg > *longest) *longest = r.seg;
        return;
    }
    uint64_t pre = r.seg;
    *work += pre;
    for (int v = 0; v < V->nv; v++) {
        iow_stack K2 = *K;
        K2.ri[r.need] = V->val[v];
        uint64_t w = 0, l = 0, lg = 0;
        fork_work(S, &K2, known | (1 << r.need), V, ro, rd, sidx, &w, &l, &lg, depth + 1);
        *work += w - pre; /* each child counts the shared prefix once */
        *leaves += l;
        if (lg > *longest) *longest = lg;
    }
}

/* per (pixel, sample): exact segments, fork work, leaves, longest branch, incoming-read mask
 * (on the exact path) -> out[(i*spp + s)*5 + k] */
int fork_stats(const float *types, const float *records, uint32_t n, const orc_camera *cam, const orc_params *p,
               const int *pix, int npix, const float *vals, int nvals, uint64_t *out) {
    const int W = p->width, H = p->height, spp = p->spp;
    float *sf = (float *)malloc(sizeof(float) * 2 * spp);
    float *fb = (float *)malloc(sizeof(float) * 3 * spp);
    int *ring = (int *)malloc(sizeof(int) * 2 * spp);
    orc_sample_tables(spp, sf, fb, ring);
    iow_scene S = {types, records, n, sf, fb, ring, spp, p->max_bounces};
    vset V;
    V.nv = nvals < MAXV ? nvals : MAXV;
    for (int i = 0; i < V.nv; i++) V.val[i] = vals[i];
    const v3 D = V3(cam->dir[0], cam->dir[1], cam->dir[2]);
    const v3 P = V3(cam->pos[0], cam->pos[1], cam->pos[2]);
    const float sd = 1.0f / (2.0f * (float)tan((double)(cam->fov_y_rad * 0.5f)));
    int grid = 1;
    while (grid * grid < spp) grid++;
#pragma omp parallel for schedule(dynamic, 1) num_threads(orc_num_threads())
    for (int i = 0; i < npix; i++) {
        int xx = pix[2 * i], yy = pix[2 * i + 1];
        iow_stack K;
        memset(&K, 0, sizeof(K));
        int w0 = 0;
        float ri0[IOW_STACK] = {0, 0, 0, 0};
        float aspect = (float)W * rcp((float)H);
        float sx = (aspect * ((float)xx * 2.0f - (float)W)) * rcp(2.0f * (float)W);
        float sy = ((float)yy * 2.0f - (float)H) * rcp(2.0f * (float)H);
        float dsx = aspect * rcp((float)(W * grid));
        float dsy = 1.0f * rcp((float)(H * grid));
        v3 look_at = add(P, mul(D, cam->focus_dist));
        v3 up = V3(0, 1, 0);
        v3 cr = cross(D, up), cu = cross(cr, D);
        for (int s = 0; s < spp; s++) {
            int ix = ring[2 * s], iy = ring[2 * s + 1];
            if (ix < 0) break;
            float rx = (sf[2 * s] * cam->aperture) * 0.5f, ry = (sf[2 * s + 1] * cam->aperture) * 0.5f;
            v3 ro = add(add(P, mul(cr, rx)), mul(cu, ry));
            v3 ld = normalize(sub(look_at, ro));
            v3 r_ = cross(ld, up), u_ = cross(cr, ld);
            v3 rd = normalize(add(add(mul(ld, sd), mul(r_, sx + dsx * (float)ix)), mul(u_, sy + dsy * (float)iy)));
            uint64_t *o0 = out + ((size_t)i * spp + s) * 12;
            for (int e = 1; e < IOW_STACK; e++) { uint32_t b; memcpy(&b, &K.ri[e], 4); o0[8 + e] = b; }
            run_t ex = run_sample(&S, &K, 0xF, ro, rd, s);
            uint64_t w = 0, l = 0, lg = 0;
            if (s == 0) { w = ex.seg; l = 1; lg = ex.seg; }
            else fork_work(&S, &K, 0x1, &V, ro, rd, s, &w, &l, &lg, 0);
            uint64_t *o = out + ((size_t)i * spp + s) * 12;
            o[0] = ex.seg; o[1] = w; o[2] = l; o[3] = lg; o[4] = (uint64_t)ex.reads;
            o[5] = 0;
            if (s > 0) { run_t r1 = run_sample(&S, &K, 0x1, ro, rd, s); o[5] = r1.complete ? ex.seg : r1.seg; }
            /* the GPU pipeline's guess (k_iow03_prep): entries sample 0 wrote keep its values,
             * others are 0 for sample 1 and the scene prior 1.5 from sample 2 */
            o[6] = ex.seg; o[7] = 0; o[8] = (uint64_t)ex.written;
            if (s == 0) { w0 = ex.written; memcpy(ri0, ex.out_ri, sizeof(ri0)); }
            else {
                iow_stack G = K;
                for (int e = 1; e < IOW_STACK; e++) G.ri[e] = (w0 & (1 << e)) ? ri0[e] : (s == 1 ? 0.0f : 1.5f);
                run_t g = run_sample(&S, &G, 0xF, ro, rd, s);
                int bad = 0;
                for (int e = 1; e < IOW_STACK; e++)
                    if ((g.reads & (1 << e)) && G.ri[e] != K.ri[e]) bad = 1;
                o[6] = g.seg; o[7] = (uint64_t)bad;
            }
            memcpy(K.ri, ex.out_ri, sizeof(K.ri)); /* stale entries carry to the next sample */
            K.size = 0;
        }
    }
    free(sf); free(fb); free(ring);
    return 0;
}
