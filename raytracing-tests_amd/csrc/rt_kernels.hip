// rt_kernels.hip -- the render hot path for gfx950 (CDNA4, wave64).
//
// One thread renders one pixel and walks its samples in order, exactly like the
// reference's invocation (IOW) or workgroup (INW) does, so the per-pixel reduction order
// is the reference's sequential one.  A 256-thread block covers a 16x16 pixel tile with
// each wave on an 8x8 quadrant (coherent camera rays).  Per-thread ray / node stacks live
// in LDS in a [slot][thread] layout: lane l of a wave touches bank (l mod 32) whatever the
// stack depth, so divergent stack pointers never conflict.
//
// Kernels and the shaders they replace (paths relative to /root/reference/Raytracing-Sandbox/Src/):
//   k_iow01 <- In-One-Weekend/01_Adding_Sphere/computeShaderSrc.glsl:98-146
//   k_iow03 <- In-One-Weekend/03_Shadows_and_Materials/computeShaderSrc.glsl:196-430
//   k_inw   <- In-Next-Week/01_BoundingVolumeHierarchy/computeShaderSrc.glsl:230-675 (LIGHTS=false)
//              In-Next-Week/04_Lights_Camera_And_Action/computeShaderSrc.glsl:243-773 (LIGHTS=true)
#include <cstdlib>
#include <type_traits>

#include "rt_kernels.hpp"
#include "rt_math.hpp"

namespace rtk {


// ----------------------------------------------------------------------- pixel mapping
struct Pix { int x, y; bool in_image; size_t out; bool valid; };

__device__ __forceinline__ Pix map_pixel(const Frame &f) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lx = ((wave & 1) << 3) | (lane & 7), ly = ((wave >> 1) << 3) | (lane >> 3);
    Pix p;
    if (f.tiles == nullptr) {
        const int nbx = (f.tw + 15) >> 4;
        const int bx = blockIdx.x % nbx, by = blockIdx.x / nbx;
        const int rx = bx * 16 + lx, ry = by * 16 + ly;
        p.x = f.x0 + rx; p.y = f.y0 + ry;
        p.valid = rx < f.tw && ry < f.th && p.x >= 0 && p.y >= 0 && p.x < f.W && p.y < f.H;
        p.in_image = p.valid;
        p.out = (size_t)p.y * f.W + p.x;
    } else {
        const int per = f.tile_size >> 4, sub = per * per;
        const int tile = blockIdx.x / sub, s = blockIdx.x % sub;
        const int ix = (s % per) * 16 + lx, iy = (s / per) * 16 + ly;
        p.x = f.tiles[2 * tile] * f.tile_size + ix;
        p.y = f.tiles[2 * tile + 1] * f.tile_size + iy;
        p.in_image = p.x < f.W && p.y < f.H;
        p.valid = true;  // packed slots outside the image are written as zero
        p.out = (size_t)tile * f.tile_size * f.tile_size + (size_t)iy * f.tile_size + ix;
    }
    return p;
}

// occupancy slots (RT_DIAG_OCC): pairs (wave iterations, lanes) of: the fold loop's iterations with
// busy lanes; wide-walk trips with walking lanes; their node steps; leaf batches; beam-list trips;
// reference-walk entries (lanes that fell back); surrounding-RI queries; node steps with the
// lanes on the first stepping lane's node; node steps where every stepping lane is on one node
enum { kOccSeg = 0, kOccWalk = 2, kOccNode = 4, kOccLeaf = 6, kOccBeam = 8, kOccRef = 10, kOccRi = 12, kOccSame = 14,
       kOccUni = 16, kOccSlots = 18 };
struct Ctr {
    uint32_t seg = 0, nodes = 0, prims = 0, shadow = 0, drops = 0, nans = 0;
    uint32_t refw = 0;  // INW closest-hit queries the wide walk / beam list handed to the LBVH walks (Frame::walk_ctr)
    unsigned long long *wdbg = nullptr;  // diagnostics: this wave's kDbg* row in LDS, or null
#ifdef RT_DIAG_SPLIT
    unsigned long long cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // INW phase cycles of this wave (k_inw_pm/sm)
    unsigned long long rnd[2] = {0, 0};  // k_inw_pm: wave cycles of the primary (0) and bounce (1) rounds
#endif
#ifdef RT_DIAG_OCC
    unsigned long long occ[kOccSlots] = {};  // INW lane occupancy per phase (OCC_TALLY), wave-uniform
#endif
};
// INW lane occupancy (diagnostic builds, -DRT_DIAG_OCC; tools/inw_occ.py): per phase, the wave
// iterations and the lanes in them doing that phase's work, summed into Frame::dbg[32 + slot] at exit
#ifdef RT_DIAG_OCC
#define OCC_TALLY(c, k, pred)                                                    \
    do {                                                                         \
        (c).occ[k] += 1;                                                         \
        (c).occ[(k) + 1] += (unsigned long long)__popcll(__ballot(pred));        \
    } while (0)
#else
#define OCC_TALLY(c, k, pred) ((void)0)
#endif
// INW phase split (diagnostic builds, -DRT_DIAG_SPLIT): shader-clock cycles per wave of a phase,
// summed into Frame::dbg slots by the fold kernels at exit
#ifdef RT_DIAG_SPLIT
#define INW_T0(t) const unsigned long long t = (unsigned long long)clock64()
#define INW_CYC(c, k, t) ((c).cyc[k] += (unsigned long long)clock64() - (t))
#else
#define INW_T0(t) ((void)0)
#define INW_CYC(c, k, t) ((void)0)
#endif
// Diagnostics (rt_debug_counters).  Tallies go to a per-wave LDS row, written by the first
// active lane, so they cost no registers when off and are exact inside divergent code.
__device__ __forceinline__ bool first_active_lane() {
    return (int)(threadIdx.x & 63) == __ffsll((long long)__ballot(1)) - 1;
}
// wave cycles of a phase (shader clock)
#define DBG_T0(f, t) const unsigned long long t = c.wdbg ? (unsigned long long)clock64() : 0ull
#define DBG_CYC(f, c, slot, t)                                                        \
    do {                                                                              \
        if ((c).wdbg) {                                                               \
            const unsigned long long d_ = (unsigned long long)clock64() - (t);        \
            if (first_active_lane()) (c).wdbg[slot] += d_;                            \
        }                                                                             \
    } while (0)
// count one wave-iteration of a phase and how many lanes take part
#define DBG_TALLY(f, c, slot, pred)                                                   \
    do {                                                                              \
        if ((c).wdbg) {                                                               \
            const unsigned long long m_ = __ballot(pred);                             \
            if (first_active_lane()) {                                                \
                (c).wdbg[slot] += 1; (c).wdbg[(slot) + 1] += (unsigned long long)__popcll(m_); \
            }                                                                         \
        }                                                                             \
    } while (0)

// Finer phase split of the wave-cooperative segment (diagnostic builds only, -DRT_DIAG_SPLIT):
// reuses tally slots that stay zero in that mode (see tools/latency_probe.py).
#ifdef RT_DIAG_SPLIT
#define SPL_T0(t) const unsigned long long t = (unsigned long long)clock64()
#define SPL_CYC(w, slot, t)                                                           \
    do {                                                                              \
        if (w) {                                                                      \
            const unsigned long long d_ = (unsigned long long)clock64() - (t);        \
            if (first_active_lane()) (w)[slot] += d_;                                 \
        }                                                                             \
    } while (0)
#else
#define SPL_T0(t) ((void)0)
#define SPL_CYC(w, slot, t) ((void)0)
#endif

__device__ __forceinline__ void flush(const Frame &f, const Ctr &c) {
    if (c.wdbg && (threadIdx.x & 63) == 0)
        for (int i = 0; i < kDbgSlots; i++) atomicAdd(f.dbg + i, c.wdbg[i]);
    if (!f.counters) return;
    unsigned long long v[6] = {c.seg, c.nodes, c.prims, c.shadow, c.drops, c.nans};
#pragma unroll
    for (int i = 0; i < 6; i++) {
        unsigned long long s = wave_sum(v[i]);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(f.counters + i, s);
    }
    if (f.walk_ctr) {
        const unsigned long long s = wave_sum((unsigned long long)c.refw);
        if ((threadIdx.x & 63) == 0 && s) atomicAdd(f.walk_ctr, s);
    }
}

// ============================================================================ IOW-01
__global__ __launch_bounds__(kBlock) void k_iow01(Frame f) {
    Pix px = map_pixel(f);
    if (!px.valid) return;  // no cross-lane work in this kernel
    f3 color = f3{0, 0, 0};
    if (px.in_image) {
        const f3 D = mk(f.dir[0], f.dir[1], f.dir[2]), P = mk(f.pos[0], f.pos[1], f.pos[2]);
        const f3 C = mk(f.sphere[0], f.sphere[1], f.sphere[2]);
        const float R = f.sphere[3];
        float aspect = (float)f.W * rcp((float)f.H);
        f3 cr = cross(D, f3{0, 1, 0}), cu = cross(cr, D);
        float sx = ((float)px.x * 2.0f - (float)f.W) * rcp(2.0f * (float)f.W);
        sx *= aspect;
        float sy = ((float)px.y * 2.0f - (float)f.H) * rcp(2.0f * (float)f.H);
        f3 pis = ((P + D * f.focus) + cr * sx) + cu * sy;
        // CreatePlane((0,-2,0),(0,-2,1),(1,-2,0))
        const f3 p1 = f3{0, -2, 0};
        f3 pn = normalize(cross(f3{0, -2, 1} - p1, f3{1, -2, 0} - p1));
        float pw = -(pn.x * p1.x + pn.y * p1.y + pn.z * p1.z);
        f3 ro = P, rd = normalize(pis - P);
        color = background(rd, false);
        float min_depth = 10000.0f;
        float t = -(pn.x * ro.x + pn.y * ro.y + pn.z * ro.z + pw) * rcp(pn.x * rd.x + pn.y * rd.y + pn.z * rd.z);
        if (min_depth > t && t > 0.0f) { color = f3{0.8f, 0.1f, 0.7f}; min_depth = t; }
        f3 rs = ro - C;
        float hb = dot(rd, rs), a = dot(rd, rd), c = dot(rs, rs) - R * R;
        float det = hb * hb - a * c;
        t = (det > 0.0f && hb < 0.0f) ? ((-hb - __builtin_sqrtf(det)) * rcp(a)) : -1.0f;
        if (min_depth > t && t > 0.0f) {
            f3 ip = ro + rd * t;
            color = f.show_normal ? normalize(ip - C) : f3{1, 0, 0};
        }
    }
    reinterpret_cast<float4 *>(f.out_rgba)[px.out] = make_float4(color.x, color.y, color.z, px.in_image ? 1.0f : 0.0f);
}

// ============================================================================ IOW-03
struct RayRet { f3 point, normal, reflected, color, material; float scat0, scat1; };

struct IowObj { f3 pos; int type; m3 M; f3 scale, is; };

__device__ __forceinline__ IowObj iow_obj(const float *__restrict__ h) {
    IowObj o;
    o.pos = mk(h[0], h[1], h[2]);
    o.type = (int)h[3];
    o.M.c0 = mk(h[4], h[5], h[6]); o.M.c1 = mk(h[7], h[8], h[9]); o.M.c2 = mk(h[10], h[11], h[12]);
    o.scale = mk(h[13], h[14], h[15]);
    o.is = mk(h[16], h[17], h[18]);
    return o;
}

// Culling-only slab test for the IOW BVH (never decides a hit: the exact object test does).
// Boxes are inflated on the host and the limit carries relative slack, so an object whose
// exact t can win is never culled.  (plane - o) * (1/d) keeps a small relative error in t;
// the fused form plane*(1/d) - o*(1/d) would cancel catastrophically for large o/d (INW uses it
// only under the bound of cull4nf below).
__device__ __forceinline__ bool cull_slab(float4 n0, float4 n1, f3 o, f3 id, float lim, float &te) {
    const float x0 = (n0.x - o.x) * id.x, x1 = (n0.w - o.x) * id.x;
    const float y0 = (n0.y - o.y) * id.y, y1 = (n1.x - o.y) * id.y;
    const float z0 = (n0.z - o.z) * id.z, z1 = (n1.y - o.z) * id.z;
    te = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    const float tx = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    return te <= tx && tx >= -1e-3f && te <= lim;
}

// Same test for one child of a 4-wide node; returns the entry t, or kMiss when culled.
constexpr float kMiss = __builtin_huge_valf();
__device__ __forceinline__ float cull_t(float lx, float ly, float lz, float hx, float hy, float hz, f3 o, f3 id,
                                        float lim) {
    const float x0 = (lx - o.x) * id.x, x1 = (hx - o.x) * id.x;
    const float y0 = (ly - o.y) * id.y, y1 = (hy - o.y) * id.y;
    const float z0 = (lz - o.z) * id.z, z1 = (hz - o.z) * id.z;
    const float te = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
    const float tx = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
    return (te <= tx && tx >= -1e-3f && te <= lim) ? te : kMiss;
}
// The four children of a 4-wide node at once.  The node is SoA over the children (lx = the
// four children's low x planes, ...), so (plane - o) * (1/d) runs on child pairs with packed
// fp32 arithmetic (v_pk_add_f32 / v_pk_mul_f32: two lanes' worth per instruction); min / max
// stay scalar.  Same operations and rounding per plane as cull_t.
typedef float pf2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ pf2 pk(float a, float b) { return pf2{a, b}; }
__device__ __forceinline__ void cull4(const float4 lx, const float4 ly, const float4 lz, const float4 hx,
                                      const float4 hy, const float4 hz, f3 o, f3 id, float lim, float &t0,
                                      float &t1, float &t2, float &t3) {
    const pf2 ox = pk(o.x, o.x), oy = pk(o.y, o.y), oz = pk(o.z, o.z);
    const pf2 ix = pk(id.x, id.x), iy = pk(id.y, id.y), iz = pk(id.z, id.z);
    const pf2 ax01 = (pk(lx.x, lx.y) - ox) * ix, bx01 = (pk(hx.x, hx.y) - ox) * ix;
    const pf2 ay01 = (pk(ly.x, ly.y) - oy) * iy, by01 = (pk(hy.x, hy.y) - oy) * iy;
    const pf2 az01 = (pk(lz.x, lz.y) - oz) * iz, bz01 = (pk(hz.x, hz.y) - oz) * iz;
    const pf2 ax23 = (pk(lx.z, lx.w) - ox) * ix, bx23 = (pk(hx.z, hx.w) - ox) * ix;
    const pf2 ay23 = (pk(ly.z, ly.w) - oy) * iy, by23 = (pk(hy.z, hy.w) - oy) * iy;
    const pf2 az23 = (pk(lz.z, lz.w) - oz) * iz, bz23 = (pk(hz.z, hz.w) - oz) * iz;
    auto one = [&](float x0, float x1, float y0, float y1, float z0, float z1) {
        const float te = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fminf(z0, z1));
        const float tx = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1));
        return (te <= tx && tx >= -1e-3f && te <= lim) ? te : kMiss;
    };
    t0 = one(ax01.x, bx01.x, ay01.x, by01.x, az01.x, bz01.x);
    t1 = one(ax01.y, bx01.y, ay01.y, by01.y, az01.y, bz01.y);
    t2 = one(ax23.x, bx23.x, ay23.x, by23.x, az23.x, bz23.x);
    t3 = one(ax23.y, bx23.y, ay23.y, by23.y, az23.y, bz23.y);
}
// The same test with the planes already split into near and far by the ray's octant (the caller
// loads plane a + 3 s_a as near and a + 3 (1 - s_a) as far, s_a = 1 when d_a < 0).  With a finite,
// nonzero reciprocal the slab value (p - o) * (1/d) is monotone in p, so the near plane's value is
// the min of the pair and the far plane's the max: te and tx have cull4's bits and the 12 min / max
// per node are gone.  A zero component (1/d = inf) keeps at least the boxes cull4 keeps: the pair
// form's fminf / fmaxf drop a NaN (origin on a plane) and then cull, the octant form keeps the box.
// The culling BVH only decides which objects get the exact test (iow_launch_ray), so that is exact.
__device__ __forceinline__ void cull4o(const float4 nx, const float4 ny, const float4 nz, const float4 fx,
                                       const float4 fy, const float4 fz, f3 o, f3 id, float lim, float &t0,
                                       float &t1, float &t2, float &t3) {
    const pf2 ox = pk(o.x, o.x), oy = pk(o.y, o.y), oz = pk(o.z, o.z);
    const pf2 ix = pk(id.x, id.x), iy = pk(id.y, id.y), iz = pk(id.z, id.z);
    const pf2 ax01 = (pk(nx.x, nx.y) - ox) * ix, bx01 = (pk(fx.x, fx.y) - ox) * ix;
    const pf2 ay01 = (pk(ny.x, ny.y) - oy) * iy, by01 = (pk(fy.x, fy.y) - oy) * iy;
    const pf2 az01 = (pk(nz.x, nz.y) - oz) * iz, bz01 = (pk(fz.x, fz.y) - oz) * iz;
    const pf2 ax23 = (pk(nx.z, nx.w) - ox) * ix, bx23 = (pk(fx.z, fx.w) - ox) * ix;
    const pf2 ay23 = (pk(ny.z, ny.w) - oy) * iy, by23 = (pk(fy.z, fy.w) - oy) * iy;
    const pf2 az23 = (pk(nz.z, nz.w) - oz) * iz, bz23 = (pk(fz.z, fz.w) - oz) * iz;
    auto one = [&](float n0, float f0, float n1, float f1, float n2, float f2) {
        const float te = fmaxf(fmaxf(n0, n1), n2);
        const float tx = fminf(fminf(f0, f1), f2);
        return (te <= tx && tx >= -1e-3f && te <= lim) ? te : kMiss;
    };
    t0 = one(ax01.x, bx01.x, ay01.x, by01.x, az01.x, bz01.x);
    t1 = one(ax01.y, bx01.y, ay01.y, by01.y, az01.y, bz01.y);
    t2 = one(ax23.x, bx23.x, ay23.x, by23.x, az23.x, bz23.x);
    t3 = one(ax23.y, bx23.y, ay23.y, by23.y, az23.y, bz23.y);
}
__device__ __forceinline__ void cswap(float &ta, int &ka, float &tb, int &kb) {
    const bool sw = tb < ta;
    const float t = sw ? tb : ta;
    const int k = sw ? kb : ka;
    tb = sw ? ta : tb; kb = sw ? ka : kb;
    ta = t; ka = k;
}

// Local ray of an object (the `M*(o-p)`, `normalize(M*d)` of t_RayXObj, 03...glsl:55-73).
// Objects whose matrix is glm::mat3(1) transform the direction identically, so M*gd and
// normalize(M*gd) are evaluated once per ray and passed in (same operations, same bits: 1*x
// folds to x, the 0*y terms are kept because IEEE forbids folding them).
__device__ __forceinline__ void iow_local(const float *h, const IowObj &ob, f3 go, f3 gd, f3 td_id, f3 nd_id, f3 &to,
                                          f3 &td, f3 &nd) {
    const m3 I = m3{f3{1.0f, 0.0f, 0.0f}, f3{0.0f, 1.0f, 0.0f}, f3{0.0f, 0.0f, 1.0f}};
    if (h[19] != 0.0f) { to = mul(I, go - ob.pos); td = td_id; nd = nd_id; }
    else { to = mul(ob.M, go - ob.pos); td = mul(ob.M, gd); nd = normalize(td); }
}
__device__ __forceinline__ void iow_id_dirs(f3 gd, f3 &td_id, f3 &nd_id) {
    const m3 I = m3{f3{1.0f, 0.0f, 0.0f}, f3{0.0f, 1.0f, 0.0f}, f3{0.0f, 0.0f, 1.0f}};
    td_id = mul(I, gd);
    nd_id = normalize(td_id);
}
// exact test of object j; keeps the reference's rule: nearer t, or the lower index on a tie
__device__ __forceinline__ void iow_test(const IowScene &S, int j, f3 go, f3 gd, f3 td_id, f3 nd_id, float &min_t,
                                         int &best) {
    const float *h = S.hot + (size_t)j * kIowHot;
    const IowObj ob = iow_obj(h);
    f3 to, td, nd;
    iow_local(h, ob, go, gd, td_id, nd_id, to, td, nd);
    float t = -1.0f;
    if (ob.type == 2) t = t_ellipsoid(to, nd, ob.is);
    else if (ob.type == 1) t = t_cuboid(to, nd, ob.scale);
    if (t > 0.0f && (t < min_t || (t == min_t && j < best))) { min_t = t; best = j; }
}

// Hit attributes of the winner `best` at min_t (LaunchRay's tail, 03...glsl:221-255): the
// closest hit's normal and attributes are evaluated once after the search.
// cold = the winner's cold record (colour3, material3, scatter2) when min_t < max_t;
// td_id / nd_id = iow_id_dirs(gd), already computed by the search
__device__ __forceinline__ RayRet iow_eval_c(const IowScene &S, f3 go, f3 gd, f3 td_id, f3 nd_id, float min_t, int best,
                                             float max_t, float contrib, float4 c0, float4 c1) {
    RayRet r;
    if (min_t < max_t) {
        const float *hb = S.hot + (size_t)best * kIowHot;
        const IowObj ob = iow_obj(hb);
        f3 best_to, best_td, best_nd;
        iow_local(hb, ob, go, gd, td_id, nd_id, best_to, best_td, best_nd);
        f3 h = best_to + best_nd * min_t;
        f3 n = ob.type == 2 ? f3{h.x * ob.is.x * ob.scale.x, h.y * ob.is.y * ob.scale.y, h.z * ob.is.z * ob.scale.z}
                            : (ob.type == 1 ? cuboid_normal(h, ob.scale) : f3{0, 0, 0});
        r.color = mk(c0.x, c0.y, c0.z);
        r.material = mk(c0.w, c1.x, c1.y);
        r.scat0 = c1.z; r.scat1 = c1.w;
        const bool inside = dot(n, best_td) > 0.0f;
        f3 n_ = sel(inside, -n, n);
        f3 refl = reflect(best_td, n_);
        if (!inside) {
            f3 nir = normalize(cross(n_, best_td));
            f3 nn = normalize(cross(nir, n_));
            float s = r.scat1;
            float k = rcp_sqrt_domain(__builtin_sqrtf(1.0f + s * s));
            f3 mr = n_ * (s * k) + nn * k;
            refl = sel(dot(refl, n_) > dot(mr, n_), refl, mr);
        }
        r.point = go + gd * min_t;
        if (hb[19] != 0.0f) {
            // M is glm::mat3(1) (iow_local): inverse(M) is the constant the same formula gives
            // for the identity, folded at compile time (IEEE folding keeps its signed zeros and
            // the 0*x products of mul), so the bits are those of the general branch
            const m3 I = m3{f3{1.0f, 0.0f, 0.0f}, f3{0.0f, 1.0f, 0.0f}, f3{0.0f, 0.0f, 1.0f}};
            const m3 inv = inverse(I);
            r.normal = normalize(mul(inv, n));
            r.reflected = normalize(mul(inv, refl));
        } else {
            const m3 inv = inverse(ob.M);
            r.normal = normalize(mul(inv, n));
            r.reflected = normalize(mul(inv, refl));
        }
        r.color = r.color * contrib;
    } else {
        r.point = f3{0, 0, 0}; r.normal = f3{0, 0, 0};
        r.reflected = r.color = r.material = f3{0, 0, 0};
        r.scat0 = r.scat1 = 0.0f;
    }
    return r;
}
__device__ __forceinline__ RayRet iow_eval(const IowScene &S, f3 go, f3 gd, f3 td_id, f3 nd_id, float min_t, int best,
                                           float max_t, float contrib) {
    float4 c0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), c1 = c0;
    if (min_t < max_t) {
        const float4 *cold = reinterpret_cast<const float4 *>(S.cold + (size_t)best * kIowCold);
        c0 = cold[0]; c1 = cold[1];
    }
    return iow_eval_c(S, go, gd, td_id, nd_id, min_t, best, max_t, contrib, c0, c1);
}

// IOW BVH-stack slot p of a lane (16-bit links), [slot][lane]: two lanes share a dword, so two
// lanes of an LDS access group whose stack depths differ hit one bank (a 2-way conflict).
// RT_IOW_BSTK_PAIR (A/B variant, round 5): [slot pair][lane][2], the lane's two slots in its own
// dword, conflict-free at any depths: C2's LDS bank-conflict cycles fell from 17.5% to 13.0% of the
// LDS-active cycles, and the frame took 3.8% longer (3,835 / 3,857 against 3,702 / 3,699 ms, same
// box, profiles/r05_ab_stackless_iow_bstk.json): the address arithmetic of every push and pop costs more
// than the conflicts did.  b = the lane's base, lds + kBstkLane * lane.
#ifdef RT_IOW_BSTK_PAIR
__device__ __forceinline__ short &bslot(short *b, int p) { return b[(p >> 1) * (2 * kBlock) + (p & 1)]; }
constexpr int kBstkLane = 2;
#else
__device__ __forceinline__ short &bslot(short *b, int p) { return b[p * kBlock]; }
constexpr int kBstkLane = 1;
#endif

// LaunchRay 03...glsl:196-256.  The reference loops over every object and keeps the first
// strictly nearer hit, i.e. the minimum t with the lowest index among exact ties.  The BVH
// walk visits a superset of the objects that can attain that minimum and applies the same
// (t, index) rule, so it returns the same object and the same t bits.
// nodes: the 4-wide BVH (NS float4 per node: in LDS, 7; in global memory, 8), or null.
template <int BCAP, int NS = 8>
__device__ RayRet iow_launch_ray(const IowScene &S, const Frame &F_, f3 go, f3 gd, float max_t, float contrib,
                                 Ctr &c, short *bstk, const float4 *nodes) {
    DBG_T0(F_, t_ray);
    float min_t = max_t;
    int best = -1;
    c.seg++;
    f3 td_id, nd_id;
    iow_id_dirs(gd, td_id, nd_id);
    auto test = [&](int j) {
        c.prims++;
        iow_test(S, j, go, gd, td_id, nd_id, min_t, best);
    };
    const float dl2 = dot(gd, gd);
    if (!(dl2 > 0.0f)) {
        // zero or NaN direction (the TIR branch pushes the uninitialised reflection_dirn,
        // 03...glsl:331-332): normalize(M*gd) is NaN for every object, so every t is -1 and
        // the reference's loop finds no hit -- skip it.
        c.prims += S.n;
    } else if (nodes != nullptr && dl2 > 0.998f && dl2 < 1.002f) {
        // Ordered walk with postponed leaves (speculative traversal): a lane that reaches a
        // leaf parks it and keeps walking inner nodes; primitive tests run when every lane
        // of the wave holds one (or has finished), so they execute with full lanes.
        const f3 id = f3{__builtin_amdgcn_rcpf(gd.x), __builtin_amdgcn_rcpf(gd.y), __builtin_amdgcn_rcpf(gd.z)};
        // 4-wide BVH.  cur = link of the next node to enter: > 0 = wide node cur-1, <= 0 =
        // leaf of object -cur.  One step loads a 112-B node (7 x float4, SoA over the four
        // children), tests the four boxes, enters the nearest hit child and pushes the others
        // farthest-first.
        DBG_T0(F_, t_trav);
#ifndef RT_IOW_NO_OCTANT
        // the ray's near / far plane of each axis (cull4o): low planes are float4 0-2, high 3-5
        const int nxo = gd.x < 0.0f ? 3 : 0, nyo = gd.y < 0.0f ? 4 : 1, nzo = gd.z < 0.0f ? 5 : 2;
        const int fxo = 3 - nxo, fyo = 5 - nyo, fzo = 7 - nzo;
#endif
        int sp = 0, pend = -1, cur = S.root_link;
        bool walking = true, ovf = false;  // ovf: a child was dropped by a full stack
        float lim = min_t * 1.0001f + 1e-3f;  // culling limit, follows min_t
        for (;;) {
            DBG_TALLY(F_, c, kDbgTrav, walking);
            if (walking) {
                bool pop;
                if (cur > 0) {
                    const float4 *nd = nodes + NS * (cur - 1);
                    const float4 lk = nd[6];  // child links as int bits (set_iow_bvh)
                    c.nodes += 4;
                    float t0, t1, t2, t3;
#ifndef RT_IOW_NO_OCTANT
                    cull4o(nd[nxo], nd[nyo], nd[nzo], nd[fxo], nd[fyo], nd[fzo], go, id, lim, t0, t1, t2, t3);
#else
                    const float4 lx = nd[0], ly = nd[1], lz = nd[2], hx = nd[3], hy = nd[4], hz = nd[5];
                    cull4(lx, ly, lz, hx, hy, hz, go, id, lim, t0, t1, t2, t3);
#endif
                    int k0 = __float_as_int(lk.x), k1 = __float_as_int(lk.y), k2 = __float_as_int(lk.z),
                        k3 = __float_as_int(lk.w);
                    // sort (t, link) ascending; misses carry t = +inf
                    cswap(t0, k0, t1, k1); cswap(t2, k2, t3, k3);
                    cswap(t0, k0, t2, k2); cswap(t1, k1, t3, k3);
                    cswap(t1, k1, t2, k2);
                    // branch-free pushes, farthest first: a miss is written above the top and
                    // overwritten before it could be popped (the array has 3 spare entries)
                    int p = sp;
                    bslot(bstk, p) = (short)k3; p += t3 != kMiss;
                    bslot(bstk, p) = (short)k2; p += t2 != kMiss;
                    bslot(bstk, p) = (short)k1; p += t1 != kMiss;
                    if (p > BCAP) { ovf = true; p = BCAP; }
                    sp = p;
                    cur = k0;
                    pop = t0 == kMiss;
                } else {
                    pop = pend < 0;  // a leaf waits while the lane still holds one
                    if (pop) pend = -cur;
                }
                if (pop) {
                    if (sp == 0) walking = false;
                    else cur = bslot(bstk, --sp);
                }
            }
            if (__all(!walking || pend >= 0) || __popcll(__ballot(pend >= 0)) >= F_.leaf_batch) {
                DBG_TALLY(F_, c, kDbgLeaf, pend >= 0);
                DBG_T0(F_, t_leaf);
                if (pend >= 0) { test(pend); pend = -1; lim = min_t * 1.0001f + 1e-3f; }
                DBG_CYC(F_, c, kDbgCycLeaf, t_leaf);
                if (__all(!walking)) break;
            }
        }
        // a dropped subtree may hold the winner: the linear loop covers every object, and the
        // (t, index) rule makes re-testing the visited ones harmless
        if (ovf) for (uint32_t j = 0; j < S.n; j++) test((int)j);
        DBG_CYC(F_, c, kDbgCycTrav, t_trav);
    } else {
        for (uint32_t j = 0; j < S.n; j++) test((int)j);  // also the path for zero / NaN directions
    }
    RayRet r = iow_eval(S, go, gd, td_id, nd_id, min_t, best, max_t, contrib);
    DBG_CYC(F_, c, kDbgCycRay, t_ray);
    return r;
}

// ---------------------------------------------------------------- wave-cooperative closest hit
// When only a few lanes of a wave still trace (the long samples at the end of a pass), the
// wave runs their closest-hit queries one ray at a time with all 64 lanes: every lane culls
// 1/64 of the objects against their conservative boxes (the BVH's leaf boxes), the survivors
// are compacted into a wave list in LDS and tested exactly in parallel, and a wave reduction
// applies the reference's (t, lowest index) rule.  The candidate set is a superset of the one
// the BVH walk tests, so the winner and its t bits are the same (DESIGN.md "k_iow03s").
// Requires all 64 lanes active.
__device__ __forceinline__ float wave_min_all(float v) {
    v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xf, 0xf, false)));   // quad [1,0,3,2]
    v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xf, 0xf, false)));   // quad [2,3,0,1]
    v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xf, 0xf, false)));  // row half-mirror
    v = fminf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xf, 0xf, false)));  // row mirror
    const float r0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 0));
    const float r1 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 16));
    const float r2 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 32));
    const float r3 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), 48));
    return fminf(fminf(r0, r1), fminf(r2, r3));
}
__device__ __forceinline__ float bcast_f(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ uint32_t lanes_below(unsigned long long m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Closest hit of one (wave-uniform) ray with the whole wave.  wl: the wave's LDS list, entry k
// at lane k & 63's BVH-stack slot k >> 6 (bslot), cap entries (a multiple of 64 * kCoopR).  Returns the
// (uniform) winner and its cold record; nbox / nprim are the boxes and objects tested.  The
// loads of a batch of kCoopR boxes per lane, and a candidate's hot and cold records, are
// issued together: a lone ray's query costs about two memory latencies, not one per step.
constexpr int kCoopR = 8;
__device__ void iow_coop_search(const IowScene &S, f3 go, f3 gd, float max_t, short *wl, int cap, float &t_out,
                                int &j_out, float4 &c0_out, float4 &c1_out, uint32_t &nbox, uint32_t &nprim,
                                unsigned long long *wdbg = nullptr) {
    const int lane = (int)(threadIdx.x & 63);
    float bt = max_t;
    int bj = -1;
    float4 b0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), b1 = b0;  // cold record of this lane's best
    nbox = 0; nprim = 0;
    t_out = max_t; j_out = -1; c0_out = b0; c1_out = b0;
    const float dl2 = dot(gd, gd);
    if (!(dl2 > 0.0f)) {  // zero / NaN direction: no object can hit (see iow_launch_ray)
        nprim = S.n;
        return;
    }
    f3 td_id, nd_id;
    iow_id_dirs(gd, td_id, nd_id);
    const bool cull = S.obox != nullptr && dl2 > 0.998f && dl2 < 1.002f;
    const f3 id = f3{__builtin_amdgcn_rcpf(gd.x), __builtin_amdgcn_rcpf(gd.y), __builtin_amdgcn_rcpf(gd.z)};
    const float lim = max_t * 1.0001f + 1e-3f;
    const uint32_t n = S.n;
    uint32_t j0 = 0;
    while (j0 < n) {
        uint32_t cnt = 0, jb = j0;
        SPL_T0(t_cull);
        if (cull) {
            for (; j0 < n && cnt + 64 * kCoopR <= (uint32_t)cap; j0 += 64 * kCoopR) {
                const float2 *ob2 = reinterpret_cast<const float2 *>(S.obox + n);
                float4 a[kCoopR];
                float2 b[kCoopR];
#pragma unroll
                for (int r = 0; r < kCoopR; r++) {
                    const uint32_t j = j0 + 64 * r + lane, jj = j < n ? j : n - 1;
                    a[r] = S.obox[jj];
                    b[r] = ob2[jj];
                }
#pragma unroll
                for (int r = 0; r < kCoopR; r++) {
                    const uint32_t j = j0 + 64 * r + lane;
                    const bool cand =
                        j < n && cull_t(a[r].x, a[r].y, a[r].z, a[r].w, b[r].x, b[r].y, go, id, lim) != kMiss;
                    const unsigned long long cm = __ballot(cand);
                    if (cand) {
                        const uint32_t k = cnt + lanes_below(cm);
                        bslot(wl + kBstkLane * (k & 63), (int)(k >> 6)) = (short)j;
                    }
                    cnt += (uint32_t)__popcll(cm);
                }
            }
            nbox += (j0 < n ? j0 : n) - jb;
        } else {
            cnt = n - j0 < (uint32_t)cap ? n - j0 : (uint32_t)cap;
            j0 += cnt;
        }
        SPL_CYC(wdbg, kDbgTrav, t_cull);
        SPL_T0(t_exact);
        for (uint32_t k0 = 0; k0 < cnt; k0 += 64) {
            const uint32_t k = k0 + lane;
            if (k < cnt) {
                const int j = cull ? (int)bslot(wl + kBstkLane * (k & 63), (int)(k >> 6)) : (int)(jb + k);
                const float4 *cold = reinterpret_cast<const float4 *>(S.cold + (size_t)j * kIowCold);
                const float4 q0 = cold[0], q1 = cold[1];
                const int was = bj;
                iow_test(S, j, go, gd, td_id, nd_id, bt, bj);
                if (bj != was) { b0 = q0; b1 = q1; }
            }
        }
        nprim += cnt;
        SPL_CYC(wdbg, kDbgTravLanes, t_exact);
    }
    SPL_T0(t_red);
    const float tm = wave_min_all(bj >= 0 ? bt : max_t);
    unsigned long long m = __ballot(bj >= 0 && bt == tm);
    if (m == 0) return;
    int jm = -1, lm = 0;
    for (; m; m &= m - 1) {  // usually one lane; exact ties keep the lowest object index
        const int l = __ffsll((long long)m) - 1;
        const int j = __builtin_amdgcn_readlane(bj, l);
        if (jm < 0 || j < jm) { jm = j; lm = l; }
    }
    t_out = tm;
    j_out = jm;
    c0_out = make_float4(bcast_f(b0.x, lm), bcast_f(b0.y, lm), bcast_f(b0.z, lm), bcast_f(b0.w, lm));
    c1_out = make_float4(bcast_f(b1.x, lm), bcast_f(b1.y, lm), bcast_f(b1.z, lm), bcast_f(b1.w, lm));
    SPL_CYC(wdbg, kDbgLeaf, t_red);
}

__device__ __forceinline__ f3 fib_dir(float4 t, float s, f3 focus) {
    float x = t.x * s, y = t.y * s, z = t.z * s;
    f3 yc = focus;
    f3 zc = normalize(cross(f3{0, 1.0f, 0}, yc));
    f3 xc = normalize(cross(yc, zc));
    return normalize(focus + ((xc * x + yc * y) + zc * z));
}

__device__ __forceinline__ float schlick(float cosine, float ri) {
    float r0 = (1.0f - ri) * rcp(1.0f + ri);
    r0 = r0 * r0;
    float q = 1.0f - cosine;
    return r0 + (1.0f - r0) * (q * q * q * q * q);
}

// IOW ray stack (03...glsl:258-283): 4 entries of {orig, dirn, contribution, RI, bounces}.
// The entries outlive a sample: the parent-RI lookup (03...glsl:316-319) may read slots above
// the stack top that an earlier sample of the same pixel wrote, so a pixel's samples stay in
// order on one lane and the LDS slots persist across them.
// Two layouts: WIDE keeps `bounced` as a ninth float (any u_NumOfBounce); NARROW keeps it as
// a byte (u_NumOfBounce <= 255), which with a 12-entry BVH stack fits 4 blocks per CU in LDS.
constexpr int kIowStack = 4;
template <bool NARROW>
struct IowStack {
    static constexpr int kSlot = NARROW ? 8 : 9;
    float *base;          // LDS, [slot][thread]
    unsigned char *bb;    // NARROW: LDS, [entry][thread]
    int size;
    // sample-parallel mode: entries written by this sample, and entries whose stale RI this
    // sample read before writing them (its dependence on the previous sample's stack)
    unsigned wmask = 0, rmask = 0;
    __device__ __forceinline__ float &at(int entry, int k) { return base[(entry * kSlot + k) * kBlock]; }
    __device__ __forceinline__ int bounced(int e) {
        if constexpr (NARROW) return bb[e * kBlock];
        else return (int)at(e, 8);
    }
    __device__ __forceinline__ void set_bounced(int e, int b) {
        if constexpr (NARROW) bb[e * kBlock] = (unsigned char)b;
        else at(e, 8) = (float)b;
    }
    __device__ __forceinline__ void push(f3 o, f3 d, float contrib, float ri, int b, Ctr &c) {
        if (size < kIowStack) {
            at(size, 0) = o.x; at(size, 1) = o.y; at(size, 2) = o.z;
            at(size, 3) = d.x; at(size, 4) = d.y; at(size, 5) = d.z;
            at(size, 6) = contrib; at(size, 7) = ri; set_bounced(size, b);
            wmask |= 1u << size;
            size++;
        } else c.drops++;
    }
};

// One ray segment of LaunchRays (03...glsl:285-358): pop, closest hit, shade and push.
struct SegIn { f3 co, cd; float contribution, ri; int bounced; float4 fib; };
template <bool NARROW>
__device__ __forceinline__ SegIn iow_seg_pop(const IowScene &S, IowStack<NARROW> &K, int sidx) {
    K.size--;
    const int e = K.size;
    SegIn in;
    in.fib = reinterpret_cast<const float4 *>(S.fib)[sidx];  // fibonacciHemiSpherePtDirn's point (03...glsl:164-184)
    in.co = mk(K.at(e, 0), K.at(e, 1), K.at(e, 2));
    in.cd = mk(K.at(e, 3), K.at(e, 4), K.at(e, 5));
    in.contribution = K.at(e, 6); in.ri = K.at(e, 7);
    in.bounced = K.bounced(e);
    return in;
}
template <bool NARROW>
__device__ __forceinline__ void iow_seg_shade(const IowScene &S, const Frame &F, IowStack<NARROW> &K, int &skip,
                                              f3 &sample, int sidx, Ctr &c, const SegIn &in, const RayRet &data) {
    const f3 cd = in.cd;
    const float contribution = in.contribution, ri = in.ri;
    int bounced = in.bounced;
    const bool hit = dot(data.normal, data.normal) > 0.9f;
    sample = sample + sel(hit, data.color, background(cd, false)) * contribution;
    if (bounced < F.max_bounces && hit) {
        bounced++;
        bool spawnRefl = false, spawnRefr = false;
        f3 refr_dir = f3{0, 0, 0}, refl_dir = f3{0, 0, 0};
        float cos_t = dot(data.normal, cd);
        float sin_t = __builtin_sqrtf(1.0f - cos_t * cos_t);
        float target_ri;
        {
            int pi = K.size - 1 - skip;
            float parent = (pi < 0) ? 1.0f : (pi < kIowStack ? K.at(pi, 7) : 0.0f);
            target_ri = cos_t > 0.0f ? parent : data.material.z;
            if (cos_t > 0.0f && pi >= 0 && pi < kIowStack && !((K.wmask >> pi) & 1u)) {
                // diagnostics (RT_DEBUG_FIRST_STALE): the segment of the first stale read replaces
                // the unit's drop counter
#ifdef RT_DIAG
                if (F.dbg_first_stale && K.rmask == 0u) c.drops = 0x80000000u | c.seg;
#endif
                K.rmask |= 1u << pi;
            }
        }
        float rr = (ri * rcp(target_ri)) * sin_t;
        float refr_c = data.material.x, refl_c = data.material.y;
        f3 n_ = sel(cos_t > 0.0f, data.normal, -data.normal);
        if (cos_t < 0.0f) {
            refl_dir = fib_dir(in.fib, data.scat1, data.reflected); spawnRefl = true;
            float inc = refr_c * schlick(-cos_t, ri * rcp(target_ri));
            refr_c -= inc; refl_c += inc;
        } else if (rr > 1.0f) {
            refr_dir = data.reflected; spawnRefl = true; refl_c = 1.0f;  // sic (03...glsl:332)
        }
        if (rr <= 1.0f) {
            f3 yc = n_ * cos_t, xc = cd - yc;
            spawnRefr = true;
            refr_dir = n_ * rr + xc * __builtin_sqrtf(1.0f - rr * rr);
            refr_dir = fib_dir(in.fib, data.scat0, refr_dir);
        }
        skip = (spawnRefl && spawnRefr) ? skip - 1 : (spawnRefl ? skip : (spawnRefr ? skip + 1 : 0));
        if (spawnRefl) {
            if (__builtin_isnan(dot(refl_dir, refl_dir))) c.nans++;
            K.push(data.point - n_ * 0.000015f, refl_dir, contribution * refl_c, ri, bounced, c);
        }
        if (spawnRefr) {
            if (__builtin_isnan(dot(refr_dir, refr_dir))) c.nans++;
            K.push(data.point + n_ * 0.000015f, refr_dir, contribution * refr_c, target_ri, bounced, c);
        }
    } else skip = 0;
}
// BS: BVH-stack slots per lane (logical depth BS - 3: 3 spare push slots); NS: node stride
template <bool NARROW, int BS, int NS>
__device__ __forceinline__ void iow_segment(const IowScene &S, const Frame &F, IowStack<NARROW> &K, int &skip,
                                            f3 &sample, int sidx, Ctr &c, short *bstk, const float4 *nodes) {
    const SegIn in = iow_seg_pop(S, K, sidx);
    const RayRet data = iow_launch_ray<BS - 3, NS>(S, F, in.co, in.cd, 32000.0f, in.contribution, c, bstk, nodes);
    iow_seg_shade(S, F, K, skip, sample, sidx, c, in, data);
}
// The segment step of a work loop, called with every lane of the wave (seg: this lane has a
// ray to trace).  With at most F.coop_max tracing lanes the wave runs their closest-hit
// queries cooperatively (iow_coop_search), one ray after another; otherwise each lane walks
// the BVH for its own ray.
template <bool NARROW, int BS, int NS>
__device__ __forceinline__ void iow_seg_step(const IowScene &S, const Frame &F, IowStack<NARROW> &K, int &skip,
                                             f3 &sample, int sidx, Ctr &c, short *bstk, const float4 *nodes, bool seg) {
    const unsigned long long m = __ballot(seg);
    if (m == 0) return;
    if (__popcll(m) > F.coop_max) {
        if (seg) iow_segment<NARROW, BS, NS>(S, F, K, skip, sample, sidx, c, bstk, nodes);
        return;
    }
    constexpr int kCap = BS * 64;  // the wave's BVH-stack slots, as a list
    short *wl = bstk - kBstkLane * (threadIdx.x & 63);
    DBG_T0(F, t_pop);
    SegIn in{};
    if (seg) in = iow_seg_pop(S, K, sidx);
    DBG_CYC(F, c, kDbgCycSpare2, t_pop);
    DBG_T0(F, t_q);
    float my_t = 32000.0f;
    int my_j = -1;
    float4 my_c0 = make_float4(0.0f, 0.0f, 0.0f, 0.0f), my_c1 = my_c0;
    uint32_t my_box = 0, my_prim = 0;
    for (unsigned long long mm = m; mm; mm &= mm - 1) {
        const int L = __ffsll((long long)mm) - 1;
        const f3 go = f3{bcast_f(in.co.x, L), bcast_f(in.co.y, L), bcast_f(in.co.z, L)};
        const f3 gd = f3{bcast_f(in.cd.x, L), bcast_f(in.cd.y, L), bcast_f(in.cd.z, L)};
        float t;
        int j;
        float4 c0, c1;
        uint32_t nb, np;
        iow_coop_search(S, go, gd, 32000.0f, wl, kCap, t, j, c0, c1, nb, np, c.wdbg);
        if ((int)(threadIdx.x & 63) == L) { my_t = t; my_j = j; my_c0 = c0; my_c1 = c1; my_box = nb; my_prim = np; }
    }
    DBG_CYC(F, c, kDbgCycSpare0, t_q);
    DBG_T0(F, t_sh);
    if (seg) {
        c.seg++; c.nodes += my_box; c.prims += my_prim;
        SPL_T0(t_ev);
        f3 td_id, nd_id;
        iow_id_dirs(in.cd, td_id, nd_id);
        const RayRet data =
            iow_eval_c(S, in.co, in.cd, td_id, nd_id, my_t, my_j, 32000.0f, in.contribution, my_c0, my_c1);
        SPL_CYC(c.wdbg, kDbgCycRay, t_ev);
        SPL_T0(t_sd);
        iow_seg_shade(S, F, K, skip, sample, sidx, c, in, data);
        SPL_CYC(c.wdbg, kDbgCycTrav, t_sd);
    }
    DBG_CYC(F, c, kDbgCycSpare1, t_sh);
}

// ---------------------------------------------------------------- persistent work queue
// Work unit = one pixel.  A wave keeps all 64 lanes busy: a lane that finishes its pixel
// takes the next one with a wave-aggregated atomic (ballot -> popcount -> one atomicAdd ->
// per-lane rank by masked popcount), so divergent path lengths never idle the wave.
struct UnitPix { int x, y; bool in_image; size_t out; };

__device__ __forceinline__ UnitPix unit_pixel(const Frame &f, uint32_t u) {
    UnitPix p;
    const int l = (int)(u & 63u);
    if (f.tiles == nullptr) {
        const int b = (int)(u >> 6), nbx = (f.tw + 7) >> 3;
        const int rx = (b % nbx) * 8 + (l & 7), ry = (b / nbx) * 8 + (l >> 3);
        p.x = f.x0 + rx; p.y = f.y0 + ry;
        p.in_image = rx < f.tw && ry < f.th && p.x >= 0 && p.y >= 0 && p.x < f.W && p.y < f.H;
        p.out = p.in_image ? (size_t)p.y * f.W + p.x : (size_t)-1;
    } else {
        const uint32_t area = (uint32_t)f.tile_size * f.tile_size;
        const int t = (int)(u / area), r = (int)(u % area), per = f.tile_size >> 3;
        const int b = r >> 6;
        const int ix = (b % per) * 8 + (l & 7), iy = (b / per) * 8 + (l >> 3);
        p.x = f.tiles[2 * t] * f.tile_size + ix;
        p.y = f.tiles[2 * t + 1] * f.tile_size + iy;
        p.in_image = p.x < f.W && p.y < f.H;
        p.out = (size_t)t * area + (size_t)iy * f.tile_size + ix;
    }
    return p;
}

__device__ __forceinline__ uint32_t units_total(const Frame &f) {
    if (f.tiles) return (uint32_t)f.n_tiles * f.tile_size * f.tile_size;
    return (uint32_t)(((f.tw + 7) >> 3) * ((f.th + 7) >> 3)) * 64u;
}

// wave-aggregated fetch: lanes with `need` get consecutive unit ids
__device__ __forceinline__ uint32_t fetch_unit(unsigned *counter, bool need) {
    const unsigned long long mask = __ballot(need);
    if (mask == 0) return 0xffffffffu;
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (unsigned)__popcll(mask));
    base = __shfl(base, leader, 64);
    const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
    return need ? base + rank : 0xffffffffu;
}

__device__ __forceinline__ void write_px(const Frame &f, const UnitPix &p, f3 c, float depth) {
    if (p.out == (size_t)-1) return;
    reinterpret_cast<float4 *>(f.out_rgba)[p.out] = make_float4(c.x, c.y, c.z, p.in_image ? 1.0f : 0.0f);
    if (f.out_depth) f.out_depth[p.out] = depth;
}

// Camera ray of sample s of a pixel, out_Pixel 03...glsl:370-406
struct IowPixelCam { float sx, sy; };
__device__ __forceinline__ void iow_camera_ray(const IowScene &S, const Frame &f, float sx, float sy, float dsx,
                                               float dsy, int s, f3 &ro, f3 &rd) {
    const f3 D = mk(f.dir[0], f.dir[1], f.dir[2]), P = mk(f.pos[0], f.pos[1], f.pos[2]);
    const f3 up = f3{0, 1, 0};
    f3 look_at = P + D * f.focus;
    f3 cr = cross(D, up), cu = cross(cr, D);
    const int ix = S.ring[2 * s], iy = S.ring[2 * s + 1];
    float rx = (S.sunflower[2 * s] * f.aperture) * 0.5f, ry = (S.sunflower[2 * s + 1] * f.aperture) * 0.5f;
    ro = (P + cr * rx) + cu * ry;
    f3 ld = normalize(look_at - ro);
    f3 r_ = cross(ld, up), u_ = cross(cr, ld);
    rd = normalize((ld * f.screen_dist + r_ * (sx + dsx * (float)ix)) + u_ * (sy + dsy * (float)iy));
}

// wave-aggregated slot allocation for parking (same ballot / popcount / rank scheme)
__device__ __forceinline__ uint32_t park_slot(unsigned *count, bool need) {
    const unsigned long long mask = __ballot(need);
    const int lane = (int)(threadIdx.x & 63);
    const int leader = __ffsll((long long)mask) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(count, (unsigned)__popcll(mask));
    base = __shfl(base, leader, 64);
    return base + (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
}
__device__ __forceinline__ float ibits(int v) { return __int_as_float(v); }
__device__ __forceinline__ float ubits(uint32_t v) { return __uint_as_float(v); }

// Kernel configurations of the IOW-03 work loops.  SUB: 256-thread sub-blocks per block, each
// with its own [slot][thread] stack arrays (stride kBlock).  LN: the whole 4-wide BVH is copied
// into the block's LDS (7 float4 per node) when it has at most kIowLdsNodes nodes: one
// 768-thread block per CU shares it, so node fetches cost LDS latency instead of L2 latency.
constexpr int kIowLdsNodes = 240;
template <bool NARROW, int SUB, bool LN>
struct IowCfg {
    static constexpr int BS = LN ? 16 : (NARROW ? 12 : kIowBvhStack);  // BVH-stack slots per lane
    static constexpr int NS = LN ? 7 : 8;                               // float4 per BVH node
    static constexpr int kThreads = SUB * kBlock;
};
// copy the BVH into LDS (7 float4 per node, dropping the pad) and return the node base
template <bool LN>
__device__ __forceinline__ const float4 *iow_stage_nodes(const IowScene &S, float4 *s_nodes) {
    if constexpr (!LN) return S.nodes;
    else {
        const uint32_t total = S.n_nodes * 7u;
        for (uint32_t i = threadIdx.x; i < total; i += blockDim.x) s_nodes[i] = S.nodes[(i / 7u) * 8u + i % 7u];
        __syncthreads();
        return s_nodes;
    }
}

template <bool NARROW, int SUB, bool LN>
__device__ __forceinline__ void iow03_body(const Frame &f, const IowScene &S, const Chunk &ch, const Cont &ct,
                                           unsigned *counter, int s_stop) {
    using Stack = IowStack<NARROW>;
    using Cfg = IowCfg<NARROW, SUB, LN>;
    constexpr int kFl = kIowStack * Stack::kSlot;  // stack floats per lane
    __shared__ float lds[SUB * kFl * kBlock];
    __shared__ unsigned char lds_b[NARROW ? SUB * kIowStack * kBlock : 1];
    __shared__ short lds_bvh[SUB * Cfg::BS * kBlock];
    __shared__ unsigned long long s_dbg[SUB * kBlock / 64][kDbgSlots];
    __shared__ float4 s_nodes[LN ? kIowLdsNodes * 7 : 1];
    const int sb = (int)(threadIdx.x / kBlock), tl = (int)(threadIdx.x % kBlock);
    short *bstk = lds_bvh + sb * Cfg::BS * kBlock + kBstkLane * tl;  // bslot's layout
    const float4 *nodes = iow_stage_nodes<LN>(S, s_nodes);
    Ctr c;
    if (f.dbg) {
        c.wdbg = s_dbg[threadIdx.x >> 6];
        if ((threadIdx.x & 63) < kDbgSlots) c.wdbg[threadIdx.x & 63] = 0;
    }
    Stack K{lds + sb * kFl * kBlock + tl, lds_b + (NARROW ? sb * kIowStack * kBlock + tl : 0), 0};
    const uint32_t total = ct.in ? *ct.in_count : (ch.order_count ? *ch.order_count : units_total(f));
    const bool may_park = ct.out != nullptr && total >= ct.park_min;
    const int W = f.W, H = f.H, spp = f.spp;
    const int s_end = ch.s_end < s_stop ? ch.s_end : s_stop;
    int grid = 1;
    while (grid * grid < spp) grid++;
    const float aspect = (float)W * rcp((float)H);
    const float dsx = aspect * rcp((float)(W * grid));
    const float dsy = 1.0f * rcp((float)(H * grid));
    bool live = true;     // lane may still find work
    bool busy = false;    // lane owns a pixel
    UnitPix px{};
    uint32_t unit = 0, urays = 0;
    float sx = 0, sy = 0;
    f3 fc = f3{0, 0, 0}, sample = f3{0, 0, 0};
    int s = 0, skip = 0;
    for (;;) {
        DBG_T0(f, t_loop);
        const uint32_t q = fetch_unit(counter, live && !busy);
        if (live && !busy) {
            if (q >= total) live = false;
            else if (ct.in) {  // resume a parked lane
                const float4 *p = ct.in + (size_t)q * kContSlots;
                const float4 m = p[0], a = p[1], b = p[2];
                unit = __float_as_uint(m.x); s = __float_as_int(m.y); skip = __float_as_int(m.z);
                K.size = __float_as_int(m.w);
                fc = f3{a.x, a.y, a.z}; urays = __float_as_uint(a.w);
                sample = f3{b.x, b.y, b.z};
                const float *fl = reinterpret_cast<const float *>(p + 3);
                for (int k = 0; k < kFl; k++) K.base[k * kBlock] = fl[k];
                if constexpr (NARROW)
                    for (int e = 0; e < kIowStack; e++) K.set_bounced(e, __float_as_int(fl[kFl + e]));
                px = unit_pixel(f, unit);
                sx = (aspect * ((float)px.x * 2.0f - (float)W)) * rcp(2.0f * (float)W);
                sy = ((float)px.y * 2.0f - (float)H) * rcp(2.0f * (float)H);
                busy = true;
            } else {
                unit = ch.order ? ch.order[q] : q;
                px = unit_pixel(f, unit);
                if (!px.in_image) {
                    if (ch.final_chunk) write_px(f, px, f3{0, 0, 0}, 0.0f);
                    if (ch.cost) ch.cost[unit] = 0;
                } else {
                    busy = true;
                    sx = (aspect * ((float)px.x * 2.0f - (float)W)) * rcp(2.0f * (float)W);
                    sy = ((float)px.y * 2.0f - (float)H) * rcp(2.0f * (float)H);
                    s = ch.per_unit_begin ? __float_as_int(ch.state[2 * (size_t)unit].w) : ch.s_begin;
                    K.size = 0;
                    urays = 0;
                    if (s == 0) {
                        fc = f3{0, 0, 0};
                        for (int e = 0; e < kIowStack; e++) K.at(e, 7) = 0.0f;  // stale RI slots start at 0
                    } else {  // resume the pixel where the previous chunk parked it
                        const float4 a0 = ch.state[2 * (size_t)unit], a1 = ch.state[2 * (size_t)unit + 1];
                        fc = f3{a0.x, a0.y, a0.z};
                        K.at(0, 7) = a1.x; K.at(1, 7) = a1.y; K.at(2, 7) = a1.z; K.at(3, 7) = a1.w;
                    }
                }
            }
        }
        if (__ballot(live) == 0) break;
        if (may_park && __ballot(!live) != 0 && __popcll(__ballot(busy)) < kParkBelow) {
            // queue drained and the wave is under half busy: park the busy lanes, free the SIMD
            const uint32_t slot = park_slot(ct.out_count, busy);
            if (busy) {
                float4 *p = ct.out + (size_t)slot * kContSlots;
                p[0] = make_float4(ubits(unit), ibits(s), ibits(skip), ibits(K.size));
                p[1] = make_float4(fc.x, fc.y, fc.z, ubits(urays));
                p[2] = make_float4(sample.x, sample.y, sample.z, 0.0f);
                float *fl = reinterpret_cast<float *>(p + 3);
                for (int k = 0; k < kFl; k++) fl[k] = K.base[k * kBlock];
                if constexpr (NARROW)
                    for (int e = 0; e < kIowStack; e++) fl[kFl + e] = ibits(K.bounced(e));
            }
            break;
        }
        DBG_TALLY(f, c, kDbgOuter, busy);
        if (ch.rec_col) {
            // take every following sample whose speculative record assumed the exact stack
            // state (the RI of the entries it read before writing them) from its record
            while (busy && K.size == 0 && s < s_end) {
                const size_t u = (size_t)unit * ch.rec_S + s;  // the record of unit s * rec_P + unit
                const float4 cl = ch.rec_col[u], a = ch.rec_assume[u];
                const uint32_t fl = __float_as_uint(cl.w), rm = fl & 15u, wm = (fl >> 4) & 15u;
                if (((rm & 2u) && __float_as_uint(a.x) != __float_as_uint(K.at(1, 7))) ||
                    ((rm & 4u) && __float_as_uint(a.y) != __float_as_uint(K.at(2, 7))) ||
                    ((rm & 8u) && __float_as_uint(a.z) != __float_as_uint(K.at(3, 7))))
                    break;
                const float4 fn = ch.rec_fin[u];
                const uint4 ct4 = ch.rec_ctr[u];
                fc = fc + f3{cl.x, cl.y, cl.z};
                if (wm & 2u) K.at(1, 7) = fn.x;
                if (wm & 4u) K.at(2, 7) = fn.y;
                if (wm & 8u) K.at(3, 7) = fn.z;
                c.seg += ct4.x; c.drops += ct4.y; c.nans += ct4.z; c.nodes += ct4.w;
                c.prims += __float_as_uint(fn.w);
                urays += ct4.x;
                s++;
            }
        }
        if (busy && K.size == 0 && s < s_end) {  // start sample s
            f3 ro, rd;
            iow_camera_ray(S, f, sx, sy, dsx, dsy, s, ro, rd);
            if (f.show_normal) {
                fc = fc + iow_launch_ray<Cfg::BS - 3, Cfg::NS>(S, f, ro, rd, 32000.0f, 1.0f, c, bstk, nodes).normal;
                s++;
                urays++;
            } else {
                K.push(ro, rd, 1.0f, 1.0f, 0, c);
                sample = f3{0, 0, 0};
                skip = 0;
            }
        }
        DBG_TALLY(f, c, kDbgSeg, busy && K.size > 0);
        DBG_CYC(f, c, kDbgCycCam, t_loop);
        DBG_T0(f, t_seg);
        {
            const bool seg = busy && K.size > 0;
            iow_seg_step<NARROW, Cfg::BS, Cfg::NS>(S, f, K, skip, sample, s, c, bstk, nodes, seg);
            if (seg) {
                urays++;
                if (K.size == 0) { fc = fc + sample; s++; }
            }
        }
        DBG_CYC(f, c, kDbgCycSeg, t_seg);
        if (busy && K.size == 0 && s >= s_end) {
            if (s_end >= s_stop) {
                if (ch.final_chunk) write_px(f, px, fc * rcp((float)s_stop), 0.0f);
                else if (ch.state) {  // early-return pixels: keep the final colour for the last launch
                    ch.state[2 * (size_t)unit] = make_float4(fc.x, fc.y, fc.z, 0.0f);
                }
            } else if (ch.state) {
                ch.state[2 * (size_t)unit] = make_float4(fc.x, fc.y, fc.z, 0.0f);
                ch.state[2 * (size_t)unit + 1] = make_float4(K.at(0, 7), K.at(1, 7), K.at(2, 7), K.at(3, 7));
            }
            if (ch.cost) ch.cost[unit] = urays;
            if (f.px_rays) f.px_rays[unit] = urays;
            busy = false;
        }
    }
    flush(f, c);
}

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3)))
void k_iow03(Frame f, IowScene S, Chunk ch, Cont ct, unsigned *counter, int s_stop) {
    iow03_body<false, 1, false>(f, S, ch, ct, counter, s_stop);
}
__global__ __launch_bounds__(3 * kBlock) void k_iow03L(Frame f, IowScene S, Chunk ch, Cont ct, unsigned *counter,
                                                       int s_stop) {
    iow03_body<false, 3, true>(f, S, ch, ct, counter, s_stop);
}
// u_NumOfBounce <= 255: byte bounce counts + 12-deep BVH stack -> 39 KB LDS per block (A/B layout)
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(3)))
void k_iow03n(Frame f, IowScene S, Chunk ch, Cont ct, unsigned *counter, int s_stop) {
    iow03_body<true, 1, false>(f, S, ch, ct, counter, s_stop);
}

// ============================================================================ IOW-03, sample-parallel
// One unit = one sample of one pixel (u = s*P + pu), so a heavy pixel's samples run on many
// lanes at once instead of one after another.  Exactness: a sample's result is a function of
// the pixel, the sample index and the RI left in stack entries 1..3 by the samples before it
// (entry 0 is always written before any read).  The sample runs with an assumed value for
// those entries (zeros in the first pass, else what the last resolve computed) and records
// which entries it read before writing (rmask) and which it wrote (wmask); the resolve replays
// the pixel in sample order and re-queues exactly the samples whose assumption was wrong.
// ---------------------------------------------------------------- alternative runs
// The slots (first, count) of unit u's alternative runs; count 0: none.  Open addressing over
// alt_hcap entries, key u + 1.
__device__ __forceinline__ uint2 alt_find(const SpecRecs &R, uint32_t u) {
    if (!R.alt_hash) return make_uint2(0u, 0u);
    uint32_t h = (u * 2654435761u) % R.alt_hcap;
    for (uint32_t i = 0; i < R.alt_hcap; i++) {
        const uint2 e = R.alt_hash[h];
        if (e.x == 0u) break;
        if (e.x == u + 1u) return make_uint2(e.y & 0xffffffu, e.y >> 24);
        h = h + 1u == R.alt_hcap ? 0u : h + 1u;
    }
    return make_uint2(0u, 0u);
}
// A finished alternative run of u (finished in a launch other than `launch`, whose records are
// stable) whose assumption holds on the entries it read under the exact state E: copied into
// u's records, which then read as a finished exact execution (flags tagged with `tag_launch`).
// Returns its slot + 1, or 0.
__device__ uint32_t alt_adopt(const SpecRecs &R, uint32_t u, uint32_t E1, uint32_t E2, uint32_t E3, uint32_t launch,
                              uint32_t tag_launch) {
    const uint2 fk = alt_find(R, u);
    for (uint32_t i = 0; i < fk.y; i++) {
        const AltRec &A = R.alt[fk.x + i];
        const uint32_t st = __hip_atomic_load(&A.state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st == 0u || st == launch + 1u || A.u != u) continue;  // (A.u: a record of this unit only)
        const unsigned fl = __float_as_uint(A.col.w), rm = fl & 15u;
        if (((rm & 2u) && __float_as_uint(A.assume.x) != E1) || ((rm & 4u) && __float_as_uint(A.assume.y) != E2) ||
            ((rm & 8u) && __float_as_uint(A.assume.z) != E3))
            continue;
        R.assume[R.ix(u)] = A.assume;
        R.fin[R.ix(u)] = A.fin;
        R.ctr[R.ix(u)] = A.ctr;
        R.col[R.ix(u)] = make_float4(A.col.x, A.col.y, A.col.z,
                               __uint_as_float((fl & ~(63u << 10)) | ((tag_launch & 63u) << 10)));
        return fk.x + i + 1u;
    }
    return 0u;
}

template <bool NARROW, int SUB, bool LN>
__device__ __forceinline__ void iow03s_body(const Frame &f, const IowScene &S, const SpecRecs &R, int mode,
                                            const Cont &ct, unsigned *counter) {
    using Stack = IowStack<NARROW>;
    using Cfg = IowCfg<NARROW, SUB, LN>;
    constexpr int kFl = kIowStack * Stack::kSlot;
    constexpr int BCAP = Cfg::BS - 3;
    __shared__ float lds[SUB * kFl * kBlock];
    __shared__ unsigned char lds_b[NARROW ? SUB * kIowStack * kBlock : 1];
    __shared__ short lds_bvh[SUB * Cfg::BS * kBlock];
    __shared__ unsigned long long s_dbg[SUB * kBlock / 64][kDbgSlots];
    __shared__ float4 s_nodes[LN ? kIowLdsNodes * 7 : 1];
    const int sb = (int)(threadIdx.x / kBlock), tl = (int)(threadIdx.x % kBlock);
    short *bstk = lds_bvh + sb * Cfg::BS * kBlock + kBstkLane * tl;  // bslot's layout
    const float4 *nodes = iow_stage_nodes<LN>(S, s_nodes);
    Ctr c;  // per unit here: written to the unit's record, never flushed
    if (f.dbg) {
        c.wdbg = s_dbg[threadIdx.x >> 6];
        if ((threadIdx.x & 63) < kDbgSlots) c.wdbg[threadIdx.x & 63] = 0;
    }
    Stack K{lds + sb * kFl * kBlock + tl, lds_b + (NARROW ? sb * kIowStack * kBlock + tl : 0), 0};
    // units: the parked lanes of ct.in first, then fresh units of the mode ([fresh_lo, fresh_hi)
    // in a mixed launch; all of them in a first launch; none in a plain resume launch)
    const uint32_t nin = ct.in ? *ct.in_count : 0u;
    const uint32_t f_lo = ct.mixed ? ct.fresh_lo : 0u;
    const uint32_t f_n = ct.mixed ? ct.fresh_hi - ct.fresh_lo
                       : (ct.in ? 0u : (mode == kSpecList ? *R.list_count
                                                          : (mode == kSpecFirst ? R.P : R.order_n * (R.S - 1))));
    const uint32_t total = nin + f_n;
    const bool may_park = ct.out != nullptr && total >= ct.park_min;
    const int park_below = ct.park_below ? ct.park_below : kParkBelow;
    const uint32_t n_waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t wcap = ct.spread ? max(1u, (total + n_waves - 1u) / n_waves) : 64u;
    const int W = f.W, H = f.H, spp = f.spp;
    int grid = 1;
    while (grid * grid < spp) grid++;
    const float aspect = (float)W * rcp((float)H);
    const float dsx = aspect * rcp((float)(W * grid));
    const float dsy = 1.0f * rcp((float)(H * grid));
    bool live = true, busy = false;
    bool solo = false;  // wave-uniform: the wave holds one unit from the sorted head
    const uint32_t solo_n = min(min(ct.solo_n, n_waves), total);
    bool solo_open = solo_n != 0;  // wave-uniform: the queue head may still be below solo_n
    uint32_t u = 0, urays = 0;
    int skip = 0;
    f3 sample = f3{0, 0, 0};
    const unsigned done_tag = (1u << 8) | ((R.epoch & 0xffffu) << 16);
    const unsigned started_tag = (1u << 9) | ((R.epoch & 0xffffu) << 16);  // heavy-first: taken, unfinished
    uint32_t useg = 0;  // segments of the current unit in this launch (ct.seg_budget)
    // exact: the unit was (re)started with its exact incoming state (a frontier or fixf restart),
    // so the state after it is exact too and the lane may go on down its pixel's chain
    bool exact = false;
    uint32_t alt_slot = 0;  // an alternative run: its slot + 1 (its record goes to R.alt)
    // the lane's state at a segment boundary -> a continuation slot (13 float4)
    auto park = [&](float4 *p) {
        p[0] = make_float4(ubits(u), ibits(skip), ibits(K.size), ubits(K.wmask | (K.rmask << 4)));
        p[1] = make_float4(sample.x, sample.y, sample.z, ubits(urays));
        p[2] = make_float4(ubits(c.seg), ubits(c.nodes), ubits(c.prims), ubits(c.drops));
        // .y: restart flag (k_iow03_fixf), .z: exact, .w: alternative slot + 1 (bits)
        p[12] = make_float4(ubits(c.nans), 0.0f, exact ? 1.0f : 0.0f, ubits(alt_slot));
        float *fl = reinterpret_cast<float *>(p + 3);
        for (int k = 0; k < kFl; k++) fl[k] = K.base[k * kBlock];
        if constexpr (NARROW)
            for (int e = 0; e < kIowStack; e++) fl[kFl + e] = ibits(K.bounced(e));
    };
    // start unit u (sample s of pixel pu) with assumed stack RI a.xyz in entries 1..3
    auto begin = [&](uint32_t u_, float4 a) {
        u = u_;
#ifdef RT_DIAG
        if (R.dbg_start) R.dbg_start[u] = (ct.launch_id & 0xffffu) | ((R.dbg_start[u] >> 16) + 1u) << 16;
#endif
        const uint32_t pu = u % R.P;
        const int s = (int)(u / R.P);
        const UnitPix px = unit_pixel(f, pu);
        busy = true;
        c.seg = c.nodes = c.prims = c.drops = c.nans = 0;
        urays = 0;
        useg = 0;
        skip = 0;
        sample = f3{0, 0, 0};
        K.size = 0; K.wmask = 0; K.rmask = 0;
        K.at(0, 7) = 0.0f; K.at(1, 7) = a.x; K.at(2, 7) = a.y; K.at(3, 7) = a.z;
        const float sx = (aspect * ((float)px.x * 2.0f - (float)W)) * rcp(2.0f * (float)W);
        const float sy = ((float)px.y * 2.0f - (float)H) * rcp(2.0f * (float)H);
        f3 ro, rd;
        iow_camera_ray(S, f, sx, sy, dsx, dsy, s, ro, rd);
        if (f.show_normal) {  // one ray, no stack: the normal is the sample
            sample = iow_launch_ray<BCAP, Cfg::NS>(S, f, ro, rd, 32000.0f, 1.0f, c, bstk, nodes).normal;
            urays = 1;
        } else K.push(ro, rd, 1.0f, 1.0f, 0, c);
    };
    for (;;) {
        // spread: a wave holds at most wcap units, so a few long samples get a wave each (and the
        // wave-cooperative closest hits) instead of sharing one
        bool want = live && !busy;
        if (wcap < 64u) {
            const int room = (int)wcap - __popcll(__ballot(busy));
            want = want && (int)lanes_below(__ballot(want)) < room;
        }
        // solo head: the queue is read only while this wave has not yet seen it pass solo_n (the
        // counter only grows), so the check costs a load per wave at the start of a launch
        if (solo) {
            if (__ballot(busy) != 0) want = false;  // keep the head unit alone
            else solo = false;
        }
        if (!solo && solo_open && __ballot(want) != 0) {
            const uint32_t head = __builtin_amdgcn_readfirstlane(__hip_atomic_load(
                counter, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (head >= solo_n) solo_open = false;
            else want = want && __ballot(busy) == 0 && lanes_below(__ballot(want)) == 0;
        }
        const uint32_t q = fetch_unit(counter, want);
        if (solo_open && __ballot(want && q < solo_n) != 0) solo = true;
        if (want) {
            if (q >= total) live = false;
            else if (q < nin && ct.in[(size_t)q * kContSlots + 12].y == 3.0f) {  // an alternative run
                const uint32_t slot = __float_as_uint(ct.in[(size_t)q * kContSlots + 12].z);
                u = __float_as_uint(ct.in[(size_t)q * kContSlots].x);
                begin(u, R.alt[slot].assume);
                exact = false;
                alt_slot = slot + 1u;
            } else if (q < nin && ct.in[(size_t)q * kContSlots + 12].y != 0.0f) {  // doomed while parked: restart exact
                u = __float_as_uint(ct.in[(size_t)q * kContSlots].x);
                begin(u, R.assume[R.ix(u)]);
                exact = ct.chain != 0;
                alt_slot = 0;
            } else if (q < nin) {  // resume a parked lane
                const float4 *p = ct.in + (size_t)q * kContSlots;
                const float4 m = p[0], a = p[1], b = p[2];
                u = __float_as_uint(m.x); skip = __float_as_int(m.y); K.size = __float_as_int(m.z);
                K.wmask = __float_as_uint(m.w) & 15u; K.rmask = __float_as_uint(m.w) >> 4;
                sample = f3{a.x, a.y, a.z}; urays = __float_as_uint(a.w);
                c.seg = __float_as_uint(b.x); c.nodes = __float_as_uint(b.y); c.prims = __float_as_uint(b.z);
                c.drops = __float_as_uint(b.w); c.nans = __float_as_uint(p[12].x);
                exact = p[12].z != 0.0f;
                alt_slot = __float_as_uint(p[12].w);
                const float *fl = reinterpret_cast<const float *>(p + 3);
                for (int k = 0; k < kFl; k++) K.base[k * kBlock] = fl[k];
                if constexpr (NARROW)
                    for (int e = 0; e < kIowStack; e++) K.set_bounced(e, __float_as_int(fl[kFl + e]));
                useg = 0;
                busy = true;
            } else {
                // kSpecFirst: sample 0 of every pixel; kSpecRest: samples 1.. pixel-major, pixels
                // in R.order (heaviest sample 0 first); kSpecList: the re-execution list
                const uint32_t qf = f_lo + (q - nin);
                bool fresh = true;
                if (ct.fresh_mode == 0) {
                    u = mode == kSpecList ? R.list[qf]
                        : (mode == kSpecFirst ? qf : (1u + qf % (R.S - 1)) * R.P + R.order[R.order_base + qf / (R.S - 1)]);
                } else {  // heavy-first enumerations of kSpecRest (a unit may come up twice: run it once)
                    const uint32_t n_px = R.order_n ? R.order_n : R.P, nr = R.S - 1u - R.n_heavy;
                    uint32_t s_, rank;
                    if (ct.fresh_mode == 1) { rank = (qf / (R.S - 1u)) * R.probe_stride; s_ = 1u + qf % (R.S - 1u); }
                    else if (ct.fresh_mode == 2) { s_ = R.sorder[qf / n_px]; rank = qf % n_px; }
                    else { s_ = R.sorder[R.n_heavy + qf % nr]; rank = qf / nr; }
                    u = s_ * R.P + R.order[R.order_base + rank];
                    const uint32_t tag = __float_as_uint(R.col[R.ix(u)].w);
                    fresh = !((tag >> 16) == (R.epoch & 0xffffu) && (tag & 0x300u) != 0u);
                }
                if (fresh && unit_pixel(f, u % R.P).in_image) {
                    if (ct.fresh_mode != 0) R.col[R.ix(u)].w = ubits(started_tag);
                    begin(u, mode == kSpecFirst ? make_float4(0.0f, 0.0f, 0.0f, 0.0f) : R.assume[R.ix(u)]);
                    exact = false;
                    alt_slot = 0;
                }
            }
        }
        if (__ballot(live) == 0) break;
        if (may_park && __ballot(!live) != 0 && __popcll(__ballot(busy)) < park_below) {
            const uint32_t slot = park_slot(ct.out_count, busy);
            if (busy) park(ct.out + (size_t)slot * kContSlots);
            break;
        }
        DBG_TALLY(f, c, kDbgOuter, busy);
        DBG_TALLY(f, c, kDbgSeg, busy && K.size > 0);
        DBG_T0(f, t_seg);
        {
            const bool seg = busy && K.size > 0;
            iow_seg_step<NARROW, Cfg::BS, Cfg::NS>(S, f, K, skip, sample, (int)(u / R.P), c, bstk, nodes, seg);
            if (seg) { urays++; useg++; }
        }
        DBG_CYC(f, c, kDbgCycSeg, t_seg);
        if (ct.seg_budget) {  // budgeted round: a unit that used its segments parks (per lane)
            const bool over = busy && K.size > 0 && useg >= ct.seg_budget;
            if (__ballot(over) != 0) {
                const uint32_t slot = park_slot(ct.out_count, over);
                if (over) { park(ct.out + (size_t)slot * kContSlots); busy = false; }
            }
        }
        if (busy && K.size == 0 && alt_slot) {  // an alternative run done: its own record
            AltRec &A = R.alt[alt_slot - 1u];
            A.col = make_float4(sample.x, sample.y, sample.z, ubits(K.rmask | (K.wmask << 4) | done_tag));
            A.fin = make_float4(K.at(1, 7), K.at(2, 7), K.at(3, 7), ubits(c.prims));
            A.ctr = make_uint4(c.seg, c.drops, c.nans, c.nodes);
            __threadfence();
            __hip_atomic_store(&A.state, ct.launch_id + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            busy = false;
            alt_slot = 0;
        }
        if (busy && K.size == 0) {  // sample done: record it
            R.col[R.ix(u)] = make_float4(sample.x, sample.y, sample.z,
                                   ubits(K.rmask | (K.wmask << 4) | done_tag | ((ct.launch_id & 63u) << 10)));
            R.fin[R.ix(u)] = make_float4(K.at(1, 7), K.at(2, 7), K.at(3, 7), ubits(c.prims));
            R.ctr[R.ix(u)] = make_uint4(c.seg, c.drops, c.nans, c.nodes);
#ifdef RT_DIAG
            if (R.dbg_end) R.dbg_end[u] = ct.launch_id;
#endif
            busy = false;
            if (exact) {
                // Chain following: the stack this exact sample left is the exact incoming state of
                // the next sample.  Walk the pixel's following finished samples while their
                // assumptions hold on the entries they read; re-run the first one that does not,
                // here and now, with the exact state.  A pixel whose samples all mispredict (each
                // reads the entry its predecessor wrote) then runs down its chain on one lane,
                // not one sample per frontier round.  Stops at an unfinished sample (running or
                // queued elsewhere), which the frontier handles.
                // Other lanes of this launch may write these records, so only records finished in
                // an earlier launch (stable since that kernel boundary) are read, with
                // device-coherent loads; a record is claimed for a re-run by a compare-and-swap of
                // its flags, and a read whose flags changed meanwhile stops the walk.
                const uint32_t pu = u % R.P;
                uint32_t E1 = __float_as_uint(K.at(1, 7)), E2 = __float_as_uint(K.at(2, 7)),
                         E3 = __float_as_uint(K.at(3, 7));
                auto ld = [](const float *p) {
                    return __hip_atomic_load(reinterpret_cast<const unsigned *>(p), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
                };
                for (uint32_t t = u / R.P + 1u; t < R.S; t++) {
                    const uint32_t v = t * R.P + pu;
                    unsigned *flp = reinterpret_cast<unsigned *>(&R.col[R.ix(v)].w);
                    const unsigned fl = ld(&R.col[R.ix(v)].w);
                    if ((fl & 0xffff0100u) != done_tag || ((fl >> 10) & 63u) == (ct.launch_id & 63u)) break;
                    const unsigned rm = fl & 15u, wm = (fl >> 4) & 15u;
                    const unsigned a1 = ld(&R.assume[R.ix(v)].x), a2 = ld(&R.assume[R.ix(v)].y), a3 = ld(&R.assume[R.ix(v)].z);
                    const unsigned f1 = ld(&R.fin[R.ix(v)].x), f2 = ld(&R.fin[R.ix(v)].y), f3v = ld(&R.fin[R.ix(v)].z);
                    __atomic_thread_fence(__ATOMIC_ACQUIRE);
                    if (ld(&R.col[R.ix(v)].w) != fl) break;
                    if (((rm & 2u) && a1 != E1) || ((rm & 4u) && a2 != E2) || ((rm & 8u) && a3 != E3)) {
                        unsigned expect = fl;
                        if (!__hip_atomic_compare_exchange_strong(flp, &expect, started_tag, __ATOMIC_ACQ_REL,
                                                                  __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))
                            break;
                        const uint32_t got = alt_adopt(R, v, E1, E2, E3, ct.launch_id, ct.launch_id);
                        if (got) {  // an alternative run already holds its exact execution
                            const AltRec &A = R.alt[got - 1u];
                            const unsigned awm = (__float_as_uint(A.col.w) >> 4) & 15u;
                            if (awm & 2u) E1 = __float_as_uint(A.fin.x);
                            if (awm & 4u) E2 = __float_as_uint(A.fin.y);
                            if (awm & 8u) E3 = __float_as_uint(A.fin.z);
                            continue;
                        }
                        const float4 e = make_float4(__uint_as_float(E1), __uint_as_float(E2), __uint_as_float(E3), 0.0f);
                        R.assume[R.ix(v)] = e;
                        begin(v, e);
                        break;
                    }
                    if (wm & 2u) E1 = f1;
                    if (wm & 4u) E2 = f2;
                    if (wm & 8u) E3 = f3v;
                }
                exact = busy;
            }
        }
    }
    if (c.wdbg && (threadIdx.x & 63) == 0)
        for (int i = 0; i < kDbgSlots; i++) atomicAdd(f.dbg + i, c.wdbg[i]);
}

__global__ __launch_bounds__(kBlock) void k_iow03s(Frame f, IowScene S, SpecRecs R, int mode, Cont ct,
                                                   unsigned *counter) {
    iow03s_body<false, 1, false>(f, S, R, mode, ct, counter);
}
__global__ __launch_bounds__(3 * kBlock) void k_iow03sL(Frame f, IowScene S, SpecRecs R, int mode, Cont ct,
                                                        unsigned *counter) {
    iow03s_body<false, 3, true>(f, S, R, mode, ct, counter);
}

// After the sample-0 pass: every later sample of a pixel assumes, for each stack entry 1..3,
// the RI sample 0 left there, or `prior` where sample 0 never wrote it (a guess, checked by
// the resolve; `prior` is the scene's most common refractive index, the value such entries
// almost always hold once any sample has pushed there).  Pixels are keyed by sample 0's ray
// count so the rest run heaviest first.
__global__ __launch_bounds__(kBlock) void k_iow03_prep(Frame f, SpecRecs R, unsigned *key, float prior,
                                                       uint32_t prior_from) {
    const uint32_t pu = blockIdx.x * kBlock + threadIdx.x;
    if (pu >= R.P) return;  // no cross-lane work in this kernel
    const UnitPix px = unit_pixel(f, pu);
    if (!px.in_image) { key[pu] = 0; return; }
    const uint32_t wm = (__float_as_uint(R.col[R.ix(pu)].w) >> 4) & 15u;
    const float4 fn = R.fin[R.ix(pu)];
    const float4 e0 = make_float4((wm & 2u) ? fn.x : 0.0f, (wm & 4u) ? fn.y : 0.0f, (wm & 8u) ? fn.z : 0.0f, 0.0f);
    // From prior_from on every entry is guessed as the prior: sample 0 starts from the all-zero
    // stack no later sample sees (a stale 0 makes target_RI 0 and forces TIR, 03...glsl:316-327),
    // so the values it leaves are a worse guess of the steady state than the scene's most common
    // RI (tests/analysis/fork_stats.py: mispredicted rays 2.6% -> 0.8% on C2).
    const float4 e1 = make_float4(prior, prior, prior, 0.0f);
    for (uint32_t s = 1; s < R.S; s++) R.assume[R.ix((size_t)s * R.P + pu)] = s >= prior_from ? e1 : e0;
#ifdef RT_DIAG
    if (R.exact && (R.exact_mode & 2))
        for (uint32_t s = 1; s < R.S; s++) R.assume[R.ix((size_t)s * R.P + pu)] = R.exact[(size_t)s * R.P + pu];
#endif
    if (R.front)  // sample 0 is exact: the frontier starts at sample 1 with its final entries
        R.front[pu] = make_uint4(1u, __float_as_uint(e0.x), __float_as_uint(e0.y), __float_as_uint(e0.z));
    if (R.front2) R.front2[pu] = make_uint4(0xffffffffu, 0u, 0u, 0u);
    key[pu] = R.ctr[R.ix(pu)].x;
}

// ---------------------------------------------------------------- checkpoint rounds
// Between the rounds of the speculative pass (kernel boundaries, so every finished record is
// visible), each pixel's frontier advances over its finished samples in sample order while
// their assumptions match the exact state E.  The first finished sample whose assumption was
// wrong gets E and is queued at once for an exact re-run in the next round (its record is
// marked unfinished until then), so a mispredicted sample -- long ones especially -- is re-run
// while the pass still has other work, not in a re-execution pass after it.  Samples behind the
// frontier keep speculating; the resolve after the pass checks everything again.
__global__ __launch_bounds__(kBlock) void k_iow03_frontier(Frame f, SpecRecs R, float4 *cont, unsigned *count,
                                                           uint32_t cap) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t n = R.order_n ? R.order_n : R.P;
    if (i >= n) return;  // no cross-lane work in this kernel
    const uint32_t pu = R.order_n ? R.order[R.order_base + i] : i;
    if (!unit_pixel(f, pu).in_image) return;
    uint4 st = R.front[pu];
    if (st.x >= R.S) return;
    const unsigned done_tag = (1u << 8) | ((R.epoch & 0xffffu) << 16);
    // queue sample u for an exact re-run with incoming state E (its record is marked unfinished)
    auto requeue = [&](size_t u, uint32_t e1, uint32_t e2, uint32_t e3) {
        const uint32_t slot = atomicAdd(count, 1u);
        if (slot >= cap) { atomicSub(count, 1u); return; }  // full: leave it to the resolve after the pass
        R.assume[R.ix(u)] = make_float4(__uint_as_float(e1), __uint_as_float(e2), __uint_as_float(e3), 0.0f);
        R.col[R.ix(u)].w = __uint_as_float((1u << 9) | ((R.epoch & 0xffffu) << 16));  // queued: unfinished
        float4 *p = cont + (size_t)slot * kContSlots;
        p[0] = make_float4(__uint_as_float((uint32_t)u), 0.0f, 0.0f, 0.0f);
        p[12] = make_float4(0.0f, 1.0f, 0.0f, 0.0f);  // restart with the (now exact) assumption
    };
    uint32_t s = st.x;
    bool queued = false;
    for (; s < R.S; s++) {
        const size_t u = (size_t)s * R.P + pu;
        unsigned fl = __float_as_uint(R.col[R.ix(u)].w);
        if ((fl & 0xffff0100u) != done_tag) {  // still running (or queued): an alternative may hold it
            if (!R.alt || !alt_adopt(R, (uint32_t)u, st.y, st.z, st.w, 0xffffffffu, 0u)) break;
            fl = __float_as_uint(R.col[R.ix(u)].w);
        }
        const float4 a = R.assume[R.ix(u)];
        const unsigned rm = fl & 15u, wm = (fl >> 4) & 15u;
        if (((rm & 2u) && __float_as_uint(a.x) != st.y) || ((rm & 4u) && __float_as_uint(a.y) != st.z) ||
            ((rm & 8u) && __float_as_uint(a.z) != st.w)) {
            if (R.alt && alt_adopt(R, (uint32_t)u, st.y, st.z, st.w, 0xffffffffu, 0u)) {
                fl = __float_as_uint(R.col[R.ix(u)].w);  // the adopted alternative is exact: go on
            } else {
                requeue(u, st.y, st.z, st.w);
                queued = true;
                break;
            }
        }
        const unsigned wm2 = (fl >> 4) & 15u;
        (void)wm;
        const float4 fn = R.fin[R.ix(u)];
        if (wm2 & 2u) st.y = __float_as_uint(fn.x);
        if (wm2 & 4u) st.z = __float_as_uint(fn.y);
        if (wm2 & 8u) st.w = __float_as_uint(fn.z);
    }
    st.x = s;
    R.front[pu] = st;
    // Anchored scan past the blocked sample s.  A finished sample that read no entry it had not
    // written (rmask 0) is exact whatever came before it, and so are the entries it wrote; a
    // finished sample whose reads are all of known entries is exact if its assumption matches
    // them.  Knowledge of entries 1..3 is tracked from s + 1 on (none known at first); once all
    // three are known, a mispredicted finished sample is re-queued at once with the exact state,
    // and the first unfinished one is handed to k_iow03_fixf (front2).  The scan goes on past
    // unfinished and mispredicted samples (knowledge restarts at the next anchor) up to
    // scan_max samples past the frontier.  So a misprediction
    // behind a long running sample is repaired without waiting for that sample (anchors --
    // samples with rmask 0 that write all three entries -- are 18% of the samples of the bench
    // scene, tests/analysis/fork_stats.py).
    if (!R.front2) return;
    uint4 f2 = make_uint4(0xffffffffu, 0u, 0u, 0u);
    if (!queued && s < R.S) {
        unsigned known = 0;
        uint32_t E[4] = {0u, 0u, 0u, 0u};
        const uint32_t k_end = min(R.S, s + 1u + R.scan_max);
        for (uint32_t k = s + 1u; k < k_end; k++) {
            const size_t u = (size_t)k * R.P + pu;
            const unsigned fl = __float_as_uint(R.col[R.ix(u)].w);
            if ((fl & 0xffff0100u) != done_tag) {  // unfinished: fixf may patch the first one
                if (known == 14u && f2.x == 0xffffffffu) f2 = make_uint4(k, E[1], E[2], E[3]);
                known = 0;  // its outputs are unknown; later anchors restore knowledge
                continue;
            }
            const unsigned rm = fl & 14u, wm = (fl >> 4) & 14u;
            if (rm & ~known) { known &= ~wm; continue; }  // read an unknown entry: its writes are unknown
            const float4 a = R.assume[R.ix(u)];
            const bool bad = ((rm & 2u) && __float_as_uint(a.x) != E[1]) ||
                             ((rm & 4u) && __float_as_uint(a.y) != E[2]) ||
                             ((rm & 8u) && __float_as_uint(a.z) != E[3]);
            unsigned wmx = wm;
            if (bad) {  // mispredicted: adopt an alternative, or re-run it now if the whole state is known
                if (known == 14u && R.alt && alt_adopt(R, (uint32_t)u, E[1], E[2], E[3], 0xffffffffu, 0u)) {
                    wmx = (__float_as_uint(R.col[R.ix(u)].w) >> 4) & 14u;
                } else {
                    if (known == 14u) requeue(u, E[1], E[2], E[3]);
                    known = 0;
                    continue;
                }
            }
            const float4 fn = R.fin[R.ix(u)];
            if (wmx & 2u) E[1] = __float_as_uint(fn.x);
            if (wmx & 4u) E[2] = __float_as_uint(fn.y);
            if (wmx & 8u) E[3] = __float_as_uint(fn.z);
            known |= wmx;
        }
    }
    R.front2[pu] = f2;
}
// Alternative runs (RT_SPEC_ALT, between tail rounds): for each pixel, every finished sample
// past the frontier that read exactly one stale entry before writing it, traced at least
// alt_min_seg segments and has no alternatives yet gets one run per other value that entry can
// hold (R.alt_vals), queued as restart records with flag 3.  Such a sample is where a dependent
// chain forms: if its guess was wrong, the frontier adopts the matching alternative instead of
// re-running a long sample once the samples before it are done.
__global__ __launch_bounds__(kBlock) void k_iow03_altspawn(Frame f, SpecRecs R, float4 *cont, unsigned *count,
                                                           uint32_t cap) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t n = R.order_n ? R.order_n : R.P;
    if (i >= n) return;  // no cross-lane work in this kernel
    const uint32_t pu = R.order_n ? R.order[R.order_base + i] : i;
    if (!unit_pixel(f, pu).in_image) return;
    const unsigned done_tag = (1u << 8) | ((R.epoch & 0xffffu) << 16);
    for (uint32_t s = R.front[pu].x; s < R.S; s++) {
        const uint32_t u = s * R.P + pu;
        const unsigned fl = __float_as_uint(R.col[R.ix(u)].w);
        if ((fl & 0xffff0100u) != done_tag) continue;
        const unsigned rm = fl & 14u;
        if (rm == 0u || (rm & (rm - 1u)) != 0u) continue;  // exactly one stale entry read
        if (R.ctr[R.ix(u)].x < R.alt_min_seg) continue;
        if (alt_find(R, u).y != 0u) continue;
        const int e = rm == 2u ? 0 : (rm == 4u ? 1 : 2);
        const float4 a = R.assume[R.ix(u)];
        const float ae = e == 0 ? a.x : (e == 1 ? a.y : a.z);
        uint32_t k = 0;
        for (int v = 0; v < R.n_alt_vals; v++) k += __float_as_uint(R.alt_vals[v]) != __float_as_uint(ae);
        if (k == 0u) continue;
        const uint32_t first = atomicAdd(R.alt_count, k);
        if (first + k > R.alt_cap) { atomicSub(R.alt_count, k); return; }
        const uint32_t slot = atomicAdd(count, k);
        if (slot + k > cap) { atomicSub(count, k); return; }  // leaves the claimed alt slots unused
        uint32_t j = 0;
        for (int v = 0; v < R.n_alt_vals; v++) {
            if (__float_as_uint(R.alt_vals[v]) == __float_as_uint(ae)) continue;
            AltRec &A = R.alt[first + j];
            A.u = u;
            A.state = 0u;
            float4 b = a;
            if (e == 0) b.x = R.alt_vals[v]; else if (e == 1) b.y = R.alt_vals[v]; else b.z = R.alt_vals[v];
            A.assume = b;
            float4 *p = cont + (size_t)(slot + j) * kContSlots;
            p[0] = make_float4(__uint_as_float(u), 0.0f, 0.0f, 0.0f);
            p[12] = make_float4(0.0f, 3.0f, __uint_as_float(first + j), 0.0f);  // start an alternative run
            j++;
        }
        // publish u -> (first, k) in the hash (open addressing, key u + 1)
        uint32_t h = (u * 2654435761u) % R.alt_hcap;
        for (uint32_t t = 0; t < R.alt_hcap; t++) {
            const unsigned prev = atomicCAS(&R.alt_hash[h].x, 0u, u + 1u);
            if (prev == 0u) { R.alt_hash[h].y = first | (k << 24); break; }
            h = h + 1u == R.alt_hcap ? 0u : h + 1u;
        }
    }
}

// Parked samples at their pixel's frontier: the exact incoming state E is known.  Entries the
// sample neither read nor wrote get E (exact: it would have started with them); if an entry it
// already read differs from E it restarts with E.  Either way its assumption becomes exact, so
// long samples stop waiting for a later resolve pass to find them wrong.
__global__ __launch_bounds__(kBlock) void k_iow03_fixf(Frame f, SpecRecs R, float4 *cont, const unsigned *count) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= *count) return;  // no cross-lane work in this kernel
    float4 *p = cont + (size_t)i * kContSlots;
    if (p[12].y != 0.0f || __float_as_uint(p[12].w) != 0u) return;  // a restart already / an alternative run
    const uint32_t u = __float_as_uint(p[0].x);
    const uint32_t pu = u % R.P, s = u / R.P;
    uint4 st = R.front[pu];
    if (st.x != s) {  // not at the frontier: past it, its exact state may come from the anchored scan
        if (!R.front2) return;
        st = R.front2[pu];
        if (st.x != s) return;
    }
    const unsigned E[3] = {st.y, st.z, st.w};
    const unsigned masks = __float_as_uint(p[0].w), wm = masks & 15u, rm = masks >> 4;
    float4 a = R.assume[R.ix(u)];
    float *av = &a.x;
    bool doomed = false;
    for (int k = 1; k <= 3; k++)
        if (((rm >> k) & 1u) && __float_as_uint(av[k - 1]) != E[k - 1]) doomed = true;
    if (doomed) {
        R.assume[R.ix(u)] = make_float4(__uint_as_float(E[0]), __uint_as_float(E[1]), __uint_as_float(E[2]), 0.0f);
        p[12].y = 1.0f;
        return;
    }
    float *fl = reinterpret_cast<float *>(p + 3);  // parked stack, [entry*9 + field], RI = field 7
    for (int k = 1; k <= 3; k++)
        if (!((wm >> k) & 1u) && !((rm >> k) & 1u)) {
            fl[k * 9 + 7] = __uint_as_float(E[k - 1]);
            av[k - 1] = __uint_as_float(E[k - 1]);
        }
    R.assume[R.ix(u)] = a;
}

// Replay of each pixel's samples in order (one lane per pixel unit; records are [s][pu], so
// consecutive lanes read consecutive records).
__global__ __launch_bounds__(kBlock) void k_iow03_resolve(Frame f, SpecRecs R, int final_pass, float4 *state) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;  // pixel i of the group (or of all units)
    const bool valid = R.order_n ? i < R.order_n : i < R.P;
    const uint32_t pu = valid ? (R.order_n ? R.order[R.order_base + i] : i) : 0;
    const UnitPix px = unit_pixel(f, valid ? pu : 0);
    bool work = valid && px.in_image;
    uint32_t E1 = 0, E2 = 0, E3 = 0;  // exact RI bits of entries 1..3 before sample s
    f3 fc = f3{0, 0, 0};
    unsigned long long seg = 0, drops = 0, nans = 0, nodes = 0, prims = 0;
    int first_bad = -1;
    uint32_t s = 0;
    for (; work && s < R.S; s++) {
        const size_t u = (size_t)s * R.P + pu;
        float4 cl = R.col[R.ix(u)];
        uint32_t fl = __float_as_uint(cl.w), rm = fl & 15u, wm = (fl >> 4) & 15u;
        float4 a = R.assume[R.ix(u)];
#ifdef RT_DIAG
        if (final_pass && R.exact && (R.exact_mode & 1) && first_bad < 0)
            R.exact[u] = make_float4(__uint_as_float(E1), __uint_as_float(E2), __uint_as_float(E3), 0.0f);
#endif
        bool bad = ((rm & 2u) && __float_as_uint(a.x) != E1) || ((rm & 4u) && __float_as_uint(a.y) != E2) ||
                   ((rm & 8u) && __float_as_uint(a.z) != E3);
        if (bad && first_bad < 0 && R.alt && alt_adopt(R, (uint32_t)u, E1, E2, E3, 0xffffffffu, 0u)) {
            cl = R.col[R.ix(u)];  // an alternative run under the exact state: adopted
            fl = __float_as_uint(cl.w); rm = fl & 15u; wm = (fl >> 4) & 15u;
            a = R.assume[R.ix(u)];
            bad = false;
        }
        if (bad) {
            if (first_bad < 0) first_bad = (int)s;
            if (final_pass) break;  // the sequential kernel takes over from here
            R.assume[R.ix(u)] = make_float4(__uint_as_float(E1), __uint_as_float(E2), __uint_as_float(E3), 0.0f);
            R.list[atomicAdd(R.list_count, 1u)] = (uint32_t)u;
        }
        if (first_bad < 0) {  // still exact: accumulate in sample order
            fc = fc + f3{cl.x, cl.y, cl.z};
            const uint4 ct4 = R.ctr[R.ix(u)];
            seg += ct4.x; drops += ct4.y; nans += ct4.z; nodes += ct4.w;
            prims += __float_as_uint(R.fin[R.ix(u)].w);
        }
        const float4 fn = R.fin[R.ix(u)];  // the record's own outputs (a guess while it is queued)
        if (wm & 2u) E1 = __float_as_uint(fn.x);
        if (wm & 4u) E2 = __float_as_uint(fn.y);
        if (wm & 8u) E3 = __float_as_uint(fn.z);
    }
    if (final_pass && valid && !px.in_image) write_px(f, px, f3{0, 0, 0}, 0.0f);  // tile padding
    if (final_pass && work) {
        if (first_bad < 0) {
            write_px(f, px, fc * rcp((float)R.S), 0.0f);
            if (f.px_rays) f.px_rays[pu] = (unsigned)seg;
        } else {  // resume state for the sequential kernel: colour sum, first sample, stack RI
            state[2 * (size_t)pu] = make_float4(fc.x, fc.y, fc.z, __int_as_float(first_bad));
            state[2 * (size_t)pu + 1] = make_float4(0.0f, __uint_as_float(E1), __uint_as_float(E2), __uint_as_float(E3));
            R.fb_list[atomicAdd(R.fb_count, 1u)] = pu;
        }
    }
    if (final_pass && f.counters) {
        const unsigned long long v[5] = {seg, nodes, prims, drops, nans};
        const int slot[5] = {0, 1, 2, 4, 5};
#pragma unroll
        for (int i = 0; i < 5; i++) {
            const unsigned long long t = wave_sum(v[i]);
            if ((threadIdx.x & 63) == 0 && t) atomicAdd(f.counters + slot[i], t);
        }
    }
}

// ============================================================================ INW
constexpr float kMaxT = 32000.0f;

struct FStack {  // FLT_STACK (01_BVH...glsl:81-107) in LDS, [slot][thread]
    float *base;
    uint32_t size;
    __device__ __forceinline__ float &at(uint32_t k) { return base[k * kBlock]; }
    __device__ __forceinline__ void push(float v, Ctr &c) {
        if (size < kFStack) { at(size) = v; size++; } else c.drops++;
    }
    __device__ __forceinline__ void push_ray(f3 o, f3 d, float contrib, float bounced, Ctr &c) {
        if (size < kFStack - 7) {
            at(size) = o.x; at(size + 1) = o.y; at(size + 2) = o.z;
            at(size + 3) = d.x; at(size + 4) = d.y; at(size + 5) = d.z;
            at(size + 6) = contrib; at(size + 7) = bounced;
            size += 8;
        } else c.drops++;
    }
    // the top ray (8 floats: origin, direction, contribution, bounced) off the stack
    __device__ __forceinline__ void pop_ray(f3 &o, f3 &d, float &contrib, float &bounced) {
        size -= 8;
        o = f3{at(size), at(size + 1), at(size + 2)};
        d = f3{at(size + 3), at(size + 4), at(size + 5)};
        contrib = at(size + 6);
        bounced = at(size + 7);
    }
    __device__ __forceinline__ void reset(uint32_t n) { size = n; }
    // the top entry is a primary ray (bounced == 0)
    __device__ __forceinline__ bool top_primary() { return size >= 8u && at(size - 1u) == 0.0f; }
    // the wide walks' node stack: the free part above the stack (+ extra floats), kBlock apart;
    // cap = entries left after `spare` slots for branch-free pushes
    __device__ __forceinline__ float *walk_stack(uint32_t extra, int spare, int &cap) {
        cap = kFStack - spare - (int)(size + extra);
        return &at(size + extra);
    }
};

// The same stack for k_inw_pm's GQ instance (DESIGN.md §5.1 "GQ"): the 40 floats in global memory
// ([slot4][lane] float4 columns, `stride` lanes apart; touched about once per segment), the top ray
// in registers -- a segment pops the ray the one before pushed last, so most pops read no memory
// -- and the wide walks' node stack in LDS (kWStack entries per lane, kBlock apart).  The
// capacity and drop semantics are FStack's: size counts every float, pushes drop when it is full.
// Invariant: a primary ray (bounced 0) is only ever the register top (pushed at a sample's start or
// by the MULTIFOCUS chain, popped by the next segment), so top_primary reads no memory.
struct GStack {
    float4 *col;        // this lane's column: slot4 k at col[k * stride]
    uint32_t stride;
    uint32_t size;
    float *ws;          // LDS node stack of the wide walks
    bool rc;            // the top 8 floats are the register ray (r0, r1); their memory is stale
    float4 r0, r1;      // o.xyz d.x | d.yz contrib bounced
    __device__ __forceinline__ float &at(uint32_t k) {
        return reinterpret_cast<float *>(col + (size_t)(k >> 2) * stride)[k & 3u];
    }
    __device__ __forceinline__ void flush() {  // the register ray to its slots size - 8 .. size - 1
        const uint32_t b = size - 8u;
        if ((b & 3u) == 0u) {
            col[(size_t)(b >> 2) * stride] = r0;
            col[(size_t)((b >> 2) + 1u) * stride] = r1;
        } else {
            at(b) = r0.x; at(b + 1) = r0.y; at(b + 2) = r0.z; at(b + 3) = r0.w;
            at(b + 4) = r1.x; at(b + 5) = r1.y; at(b + 6) = r1.z; at(b + 7) = r1.w;
        }
        rc = false;
    }
    __device__ __forceinline__ void push(float v, Ctr &c) {
        if (size < kFStack) {
            if (rc) flush();
            at(size) = v;
            size++;
        } else c.drops++;
    }
    __device__ __forceinline__ void push_ray(f3 o, f3 d, float contrib, float bounced, Ctr &c) {
        if (size < kFStack - 7) {
            if (rc) flush();
            r0 = make_float4(o.x, o.y, o.z, d.x);
            r1 = make_float4(d.y, d.z, contrib, bounced);
            rc = true;
            size += 8;
        } else c.drops++;
    }
    __device__ __forceinline__ void pop_ray(f3 &o, f3 &d, float &contrib, float &bounced) {
        size -= 8;
        if (!rc) {
            if ((size & 3u) == 0u) {
                r0 = col[(size_t)(size >> 2) * stride];
                r1 = col[(size_t)((size >> 2) + 1u) * stride];
            } else {
                r0 = make_float4(at(size), at(size + 1), at(size + 2), at(size + 3));
                r1 = make_float4(at(size + 4), at(size + 5), at(size + 6), at(size + 7));
            }
        }
        rc = false;
        o = f3{r0.x, r0.y, r0.z};
        d = f3{r0.w, r1.x, r1.y};
        contrib = r1.z;
        bounced = r1.w;
    }
    __device__ __forceinline__ void reset(uint32_t n) { size = n; rc = false; }
    __device__ __forceinline__ bool top_primary() { return rc && r1.w == 0.0f; }
    __device__ __forceinline__ float *walk_stack(uint32_t, int spare, int &cap) {
        cap = kWStack - spare;
        return ws;
    }
};

// ident: the rotation is exactly the identity (the host marks the record's type field with + 0.5;
// int(type + 0.1) still reads the type): the wide walk's object test then skips both 3 x 3 products
// and, for a cuboid, reuses the ray's reciprocals (DESIGN.md §5.2 "Unrotated objects")
struct Xf { f3 pos, scale, delta, is, is2; m3 R; int type; bool ident; float extra, ri_acc; };

__device__ __forceinline__ Xf load_xf(const InwScene &S, int g) {
    const float4 *h = S.hot + (size_t)g * 7;
    float4 a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], q = h[6];
    Xf x;
    x.pos = mk(a.x, a.y, a.z);
    x.R.c0 = mk(a.w, b.x, b.y); x.R.c1 = mk(b.z, b.w, c.x); x.R.c2 = mk(c.y, c.z, c.w);
    x.scale = mk(d.x, d.y, d.z);
    x.delta = mk(d.w, e.x, e.y);
    x.type = (int)(e.z + 0.1f);
    x.ident = e.z - (float)x.type > 0.25f;
    x.extra = e.w;
    x.is = mk(f.x, f.y, f.z);
    x.is2 = mk(f.w, q.x, q.y);
    x.ri_acc = q.z;
    return x;
}

// TestIntersectAABB 01_BVH...glsl:187-208 (reciprocals of the ray direction hoisted)
// EO (default): the shader's early outs.  !EO: every axis evaluated -- the same result, with the
// node's two loads issued together (see test_aabb_te below); INW-04's reference walks (its
// axis-aligned rays) run 1.1% faster that way at C5, INW-01's early-out code generation is 1% faster at C3
template <bool EO = true>
__device__ __forceinline__ bool test_aabb(float4 n0, float4 n1, f3 o, f3 id, float tlim) {
    float a = (n0.x - o.x) * id.x, b = (n0.w - o.x) * id.x;
    float tmin = fminf(a, b), tmax = fmaxf(a, b);
    if constexpr (EO) {
        if (tmax <= tmin) return false;  // axis 0 re-applied by the loop is idempotent
        a = (n0.y - o.y) * id.y; b = (n1.x - o.y) * id.y;
        tmin = fmaxf(fminf(a, b), tmin); tmax = fminf(fmaxf(a, b), tmax);
        if (tmax <= tmin) return false;
        a = (n0.z - o.z) * id.z; b = (n1.y - o.z) * id.z;
        tmin = fmaxf(fminf(a, b), tmin); tmax = fminf(fmaxf(a, b), tmax);
        if (tmax <= tmin) return false;
        return tlim > 0.0f ? tlim > tmin : true;
    } else {
        bool ok = !(tmax <= tmin);
        a = (n0.y - o.y) * id.y; b = (n1.x - o.y) * id.y;
        tmin = fmaxf(fminf(a, b), tmin); tmax = fminf(fmaxf(a, b), tmax);
        ok = ok && !(tmax <= tmin);
        a = (n0.z - o.z) * id.z; b = (n1.y - o.z) * id.z;
        tmin = fmaxf(fminf(a, b), tmin); tmax = fminf(fmaxf(a, b), tmax);
        ok = ok && !(tmax <= tmin);
        return ok && (tlim > 0.0f ? tlim > tmin : true);
    }
}

// The same test, also returning the entry t it compares (te) -- the wide walk's guard below.  Every
// axis is evaluated (test_aabb returns at the first failing one): the same result and, when it
// passes, the same te.  Without the early outs the compiler issues the box's loads together
// instead of one round trip per axis: C3 201.7 -> 196.5 ms, C5 6.92 -> 6.79 s (same-box A/B,
// profiles/r05_ab_leaf_test.json)
__device__ __forceinline__ bool test_aabb_te(float4 n0, float4 n1, f3 o, f3 id, float tlim, float &te) {
    float a = (n0.x - o.x) * id.x, b = (n0.w - o.x) * id.x;
    float tmin = fminf(a, b), tmax = fmaxf(a, b);
    bool ok = !(tmax <= tmin);
    a = (n0.y - o.y) * id.y; b = (n1.x - o.y) * id.y;
    tmin = fmaxf(fminf(a, b), tmin); tmax = fminf(fmaxf(a, b), tmax);
    ok = ok && !(tmax <= tmin);
    a = (n0.z - o.z) * id.z; b = (n1.y - o.z) * id.z;
    tmin = fmaxf(fminf(a, b), tmin); tmax = fminf(fmaxf(a, b), tmax);
    ok = ok && !(tmax <= tmin);
    te = tmin;
    return ok && (tlim > 0.0f ? tlim > tmin : true);
}

// closest-hit LBVH DFS (01_BVH...glsl:431-473, 04...glsl:524-563, shadow 620-657)
template <bool WANT_NORMAL, bool EO = true, class KS = FStack>
__device__ float inw_traverse(const InwScene &S, KS &K, f3 o, f3 d, float ratio, bool invert,
                              float &tlim, f3 &normal, float &extra, float init_geom, Ctr &c) {
    float final_geom = init_geom;
    const uint32_t I = K.size;
    const f3 id = f3{rcp(d.x), rcp(d.y), rcp(d.z)};
    K.push(0.0f, c);
    for (;;) {
        float geom = -1.0f;
        while (K.size > I) {
            K.size--;
            const int node = (int)K.at(K.size);
            const float4 n0 = S.nodes[2 * node], n1 = S.nodes[2 * node + 1];
            c.nodes++;
            if (test_aabb<EO>(n0, n1, o, id, tlim)) {
                const float left = n1.z;
                if (left > 0.1f) {
                    const float right = left + 1.0f;
                    K.push(invert ? right : left, c);
                    K.push(invert ? left : right, c);
                } else { geom = -left; break; }
            }
        }
        if (!(geom > -0.9f)) break;
        c.prims++;
        // IntersectRay / IntersectRayMinimal
        const Xf x = load_xf(S, (int)geom);
        f3 ov = (o - x.pos) + x.delta * (1.0f - ratio);
        f3 to = tmul(x.R, ov), td = tmul(x.R, d);
        float t = -1.0f;
        if (x.type == 1) t = t_ellipsoid(to, td, x.is);
        else if (x.type == 2) t = t_cuboid(to, td, x.scale);
        if (t > 0.0f && t < tlim) {
            tlim = t;
            final_geom = geom;
            if (WANT_NORMAL) {
                f3 h = to + td * t, nl;
                if (x.type == 1) nl = normalize(f3{h.x * x.is2.x, h.y * x.is2.y, h.z * x.is2.z});
                else if (x.type == 2) nl = cuboid_normal(h, x.scale);
                else nl = f3{0, 0, 0};
                normal = mul(x.R, nl);
                extra = x.extra;
            }
        }
    }
    K.size = I;
    return final_geom;
}

// Surrounding refractive index (01_BVH...glsl:272-345, 486-502)
template <class KS = FStack>
__device__ float inw_surrounding_ri(const InwScene &S, KS &K, f3 hp, float ratio, Ctr &c) {
    float acc = 0.0f;
    uint32_t cnt = 0;
    const uint32_t I = K.size;
    K.push(0.0f, c);
    while (K.size > I) {
        K.size--;
        const int node = (int)K.at(K.size);
        const float4 n0 = S.nodes[2 * node], n1 = S.nodes[2 * node + 1];
        c.nodes++;
        if (hp.x <= n0.w && hp.y <= n1.x && hp.z <= n1.y && hp.x >= n0.x && hp.y >= n0.y && hp.z >= n0.z) {
            const float left = n1.z;
            if (left < 0.1f) {
                c.prims++;
                const Xf x = load_xf(S, (int)(-left));
                f3 v = (hp - x.pos) + x.delta * (1.0f - ratio);
                v = tmul(x.R, v);
                v.x *= x.is.x; v.y *= x.is.y; v.z *= x.is.z;
                bool inside;
                if (x.type == 1) inside = dot(v, v) <= 1.0f;
                else if (x.type == 2) inside = fabsf(v.x) <= 0.5f && fabsf(v.y) <= 0.5f && fabsf(v.z) <= 0.5f;
                else inside = false;
                if (inside) { acc += x.ri_acc; cnt++; }
            } else {
                K.push(left, c);
                K.push(left + 1.0f, c);
            }
        }
    }
    if (acc > 1.0f) acc *= rcp((float)cnt);
    else acc = 1.0f;
    return acc;
}

// ---------------------------------------------------------------- LDS-staged top of the wide BVH
// (measured in DESIGN.md §5): kernels instantiated with LN copy the first n_lnodes wide
// nodes -- the top levels, as bvh4_collapse numbers them breadth first -- into LDS and read them
// there; deeper nodes come from global memory.
// INW wide node: 10 float4, SoA over the 4 children: planes lx ly lz hx hy hz, then lx ly lz again,
// then the child links.  The repeat lets a ray read its near and far planes of axis a at
// a + 3*s_a and a + 3 + 3*s_a (s_a = 1 when d_a < 0): one per-lane offset per axis (inw_wnode_nf).
constexpr int kInwNodeF4 = 10;
// 236 nodes (36.9 KB): what the 3 x 256-lane stacks (120 KB) and k_inw_pm's depth slots (3 KB)
// leave of 160 KB
// (kInwLdsNodes = 236: rt_kernels.hpp)
__shared__ float4 g_inw_lnodes[kInwLdsNodes * kInwNodeF4];
// k_inw_pm / k_inw_sm with LN and InwScene::lring / lring_sm: room for kPmLdsNodes nodes, then the
// 12 waves' fold rings of kPmLdsRing entries (r, g, b planes) in the same LDS (a
// 256-entry window costs 0.5% against 1024, 128 entries 7%; the ring takes the LDS of all but 5
// nodes, which were worth 1.5%, and saves 1% of global ring traffic -- 0.57 against 42 GB of
// L2-to-fabric traffic per C3 frame).  k_inw_pm's ring instances leave those 5 slots unused (its
// walks read no staged node), k_inw_sm's stage the BVH there when it fits
static_assert(kPmLdsNodes * kInwNodeF4 * 16 + 12 * 3 * kPmLdsRing * 4 <= kInwLdsNodes * kInwNodeF4 * 16, "LDS ring");
template <bool LN>
__device__ __forceinline__ const float4 *inw_node_ptr(const InwScene &S, int cur) {
    if (LN && (uint32_t)(cur - 1) < S.n_lnodes) return g_inw_lnodes + kInwNodeF4 * (cur - 1);
    return S.wnodes + kInwNodeF4 * (cur - 1);
}
template <bool LN>
__device__ __forceinline__ void inw_wnode(const InwScene &S, int cur, float4 &lx, float4 &ly, float4 &lz, float4 &hx,
                                          float4 &hy, float4 &hz, float4 &lk) {
    const float4 *nd = inw_node_ptr<LN>(S, cur);
    lx = nd[0]; ly = nd[1]; lz = nd[2]; hx = nd[3]; hy = nd[4]; hz = nd[5]; lk = nd[9];
}
// The near and far planes of the four children for this ray's octant (oa = a + 3*s_a).
template <bool LN>
__device__ __forceinline__ void inw_wnode_nf(const InwScene &S, int cur, uint32_t ox, uint32_t oy, uint32_t oz,
                                             float4 &nx, float4 &ny, float4 &nz, float4 &fx, float4 &fy, float4 &fz,
                                             float4 &lk) {
#ifndef RT_INW_FLAT
    if (LN && (uint32_t)(cur - 1) < S.n_lnodes) {  // ds_read_b128 (a generic pointer would make flat loads)
        const float4 *nd = g_inw_lnodes + kInwNodeF4 * (cur - 1);
        const float4 *px = nd + ox, *py = nd + oy, *pz = nd + oz;
        nx = px[0]; fx = px[3]; ny = py[0]; fy = py[3]; nz = pz[0]; fz = pz[3]; lk = nd[9];
        return;
    }
    const float4 *nd = S.wnodes + kInwNodeF4 * (cur - 1);
#else
    const float4 *nd = inw_node_ptr<LN>(S, cur);
#endif
    const float4 *px = nd + ox, *py = nd + oy, *pz = nd + oz;
    nx = px[0]; fx = px[3]; ny = py[0]; fy = py[3]; nz = pz[0]; fz = pz[3]; lk = nd[9];
}
// The same fetch from global memory as buffer loads: the node's byte offset is 32 bits (a node
// index times 160), the octant offsets and the far planes' +48 / the links' +144 fold into the
// instructions, so a node step spends 4 VALU on addresses instead of the 64-bit pointer sums (~10)
// (C3 185.9 -> 184.2 ms on one box, profiles/r06_ab2_gq.json; -DRT_INW_NO_BUFLOAD: the pointer form)
__device__ __forceinline__ float4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
// The buffer-load walk's node layout: 10 float4 (wnodes: the far planes 48 B after the near ones)
// or, with InwScene::cnodes, 7 float4 (the far plane of axis a at a + 3 (1 - s_a): its own offset)
struct WnodeBuf {
    __amdgpu_buffer_rsrc_t rs;
    uint32_t stride, lk;     // bytes per node, offset of the links
    uint32_t fx, fy, fz;     // far-plane offsets of this ray's octant
};
__device__ __forceinline__ WnodeBuf wnode_buf(const InwScene &S, uint32_t oxb, uint32_t oyb, uint32_t ozb) {
    WnodeBuf w;
    const bool c = S.cnodes != nullptr;
    w.stride = c ? 112u : (uint32_t)kInwNodeF4 * 16u;
    w.lk = c ? 96u : 144u;
    // cnodes: near at 16 a + 48 s_a, far at 16 a + 48 (1 - s_a): near + far = 32 a + 48
    w.fx = c ? 48u - oxb : oxb + 48u;
    w.fy = c ? 80u - oyb : oyb + 48u;
    w.fz = c ? 112u - ozb : ozb + 48u;
    // dword 3 = 0x00020000: the gfx9-family raw-buffer format word; num_records bounds the nodes
    w.rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float4 *>(c ? S.cnodes : S.wnodes), (short)0,
                                             (int)(S.n_wnodes * w.stride), 0x00020000);
    return w;
}
template <bool LN>
__device__ __forceinline__ void inw_wnode_nf_buf(const InwScene &S, const WnodeBuf &W, int cur, uint32_t oxb,
                                                 uint32_t oyb, uint32_t ozb, float4 &nx, float4 &ny, float4 &nz,
                                                 float4 &fx, float4 &fy, float4 &fz, float4 &lk) {
    if (LN && (uint32_t)(cur - 1) < S.n_lnodes) {
        const float4 *nd = g_inw_lnodes + kInwNodeF4 * (cur - 1);
        const float4 *px = nd + (oxb >> 4), *py = nd + (oyb >> 4), *pz = nd + (ozb >> 4);
        nx = px[0]; fx = px[3]; ny = py[0]; fy = py[3]; nz = pz[0]; fz = pz[3]; lk = nd[9];
        return;
    }
    const uint32_t b = __umul24((uint32_t)(cur - 1), W.stride);  // v_mul_u32_u24 (ids < 2^24)
    nx = bload4(W.rs, b + oxb); fx = bload4(W.rs, b + W.fx);
    ny = bload4(W.rs, b + oyb); fy = bload4(W.rs, b + W.fy);
    nz = bload4(W.rs, b + ozb); fz = bload4(W.rs, b + W.fz);
    lk = bload4(W.rs, b + W.lk);
}
// FU: one fused multiply-add per plane, plane * (1/d) + (-o * (1/d)), the second term computed
// once per ray (noid).  Its rounding error in t is at most |o| * 2^-23 * |1/d| per axis, against a
// culling-box inflation of e >= 1e-3 (x |1/d| in t), so it stays conservative while
// |o| * 2^-23 < e: the host enables it (InwScene::fused) only when every ray origin (the camera,
// the scene's boxes) lies within 1000 of the origin.  The wide walk runs with finite reciprocals
// only (an infinite one would make every plane's fma NaN).
// The culling test with the planes already split into near and far by the ray's octant.  With a
// finite, nonzero reciprocal, the slab value of a plane is monotone in the plane (each step is a
// correctly rounded monotone function), so the near plane's value is the min of the pair and the
// far plane's the max: the same te and tx bits as min / max of the pair, without the 6 min/max per child.
// The test te <= tx && tx >= -1e-3 && te <= lim is max(te, -1e-3) <= min(tx, lim) (lim > 0).
template <bool FU>
__device__ __forceinline__ void cull4nf(const float4 nx, const float4 ny, const float4 nz, const float4 fx,
                                        const float4 fy, const float4 fz, f3 o, f3 id, f3 noid, float lim, float &t0,
                                        float &t1, float &t2, float &t3) {
    const pf2 ix = pk(id.x, id.x), iy = pk(id.y, id.y), iz = pk(id.z, id.z);
    pf2 a[12];
    const float4 *pl[6] = {&nx, &ny, &nz, &fx, &fy, &fz};
    const pf2 iv[3] = {ix, iy, iz};
    if constexpr (FU) {
        const pf2 nv[3] = {pk(noid.x, noid.x), pk(noid.y, noid.y), pk(noid.z, noid.z)};
#pragma unroll
        for (int k = 0; k < 6; k++) {
            a[2 * k] = __builtin_elementwise_fma(pk(pl[k]->x, pl[k]->y), iv[k % 3], nv[k % 3]);
            a[2 * k + 1] = __builtin_elementwise_fma(pk(pl[k]->z, pl[k]->w), iv[k % 3], nv[k % 3]);
        }
    } else {
        const pf2 ov[3] = {pk(o.x, o.x), pk(o.y, o.y), pk(o.z, o.z)};
#pragma unroll
        for (int k = 0; k < 6; k++) {
            a[2 * k] = (pk(pl[k]->x, pl[k]->y) - ov[k % 3]) * iv[k % 3];
            a[2 * k + 1] = (pk(pl[k]->z, pl[k]->w) - ov[k % 3]) * iv[k % 3];
        }
    }
    // a[2k + h]: plane k (near x, y, z, far x, y, z) of children 2h, 2h + 1
    auto one = [&](float n0, float n1, float n2, float f0, float f1, float f2) {
        const float te = fmaxf(fmaxf(n0, n1), n2), tx = fminf(fminf(f0, f1), f2);
        return fmaxf(te, -1e-3f) <= fminf(tx, lim) ? te : kMiss;
    };
    t0 = one(a[0].x, a[2].x, a[4].x, a[6].x, a[8].x, a[10].x);
    t1 = one(a[0].y, a[2].y, a[4].y, a[6].y, a[8].y, a[10].y);
    t2 = one(a[1].x, a[3].x, a[5].x, a[7].x, a[9].x, a[11].x);
    t3 = one(a[1].y, a[3].y, a[5].y, a[7].y, a[9].y, a[11].y);
}

// ---------------------------------------------------------------- quantised wide nodes (GQ)
// DESIGN.md §5.2 "Quantised nodes": 4 float4 per node instead of 10 (InwScene::qnodes; built by
// rt_build.hip: k_quantize_wnodes), so a node step is 4 loads (64 B, half a cache line) instead of 7
// (112 B), and 1,168 nodes fit the LDS the global FStack frees.  k_inw_pm's GQ instance stages the
// first n_lnodes of them (the top levels, breadth first) in g_inw_qlds.
__shared__ float4 g_inw_qlds[kQLdsNodes * kQNodeF4];
template <bool LN>
__device__ __forceinline__ void inw_qnode(const InwScene &S, int cur, float4 &a, float4 &b, float4 &c, float4 &lk) {
    if (LN && (uint32_t)(cur - 1) < S.n_lnodes) {  // ds_read_b128
        const float4 *nd = g_inw_qlds + kQNodeF4 * (cur - 1);
        a = nd[0]; b = nd[1]; c = nd[2]; lk = nd[3];
        return;
    }
    const float4 *nd = S.qnodes + kQNodeF4 * (cur - 1);
    a = nd[0]; b = nd[1]; c = nd[2]; lk = nd[3];
}
// The fused cull of a quantised node: per axis sf = s * (1/d), of = fma(o, 1/d, -ray.o * (1/d)),
// and each plane's t = fma(byte, sf, of) (one v_cvt_f32_ubyte per plane, pairs of fma packed).
// hx/hy/hz: the ray's direction is negative on that axis, so its near planes are the high ones.
__device__ __forceinline__ float ub(uint32_t v, int k) { return (float)((v >> (8 * k)) & 0xffu); }
__device__ __forceinline__ void cull4q(const float4 a, const float4 b, const float4 c, bool hx, bool hy, bool hz, f3 fid,
                                      f3 noid, float lim, float &t0, float &t1, float &t2, float &t3) {
    const float sf[3] = {a.w * fid.x, b.x * fid.y, b.y * fid.z};
    const float of[3] = {__builtin_fmaf(a.x, fid.x, noid.x), __builtin_fmaf(a.y, fid.y, noid.y),
                         __builtin_fmaf(a.z, fid.z, noid.z)};
    const uint32_t lx = __float_as_uint(b.z), ly = __float_as_uint(b.w), lz = __float_as_uint(c.x);
    const uint32_t ux = __float_as_uint(c.y), uy = __float_as_uint(c.z), uz = __float_as_uint(c.w);
    const uint32_t q[6] = {hx ? ux : lx, hy ? uy : ly, hz ? uz : lz, hx ? lx : ux, hy ? ly : uy, hz ? lz : uz};
    pf2 t[12];  // t[2p + h]: plane p (near x, y, z, far x, y, z) of children 2h, 2h + 1
#pragma unroll
    for (int p = 0; p < 6; p++) {
        const pf2 s2 = pk(sf[p % 3], sf[p % 3]), o2 = pk(of[p % 3], of[p % 3]);
        t[2 * p] = __builtin_elementwise_fma(pk(ub(q[p], 0), ub(q[p], 1)), s2, o2);
        t[2 * p + 1] = __builtin_elementwise_fma(pk(ub(q[p], 2), ub(q[p], 3)), s2, o2);
    }
    auto one = [&](float n0, float n1, float n2, float f0, float f1, float f2) {
        const float te = fmaxf(fmaxf(n0, n1), n2), tx = fminf(fminf(f0, f1), f2);
        return fmaxf(te, -1e-3f) <= fminf(tx, lim) ? te : kMiss;
    };
    t0 = one(t[0].x, t[2].x, t[4].x, t[6].x, t[8].x, t[10].x);
    t1 = one(t[0].y, t[2].y, t[4].y, t[6].y, t[8].y, t[10].y);
    t2 = one(t[1].x, t[3].x, t[5].x, t[7].x, t[9].x, t[11].x);
    t3 = one(t[1].y, t[3].y, t[5].y, t[7].y, t[9].y, t[11].y);
}

// An empty asm that reads the object-space ray: the compiler must have it (so the object record's
// loads) before the caller's box-test branch, instead of sinking the loads behind the branch --
// one round trip for box and record instead of two or three (leaf tests, beam candidates)
__device__ __forceinline__ void keep_before_branch(f3 to, f3 td) {
#ifndef RT_LEAF_SINK
    asm volatile("" ::"v"(to.x), "v"(to.y), "v"(to.z), "v"(td.x), "v"(td.y), "v"(td.z));
#endif
}

// Scalar loads of wave-uniform records (constant address space: s_load through the scalar cache,
// no vector-memory / TA work)
typedef float sv4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(4))) const sv4f csv4f;
__device__ __forceinline__ float4 sload4(const float4 *p, int i) {
    const sv4f v = ((const csv4f *)(const void *)p)[i];
    return make_float4(v.x, v.y, v.z, v.w);
}

// ---------------------------------------------------------------- INW wide walk
// The reference's closest hit (01_BVH...glsl:431-473) is the nearest hit among the objects whose
// LBVH leaf box its depth-first walk reaches, ties to the one it reaches first.  With finite ray
// reciprocals the walk reaches every leaf whose own box test passes (an ancestor box holds the
// leaf box, and the slab intervals are monotone in the planes), as long as its 40-float stack
// drops no push -- guaranteed while size + dfs_high <= 40.  Under those conditions the ordered
// walk of the 4-wide culling BVH below, the reference's test of the leaf box with the initial
// limit, the exact object test and the (t, depth-first rank) rule pick the same object with the
// same t; its normal and extra data are then computed as the reference computes them.  The
// walk's stack lives in the free part of the shared stack above K.size.  Node and primitive
// counters count this walk's own work.  ok = false: the conditions do not hold (or the walk's
// stack overflowed) and the caller runs the reference walk.
// One more condition: the reference tests a leaf box against its running limit, so it skips an
// object whose box entry te is not below the best t found so far.  Normally t >= te for a hit
// inside its own box, and then skipping it changes nothing; but where an object's face coincides
// with its box face, rounding can put t an ulp below te.  Any accepted candidate with t < te
// therefore hands the ray to the reference walk (ok = false).
// Walk parking (RT_INW_PARK experiment, DESIGN.md §5 "Walk parking"): a wave's walk loop runs
// as long as its slowest lane; with PK, once at most kParkLanes lanes still walk (after at least
// kParkMinTrips trips) the wave tests the pending leaves, saves those lanes' walk state to their
// slot (2 float4: cur, sp, best object, its rank; best t, culling limit) and leaves the loop, so
// the other lanes shade and start their next segments; the parked lanes resume their walk in the
// next iteration of the fold kernel, next to the new walks.  The segment's ray stays in the
// shared stack (the walk's stack starts 8 floats above it).  The walk's result does not depend on
// when its node steps run, so the image and the counters are unchanged.
#ifndef RT_INW_PARK_LANES
#define RT_INW_PARK_LANES 8
#endif
#ifndef RT_INW_PARK_MIN
#define RT_INW_PARK_MIN 4
#endif
constexpr int kParkLanes = RT_INW_PARK_LANES, kParkMinTrips = RT_INW_PARK_MIN;
#ifndef RT_INW_LEAF_BATCH
#define RT_INW_LEAF_BATCH 65
#endif
constexpr int kInwLeafBatch = RT_INW_LEAF_BATCH;
struct WalkPark {
    float4 *slot;   // this lane's 2 float4
    bool resume;    // the walk was parked in an earlier iteration: restore it
    bool parked;    // out: parked again
};
// QN: the quantised nodes (S.qnodes, cull4q; requires FU), LN then meaning the staged ones in g_inw_qlds.
// The hit object's normal and extra data (01_BVH...glsl:FillHitData's inputs) at t = bt.  SP with
// sphere records: from their third float4 (RN(1/RN(s*s)) per axis, extra) -- R = I, so the
// object-space ray is the world one (h's components are nonzero products: the same floats) and
// mul(I, nl) is evaluated with the literal identity, the same operations as with R loaded
template <bool SP>
__device__ __forceinline__ void inw_hit_normal(const InwScene &S, int bg, f3 o, f3 d, float ratio, float bt, f3 &normal,
                                               float &extra) {
#ifndef RT_INW_SPH_NO_NORMAL
    if (SP && S.sph) {
        const float4 p = S.sph[3 * bg], q = S.sph[3 * bg + 1], w = S.sph[3 * bg + 2];
        const f3 ov = (o - mk(p.x, p.y, p.z)) + mk(q.x, q.y, q.z) * (1.0f - ratio);
        const f3 h = ov + d * bt;
        const f3 nl = normalize(f3{h.x * w.x, h.y * w.y, h.z * w.z});
        const m3 I = m3{f3{1.0f, 0.0f, 0.0f}, f3{0.0f, 1.0f, 0.0f}, f3{0.0f, 0.0f, 1.0f}};
        normal = mul(I, nl);
        extra = w.w;
        return;
    }
#endif
    const Xf x = load_xf(S, bg);
    f3 ov = (o - x.pos) + x.delta * (1.0f - ratio);
#ifndef RT_INW_NO_IDENT
    if (x.ident) {  // R = I: h = ov + d bt has the same floats (d has no zero component here), and
                    // mul(I, nl) with the literal identity repeats the loaded R's operations
        const f3 h = ov + d * bt;
        f3 nl;
        if (x.type == 1) nl = normalize(f3{h.x * x.is2.x, h.y * x.is2.y, h.z * x.is2.z});
        else if (x.type == 2) nl = cuboid_normal(h, x.scale);
        else nl = f3{0, 0, 0};
        const m3 I = m3{f3{1.0f, 0.0f, 0.0f}, f3{0.0f, 1.0f, 0.0f}, f3{0.0f, 0.0f, 1.0f}};
        normal = mul(I, nl);
        extra = x.extra;
        return;
    }
#endif
    f3 to = tmul(x.R, ov), td = tmul(x.R, d);
    f3 h = to + td * bt, nl;
    if (x.type == 1) nl = normalize(f3{h.x * x.is2.x, h.y * x.is2.y, h.z * x.is2.z});
    else if (x.type == 2) nl = cuboid_normal(h, x.scale);
    else nl = f3{0, 0, 0};
    normal = mul(x.R, nl);
    extra = x.extra;
}

// SP: the sphere-record object test is compiled in (INW-01 kernels; INW-04's keep their registers)
template <bool WANT_NORMAL, bool LN = false, bool FU = false, bool PK = false, bool QN = false, class KS = FStack,
          bool SP = true>
__device__ float inw_traverse_wide(const InwScene &S, KS &K, f3 o, f3 d, float ratio, bool invert, float &tlim,
                                   f3 &normal, float &extra, float init_geom, Ctr &c, bool &ok,
                                   WalkPark *wp = nullptr) {
    static_assert(!QN || FU, "quantised nodes are culled with the fused planes");
    const f3 id = f3{rcp(d.x), rcp(d.y), rcp(d.z)};  // the reference's reciprocals (test_aabb)
    ok = S.wnodes != nullptr && K.size + S.dfs_high <= (uint32_t)kFStack && __builtin_isfinite(id.x) &&
         __builtin_isfinite(id.y) && __builtin_isfinite(id.z) && d.x != 0.0f && d.y != 0.0f && d.z != 0.0f;
    if (!__any(ok)) return init_geom;
    const float tlim0 = tlim;
    float bt = tlim0;
    int bg = -1;
    uint32_t br = 0xffffffffu;
    const uint32_t *rank = S.rank + (invert ? S.n : 0u);
    // the culling planes use the reference's (correctly rounded) reciprocals too: no second set of
    // three (round 5 took v_rcp approximations), C3 184.6 -> 184.0 ms (profiles/r06_ab_walk_tweaks.json)
    const f3 fid = id;
    const f3 noid = f3{-(o.x * fid.x), -(o.y * fid.y), -(o.z * fid.z)};  // the fused cull's per-ray term (FU)
    // the fused planes need a finite per-ray term: a direction component near the smallest normal
    // float with |o| ~ 10^3 overflows it, and every fma would be -inf or NaN (every child culled);
    // such a ray takes the reference walk
    if (FU) ok = ok && __builtin_isfinite(noid.x) && __builtin_isfinite(noid.y) && __builtin_isfinite(noid.z);
    // 3 spare slots for branch-free pushes; PK: the segment's ray (8 floats) stays below the walk
    int cap;
    float *const wsb = K.walk_stack(PK ? 8u : 0u, 3, cap);  // entry p at wsb[p * kBlock]
    const uint32_t ox = d.x < 0.0f ? 3u : 0u, oy = d.y < 0.0f ? 4u : 1u, oz = d.z < 0.0f ? 5u : 2u;
#ifndef RT_INW_NO_BUFLOAD
    const WnodeBuf wrs = wnode_buf(S, ox * 16u, oy * 16u, oz * 16u);
#endif
    int sp = 0, pend = -1, cur = S.wroot;
    if (!LN && S.wbins > 1u) {  // the ray's time-bin tree (the staged nodes are the swept tree's)
        const int b = min((int)(ratio * (float)S.wbins), (int)S.wbins - 1);
        cur = 1 + (int)S.wbin_base + b * (int)S.wbin_stride;
    }
    bool walking = ok, ovf = false;
    float lim = bt * 1.0001f + 1e-3f;
    // the leaf-entry guard: the best hit's leaf-box entry, and the smallest t of the
    // other hits; the reference's walk accepts the best hit for certain when t2 > bte
    float bte = 0.0f, t2 = tlim0;
    if constexpr (PK) {
        if (wp->resume) {  // a parked walk: its state from the slot (ok held when it parked)
            const float4 a = wp->slot[0], b = wp->slot[1];
            cur = __float_as_int(a.x); sp = __float_as_int(a.y); bg = __float_as_int(a.z); br = __float_as_uint(a.w);
            bt = b.x; lim = b.y; bte = b.z; t2 = b.w;
        }
        wp->parked = false;
    }
    int trips = 0;
    auto leaf = [&](int g) {
        c.prims++;
        const float4 n0 = S.leafbox[2 * g], n1 = S.leafbox[2 * g + 1];
        float te, t = -1.0f;
        if (SP && S.sph) {  // a sphere scene: 2 float4 instead of 7, no rotation (R = I: tmul(R, v) = v)
            const float4 p = S.sph[3 * g], q = S.sph[3 * g + 1];
            const bool inb = test_aabb_te(n0, n1, o, id, tlim0, te);
            const f3 to = (o - mk(p.x, p.y, p.z)) + mk(q.x, q.y, q.z) * (1.0f - ratio);
            keep_before_branch(to, d);
            if (!inb) return;
            t = t_ellipsoid(to, d, f3{p.w, p.w, p.w});
        } else {
            const Xf x = load_xf(S, g);  // loaded with the box, before its test: one memory latency
            const bool inb = test_aabb_te(n0, n1, o, id, tlim0, te);
            const f3 ov = (o - x.pos) + x.delta * (1.0f - ratio);
#ifndef RT_INW_NO_IDENT
            if (x.ident) {  // R = I: tmul(R, v) is v (up to zero signs, which t cannot see; d has no
                            // zero component here), and rcp(d) is the ray's own id
                keep_before_branch(ov, d);
                if (!inb) return;
                if (x.type == 1) t = t_ellipsoid(ov, d, x.is);
                else if (x.type == 2) t = t_cuboid_rcp(ov, id, x.scale);
            } else
#endif
            {
                f3 to = tmul(x.R, ov), td = tmul(x.R, d);
                keep_before_branch(to, td);
                if (!inb) return;
                if (x.type == 1) t = t_ellipsoid(to, td, x.is);
                else if (x.type == 2) t = t_cuboid(to, td, x.scale);
            }
        }
        if (t > 0.0f && t < tlim0) {
            const uint32_t r = rank[g];
#ifdef RT_INW_GUARD_ANY
            if (t < te) ovf = true;  // round-5 guard: any hit below its leaf-box entry
#endif
            if (t < bt || (t == bt && r < br)) {
                if (bg >= 0) t2 = fminf(t2, bt);
                bt = t; bg = g; br = r; bte = te; lim = bt * 1.0001f + 1e-3f;
            } else {
                t2 = fminf(t2, t);
            }
        }
    };
    for (;;) {
        OCC_TALLY(c, kOccWalk, walking);
        OCC_TALLY(c, kOccNode, walking && cur > 0);
#ifdef RT_DIAG_OCC
        {  // how often a node step's lanes share one node (a wave-uniform node load would serve them)
            const unsigned long long m = __ballot(walking && cur > 0);
            if (m) {
                const int c0 = __builtin_amdgcn_readlane(cur, (int)__builtin_ctzll(m));
                const bool on = walking && cur == c0;
                OCC_TALLY(c, kOccSame, on);
                if (__ballot(walking && cur > 0 && cur != c0) == 0ull) OCC_TALLY(c, kOccUni, on);
            }
        }
#endif
        if (walking) {
            bool pop;
            if (cur > 0) {
                float4 lk;
                float t0, t1, t2, t3;
                if constexpr (QN) {
                    float4 qa, qb, qc;
                    inw_qnode<LN>(S, cur, qa, qb, qc, lk);
                    cull4q(qa, qb, qc, ox != 0u, oy != 1u, oz != 2u, fid, noid, lim, t0, t1, t2, t3);
                } else {
                    float4 nx, ny, nz, fx, fy, fz;
#ifndef RT_INW_NO_BUFLOAD
#ifdef RT_INW_NODE_SLOAD
                    // every stepping lane at one node with one octant (30% of C3's node steps are at one
                    // node): the node's planes by scalar loads, off the TA path
                    const int c0 = __builtin_amdgcn_readfirstlane(cur);
                    const uint32_t oc = ox + 8u * oy + 64u * oz, oc0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)oc);
                    if (S.cnodes && (!LN || (uint32_t)(c0 - 1) >= S.n_lnodes) && __ballot(cur != c0 || oc != oc0) == 0ull) {
                        const float4 *nd = S.cnodes + 7 * (c0 - 1);
                        const int sx = (int)(oc0 & 7u), sy = (int)((oc0 >> 3) & 7u), sz = (int)(oc0 >> 6);  // 0|3, 1|4, 2|5
                        nx = sload4(nd, sx); fx = sload4(nd, 3 - sx);
                        ny = sload4(nd, sy); fy = sload4(nd, 5 - sy);
                        nz = sload4(nd, sz); fz = sload4(nd, 7 - sz);
                        lk = sload4(nd, 6);
                    } else
#endif
                    inw_wnode_nf_buf<LN>(S, wrs, cur, ox * 16u, oy * 16u, oz * 16u, nx, ny, nz, fx, fy, fz, lk);
#else
                    inw_wnode_nf<LN>(S, cur, ox, oy, oz, nx, ny, nz, fx, fy, fz, lk);
#endif
                    cull4nf<FU>(nx, ny, nz, fx, fy, fz, o, fid, noid, lim, t0, t1, t2, t3);
                }
                c.nodes += 4;
                int k0 = __float_as_int(lk.x), k1 = __float_as_int(lk.y), k2 = __float_as_int(lk.z),
                    k3 = __float_as_int(lk.w);
                cswap(t0, k0, t1, k1); cswap(t2, k2, t3, k3);
                cswap(t0, k0, t2, k2); cswap(t1, k1, t3, k3);
                cswap(t1, k1, t2, k2);
                int p = sp;  // branch-free pushes, farthest first (a miss is overwritten before a pop)
                wsb[p * kBlock] = __int_as_float(k3); p += t3 != kMiss;
                wsb[p * kBlock] = __int_as_float(k2); p += t2 != kMiss;
                wsb[p * kBlock] = __int_as_float(k1); p += t1 != kMiss;
                if (p > cap) { ovf = true; p = cap; }
                sp = p;
                cur = k0;
                pop = t0 == kMiss;
            } else {
                pop = pend < 0;  // a leaf waits while the lane still holds one
                if (pop) pend = -cur;
            }
            if (pop) {
                if (sp == 0) walking = false;
                else cur = __float_as_int(wsb[(--sp) * kBlock]);
            }
            if (ovf) walking = false;
        }
        // postponed leaves are tested once every walking lane holds one (RT_INW_LEAF_BATCH < 65: or
        // once that many lanes hold one, an experiment)
        if (__all(!walking || pend >= 0) ||
            (kInwLeafBatch < 65 && __popcll(__ballot(pend >= 0)) >= (unsigned)kInwLeafBatch)) {
            OCC_TALLY(c, kOccLeaf, pend >= 0);
            if (pend >= 0) { leaf(pend); pend = -1; }
            if (__all(!walking)) break;
        }
        if constexpr (PK) {
            if (++trips >= kParkMinTrips && __popcll(__ballot(walking)) <= kParkLanes) {
                if (__any(pend >= 0)) {  // every pending leaf is tested before the lanes part
                    OCC_TALLY(c, kOccLeaf, pend >= 0);
                    if (pend >= 0) { leaf(pend); pend = -1; }
                }
                if (ovf) walking = false;
                if (walking) {
                    wp->slot[0] = make_float4(__int_as_float(cur), __int_as_float(sp), __int_as_float(bg), __uint_as_float(br));
                    wp->slot[1] = make_float4(bt, lim, bte, t2);
                    wp->parked = true;
                }
                break;
            }
        }
    }
    if (PK && wp->parked) return init_geom;
    // the best hit passes the reference's leaf-box test for certain unless another hit's t could
    // have lowered its running limit to the box entry first (rare: a face on its box, C5)
    if (bg >= 0 && !(t2 > bte)) ovf = true;
    if (ovf) ok = false;
    if (!ok) return init_geom;
    if (bg < 0) return init_geom;
    tlim = bt;
    if (WANT_NORMAL) inw_hit_normal<SP>(S, bg, o, d, ratio, bt, normal, extra);
    return (float)bg;
}

// load_xf by scalar loads (sload4): the beam lists' candidates are the same object for every active
// lane of one pixel (they step through the list together)
__device__ __forceinline__ Xf load_xf_s(const InwScene &S, int g) {  // load_xf of a wave-uniform g
    const float4 a = sload4(S.hot, 7 * g), b = sload4(S.hot, 7 * g + 1), c = sload4(S.hot, 7 * g + 2),
                 d = sload4(S.hot, 7 * g + 3), e = sload4(S.hot, 7 * g + 4), f = sload4(S.hot, 7 * g + 5),
                 q = sload4(S.hot, 7 * g + 6);
    Xf x;
    x.pos = mk(a.x, a.y, a.z);
    x.R.c0 = mk(a.w, b.x, b.y); x.R.c1 = mk(b.z, b.w, c.x); x.R.c2 = mk(c.y, c.z, c.w);
    x.scale = mk(d.x, d.y, d.z);
    x.delta = mk(d.w, e.x, e.y);
    x.type = (int)(e.z + 0.1f);
    x.ident = e.z - (float)x.type > 0.25f;
    x.extra = e.w;
    x.is = mk(f.x, f.y, f.z);
    x.is2 = mk(f.w, q.x, q.y);
    x.ri_acc = q.z;
    return x;
}

// Closest hit of a primary ray from its pixel's beam list (DESIGN.md §5 "Pixel beams").  The list
// holds every object whose culling box the beam of the pixel's primary rays can cross, in the
// order of the central ray's entry t into the box inflated by beam_R; a sample ray hitting object
// j at t has entry(j) <= t * beam_kappa, so the candidates past bt * kappa (+ slack) cannot win.
// Each candidate gets the wide walk's leaf test (the reference's leaf box with the initial limit,
// the exact test, the leaf-entry guard, the (t, depth-first rank) rule), so the winner is the
// wide walk's and the reference walk's.  ok = false: the list does not decide this ray (no list,
// the wide walk's conditions fail, or candidates beyond the stored ones could still win).
template <bool WANT_NORMAL, class KS = FStack>
__device__ float inw_closest_beam(const InwScene &S, const KS &K, f3 o, f3 d, float ratio, bool invert, float &tlim,
                                  f3 &normal, float &extra, float init_geom, Ctr &c, uint32_t unit, bool &ok) {
    const f3 id = f3{rcp(d.x), rcp(d.y), rcp(d.z)};  // the reference's reciprocals (test_aabb)
    // the ray's time bin's list (beam_bins > 1): bin b's counts, cuts and lists after those of bins < b
    const uint32_t bo = S.beam_bins > 1u ? min((uint32_t)(ratio * (float)S.beam_bins), S.beam_bins - 1u) * S.beam_units : 0u;
    const uint32_t nw = S.beam_n[bo + unit], n = nw & 0xffu;  // k_inw_beam: offset in the block's region << 8 | count
    ok = nw != kBeamOff && K.size + S.dfs_high <= (uint32_t)kFStack && __builtin_isfinite(id.x) &&
         __builtin_isfinite(id.y) && __builtin_isfinite(id.z) && d.x != 0.0f && d.y != 0.0f && d.z != 0.0f;
    const float tlim0 = tlim;
    float bt = tlim0;
    int bg = -1;
    uint32_t br = 0xffffffffu;
    const uint32_t *rank = S.rank + (invert ? S.n : 0u);
    const size_t lbase = ((size_t)bo + (unit & ~63u)) * S.beam_cap + (nw >> 8);
    const uint2 *list = S.beam + lbase;
    const uint32_t *list16 = reinterpret_cast<const uint32_t *>(S.beam) + lbase;
    const float kap = S.beam_kappa;
    float lim = bt * kap + 0.01f;
    bool ovf = false;
    float bte = 0.0f, t2 = tlim0;  // the leaf-entry guard's state (inw_traverse_wide)
    uint32_t k = 0;
    // packed entries hold t rounded down (and 0 for a negative entry): the list stays sorted, and a
    // ray stops at a stored t above lim no earlier than at the exact one
    auto entry = [&](uint32_t j) {
        if (S.beam16) {
            const uint32_t p = list16[j];
            return make_uint2(p & 0xffffu, p & 0xffff0000u);
        }
        return list[j];
    };
    uint2 en = ok && n > 0u ? entry(0) : make_uint2(0u, 0u);  // the next entry, loaded a candidate ahead
    for (;;) {
        bool act = ok && k < n;
        uint2 e = make_uint2(0u, 0u);
        if (act) {
            e = en;
            act = __uint_as_float(e.y) <= lim;
        }
        if (!__any(act)) break;
        OCC_TALLY(c, kOccBeam, act);
        if (act) {
            if (k + 1u < n) en = entry(k + 1u);
            const int g = (int)e.x;
            c.prims++;
            float4 n0, n1;
            float te, t = -1.0f;
            bool inb;
#ifndef RT_INW_BEAM_VLOAD
            // one candidate for every active lane (a wave's lanes trace samples of one pixel and step
            // through its list together): scalar loads, C3 184.7 -> 182.5 ms
            // (profiles/r06_ab_beam_sload_ring_il.json; -DRT_INW_BEAM_VLOAD: vector loads only)
            const int g0 = __builtin_amdgcn_readfirstlane(g);
            const bool uni_g = __ballot(g != g0) == 0ull;
#else
            const int g0 = g;
            const bool uni_g = false;
#endif
            if (S.sph) {  // a sphere scene (inw_traverse_wide's leaf test): 2 float4, R = I
                float4 p, q;
                if (uni_g) {
                    n0 = sload4(S.leafbox, 2 * g0); n1 = sload4(S.leafbox, 2 * g0 + 1);
                    p = sload4(S.sph, 3 * g0); q = sload4(S.sph, 3 * g0 + 1);
                } else {
                    n0 = S.leafbox[2 * g]; n1 = S.leafbox[2 * g + 1];
                    p = S.sph[3 * g]; q = S.sph[3 * g + 1];
                }
                inb = test_aabb_te(n0, n1, o, id, tlim0, te);
                const f3 to = (o - mk(p.x, p.y, p.z)) + mk(q.x, q.y, q.z) * (1.0f - ratio);
                keep_before_branch(to, d);
                if (inb) t = t_ellipsoid(to, d, f3{p.w, p.w, p.w});
            } else {
                Xf x;
                if (uni_g) {
                    n0 = sload4(S.leafbox, 2 * g0); n1 = sload4(S.leafbox, 2 * g0 + 1);
                    x = load_xf_s(S, g0);
                } else {
                    n0 = S.leafbox[2 * g]; n1 = S.leafbox[2 * g + 1];
                    x = load_xf(S, g);
                }
                inb = test_aabb_te(n0, n1, o, id, tlim0, te);
                f3 ov = (o - x.pos) + x.delta * (1.0f - ratio);
                f3 to = tmul(x.R, ov), td = tmul(x.R, d);
                keep_before_branch(to, td);
                if (inb) {
                    if (x.type == 1) t = t_ellipsoid(to, td, x.is);
                    else if (x.type == 2) t = t_cuboid(to, td, x.scale);
                }
            }
            if (inb) {
                if (t > 0.0f && t < tlim0) {
                    const uint32_t r = rank[g];
#ifdef RT_INW_GUARD_ANY
                    if (t < te) ovf = true;
#endif
                    if (t < bt || (t == bt && r < br)) {  // the leaf-entry guard as in inw_traverse_wide
                        if (bg >= 0) t2 = fminf(t2, bt);
                        bt = t; bg = g; br = r; bte = te; lim = bt * kap * 1.00001f + 0.01f;
                    } else {
                        t2 = fminf(t2, t);
                    }
                }
            }
            k++;
        }
    }
    if (bg >= 0 && !(t2 > bte)) ovf = true;
    // candidates not stored (entry >= cut) could still be reached below lim
    if (ok && (ovf || !(lim < S.beam_cut[bo + unit]))) ok = false;
    if (!ok) return init_geom;
    if (bg < 0) return init_geom;
    tlim = bt;
    if (WANT_NORMAL) inw_hit_normal<true>(S, bg, o, d, ratio, bt, normal, extra);
    return (float)bg;
}

// The surrounding-RI walk (01_BVH...glsl:486-502) sums the RI of every object holding the point,
// in its depth-first order (right child first).  Same conditions as above: the objects are those
// whose leaf box holds the point (inclusive, as the reference compares) and whose inside test
// passes, found by a walk of the culling BVH and summed in rank order.  ok = false: fall back.
constexpr int kRiMax = 8;
template <bool LN = false, class KS = FStack>
__device__ float inw_surrounding_ri_wide(const InwScene &S, KS &K, f3 hp, float ratio, Ctr &c, bool &ok) {
    ok = S.wnodes != nullptr && K.size + S.dfs_high <= (uint32_t)kFStack;
    if (!__any(ok)) return 1.0f;
    int cap;
    float *const wsb = K.walk_stack(0u, 4, cap);  // entry p at wsb[p * kBlock]
    uint32_t rk[kRiMax];
    float rv[kRiMax];
    int nin = 0;
    int sp = 0, cur = S.wroot;
    bool walking = ok;
    while (walking) {
        if (cur > 0) {
            float4 lx, ly, lz, hx, hy, hz, lk;
            inw_wnode<LN>(S, cur, lx, ly, lz, hx, hy, hz, lk);
            c.nodes += 4;
            const bool i0 = hp.x >= lx.x && hp.x <= hx.x && hp.y >= ly.x && hp.y <= hy.x && hp.z >= lz.x && hp.z <= hz.x;
            const bool i1 = hp.x >= lx.y && hp.x <= hx.y && hp.y >= ly.y && hp.y <= hy.y && hp.z >= lz.y && hp.z <= hz.y;
            const bool i2 = hp.x >= lx.z && hp.x <= hx.z && hp.y >= ly.z && hp.y <= hy.z && hp.z >= lz.z && hp.z <= hz.z;
            const bool i3 = hp.x >= lx.w && hp.x <= hx.w && hp.y >= ly.w && hp.y <= hy.w && hp.z >= lz.w && hp.z <= hz.w;
            int p = sp;
            wsb[p * kBlock] = lk.x; p += i0;
            wsb[p * kBlock] = lk.y; p += i1;
            wsb[p * kBlock] = lk.z; p += i2;
            wsb[p * kBlock] = lk.w; p += i3;
            if (p > cap) { ok = false; break; }
            sp = p;
        } else {
            const int g = -cur;
            c.prims++;
            const float4 n0 = S.leafbox[2 * g], n1 = S.leafbox[2 * g + 1];
            const Xf x = load_xf(S, g);  // loaded with the box, before its test
            if (hp.x <= n0.w && hp.y <= n1.x && hp.z <= n1.y && hp.x >= n0.x && hp.y >= n0.y && hp.z >= n0.z) {
                f3 v = (hp - x.pos) + x.delta * (1.0f - ratio);
                v = tmul(x.R, v);
                v.x *= x.is.x; v.y *= x.is.y; v.z *= x.is.z;
                bool inside;
                if (x.type == 1) inside = dot(v, v) <= 1.0f;
                else if (x.type == 2) inside = fabsf(v.x) <= 0.5f && fabsf(v.y) <= 0.5f && fabsf(v.z) <= 0.5f;
                else inside = false;
                if (inside) {
                    if (nin == kRiMax) { ok = false; break; }
                    rk[nin] = S.rank[g];
                    rv[nin] = x.ri_acc;
                    nin++;
                }
            }
        }
        if (sp == 0) walking = false;
        else cur = __float_as_int(wsb[(--sp) * kBlock]);
    }
    if (!ok) return 1.0f;
    // sum in the reference's order (insertion sort by rank; a handful of objects at most)
    for (int i = 1; i < nin; i++)
        for (int j = i; j > 0 && rk[j] < rk[j - 1]; j--) {
            const uint32_t tr = rk[j]; rk[j] = rk[j - 1]; rk[j - 1] = tr;
            const float tv = rv[j]; rv[j] = rv[j - 1]; rv[j - 1] = tv;
        }
    float acc = 0.0f;
    for (int i = 0; i < nin; i++) acc += rv[i];
    if (acc > 1.0f) acc *= rcp((float)nin);
    else acc = 1.0f;
    return acc;
}

// The surrounding-RI walk (inw_surrounding_ri_wide) through the RI grid: the objects whose
// leaf box holds the point are all listed in the point's cell (their boxes were entered with a
// margin wider than the rounding of the cell index), so testing that cell's objects with the
// walk's comparisons finds the same objects; they are summed in depth-first rank order.
__device__ float inw_ri_grid(const InwScene &S, f3 hp, float ratio, Ctr &c, bool &ok) {
    ok = true;
    if (!(hp.x >= S.ri_lo[0] && hp.y >= S.ri_lo[1] && hp.z >= S.ri_lo[2] && hp.x <= S.ri_hi[0] &&
          hp.y <= S.ri_hi[1] && hp.z <= S.ri_hi[2]))
        return 1.0f;  // outside every leaf box (or NaN: no comparison holds, as in the walk)
    const int cx = min(max((int)((hp.x - S.ri_lo[0]) * S.ri_inv[0]), 0), S.ri_dim[0] - 1);
    const int cy = min(max((int)((hp.y - S.ri_lo[1]) * S.ri_inv[1]), 0), S.ri_dim[1] - 1);
    const int cz = min(max((int)((hp.z - S.ri_lo[2]) * S.ri_inv[2]), 0), S.ri_dim[2] - 1);
    const uint32_t cell = ((uint32_t)cz * (uint32_t)S.ri_dim[1] + (uint32_t)cy) * (uint32_t)S.ri_dim[0] + (uint32_t)cx;
    const uint32_t b = S.ri_cells[cell], e = S.ri_cells[cell + 1];
    uint32_t rk[kRiMax];
    float rv[kRiMax];
    int nin = 0;
    // an object's leaf box, record and rank are loaded together (one round trip; the hit object
    // itself is always listed and inside its box), the next id while this one is tested
    uint32_t gn = b < e ? S.ri_ids[b] : 0u;
    for (uint32_t k = b; k < e; k++) {
        const int g = (int)gn;
        if (k + 1 < e) gn = S.ri_ids[k + 1];
        c.prims++;
        const float4 n0 = S.leafbox[2 * g], n1 = S.leafbox[2 * g + 1];
        const uint32_t rg = S.rank[g];
        bool inside;
        float ri;
        if (S.sph) {  // sphere records (RI in q.w): R = I, so v = ov * is, the same floats
            const float4 p = S.sph[3 * g], q = S.sph[3 * g + 1];
            if (!(hp.x <= n0.w && hp.y <= n1.x && hp.z <= n1.y && hp.x >= n0.x && hp.y >= n0.y && hp.z >= n0.z)) continue;
            f3 v = (hp - mk(p.x, p.y, p.z)) + mk(q.x, q.y, q.z) * (1.0f - ratio);
            v.x *= p.w; v.y *= p.w; v.z *= p.w;
            inside = dot(v, v) <= 1.0f;
            ri = q.w;
        } else {
            const Xf x = load_xf(S, g);
            if (!(hp.x <= n0.w && hp.y <= n1.x && hp.z <= n1.y && hp.x >= n0.x && hp.y >= n0.y && hp.z >= n0.z)) continue;
            f3 v = (hp - x.pos) + x.delta * (1.0f - ratio);
            v = tmul(x.R, v);
            v.x *= x.is.x; v.y *= x.is.y; v.z *= x.is.z;
            if (x.type == 1) inside = dot(v, v) <= 1.0f;
            else if (x.type == 2) inside = fabsf(v.x) <= 0.5f && fabsf(v.y) <= 0.5f && fabsf(v.z) <= 0.5f;
            else inside = false;
            ri = x.ri_acc;
        }
        if (inside) {
            if (nin == kRiMax) { ok = false; return 1.0f; }
            rk[nin] = rg;
            rv[nin] = ri;
            nin++;
        }
    }
    for (int i = 1; i < nin; i++)
        for (int j = i; j > 0 && rk[j] < rk[j - 1]; j--) {
            const uint32_t tr = rk[j]; rk[j] = rk[j - 1]; rk[j - 1] = tr;
            const float tv = rv[j]; rv[j] = rv[j - 1]; rv[j - 1] = tv;
        }
    float acc = 0.0f;
    for (int i = 0; i < nin; i++) acc += rv[i];
    if (acc > 1.0f) acc *= rcp((float)nin);
    else acc = 1.0f;
    return acc;
}

// ---------------------------------------------------------------- stackless LBVH walks
// The reference walks its LBVH depth first with the shared 40-float stack (01_BVH...glsl:431-476;
// RI: 486-502, 272-345).  Its node buffer is written breadth first with the two children of a node
// next to each other and rightData = the parent (lbvh.h:236-269), so the left children sit at odd
// indices and their right siblings at the next one; the host checks that layout (InwScene::sl).
// The same depth-first order then needs no stack: the closest-hit walk pops (invert ? left :
// right) first (it pushes the other one first, :456-460), so after the first child's subtree
// comes its sibling, and after the second child's subtree the walk climbs to the parent and on.
// Every node the reference pops is visited once, in the same order, with the same running limit:
// the same box tests, leaves, hit, node and primitive counts.  Where a reference push could drop
// (size + dfs_high > 40) the result depends on the stack, and the caller runs the stack walk.
// Climbing past a second child reads one float, the parent's own parent link.
template <bool LN>
__device__ __forceinline__ void lbvh_node(const InwScene &S, uint32_t i, float4 &n0, float4 &n1) {
    if (LN && i < S.n_blds) {  // LDS-staged top of the LBVH (ds_read_b128)
        n0 = g_inw_lnodes[2 * i];
        n1 = g_inw_lnodes[2 * i + 1];
        return;
    }
    n0 = S.nodes[2 * i];
    n1 = S.nodes[2 * i + 1];
}
template <bool LN>
__device__ __forceinline__ float lbvh_parent(const InwScene &S, uint32_t i) {
    if (LN && i < S.n_blds) return g_inw_lnodes[2 * i + 1].w;
    return reinterpret_cast<const float *>(S.nodes)[8 * (size_t)i + 7];
}
// The node after the subtree of `cur` in depth-first order (0 = the walk is over).  first_odd:
// the first-visited child of a node has an odd index (invert) or an even one.  par: cur's parent.
template <bool LN>
__device__ __forceinline__ uint32_t lbvh_next(const InwScene &S, uint32_t cur, float par, uint32_t first_odd) {
    for (;;) {
        if (cur == 0u) return 0u;
        if ((cur & 1u) == first_odd) return first_odd ? cur + 1u : cur - 1u;  // its sibling comes next
        cur = (uint32_t)par;  // a second child: its parent's subtree is done
        if (cur == 0u) return 0u;
        par = lbvh_parent<LN>(S, cur);
    }
}

template <bool WANT_NORMAL, bool LN = false, bool EO = true>
__device__ float inw_traverse_sl(const InwScene &S, f3 o, f3 d, float ratio, bool invert, float &tlim, f3 &normal,
                                 float &extra, float init_geom, Ctr &c) {
    float final_geom = init_geom;
    const f3 id = f3{rcp(d.x), rcp(d.y), rcp(d.z)};
    const uint32_t first_odd = invert ? 1u : 0u;
    uint32_t cur = 0u;
    for (;;) {
        float4 n0, n1;
        lbvh_node<LN>(S, cur, n0, n1);
        c.nodes++;
        if (test_aabb<EO>(n0, n1, o, id, tlim)) {
            const float left = n1.z;
            if (left > 0.1f) {  // descend: the child the reference pops first
                const uint32_t L = (uint32_t)left;
                cur = invert ? L : L + 1u;
                continue;
            }
            c.prims++;  // IntersectRay / IntersectRayMinimal (as inw_traverse)
            const float geom = -left;
            const Xf x = load_xf(S, (int)geom);
            f3 ov = (o - x.pos) + x.delta * (1.0f - ratio);
            f3 to = tmul(x.R, ov), td = tmul(x.R, d);
            float t = -1.0f;
            if (x.type == 1) t = t_ellipsoid(to, td, x.is);
            else if (x.type == 2) t = t_cuboid(to, td, x.scale);
            if (t > 0.0f && t < tlim) {
                tlim = t;
                final_geom = geom;
                if (WANT_NORMAL) {
                    f3 h = to + td * t, nl;
                    if (x.type == 1) nl = normalize(f3{h.x * x.is2.x, h.y * x.is2.y, h.z * x.is2.z});
                    else if (x.type == 2) nl = cuboid_normal(h, x.scale);
                    else nl = f3{0, 0, 0};
                    normal = mul(x.R, nl);
                    extra = x.extra;
                }
            }
        }
        cur = lbvh_next<LN>(S, cur, n1.w, first_odd);
        if (cur == 0u) break;
    }
    return final_geom;
}

// the surrounding-RI point walk (01_BVH...glsl:486-502): pushes left, then left + 1, so it pops
// the right (even) child first
template <bool LN = false>
__device__ float inw_surrounding_ri_sl(const InwScene &S, f3 hp, float ratio, Ctr &c) {
    float acc = 0.0f;
    uint32_t cnt = 0, cur = 0u;
    for (;;) {
        float4 n0, n1;
        lbvh_node<LN>(S, cur, n0, n1);
        c.nodes++;
        if (hp.x <= n0.w && hp.y <= n1.x && hp.z <= n1.y && hp.x >= n0.x && hp.y >= n0.y && hp.z >= n0.z) {
            const float left = n1.z;
            if (!(left < 0.1f)) {
                cur = (uint32_t)left + 1u;
                continue;
            }
            c.prims++;
            const Xf x = load_xf(S, (int)(-left));
            f3 v = (hp - x.pos) + x.delta * (1.0f - ratio);
            v = tmul(x.R, v);
            v.x *= x.is.x; v.y *= x.is.y; v.z *= x.is.z;
            bool inside;
            if (x.type == 1) inside = dot(v, v) <= 1.0f;
            else if (x.type == 2) inside = fabsf(v.x) <= 0.5f && fabsf(v.y) <= 0.5f && fabsf(v.z) <= 0.5f;
            else inside = false;
            if (inside) { acc += x.ri_acc; cnt++; }
        }
        cur = lbvh_next<LN>(S, cur, n1.w, 0u);
        if (cur == 0u) break;
    }
    if (acc > 1.0f) acc *= rcp((float)cnt);
    else acc = 1.0f;
    return acc;
}

// EO: the reference walks' box test with the shader's early outs (INW-01) or all axes (INW-04)
// QN: the wide walk reads the quantised nodes (LN: the staged ones); the LBVH walks then read no
// staged node (their LDS is not filled in the GQ instance)
template <bool WANT_NORMAL, bool LN = false, bool FU = false, bool PK = false, bool EO = true, bool QN = false,
          class KS = FStack>
__device__ __forceinline__ float inw_closest(const InwScene &S, KS &K, f3 o, f3 d, float ratio, bool invert,
                                             float &tlim, f3 &normal, float &extra, float init_geom, Ctr &c,
                                             WalkPark *wp = nullptr) {
    bool ok = false;
    const float g = inw_traverse_wide<WANT_NORMAL, LN, FU, PK, QN, KS, EO>(S, K, o, d, ratio, invert, tlim, normal, extra,
                                                                   init_geom, c, ok, wp);
    if (PK && wp->parked) return g;
    OCC_TALLY(c, kOccRef, !ok);
    if (ok) return g;
    c.refw++;
    if (S.sl && K.size + S.dfs_high <= (uint32_t)kFStack)  // no push of the reference walk could drop
        return inw_traverse_sl<WANT_NORMAL, LN && !QN, EO>(S, o, d, ratio, invert, tlim, normal, extra, init_geom, c);
    return inw_traverse<WANT_NORMAL, EO>(S, K, o, d, ratio, invert, tlim, normal, extra, init_geom, c);
}
template <bool LN = false, class KS = FStack>
__device__ __forceinline__ float inw_ri(const InwScene &S, KS &K, f3 hp, float ratio, Ctr &c) {
    bool ok = false;
    if (S.ri_cells && K.size + S.dfs_high <= (uint32_t)kFStack) {  // no push of the walk could drop
        const float g = inw_ri_grid(S, hp, ratio, c, ok);
        if (ok) return g;
    }
    const float r = inw_surrounding_ri_wide<LN>(S, K, hp, ratio, c, ok);
    if (ok) return r;
    if (S.sl && K.size + S.dfs_high <= (uint32_t)kFStack) return inw_surrounding_ri_sl<LN>(S, hp, ratio, c);
    return inw_surrounding_ri(S, K, hp, ratio, c);
}

__device__ __forceinline__ bool is_lit_geom(const InwScene &S, uint32_t in) {  // 04...glsl:468-474
    bool r = false;
    for (uint32_t i = 0; i < S.n_lights && !r; i++) r = in == __float_as_uint(S.lights[i * 7 + 6]);
    return r;
}
__device__ __forceinline__ uint32_t f2u(float f) { return f <= 0.0f ? 0u : (uint32_t)f; }

// deviateWithLinmit90deg 01_BVH...glsl:28-46, power = 1
__device__ __forceinline__ f3 deviate(const InwScene &S, f3 dir, float tan_theta, int s) {
    float ap = (2.0f * tan_theta) * 0.5f;
    float nx = S.sunflower[2 * s] * ap, ny = S.sunflower[2 * s + 1] * ap;
    f3 right = cross(dir, f3{0, 1, 0});
    f3 up = cross(right, dir);
    return normalize(dir + (right * nx + up * ny) * 0.1f);
}

// Camera ray of sample s (out_Pixel prologue, 01_BVH...glsl:366-410): push it, reset the sample.
// the pixel's camera direction (01_BVH...glsl:366-386)
__device__ __forceinline__ f3 inw_pixel_dir(const Frame &F, int px, int py) {
    const f3 D = mk(F.dir[0], F.dir[1], F.dir[2]);
    float aspect = (float)F.W * rcp((float)F.H);
    float srx = (float)px * rcp((float)F.W) - 0.5f;
    float sry = (float)py * rcp((float)F.H) - 0.5f;
    srx *= aspect;
    const f3 up = f3{0, 1, 0};
    f3 cr = cross(D, up), cu = cross(cr, D);
    return normalize((D * F.screen_dist + cr * srx) + cu * sry);
}
// cd: the pixel's direction (inw_pixel_dir), which callers that keep it per pixel pass in
template <class KS>
__device__ __forceinline__ void inw_start_sample_cd(const InwScene &S, const Frame &F, KS &K, f3 cd, int s, Ctr &c) {
    K.reset(0);
    const f3 up = f3{0, 1, 0};
    f3 co = mk(F.pos[0], F.pos[1], F.pos[2]);
    float ox = S.sunflower[2 * s] * (F.aperture * 0.5f), oy = S.sunflower[2 * s + 1] * (F.aperture * 0.5f);
    f3 rr = cross(cd, up), ru = cross(rr, cd);
    if (F.n_focus > 0) {  // MULTIFOCUS lens record (01_BVH...glsl:388-400): stack floats 0..5
        const float first_limit = F.focus_list[0] * 0.5f;
        const f3 nd = normalize((cd * first_limit + rr * ox) + ru * oy);
        const f3 rn = normalize((-rr) * ox - ru * oy);
        const float mult = rcp(dot(cd, nd));
        K.push(rn.x, c); K.push(rn.y, c); K.push(rn.z, c);
        K.push(mult, c); K.push(first_limit, c); K.push(0.0f, c);
        K.push_ray(co, nd, 1.0f, 0.0f, c);
        return;
    }
    f3 tip = ((co + cd) + rr * ox) + ru * oy;
    f3 la = normalize((co + cd * F.focus) - tip);
    K.push_ray(tip - la, la, 1.0f, 0.0f, c);
}
template <class KS>
__device__ __forceinline__ void inw_start_sample(const InwScene &S, const Frame &F, KS &K, int px, int py, int s,
                                                 Ctr &c) {
    inw_start_sample_cd(S, F, K, inw_pixel_dir(F, px, py), s, c);
}

// texture(u_MaterialTextures[k], st) in a compute shader: lambda = 0, so the magnification
// filter GL_NEAREST applies (utility.cpp:182), with GL_REPEAT (utility.cpp:191-192)
__device__ __forceinline__ int tex_wrap(float u, int size) {
    const float f = __builtin_floorf(u);
    if (!(f == f) || f > 2147483520.0f || f < -2147483520.0f) return 0;  // NaN / inf: texel 0
    const int i = (int)f % size;
    return i < 0 ? i + size : i;
}
// FillHitMaterialData 04...glsl:416-464 (TextureIndex > 0): cube projection of the
// object-space hit position onto a 6-face strip, nearest texel
__device__ f3 inw_tex_color(const InwScene &S, uint32_t k, f3 lp) {
    lp = normalize(lp);
    float mx = lp.x;
    uint32_t face = mx > 0 ? 1u : 3u;
    f3 fd = f3{1, 0, 0} * (mx > 0 ? 1.0f : -1.0f);
    if (__builtin_fabsf(mx) < __builtin_fabsf(lp.y)) {
        mx = lp.y;
        face = mx > 0 ? 0u : 5u;
        fd = f3{0, 1, 0} * (mx > 0 ? 1.0f : -1.0f);
    }
    if (__builtin_fabsf(mx) < __builtin_fabsf(lp.z)) {
        mx = lp.z;
        face = mx > 0 ? 2u : 4u;
        fd = f3{0, 0, 1} * (mx > 0 ? 1.0f : -1.0f);
    }
    lp = lp * rcp(dot(lp, fd));
    lp = lp * 0.5f;
    lp = lp + f3{0.5f, 0.5f, 0.5f};
    float u, v;
    switch (face) {
        case 0: u = lp.x; v = 1.0f - lp.z; break;
        case 1: u = 1.0f - lp.y; v = 1.0f - lp.z; break;
        case 2: u = lp.x; v = lp.y; break;
        case 3: u = lp.z; v = lp.y; break;
        case 4: u = 1.0f - lp.y; v = 1.0f - lp.x; break;
        default: u = lp.z; v = 1.0f - lp.x; break;
    }
    const int4 ti = S.tex_info[k];
    const int i = tex_wrap(((float)face * 0.16666f + u * 0.16666f) * (float)ti.y, ti.y);
    const int j = tex_wrap(v * (float)ti.z, ti.z);
    const float4 c = S.tex[(size_t)ti.x + (size_t)j * (size_t)ti.y + (size_t)i];
    return f3{c.x, c.y, c.z};
}

// One iteration of out_Pixel's ray loop (01_BVH...glsl:414-597 / 04...glsl:510-713):
// pop a ray, closest hit, surrounding RI, shadow rays, push reflect/refract, accumulate.
// bunit: the lane's pixel unit when its primary ray may use the pixel's beam list (k_inw_pm), else kBeamOff
// PK (walk parking, above): wp->resume continues a parked walk of this segment (its ray still
// sits above K.size); wp->parked on return: the walk parked again and the segment is not done.
// QN (k_inw_pm's GQ instance): the wide closest-hit walks read the quantised nodes (inw_closest)
template <bool LIGHTS, bool LN = false, bool FU = false, bool PK = false, bool QN = false, class KS = FStack>
__device__ void inw_segment(const InwScene &S, const Frame &F, KS &K, int s, f3 &color, float &depth, Ctr &c,
                            uint32_t bunit = kBeamOff, WalkPark *wp = nullptr) {
    static_assert(!PK || !QN, "walk parking keeps the segment's ray in the stack (FStack only)");
    constexpr bool RLN = LN && !QN;  // the LBVH / RI walks' staged nodes (none in the GQ instance)
    const f3 D = mk(F.dir[0], F.dir[1], F.dir[2]);
    const float ratio = (float)s * F.inv_spp;
    const bool invert = dot(D, f3{1, 1, 1}) > 0.0f;
    INW_T0(t_fn);
#ifdef RT_DIAG_SPLIT
    unsigned long long t_tail = 0;  // the scatter and pushes after the RI (phase 7)
#endif
    do {
        const bool resumed = PK && wp->resume;
        f3 co, cd;
        float contribution, bounced;
        if (!resumed) K.pop_ray(co, cd, contribution, bounced);
        else {  // a parked walk: its ray still sits above K.size
            const uint32_t b = K.size;
            co = mk(K.at(b), K.at(b + 1), K.at(b + 2));
            cd = mk(K.at(b + 3), K.at(b + 4), K.at(b + 5));
            contribution = K.at(b + 6);
            bounced = K.at(b + 7);
        }
        bounced = (float)(int)bounced;
        if (!resumed) c.seg++;
        // SET LIMIT (01_BVH...glsl:424-428): a MULTIFOCUS primary ray stops at the lens
        const bool mf0 = !LIGHTS && F.n_focus > 0 && (int)(bounced + 0.1f) == 0;
        const float tlim0 = mf0 ? K.at(4) : kMaxT;
        float tlim = tlim0, extra = 0.0f;
        f3 normal = f3{0, 0, 0};
        INW_CYC(c, 5, t_fn);  // the pop and the segment's prologue
        INW_T0(t_ch);
        float fg;
        bool beam_ok = false;
        if (!resumed && bunit != kBeamOff && (int)(bounced + 0.1f) == 0 && !mf0)  // a primary ray (pushed rays have bounced >= 1)
            fg = inw_closest_beam<true>(S, K, co, cd, ratio, invert, tlim, normal, extra, LIGHTS ? -1.0f : 0.0f, c, bunit,
                                        beam_ok);
        if (!beam_ok) {
            fg = inw_closest<true, LN, FU, PK, !LIGHTS, QN>(S, K, co, cd, ratio, invert, tlim, normal, extra,
                                                            LIGHTS ? -1.0f : 0.0f, c, wp);
            if (PK && wp->parked) return;  // the walk goes on in the next iteration
        }
        INW_CYC(c, 0, t_ch);
        INW_T0(t_mat);
        const f3 hitpoint = co + cd * tlim;
        if (!(tlim < tlim0)) {
            if (mf0 && (int)(K.at(5) + 0.1f) < F.n_focus) {  // next focal lens, 01_BVH...glsl:506-528
                const f3 rn = mk(K.at(0), K.at(1), K.at(2));
                K.at(0) = -K.at(0); K.at(1) = -K.at(1); K.at(2) = -K.at(2);
                const float mult = K.at(3), dist = K.at(4);
                const f3 no = co + cd * (mult * dist), nd = reflect(cd, rn);
                const int lens = (int)(K.at(5) + 0.1f);
                if (lens < F.n_focus - 1)
                    K.at(4) = (F.focus_list[lens + 1] - F.focus_list[lens]) * 0.5f +
                              (F.focus_list[lens] - (lens > 0 ? F.focus_list[lens - 1 > 0 ? lens - 1 : 0] : 0.0f)) *
                                  0.5f;
                else K.at(4) = kMaxT - mult * K.at(4);
                K.at(5) = K.at(5) + 1.0f;
                K.reset(6);
                K.push_ray(no, nd, 1.0f, 0.0f, c);
                break;
            }
            color = color + background(cd, LIGHTS && S.n_lights > 0) * contribution;
            depth = tlim;
            if (mf0) K.reset(0);  // 01_BVH...glsl:531-535
            break;
        }
        const float4 m0 = S.cold[2 * (int)fg], m1 = S.cold[2 * (int)fg + 1];
        const float m_refr = m0.x, m_refl = m0.y, m_srfr = m0.z, m_srfl = m0.w;
        f3 m_color = mk(m1.x, m1.y, m1.z);
        const float m_ri = LIGHTS ? extra : m1.w;
        if (LIGHTS && S.n_tex) {  // layout 4 keeps the TextureIndex (uint bits) in m1.w
            const uint32_t ti = __float_as_uint(m1.w);
            if (ti - 1u < S.n_tex) {  // 04...glsl:416; local position :569 (no motion offset)
                const float4 h0 = S.hot[7 * (int)fg], h1 = S.hot[7 * (int)fg + 1], h2 = S.hot[7 * (int)fg + 2];
                const m3 R{mk(h0.w, h1.x, h1.y), mk(h1.z, h1.w, h2.x), mk(h2.y, h2.z, h2.w)};
                m_color = mulv(m_color, inw_tex_color(S, ti - 1u, tmul(R, hitpoint - mk(h0.x, h0.y, h0.z))));
            }
        }
        // The surrounding RI (01_BVH...glsl:486-502) is read only by the refract calls below: on an
        // outer hit of a refractive object, or on an inner hit.  Where the scatter branch will not
        // run or reads no RI, the walk is skipped -- when it cannot drop a push (the wide walk's
        // condition; its drops are counted) and the walk is the wide one (whose node counts are
        // this build's own).  INW-04 decides after its shadow rays, which scale the contribution.
        INW_CYC(c, 6, t_mat);  // a hit's material (and texture)
        const bool ri_forced = S.wnodes == nullptr || K.size + S.dfs_high > (uint32_t)kFStack;
        const bool ri_read = (m_refl > 0.002f || m_refr > 0.002f) && (m_refr > 0.002f || dot(normal, cd) > 0.0f);
        float surr = 1.0f;
        if (!LIGHTS && (ri_forced || (ri_read && contribution > 0.01f && bounced + 1.0f < (float)F.max_bounces)))
        {
            INW_T0(t_ri);
            OCC_TALLY(c, kOccRi, true);
            surr = inw_ri<RLN>(S, K, hitpoint + normal * 0.001f, ratio, c);
            INW_CYC(c, 1, t_ri);
        }
#ifdef RT_DIAG_SPLIT
        t_tail = clock64();
#endif
        if (mf0) K.reset(0);  // 01_BVH...glsl:544-549: the lens record goes after a primary hit
        if (LIGHTS) {  // 04...glsl:604-665
            uint32_t is_lit = S.n_lights > 0 ? 0u : (uint32_t)is_lit_geom(S, f2u(fg + 0.1f));
            if (is_lit == 0) {
                for (uint32_t i = 0; i < S.n_lights; i++) {
                    const float *lt = S.lights + i * 7;
                    f3 bmin = mk(lt[0], lt[1], lt[2]), bmax = mk(lt[3], lt[4], lt[5]);
                    f3 so = hitpoint + normal * 0.0001f;
                    float sl = len((bmax + bmin) * 0.5f - so) + len(bmax - bmin);
                    f3 sd = normalize((bmin + (bmax - bmin) * ratio) - so);
                    c.shadow++;
                    f3 dummy_n; float dummy_e;
                    float sg = inw_closest<false, LN, FU, false, !LIGHTS, QN>(S, K, so, sd, ratio, invert, sl, dummy_n,
                                                                              dummy_e, -1.0f, c);
                    is_lit += (uint32_t)is_lit_geom(S, f2u(sg + 0.1f));
                }
                const uint32_t nl = S.n_lights > 1 ? S.n_lights : 1u;
                contribution *= (float)is_lit * rcp((float)nl);
                if (ri_forced || (ri_read && contribution > 0.01f && bounced < (float)F.max_bounces))
                    surr = inw_ri<RLN>(S, K, hitpoint + normal * 0.001f, ratio, c);
            } else {
                if (ri_forced) (void)inw_ri<RLN>(S, K, hitpoint + normal * 0.001f, ratio, c);
                color = f3{1, 1, 1};
                K.reset(0);
                break;
            }
        }
        bool ok;
        if (!LIGHTS) { bounced += 1.0f; ok = bounced < (float)F.max_bounces; }
        else ok = bounced < (float)F.max_bounces;
        if ((m_refl > 0.002f || m_refr > 0.002f) && contribution > 0.01f && ok) {
            if (LIGHTS) bounced += 1.0f;
            f3 refl = f3{0, 0, 0}, refr = f3{0, 0, 0};
            f3 nrm = normal;
            if (!(dot(nrm, cd) > 0.0f)) {
                if (m_refl > 0.002f) {
                    refl = normalize(reflect(cd, nrm));
                    if (m_srfl > 0.001f) refl = deviate(S, refl, m_srfl, s);
                }
                if (m_refr > 0.002f) {
                    refr = normalize(refract(cd, nrm, surr * rcp(m_ri)));
                    if (m_srfr > 0.001f) refr = deviate(S, refr, m_srfr, s);
                }
            } else {
                nrm = nrm * -1.0f;
                refr = refract(cd, nrm, m_ri * rcp(surr));
                if (dot(refr, refr) < 0.1f) refl = reflect(cd, nrm);
            }
            float carried = 0.0f;
            const float rr2 = dot(refr, refr);
            if (__builtin_isnan(rr2)) c.nans++;
            if (rr2 > 0.1f) {
                carried += m_refr;
                K.push_ray(hitpoint - nrm * 0.0001f, refr, contribution * m_refr, bounced, c);
            }
            if (dot(refl, refl) > 0.1f) {
                carried += m_refl;
                K.push_ray(hitpoint + nrm * 0.0001f, refl, contribution * m_refl, bounced, c);
            }
            contribution *= (1.0f - 0.5f * carried);
        }
        color = color + m_color * contribution;
    } while (false);
#ifdef RT_DIAG_SPLIT
    if (t_tail) c.cyc[7] += clock64() - t_tail;
#endif
}

template <bool LIGHTS>
__global__ __launch_bounds__(kBlock) void k_inw(Frame f, InwScene S, Chunk ch, Cont ct, unsigned *counter) {
    __shared__ float lds[kFStack * kBlock];
    Ctr c;
    FStack K{lds + threadIdx.x, 0};
    const uint32_t total = ct.in ? *ct.in_count : units_total(f);
    const bool may_park = ct.out != nullptr && total >= ct.park_min;
    const int s_end = ch.s_end < f.spp ? ch.s_end : f.spp;
    bool live = true, busy = false;
    UnitPix px{};
    uint32_t unit = 0, urays = 0;
    f3 acc = f3{0, 0, 0}, col = f3{0, 0, 0};
    float dmid = 0.0f, dep = 0.0f;
    int s = 0;
    K.size = 0;
    for (;;) {
        const uint32_t q = fetch_unit(counter, live && !busy);
        if (live && !busy) {
            if (q >= total) live = false;
            else if (ct.in) {  // resume a parked lane
                const float4 *p = ct.in + (size_t)q * kContSlots;
                const float4 m = p[0], a = p[1], b = p[2];
                unit = __float_as_uint(m.x); s = __float_as_int(m.y); K.size = __float_as_uint(m.z);
                urays = __float_as_uint(m.w);
                acc = f3{a.x, a.y, a.z}; dmid = a.w;
                col = f3{b.x, b.y, b.z}; dep = b.w;
                const float *fl = reinterpret_cast<const float *>(p + 3);
                for (int k = 0; k < kFStack; k++) K.base[k * kBlock] = fl[k];
                px = unit_pixel(f, unit);
                busy = true;
            } else {
                unit = ch.order ? ch.order[q] : q;
                px = unit_pixel(f, unit);
                if (!px.in_image) {
                    if (ch.final_chunk) write_px(f, px, f3{0, 0, 0}, 0.0f);
                    if (ch.cost) ch.cost[unit] = 0;
                } else {
                    busy = true;
                    s = ch.s_begin;
                    K.size = 0;
                    urays = 0;
                    if (s == 0) { acc = f3{0, 0, 0}; dmid = 0.0f; }
                    else {
                        const float4 a0 = ch.state[2 * (size_t)unit];
                        acc = f3{a0.x, a0.y, a0.z};
                        dmid = a0.w;
                    }
                }
            }
        }
        if (__ballot(live) == 0) break;
        if (may_park && __ballot(!live) != 0 && __popcll(__ballot(busy)) < kParkBelow) {
            const uint32_t slot = park_slot(ct.out_count, busy);
            if (busy) {
                float4 *p = ct.out + (size_t)slot * kContSlots;
                p[0] = make_float4(ubits(unit), ibits(s), ubits(K.size), ubits(urays));
                p[1] = make_float4(acc.x, acc.y, acc.z, dmid);
                p[2] = make_float4(col.x, col.y, col.z, dep);
                float *fl = reinterpret_cast<float *>(p + 3);
                for (int k = 0; k < kFStack; k++) fl[k] = K.base[k * kBlock];
            }
            break;
        }
        DBG_TALLY(f, c, kDbgOuter, busy);
        if (!busy) continue;
        // one ray segment per iteration (samples of a pixel are independent invocations)
        if (K.size == 0) { inw_start_sample(S, f, K, px.x, px.y, s, c); col = f3{0, 0, 0}; dep = 0.0f; }
        DBG_TALLY(f, c, kDbgSeg, true);
        inw_segment<LIGHTS>(S, f, K, s, col, dep, c);
        urays++;
        if (K.size == 0) {  // sample done: End() accumulates sqrt(colour) in sample order
            f3 g = f3{__builtin_sqrtf(col.x), __builtin_sqrtf(col.y), __builtin_sqrtf(col.z)};
            acc = sel(s == 0, g, acc + g);
            if (s == f.spp / 2) dmid = dep;
            s++;
            if (s >= s_end) {
                if (ch.final_chunk) write_px(f, px, acc * rcp((float)f.spp), dmid);
                else ch.state[2 * (size_t)unit] = make_float4(acc.x, acc.y, acc.z, dmid);
                if (ch.cost) ch.cost[unit] = urays;
                busy = false;
            }
        }
    }
    flush(f, c);
}

// ---------------------------------------------------------------- INW wave counts
// Waves per SIMD of the 256-lane INW kernels: INW-04 (LIGHTS) at 3 (159 VGPRs, no spills);
// INW-01 at 4 (128 VGPRs with a few spills, 8% faster on C3 than 3 waves in round 2).
#ifndef RT_INW_WAVES
#define RT_INW_WAVES 3
#endif
#ifndef RT_INW01_WAVES
#define RT_INW01_WAVES 4  // INW-01: 128 VGPRs with a few spills, 8% faster on C3 than 3 waves
#endif

// ---------------------------------------------------------------- INW: on-chip End() folds
// End() (01_BVH...glsl:625-653, 664-675) adds each sample's sqrt(colour) in sample order and
// stores the mean.  The INW kernels below keep that sum on chip.  A wave claims work from the
// global queue, hands its samples to its lanes as a stream g = 0, 1, 2, ... in a fixed order, and
// a lane that finishes a sample takes the next stream entry at once (lane persistence).  A
// finished sample stores its sqrt(colour) into the wave's private ring; the wave folds the ring in
// each pixel's sample order, End()'s float order, and writes a pixel when its last sample is
// folded.  The ring: k_inw_pm's 768-lane instances keep it in LDS (InwScene::lring, the default:
// 256 entries per wave as r, g, b planes; an entry is finished when no busy lane holds it); the
// other kernels keep a global ring of {sqrt(colour), tag g} per wave (16 KB per wave at 1024
// entries, not L2-resident at the chip's 3,000-odd waves: it reaches the fabric).
// The middle sample's depth goes with the pixel's colour.  Entries beyond the oldest unfolded one + ring size are not issued (a
// straggling sample holds the window; the other lanes keep running until it fills).  Counters
// accumulate per lane.  Two stream orders, one per kind of ray coherence:
//  - k_inw_pm (pixel-major): the wave claims pixels and runs all samples of one pixel back to
//    back, so its 64 lanes trace 64 consecutive samples of one pixel -- nearly the same ray where
//    lens, motion and scatter offsets are small next to the scene's detail (C3: 10k small
//    spheres, neighbouring pixels see different spheres).  The fold is wave-serial: once per
//    iteration the wave loads the next 64 ring entries and every lane adds the leading finished
//    run in order (each lane computes the same sum).
//  - k_inw_sm (sample-major): the wave claims 8x8 pixel blocks and runs one sample index over the
//    64 pixels of the block at a time (rows s = 0, 1, ...), so its lanes trace neighbouring
//    pixels at one lens offset, time and scatter direction -- the same ray where the scene is
//    coarse next to a pixel (C5: the Cornell walls).  The fold is lane-parallel: lane p holds
//    pixel p's sum and adds its own samples as they finish.
// k_inw_probe picks one per frame on the device (mode[]): over a sparse set of 8x8 blocks it
// traces one primary ray per pixel; the frame is "coarse" when most blocks with a hit see one
// object in all their pixels.  Both kernels are launched; the one not picked exits at once.
// A fold-ring entry's tag: the low 26 bits of its stream position and the frame's ring epoch
// (0..62) in the high 6 (InwScene::ring_epoch).  An entry left by one of the 62 frames before
// carries another epoch, and the host clears the rings with 0xff bytes (an epoch of 63, never
// valid) whenever the epoch wraps to 0, so a stale entry never passes for a finished one and no
// per-frame clear is needed.  Within a frame, slot g mod R last held g - R (R <= 2^16 < 2^26).
// The fold kernels' framebuffer stores.  Measured and not kept (round 5): nontemporal stores here
// raised C5's L2-to-fabric writes from 4.7 to 37 GB per frame (each streaming 16-B store leaves L2
// as its own partial-line write) at the same frame time.
__device__ __forceinline__ void fb_store(const Frame &f, size_t o, float4 v) {
    reinterpret_cast<float4 *>(f.out_rgba)[o] = v;
}
__device__ __forceinline__ void depth_store(const Frame &f, size_t o, float d) { f.out_depth[o] = d; }
__device__ __forceinline__ uint32_t ring_tag(const InwScene &S, uint32_t g) {
    return (g & 0x03ffffffu) | S.ring_epoch;
}
__device__ __forceinline__ float rdl(float v, uint32_t l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)l));
}
__device__ __forceinline__ uint32_t uni(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
// the probe's verdict: mode[0] = blocks with a hit, mode[1] = those whose pixels all see one object
__device__ __forceinline__ bool inw_sample_major(const uint32_t *mode, uint32_t force) {
    if (force == 1u) return false;
    if (force == 2u) return true;
    const uint32_t hit = uni(mode[0]), same = uni(mode[1]);
    return 2u * same >= hit && hit > 0u;
}
// Pixel beams (DESIGN.md §5 "Pixel beams").  A pixel's primary rays all pass through its focal
// point F = co + cd * focus and leave the lens disk around C0 = co + cd (radius <= delta0), so they
// lie within beam_R of the central ray C0 + t * cd over t in [beam_tmin, beam_tfar] (host bounds).
// One lane per pixel unit walks the culling BVH with that ray against the boxes inflated by
// beam_R and keeps the beam_cap leaves of smallest entry t, sorted; beam_cut is the smallest
// entry t of a leaf it could not keep.
constexpr int kBeamBlock = 128, kBeamStack = 48, kBeamCapMax = 32;
__global__ __launch_bounds__(kBeamBlock) void k_inw_beam(Frame f, InwScene S, const uint32_t *mode, uint32_t force) {
    if (inw_sample_major(mode, force)) return;
    __shared__ int st[kBeamStack * kBeamBlock];
    __shared__ uint2 lst[kBeamCapMax * kBeamBlock];
    const uint32_t u = blockIdx.x * kBeamBlock + threadIdx.x, lane = threadIdx.x & 63u;
    if (u >= units_total(f)) return;  // whole waves (units come in 8x8 blocks of 64)
    const UnitPix px = unit_pixel(f, u);
    const uint32_t bo = blockIdx.y * S.beam_units;  // time bin blockIdx.y (beam_bins > 1): its tree, its lists
    uint32_t *nout = const_cast<uint32_t *>(S.beam_n) + bo;
    float *cout = const_cast<float *>(S.beam_cut) + bo;
    const uint32_t cap = S.beam_cap;
    uint2 *L = lst + threadIdx.x;
    uint32_t nl = 0;
    float cut = kMiss;
    bool off = false;
    if (px.in_image) {
        const f3 cd = inw_pixel_dir(f, px.x, px.y);
        const f3 o = mk(f.pos[0], f.pos[1], f.pos[2]) + cd;
        const f3 id = f3{rcp(cd.x), rcp(cd.y), rcp(cd.z)};
        off = !(__builtin_isfinite(id.x) && __builtin_isfinite(id.y) && __builtin_isfinite(id.z));
        const float R = S.beam_R, t0 = S.beam_tmin, t1 = S.beam_tfar;
        // near / far planes of each axis for this direction, inflated outward by R
        const uint32_t ox = cd.x < 0.0f ? 3u : 0u, oy = cd.y < 0.0f ? 4u : 1u, oz = cd.z < 0.0f ? 5u : 2u;
        const f3 rn = f3{cd.x < 0.0f ? R : -R, cd.y < 0.0f ? R : -R, cd.z < 0.0f ? R : -R};
        int *stk = st + threadIdx.x;
        int sp = 0, cur = S.beam_bins > 1u ? (int)(1u + S.wbin_base + blockIdx.y * S.wbin_stride) : S.wroot;
        while (!off) {
            const float4 *nd = S.wnodes + kInwNodeF4 * (cur - 1);
            const float4 nx = nd[ox], fx = nd[ox + 3], ny = nd[oy], fy = nd[oy + 3], nz = nd[oz], fz = nd[oz + 3];
            const float4 lk = nd[9];
            const float nxa[4] = {nx.x, nx.y, nx.z, nx.w}, fxa[4] = {fx.x, fx.y, fx.z, fx.w};
            const float nya[4] = {ny.x, ny.y, ny.z, ny.w}, fya[4] = {fy.x, fy.y, fy.z, fy.w};
            const float nza[4] = {nz.x, nz.y, nz.z, nz.w}, fza[4] = {fz.x, fz.y, fz.z, fz.w};
            const int lka[4] = {__float_as_int(lk.x), __float_as_int(lk.y), __float_as_int(lk.z), __float_as_int(lk.w)};
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const float te = fmaxf(fmaxf(((nxa[k] + rn.x) - o.x) * id.x, ((nya[k] + rn.y) - o.y) * id.y),
                                       ((nza[k] + rn.z) - o.z) * id.z);
                const float tx = fminf(fminf(((fxa[k] - rn.x) - o.x) * id.x, ((fya[k] - rn.y) - o.y) * id.y),
                                       ((fza[k] - rn.z) - o.z) * id.z);
                if (!(fmaxf(te, t0) <= fminf(tx, t1))) continue;
                const int l = lka[k];
                if (l > 0) {
                    if (sp == kBeamStack) off = true;
                    else stk[(sp++) * kBeamBlock] = l;
                } else {  // keep the cap smallest entries, sorted (insertion)
                    float tv = te;
                    uint32_t gv = (uint32_t)(-l);
                    if (nl == cap) {
                        const float last = __uint_as_float(L[(cap - 1) * kBeamBlock].y);
                        if (!(tv < last)) { cut = fminf(cut, tv); continue; }
                        cut = fminf(cut, last);
                        nl--;
                    }
                    uint32_t j = nl;
                    while (j > 0 && __uint_as_float(L[(j - 1) * kBeamBlock].y) > tv) {
                        L[j * kBeamBlock] = L[(j - 1) * kBeamBlock];
                        j--;
                    }
                    L[j * kBeamBlock] = make_uint2(gv, __float_as_uint(tv));
                    nl++;
                }
            }
            if (off || sp == 0) break;
            cur = stk[(--sp) * kBeamBlock];
        }
    }
    // The block's 64 lists packed densely in its region of 64 * cap entries, in unit order (the
    // fold kernel claims a block's pixels one after another, so their lists share cache lines):
    // beam_n[u] = offset in the region << 8 | count
    const uint32_t cnt = off ? 0u : nl;
    uint32_t incl = cnt;
    for (uint32_t d = 1; d < 64u; d <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)incl, d, 64);
        if (lane >= d) incl += y;
    }
    const uint32_t at = incl - cnt;
    const size_t base = ((size_t)bo + (u & ~63u)) * cap + at;
    if (S.beam16) {  // object ids < 2^16: the id and the high half of max(t, 0) (t rounded down)
        uint32_t *dst = reinterpret_cast<uint32_t *>(const_cast<uint2 *>(S.beam)) + base;
        for (uint32_t j = 0; j < cnt; j++) {
            const uint2 e = L[j * kBeamBlock];
            const uint32_t tb = __uint_as_float(e.y) > 0.0f ? e.y : 0u;
            dst[j] = (e.x & 0xffffu) | (tb & 0xffff0000u);
        }
    } else {
        uint2 *dst = const_cast<uint2 *>(S.beam) + base;
        for (uint32_t j = 0; j < cnt; j++) dst[j] = L[j * kBeamBlock];
    }
    nout[u] = off ? kBeamOff : (at << 8) | nl;
    cout[u] = px.in_image ? cut : kMiss;
}

template <bool LIGHTS>
__global__ __launch_bounds__(kBlock) void k_inw_probe(Frame f, InwScene S, uint32_t stride, uint32_t *mode) {
    __shared__ float lds[kFStack * kBlock];
    Ctr c;  // not flushed: the probe's rays are not the frame's
    FStack K{lds + threadIdx.x, 0};
    const uint32_t lane = threadIdx.x & 63u, nblk = units_total(f) / 64u;
    const uint32_t blk = ((blockIdx.x * kBlock + threadIdx.x) >> 6) * stride;
    if (blk >= nblk) return;  // whole waves (blk is per wave)
    const UnitPix px = unit_pixel(f, blk * 64u + lane);
    int id = -2;  // -2: outside the image, -1: no hit, else the object
    if (px.in_image) {
        const int s = f.spp / 2;
        inw_start_sample(S, f, K, px.x, px.y, s, c);
        K.size -= 8;
        const uint32_t b = K.size;
        const f3 o = mk(K.at(b), K.at(b + 1), K.at(b + 2)), d = mk(K.at(b + 3), K.at(b + 4), K.at(b + 5));
        const f3 D = mk(f.dir[0], f.dir[1], f.dir[2]);
        float tlim = kMaxT, extra = 0.0f;
        f3 nrm;
        const float g = inw_closest<false>(S, K, o, d, (float)s * f.inv_spp, dot(D, f3{1, 1, 1}) > 0.0f, tlim, nrm,
                                           extra, -1.0f, c);
        id = tlim < kMaxT ? (int)g : -1;
    }
    const int id0 = __shfl(id, __ffsll((long long)__ballot(id != -2)) - 1, 64);
    const bool any_hit = __ballot(id >= 0) != 0ull, same = __ballot(id != -2 && id != id0) == 0ull;
    if (lane == 0 && any_hit) {
        atomicAdd(mode, 1u);
        if (same) atomicAdd(mode + 1, 1u);
    }
}

// Claim order (DESIGN.md §5 "Claim order"): a persistent fold kernel's tail is the last pixels
// it claims -- a wave needs spp / 64 rounds of samples for one pixel, so expensive pixels claimed
// last leave the rest of the chip idle.  k_inw_cost estimates each pixel's cost from the primary
// rays of two of its samples, the costlier (a miss or a diffuse hit ends the sample; a reflective /
// refractive hit starts a chain of about log(0.01) / log(coefficient) segments, two-sided for
// refraction), keys each 8x8 block by its costliest pixel and buckets it (256 log-scale keys);
// k_inw_order_scan / k_inw_order_scatter lay
// the blocks out costliest first, and k_inw_pm claims through that order.  The order only decides
// which wave traces which pixel when: every pixel's samples and sums are the same.  Pixel-major
// frames only: the three kernels exit at once when the probe picked k_inw_sm, whose 8x8 blocks
// keep their spatial order (measured: C5 3% slower with it, the blocks' locality lost).
template <bool LIGHTS>
__global__ __launch_bounds__(kBlock) void k_inw_cost(Frame f, InwScene S, uint32_t *key, uint32_t *hist,
                                                     const uint32_t *mode, uint32_t force) {
    if (inw_sample_major(mode, force)) return;
    __shared__ float lds[kFStack * kBlock];
    Ctr c;  // not flushed: these rays are not the frame's
    FStack K{lds + threadIdx.x, 0};
    // every pixel of the block (a wave per block), two samples each; the block's key is its
    // costliest pixel's, so the blocks claimed last hold no expensive pixel
    const uint32_t lane = threadIdx.x & 63u, nblk = units_total(f) / 64u, p = lane;
    const uint32_t blk = ((blockIdx.x * kBlock + threadIdx.x) >> 6);
    float est = 0.0f;
    if (blk < nblk) {
        const UnitPix px = unit_pixel(f, blk * 64u + p);
        for (int si = 0; si < 2 && px.in_image; si++) {
            const int s = si == 0 ? f.spp / 2 : f.spp / 4;
            K.size = 0;
            inw_start_sample(S, f, K, px.x, px.y, s, c);
            K.size -= 8;
            const uint32_t b = K.size;
            const f3 o = mk(K.at(b), K.at(b + 1), K.at(b + 2)), d = mk(K.at(b + 3), K.at(b + 4), K.at(b + 5));
            const f3 D = mk(f.dir[0], f.dir[1], f.dir[2]);
            float tlim = kMaxT, extra = 0.0f;
            f3 nrm;
            const float g = inw_closest<false>(S, K, o, d, (float)s * f.inv_spp, dot(D, f3{1, 1, 1}) > 0.0f, tlim,
                                               nrm, extra, -1.0f, c);
            float e1 = 1.0f;
            if (tlim < kMaxT) {
                const float4 m0 = S.cold[2 * (int)g];
                const float m = fminf(fmaxf(m0.x, m0.y), 0.99f);
                if (LIGHTS) e1 += (float)S.n_lights;
                if (m > 0.002f) {
                    const float n = fminf((float)f.max_bounces, 1.0f + __logf(0.01f) / __logf(m));
                    e1 += n * (m0.x > 0.002f ? 2.0f : 1.0f) * (LIGHTS ? 1.0f + (float)S.n_lights : 1.0f);
                }
            }
            est = fmaxf(est, e1);
        }
    }
    for (int o = 32; o >= 1; o >>= 1) est = fmaxf(est, __shfl_xor(est, o, 64));
    est *= 16.0f;  // the scale of the 16-pixel sums this key replaced
    if (p == 0 && blk < nblk) {
        const uint32_t k = (uint32_t)fminf(255.0f, 16.0f * __log2f(1.0f + est));
        key[blk] = k;
        atomicAdd(hist + (255u - k), 1u);
    }
}
// exclusive scan of the 256 bucket counts (one 256-lane block)
__global__ __launch_bounds__(256) void k_inw_order_scan(uint32_t *hist, const uint32_t *mode, uint32_t force) {
    if (inw_sample_major(mode, force)) return;
    __shared__ uint32_t t[256];
    const uint32_t i = threadIdx.x;
    const uint32_t v = hist[i];
    t[i] = v;
    __syncthreads();
    for (uint32_t o = 1; o < 256u; o <<= 1) {
        const uint32_t a = i >= o ? t[i - o] : 0u;
        __syncthreads();
        t[i] += a;
        __syncthreads();
    }
    hist[i] = t[i] - v;
}
__global__ __launch_bounds__(kBlock) void k_inw_order_scatter(const uint32_t *key, uint32_t *off, uint32_t *order,
                                                               uint32_t nblk, const uint32_t *mode, uint32_t force) {
    if (inw_sample_major(mode, force)) return;
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= nblk) return;
    order[atomicAdd(off + (255u - key[i]), 1u)] = i;
}

// pixel-major stream (see above): entry g = (claimed pixel ordinal j, sample s).  LN: 768-lane
// blocks (3 waves per SIMD) that stage the top of the wide BVH in the LDS their three 256-lane
// stacks leave free (kInwLdsNodes nodes)
// GQ (DESIGN.md §5.1 "GQ"; LN, FU, LRING and INW-01 only): the reference's 40-float stacks in
// global memory (GStack, S.gstk), the wide walks' node stacks in LDS (kWStack entries per lane), the
// closest-hit walks over the quantised nodes, the top kQLdsNodes of them staged in LDS
#ifndef RT_GQ_STAGE
#define RT_GQ_STAGE 1
#endif
// k_inw_pm's LDS fold ring: channel c of entry e.  Planes (r, g, b of 256 entries each): the fold's
// lanes 0, 1, 2 read one plane each at the same entry, addresses 1 KB apart, one bank: a 3-way
// conflict per read.  RT_RING_IL interleaves the channels (3 e + c): the three lanes hit 3 banks,
// but C3 ran 0.5% slower (185.7 against 184.7 ms, profiles/r06_ab_beam_sload_ring_il.json).
#ifdef RT_RING_IL
#define RIX(c, e) (3u * (e) + (c))
#else
#define RIX(c, e) ((c) * kPmLdsRing + (e))
#endif
#ifndef RT_INW_R1_MIN
#define RT_INW_R1_MIN 0
#endif
constexpr int kR1Min = RT_INW_R1_MIN;  // k_inw_pm: round 1 waits for this many lanes with a ray (0 = off)
#ifdef RT_GQ_FSTACK
constexpr bool kGqGlobalStack = false;
#else
constexpr bool kGqGlobalStack = true;
#endif
constexpr bool kGqStage = RT_GQ_STAGE != 0;
static_assert(kGqLdsFree >= kInwLdsNodes * kInwNodeF4 * 16, "GQ: room for the 236 full nodes");
template <bool LN, bool GQ>
constexpr int pm_sub() { return GQ && kGqGlobalStack ? kGqSub : (LN ? 3 : 1); }
template <bool LIGHTS, bool LN = false, bool FU = false, bool LRING = false, bool GQ = false>
__global__ __launch_bounds__((pm_sub<LN, GQ>() * kBlock)) __attribute__((amdgpu_waves_per_eu((LN ? pm_sub<LN, GQ>() : (LIGHTS ? RT_INW_WAVES : RT_INW01_WAVES))))) void k_inw_pm(Frame f, InwScene S0, float4 *ring, uint32_t rmask, unsigned *counter, const uint32_t *mode, uint32_t force, const uint32_t *border) {
    static_assert(!GQ || (LN && FU && LRING && !LIGHTS), "GQ: the C3 instance only");
    if (inw_sample_major(mode, force)) return;  // the probe picked k_inw_sm for this frame
    constexpr int SUB = pm_sub<LN, GQ>();
    // GS: the global 40-float stacks (GQ; the RT_GQ_FSTACK experiment keeps FStack), GST: the top
    // of the culling BVH staged in the LDS that frees (RT_GQ_STAGE=0: none, an experiment), QN:
    // quantised nodes (else the full ones, 236 in g_inw_lnodes)
    constexpr bool GS = GQ && kGqGlobalStack, GST = GS && kGqStage, QN = GQ && kGqQn;
    // FStack instances: the three 256-lane 40-float stacks; GS: the wide walks' node stacks
    __shared__ float lds[SUB * (GS ? kWStack : kFStack) * kBlock];
    // per wave: the middle sample's depth of claimed ordinal j (slot j % 64; at most 64 ordinals lie
    // between the fold and the issue), written out with the pixel's colour
    __shared__ float s_pdep[SUB * kBlock];
    InwScene S = S0;
    // LRING: the fold ring in LDS, after the first kPmLdsNodes staged nodes (InwScene::lring; an
    // instance of its own: as a per-frame branch it cost 1% of C3 in either mode)
    constexpr bool LR = LN && LRING;
    // WLN: the walks read staged nodes.  The LDS-ring instances stage none: the top 5 nodes the
    // ring leaves room for sit in L1 anyway, and the walk loop without the LDS branch (its exec
    // masking and the base pointer kept in a VGPR lane) ran C3 2% faster.  GQ
    // stages kQLdsNodes quantised nodes beside its ring
    constexpr bool WLN = LN && (!LR || GST);
    float *lr;  // LR: this wave's ring, three planes (r, g, b) of kPmLdsRing floats
    if constexpr (GS) {
        __shared__ float s_ring[SUB * kBlock / 64 * 3 * kPmLdsRing];
        lr = s_ring + uni((threadIdx.x >> 6) * (3u * kPmLdsRing));
        if constexpr (GST && QN) {
            const uint32_t n = S.qnodes ? (S.n_wnodes < (uint32_t)kQLdsNodes ? S.n_wnodes : (uint32_t)kQLdsNodes) : 0u;
            for (uint32_t i = threadIdx.x; i < n * (uint32_t)kQNodeF4; i += SUB * kBlock) g_inw_qlds[i] = S.qnodes[i];
            __syncthreads();
            S.n_lnodes = n;
        } else if constexpr (GST) {
            const uint32_t n = S.wnodes ? (S.n_wnodes < (uint32_t)kInwLdsNodes ? S.n_wnodes : (uint32_t)kInwLdsNodes) : 0u;
            for (uint32_t i = threadIdx.x; i < n * (uint32_t)kInwNodeF4; i += SUB * kBlock) g_inw_lnodes[i] = S.wnodes[i];
            __syncthreads();
            S.n_lnodes = n;
        }
    } else {
        lr = reinterpret_cast<float *>(g_inw_lnodes + kPmLdsNodes * kInwNodeF4) + uni((threadIdx.x >> 6) * (3u * kPmLdsRing));
        if constexpr (WLN) {
            const uint32_t cap = (uint32_t)kInwLdsNodes;
            const uint32_t n = S.wnodes ? (S.n_wnodes < cap ? S.n_wnodes : cap) : 0u;
            for (uint32_t i = threadIdx.x; i < n * (uint32_t)kInwNodeF4; i += SUB * kBlock) g_inw_lnodes[i] = S.wnodes[i];
            // no wide walk: the stackless LBVH walks read the top of the LBVH (2 float4 per node) there
            const uint32_t nb = (!S.wnodes && S.sl) ? min(2u * S.n - 1u, cap * (uint32_t)kInwNodeF4 / 2u) : 0u;
            for (uint32_t i = threadIdx.x; i < 2u * nb; i += SUB * kBlock) g_inw_lnodes[i] = S.nodes[i];
            __syncthreads();
            S.n_lnodes = n;
            S.n_blds = nb;
        }
    }
    Ctr c;
#ifdef RT_DIAG_SPLIT
    const unsigned long long t_start = wall_clock64();  // the tail split (tools/inw_split.py)
    unsigned long long t_qd = 0;
#endif
    using KS = std::conditional_t<GS, GStack, FStack>;
    KS K;
    if constexpr (GS) {
        K.col = S.gstk + ((size_t)blockIdx.x * (SUB * kBlock) + threadIdx.x);
        K.stride = gridDim.x * (SUB * kBlock);
        K.ws = lds + (threadIdx.x / kBlock) * (kWStack * kBlock) + (threadIdx.x % kBlock);
        K.rc = false;
    } else {
        K.base = lds + (threadIdx.x / kBlock) * (kFStack * kBlock) + (threadIdx.x % kBlock);
    }
    K.size = 0;
    const uint32_t lane = threadIdx.x & 63u;
    if constexpr (LR) rmask = kPmLdsRing - 1u;
    const uint32_t rsize = rmask + 1u;
    float4 *wr = ring + (size_t)uni((blockIdx.x * (SUB * kBlock) + threadIdx.x) >> 6) * rsize;
    float *pdep = s_pdep + (threadIdx.x & ~63u);
    const uint32_t spp = (uint32_t)f.spp, mid = spp / 2u, total = units_total(f);
    const float inv = rcp((float)f.spp);
    // wave-uniform: stream positions (entry gi / fold gf) as (pixel ordinal, sample), claims
    uint32_t gi = 0, ji = 0, si = 0;   // next entry to issue: pixel ordinal ji, sample si
    uint32_t gf = 0, jf = 0, sf = 0;   // next entry to fold
    uint32_t nclaimed = 0;             // pixel ordinals claimed so far
    bool qdone = false;
    uint32_t xq = 0;                   // S.xcdq: queues found empty (from this block's XCD on)
    const uint32_t nblk8 = total / 64u;  // 8x8 blocks (units come in whole blocks)
    f3 acc = f3{0, 0, 0};              // running End() sum of pixel jf (the same in every lane)
    float accc = 0.0f;                 // LR: lane c < 3 holds channel c of that sum
    uint32_t pix_slot = 0xffffffffu;   // lane l: the unit of the claimed ordinal j with j % 64 == l
    // per lane: the sample it traces
    bool busy = false;
    uint32_t g = 0, pj = 0;  // the lane's stream entry and its pixel's ordinal slot (j % 64)
    int s = 0;
    UnitPix px{};
    uint32_t bu = kBeamOff;  // the lane's pixel unit for its beam list (S.beam)
    uint32_t pu = 0xffffffffu;  // the unit px and pcd belong to: a lane's next sample is mostly the same pixel's
#ifdef RT_INW_PARK
    constexpr bool PK = true;
#else
    constexpr bool PK = false;
#endif
    bool parked = false;  // PK: this lane's walk is parked (its segment resumes next iteration)
    float4 *pslot = S.park ? S.park + 2 * ((size_t)blockIdx.x * blockDim.x + threadIdx.x) : nullptr;
    f3 pcd = f3{0, 0, 0};
    f3 col = f3{0, 0, 0};
    float dep = 0.0f;
    K.size = 0;
    for (;;) {
        // ---- fold the finished entries gf, gf+1, ... (stored in earlier iterations)
        INW_T0(t_fold);
        if (gf != gi) {
            const uint32_t k = gf + lane;
            float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            uint32_t n;
            bool continue_fold = true;  // (the LDS-ring fold below finishes the run itself)
            if constexpr (LR) {
                // Every issued entry is either held by a busy lane or stored, so the entries below
                // the smallest one a busy lane holds are finished: no tags.  LDS ops of one wave
                // complete in order, so the stores of earlier iterations are visible.
                n = uni(__ockl_wfred_min_u32(busy ? g - gf : 0xffffffffu));  // DPP reduction
                if (n > gi - gf) n = gi - gf;
                if (n > 64u) n = 64u;
                if (lane < n) {
                    const uint32_t e = k & rmask;
                    v = make_float4(lr[RIX(0u, e)], lr[RIX(1u, e)], lr[RIX(2u, e)], 0.0f);
                }
            } else {
                __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's ring stores have landed (same CU: L1 write-through)
                bool fin = false;
                if (k - gf < gi - gf) {
                    v = wr[k & rmask];
                    fin = __float_as_uint(v.w) == ring_tag(S, k);
                }
                const unsigned long long m = __ballot(fin);
                n = ~m == 0ull ? 64u : (uint32_t)__builtin_ctzll(~m);
            }
#ifndef RT_FOLD_READLANE
            if constexpr (LR) {
                // LDS ring: lanes 0, 1, 2 add the r, g, b planes' entries straight from LDS, each
                // its channel in sample order (the same float additions, two instructions per entry
                // instead of three readlanes and three adds); the run splits at pixel ends
                const uint32_t lc = lane < 3u ? lane : 0u;  // this lane's channel
                for (uint32_t i = 0; i < n;) {
                    const uint32_t e = i + (n - i < spp - sf ? n - i : spp - sf);
                    if (lane < 3u) {
                        uint32_t j = i;
                        if (sf == 0) { accc = lr[RIX(lc, (gf + j) & rmask)]; j++; }
                        constexpr uint32_t kFU = 4;  // loads in flight, then the adds in order (8, 16: same time)
                        for (; j + kFU <= e; j += kFU) {
                            float a[kFU];
#pragma unroll
                            for (uint32_t u = 0; u < kFU; u++) a[u] = lr[RIX(lc, (gf + j + u) & rmask)];
#pragma unroll
                            for (uint32_t u = 0; u < kFU; u++) accc = accc + a[u];
                        }
                        for (; j < e; j++) accc = accc + lr[RIX(lc, (gf + j) & rmask)];
                    }
                    sf += e - i;
                    i = e;
                    if (sf == spp) {  // pixel jf complete: End()'s imageStores (01_BVH...glsl:652, 667-668)
                        const uint32_t unit = uni((uint32_t)__builtin_amdgcn_readlane((int)pix_slot, (int)(jf & 63u)));
                        const float ax = rdl(accc, 0u), ay = rdl(accc, 1u), az = rdl(accc, 2u);
                        if (lane == 0) {
                            const UnitPix p = unit_pixel(f, unit);
                            if (p.out != (size_t)-1) {
                                fb_store(f, p.out,
                                         make_float4(p.in_image ? ax * inv : 0.0f, p.in_image ? ay * inv : 0.0f,
                                                     p.in_image ? az * inv : 0.0f, p.in_image ? 1.0f : 0.0f));
                                if (f.out_depth) depth_store(f, p.out, pdep[jf & 63u]);
                            }
                        }
                        sf = 0;
                        jf++;
                    }
                }
                gf += n;
                continue_fold = false;
            }
#endif
            // the run splits at pixel ends: per pixel, its entries are added with no test between them
            for (uint32_t i = 0; continue_fold && i < n;) {
                const uint32_t e = i + (n - i < spp - sf ? n - i : spp - sf);
                uint32_t j = i;
                if (sf == 0) { acc = f3{rdl(v.x, j), rdl(v.y, j), rdl(v.z, j)}; j++; }
                for (; j + 4u <= e; j += 4u) {  // four adds in order, one loop test
                    acc = acc + f3{rdl(v.x, j), rdl(v.y, j), rdl(v.z, j)};
                    acc = acc + f3{rdl(v.x, j + 1u), rdl(v.y, j + 1u), rdl(v.z, j + 1u)};
                    acc = acc + f3{rdl(v.x, j + 2u), rdl(v.y, j + 2u), rdl(v.z, j + 2u)};
                    acc = acc + f3{rdl(v.x, j + 3u), rdl(v.y, j + 3u), rdl(v.z, j + 3u)};
                }
                for (; j < e; j++) acc = acc + f3{rdl(v.x, j), rdl(v.y, j), rdl(v.z, j)};
                sf += e - i;
                i = e;
                if (sf == spp) {  // pixel jf complete: End()'s imageStores (01_BVH...glsl:652, 667-668)
                    const uint32_t unit = uni((uint32_t)__builtin_amdgcn_readlane((int)pix_slot, (int)(jf & 63u)));
                    if (lane == 0) {
                        const UnitPix p = unit_pixel(f, unit);
                        if (p.out != (size_t)-1) {
                            fb_store(f, p.out,
                                     make_float4(p.in_image ? acc.x * inv : 0.0f, p.in_image ? acc.y * inv : 0.0f,
                                                 p.in_image ? acc.z * inv : 0.0f, p.in_image ? 1.0f : 0.0f));
                            if (f.out_depth) depth_store(f, p.out, pdep[jf & 63u]);
                        }
                    }
                    sf = 0;
                    jf++;
                }
            }
            if (continue_fold) gf += n;
        }
        INW_CYC(c, 2, t_fold);
        INW_T0(t_issue);
        // ---- claim pixels for the free lanes (at most 64 pixels between fold and issue)
        const unsigned long long fm = __ballot(!busy);
        const uint32_t nfree = (uint32_t)__popcll(fm);
        if (!qdone && nfree) {
            // ordinals the free lanes would reach: ji + (si + nfree - 1) / spp, capped at jf + 63
            uint32_t need = ji + (si + nfree - 1u) / spp + 1u;
            if (need > jf + 64u) need = jf + 64u;
            if (need > nclaimed) {
                const uint32_t want = need - nclaimed;
                uint32_t base = 0, got = 0, qx = 0;
                if (S.xcdq) {
                    // per-XCD queues (rt_options.inw_claim_xcd): queue x holds the blocks of claim
                    // ordinal b = x mod 8, in claim order, so a block's pixels -- whole 128-B lines of
                    // the framebuffer per block row -- are written through one XCD's L2 (workgroups go
                    // to the XCDs round robin); a wave whose queue is empty takes from the next ones
                    while (xq < 8u) {  // wave-uniform
                        qx = (blockIdx.x + xq) & 7u;
                        const uint32_t nb = nblk8 > qx ? (nblk8 - qx + 7u) >> 3 : 0u, qt = nb * 64u;
                        if (lane == 0) base = atomicAdd(counter + 64u + 16u * qx, want);
                        base = uni((uint32_t)__shfl((int)base, 0, 64));
                        if (base < qt) {
                            got = min(want, qt - base);
                            if (base + want >= qt) xq++;
                            break;
                        }
                        xq++;
                    }
                    if (xq >= 8u) qdone = true;
                } else {
                    if (lane == 0) base = atomicAdd(counter, want);
                    base = uni((uint32_t)__shfl((int)base, 0, 64));
                    got = want;
                    if (base >= total) { got = 0; qdone = true; }
                    else if (base + want >= total) { got = total - base; qdone = true; }
                }
#ifdef RT_DIAG_SPLIT
                if (qdone && t_qd == 0) t_qd = wall_clock64();
#endif
                const uint32_t rel = (lane - nclaimed) & 63u;
                if (rel < got) {  // ordinal -> unit through the claim order (block-wise)
                    uint32_t u = base + rel;
                    if (S.xcdq) u = (((u >> 6) << 3) + qx) * 64u + (u & 63u);  // queue ordinal -> claim ordinal
                    pix_slot = border ? border[u >> 6] * 64u + (u & 63u) : u;
                }
                nclaimed += got;
            }
        }
        // ---- issue: free lanes take stream entries in lane order, within the window
        {
            const uint32_t rank = (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
            uint32_t avail = rsize - (gi - gf);
            const uint64_t left = (uint64_t)(nclaimed - ji) * spp - si;  // entries of claimed pixels not issued
            if ((uint64_t)avail > left) avail = (uint32_t)left;
            const uint32_t take = nfree < avail ? nfree : avail;
            if (take) {
                // this lane's entry: pixel ji + adv / spp, sample adv % spp (adv < spp + 64: one
                // subtraction when spp >= 64)
                const uint32_t adv = si + rank;
                const uint32_t q = spp >= 64u ? (adv >= spp ? 1u : 0u) : adv / spp;
                const uint32_t jl = ji + q;
                const uint32_t unit = (uint32_t)__shfl((int)pix_slot, (int)(jl & 63u), 64);
                if (!busy && rank < take) {
                    g = gi + rank;
                    pj = jl & 63u;
                    s = (int)(adv - q * spp);
                    if (unit != pu) {
                        pu = unit;
                        px = unit_pixel(f, unit);
                        if (px.in_image) pcd = inw_pixel_dir(f, px.x, px.y);
                    }
                    bu = S.beam ? unit : kBeamOff;
                    col = f3{0, 0, 0};
                    dep = 0.0f;
                    if (px.in_image) {
                        busy = true;
                        inw_start_sample_cd(S, f, K, pcd, s, c);
                    } else {  // a padding slot: an empty sample, folded as zero
                        if ((uint32_t)s == mid) pdep[pj] = 0.0f;
                        if constexpr (LR) {
                            const uint32_t e = g & rmask;
                            lr[RIX(0u, e)] = 0.0f; lr[RIX(1u, e)] = 0.0f; lr[RIX(2u, e)] = 0.0f;
                        } else {
                            wr[g & rmask] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(ring_tag(S, g)));
                        }
                    }
                }
                gi += take;
                const uint32_t a2 = si + take;
                ji += a2 / spp;
                si = a2 % spp;
            }
        }
        INW_CYC(c, 3, t_issue);
        if (qdone && ji == nclaimed && gf == gi && __ballot(busy) == 0) break;
        // ---- one ray segment per busy lane (samples are independent invocations)
        INW_T0(t_seg);
        OCC_TALLY(c, kOccSeg, busy);
        // Two rounds per iteration (DESIGN.md §5 "Primary and bounce rounds"): primary rays take
        // the beam lists, bounce rays the wide walk, two code paths a wave runs one after the other
        // (one walk trip then carries only the lanes with a bounce ray).  Round 0 runs the lanes
        // whose next ray is a primary one; round 1 every lane with a ray left, the bounce rays those
        // primaries just pushed included, so the walk runs with the bounce rays of the whole wave.
        // INW-04 (LIGHTS) keeps one round: with its shadow walks the two-round loop spills 17 VGPRs
        constexpr int kRounds = LIGHTS ? 1 : 2;
#pragma unroll 1
        for (int round = 2 - kRounds; round < 2; round++) {
            const bool prim = bu != kBeamOff && !parked && K.top_primary();
            const bool go = busy && (round == 0 ? prim : (parked || K.size > 0u));
            INW_T0(t_rnd);
            if (go) {
                WalkPark wp{pslot, parked, false};
                if (f.px_rays && !parked) atomicAdd(f.px_rays + px.out, 1u);  // rt_debug_pixel_rays (diagnostics only)
                inw_segment<LIGHTS, WLN, FU, PK, QN>(S, f, K, s, col, dep, c, bu, &wp);
                parked = PK && wp.parked;
            }
#ifdef RT_DIAG_SPLIT
            c.rnd[round] += (unsigned long long)clock64() - t_rnd;
#endif
            if (busy && !parked && K.size == 0) {  // sample done: its sqrt(colour) (01_BVH...glsl:670) to the ring
                if constexpr (LR) {
                    const uint32_t e = g & rmask;
                    lr[RIX(0u, e)] = __builtin_sqrtf(col.x);
                    lr[RIX(1u, e)] = __builtin_sqrtf(col.y);
                    lr[RIX(2u, e)] = __builtin_sqrtf(col.z);
                } else {
                    wr[g & rmask] = make_float4(__builtin_sqrtf(col.x), __builtin_sqrtf(col.y), __builtin_sqrtf(col.z),
                                                __uint_as_float(ring_tag(S, g)));
                }
                if ((uint32_t)s == mid) pdep[pj] = dep;  // 01_BVH...glsl:667-668, stored with the pixel's colour
                busy = false;
            }
            // Bounce-walk fill: the wide walk of round 1 costs a wave the same
            // trips however few of its lanes hold a bounce ray, and primary rays (beam lists) are
            // cheap.  While fewer than kR1Min lanes hold a ray for round 1 and free lanes could take
            // more samples, skip round 1: the next iteration issues samples to the free lanes and
            // runs their primaries, and the bounce rays pile up for one fuller walk.  Every
            // iteration issues at least one entry while that holds, so the loop always advances.
            if (kR1Min > 0 && round == 0) {
                const uint32_t nb = (uint32_t)__popcll(__ballot(busy && K.size > 0u));
                const bool nfree = __ballot(!busy) != 0ull;
                const bool more = nfree && (uint64_t)(nclaimed - ji) * spp - si + (qdone ? 0u : 1u) > 0u &&
                                  gi - gf < rsize;
                if (nb < (uint32_t)kR1Min && more) break;
            }
        }
        INW_CYC(c, 4, t_seg);
    }
#ifdef RT_DIAG_SPLIT
    // phases 0-1 and 5-7 run inside `if (busy)`: the wave's time there is the largest of its lanes'
    for (int k = 0; k < 8; k++) {
        if (k >= 2 && k < 5) continue;
        for (int o = 32; o >= 1; o >>= 1) {
            const unsigned long long t = __shfl_xor(c.cyc[k], o, 64);
            c.cyc[k] = t > c.cyc[k] ? t : c.cyc[k];
        }
    }
    if (f.dbg && lane == 0) {
        for (int k = 0; k < 8; k++) atomicAdd(f.dbg + 8 + k, c.cyc[k]);
        atomicAdd(f.dbg + 24, c.rnd[0]);
        atomicAdd(f.dbg + 25, c.rnd[1]);
        // wall clock (100 MHz): first / last wave start, first queue drain, first / last wave exit
        const unsigned long long t_end = wall_clock64();
        unsigned long long *t = reinterpret_cast<unsigned long long *>(f.dbg) + 16;
        atomicMin(t, t_start); atomicMax(t + 1, t_start);
        if (t_qd) atomicMin(t + 2, t_qd);
        atomicMin(t + 3, t_end); atomicMax(t + 4, t_end);
    }
#endif
#ifdef RT_DIAG_OCC
    if (f.dbg && lane == 0)
        for (int k = 0; k < kOccSlots; k++) atomicAdd(f.dbg + 32 + k, c.occ[k]);
#endif
    flush(f, c);
}

// sample-major stream (see above): entry g = block ordinal b, sample s, pixel p (b * 64 * spp + s * 64 + p)
// LRING: the fold ring in LDS after the first kPmLdsNodes staged nodes, as k_inw_pm's (InwScene::
// lring_sm: chosen when the scene's BVH top fits those nodes, so the staging loses nothing)
template <bool LIGHTS, bool LN = false, bool FU = false, bool LRING = false>
__global__ __launch_bounds__(LN ? 3 * kBlock : kBlock) __attribute__((amdgpu_waves_per_eu(LN ? 3 : (LIGHTS ? RT_INW_WAVES : RT_INW01_WAVES)))) void k_inw_sm(Frame f, InwScene S0, float4 *ring, uint32_t rmask, unsigned *counter, const uint32_t *mode, uint32_t force, const uint32_t *) {
    if (!inw_sample_major(mode, force)) return;  // the probe picked k_inw_pm for this frame
    constexpr int SUB = LN ? 3 : 1;
    constexpr bool LR = LN && LRING;
    __shared__ float lds[SUB * kFStack * kBlock];
    InwScene S = S0;
    if constexpr (LN) {
        const uint32_t cap = LR ? (uint32_t)kPmLdsNodes : (uint32_t)kInwLdsNodes;
        const uint32_t n = S.wnodes ? (S.n_wnodes < cap ? S.n_wnodes : cap) : 0u;
        for (uint32_t i = threadIdx.x; i < n * (uint32_t)kInwNodeF4; i += SUB * kBlock) g_inw_lnodes[i] = S.wnodes[i];
        const uint32_t nb = (!S.wnodes && S.sl) ? min(2u * S.n - 1u, cap * (uint32_t)kInwNodeF4 / 2u) : 0u;
        for (uint32_t i = threadIdx.x; i < 2u * nb; i += SUB * kBlock) g_inw_lnodes[i] = S.nodes[i];
        __syncthreads();
        S.n_lnodes = n;
        S.n_blds = nb;
    }
    Ctr c;
    FStack K{lds + (threadIdx.x / kBlock) * (kFStack * kBlock) + (threadIdx.x % kBlock), 0};
    const uint32_t lane = threadIdx.x & 63u;
    if constexpr (LR) rmask = kPmLdsRing - 1u;
    const uint32_t rsize = rmask + 1u;
    float4 *wr = ring + (size_t)uni((blockIdx.x * (SUB * kBlock) + threadIdx.x) >> 6) * rsize;
    // LR: this wave's ring, three planes (r, g, b) of kPmLdsRing floats
    float *lr = reinterpret_cast<float *>(g_inw_lnodes + kPmLdsNodes * kInwNodeF4) + uni((threadIdx.x >> 6) * (3u * kPmLdsRing));
    const uint32_t spp = (uint32_t)f.spp, mid = spp / 2u, nblk = units_total(f) / 64u;
    const uint32_t E = 64u * spp;  // entries per block
    const float inv = rcp((float)f.spp);
    // wave-uniform issue state: next entry = offset ei of block ordinal bi; gi = bi * E + ei
    uint32_t gi = 0, bi = 0, ei = 0, nclaimed = 0;
    bool qdone = false;
    uint32_t blk_slot = 0xffffffffu;  // lane l: the block id of ordinal j with j % 64 == l
    // per-lane fold state: pixel `lane` of block ordinal bf, next sample sf
    uint32_t bf = 0, sf = 0;
    f3 acc = f3{0, 0, 0};
    // per-lane trace state
    bool busy = false;
    uint32_t g = 0;
    int s = 0;
    UnitPix px{};
    f3 col = f3{0, 0, 0};
    float dep = 0.0f;
    K.size = 0;
    for (;;) {
        // ---- fold: lane p adds the finished samples of its pixel, in order (up to 2 per iteration)
        {
            if constexpr (!LR) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): this wave's ring stores have landed (same CU: L1 write-through)
            // LR: every issued entry is either held by a busy lane or stored (LDS ops of one wave
            // complete in order), so the issued entries below the oldest one a busy lane holds are
            // finished: no tags (the window keeps every unfolded entry from being overwritten)
            uint32_t hold = 0u;
            if constexpr (LR) hold = uni(__ockl_wfred_min_u32(busy ? g - (gi - rsize) : 0xffffffffu));
            const uint32_t my_blk = (uint32_t)__shfl((int)blk_slot, (int)(bf & 63u), 64);
            if (bf != nclaimed) {
                uint32_t gg[2];
                float4 v[2];
                bool fin[2];
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    const uint32_t sk = sf + (uint32_t)k;
                    gg[k] = bf * E + (sk < spp ? sk : spp - 1u) * 64u + lane;
                    const uint32_t rel = gg[k] - (gi - rsize);
                    const bool ok = sk < spp && rel < rsize;  // issued (and inside the window)
                    if constexpr (LR) {
                        fin[k] = ok && rel < hold;
                        const uint32_t e = gg[k] & rmask;
                        v[k] = fin[k] ? make_float4(lr[e], lr[kPmLdsRing + e], lr[2u * kPmLdsRing + e], 0.0f)
                                      : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    } else {
                        v[k] = ok ? wr[gg[k] & rmask] : make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(~ring_tag(S, gg[k])));
                        fin[k] = __float_as_uint(v[k].w) == ring_tag(S, gg[k]);
                    }
                }
#pragma unroll
                for (int k = 0; k < 2; k++) {
                    if (!fin[k] || sf == spp) break;
                    const f3 gv = f3{v[k].x, v[k].y, v[k].z};
                    acc = sf == 0 ? gv : acc + gv;
                    if (++sf == spp) {  // pixel complete: End()'s imageStore (01_BVH...glsl:652)
                        const UnitPix p = unit_pixel(f, my_blk * 64u + lane);
                        if (p.out != (size_t)-1)
                            fb_store(f, p.out,
                                     make_float4(p.in_image ? acc.x * inv : 0.0f, p.in_image ? acc.y * inv : 0.0f,
                                                 p.in_image ? acc.z * inv : 0.0f, p.in_image ? 1.0f : 0.0f));
                    }
                }
                if (sf == spp) { sf = 0; bf++; }
            }
        }
        // the ring window starts at the oldest unfolded entry of the wave (a lane whose next sample
        // is not issued yet holds nothing back)
        const uint32_t gnext = bf == nclaimed ? gi : bf * E + sf * 64u + lane;
        const int dl = (int)(gi - gnext);
        uint32_t dmax = dl > 0 ? (uint32_t)dl : 0u, bmin = bf;
        for (int o = 32; o >= 1; o >>= 1) {
            const uint32_t t = (uint32_t)__shfl_xor((int)dmax, o, 64), tb = (uint32_t)__shfl_xor((int)bmin, o, 64);
            dmax = t > dmax ? t : dmax;
            bmin = tb < bmin ? tb : bmin;
        }
        dmax = uni(dmax);
        bmin = uni(bmin);
        // ---- claim blocks for the free lanes (at most 64 blocks between fold and issue)
        const unsigned long long fm = __ballot(!busy);
        const uint32_t nfree = (uint32_t)__popcll(fm);
        if (!qdone && nfree) {
            uint32_t need = bi + (ei + nfree - 1u) / E + 1u;
            if (need > bmin + 64u) need = bmin + 64u;
            if (need > nclaimed) {
                const uint32_t want = need - nclaimed;
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(counter, want);
                base = uni((uint32_t)__shfl((int)base, 0, 64));
                uint32_t got = want;
                if (base >= nblk) { got = 0; qdone = true; }
                else if (base + want >= nblk) { got = nblk - base; qdone = true; }
                const uint32_t rel = (lane - nclaimed) & 63u;
                if (rel < got) blk_slot = base + rel;
                nclaimed += got;
            }
        }
        // ---- issue: free lanes take the next stream entries in lane order, inside the window
        {
            const uint32_t rank = (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
            uint32_t avail = rsize - dmax;
            const uint64_t left = (uint64_t)(nclaimed - bi) * E - ei;
            if ((uint64_t)avail > left) avail = (uint32_t)left;
            const uint32_t take = nfree < avail ? nfree : avail;
            if (take) {
                uint32_t b = bi, e = ei + rank;
                if (e >= E) { e -= E; b++; }
                const uint32_t blk = (uint32_t)__shfl((int)blk_slot, (int)(b & 63u), 64);
                if (!busy && rank < take) {
                    g = gi + rank;
                    s = (int)(e >> 6);
                    px = unit_pixel(f, blk * 64u + (e & 63u));
                    col = f3{0, 0, 0};
                    dep = 0.0f;
                    if (px.in_image) {
                        busy = true;
                        inw_start_sample(S, f, K, px.x, px.y, s, c);
                    } else {  // a padding slot: an empty sample, folded as zero
                        if ((uint32_t)s == mid && f.out_depth && px.out != (size_t)-1) depth_store(f, px.out, 0.0f);
                        if constexpr (LR) {
                            const uint32_t e = g & rmask;
                            lr[e] = 0.0f; lr[kPmLdsRing + e] = 0.0f; lr[2u * kPmLdsRing + e] = 0.0f;
                        } else wr[g & rmask] = make_float4(0.0f, 0.0f, 0.0f, __uint_as_float(ring_tag(S, g)));
                    }
                }
                gi += take;
                ei += take;
                if (ei >= E) { ei -= E; bi++; }
            }
        }
        if (qdone && bi == nclaimed && bmin == nclaimed && __ballot(busy) == 0) break;
        OCC_TALLY(c, kOccSeg, busy);
        if (busy) {
            inw_segment<LIGHTS, LN, FU>(S, f, K, s, col, dep, c);
            if (f.px_rays) atomicAdd(f.px_rays + px.out, 1u);  // rt_debug_pixel_rays (diagnostics only)
        }
        if (busy && K.size == 0) {  // sample done: its sqrt(colour) (01_BVH...glsl:670) to the ring
            if constexpr (LR) {
                const uint32_t e = g & rmask;
                lr[e] = __builtin_sqrtf(col.x);
                lr[kPmLdsRing + e] = __builtin_sqrtf(col.y);
                lr[2u * kPmLdsRing + e] = __builtin_sqrtf(col.z);
            } else
                wr[g & rmask] = make_float4(__builtin_sqrtf(col.x), __builtin_sqrtf(col.y), __builtin_sqrtf(col.z),
                                            __uint_as_float(ring_tag(S, g)));
            if ((uint32_t)s == mid && f.out_depth) depth_store(f, px.out, dep);  // 01_BVH...glsl:667-668
            busy = false;
        }
    }
#ifdef RT_DIAG_OCC
    if (f.dbg && lane == 0)
        for (int k = 0; k < kOccSlots; k++) atomicAdd(f.dbg + 32 + k, c.occ[k]);
#endif
    flush(f, c);
}


// ============================================================================ launch
uint32_t units_of(const Frame &f) {
    return f.tiles ? (uint32_t)f.n_tiles * f.tile_size * f.tile_size
                   : (uint32_t)(((f.tw + 7) >> 3) * ((f.th + 7) >> 3)) * 64u;
}
static unsigned grid_of(uint32_t units, int blocks_cap) {
    uint64_t b = ((uint64_t)units + kBlock - 1) / kBlock;
    if (b > (uint64_t)blocks_cap) b = blocks_cap;
    return (unsigned)(b ? b : 1);
}
static dim3 grid_iow01(const Frame &f) {
    if (f.tiles) { const int per = f.tile_size >> 4; return dim3((unsigned)(f.n_tiles * per * per)); }
    return dim3((unsigned)(((f.tw + 15) >> 4) * ((f.th + 15) >> 4)));
}

bool iow_narrow(const Frame &f) {  // A/B switch (measured slower: VGPR spills)
    return f.max_bounces <= 255 && f.narrow != 0;
}

// the LDS-node kernels (k_iow03L / k_iow03sL) when the BVH fits and rt_options.iow_lds_bvh is on
bool iow_lds(const IowScene &sc) {
    return sc.lds_on && sc.nodes != nullptr && sc.n_nodes > 0 && sc.n_nodes <= (uint32_t)kIowLdsNodes;
}

int resident_blocks_per_cu(int kind) {
    int nb = 0;
    hipError_t e;
    if (kind == 3) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_iow03, kBlock, 0);
    else if (kind == 9) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_iow03L, 3 * kBlock, 0);
    else if (kind == 10) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_iow03sL, 3 * kBlock, 0);
    else if (kind == 4) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_iow03n, kBlock, 0);
    else if (kind == 5) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_iow03s, kBlock, 0);
    else if (kind == 14) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_inw<true>, kBlock, 0);
    else if (kind == 15) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_inw_pm<false>, kBlock, 0);
    else if (kind == 16) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_inw_pm<true>, kBlock, 0);
    else if (kind == 17) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_inw_pm<false, true>, 3 * kBlock, 0);
    else if (kind == 18) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_inw_pm<true, true>, 3 * kBlock, 0);
    else if (kind == 19)
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_inw_pm<false, true, true, true, true>, pm_sub<true, true>() * kBlock, 0);
    else e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_inw<false>, kBlock, 0);
    return (e == hipSuccess && nb > 0) ? nb : 2;
}

hipError_t launch_iow01(const Frame &f, hipStream_t s) {
    hipLaunchKernelGGL(k_iow01, grid_iow01(f), dim3(kBlock), 0, s, f);
    return hipGetLastError();
}
hipError_t launch_iow03(const Frame &f, const IowScene &sc, const Chunk &ch, const Cont &ct, uint32_t n_units,
                        unsigned *counter, int s_stop, int blocks_cap, hipStream_t s) {
    hipError_t e = hipMemsetAsync(counter, 0, sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    if (!iow_narrow(f) && iow_lds(sc)) {
        const dim3 g(grid_of((n_units + 2) / 3, blocks_cap / 3));  // blocks_cap counts 256-lane slots
        hipLaunchKernelGGL(k_iow03L, g, dim3(3 * kBlock), 0, s, f, sc, ch, ct, counter, s_stop);
        return hipGetLastError();
    }
    const dim3 g(grid_of(n_units, blocks_cap));
    if (iow_narrow(f)) hipLaunchKernelGGL(k_iow03n, g, dim3(kBlock), 0, s, f, sc, ch, ct, counter, s_stop);
    else hipLaunchKernelGGL(k_iow03, g, dim3(kBlock), 0, s, f, sc, ch, ct, counter, s_stop);
    return hipGetLastError();
}
hipError_t launch_iow03_spec(const Frame &f, const IowScene &sc, const SpecRecs &R, int mode, const Cont &ct,
                             uint32_t n_units, unsigned *counter, int blocks_cap, hipStream_t s) {
    hipError_t e = hipMemsetAsync(counter, 0, sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    if (iow_lds(sc))
        hipLaunchKernelGGL(k_iow03sL, dim3(grid_of((n_units + 2) / 3, blocks_cap / 3)), dim3(3 * kBlock), 0, s, f, sc, R,
                           mode, ct, counter);
    else
        hipLaunchKernelGGL(k_iow03s, dim3(grid_of(n_units, blocks_cap)), dim3(kBlock), 0, s, f, sc, R, mode, ct,
                           counter);
    return hipGetLastError();
}
// diagnostics: log2 histogram of rays per sample over the last sample-parallel render
__global__ void k_spec_hist(const uint4 *ctr, size_t n, unsigned long long *out) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned v = ctr[i].x;
        if (v == 0) continue;
        const int b = 31 - __clz(v);
        atomicAdd(out + 2 + b, 1ull);
        atomicAdd(out + 34 + b, (unsigned long long)v);
        atomicMax(out, (unsigned long long)v);
        atomicAdd(out + 1, 1ull);
    }
}
// diagnostics: per pixel unit (sample-0 rays, max rays of a sample, that sample, rank in `order`)
__global__ void k_spec_pixels(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *order, uint32_t *out) {
    const uint32_t pu = blockIdx.x * blockDim.x + threadIdx.x;
    if (pu >= P) return;  // no cross-lane work in this kernel
    uint32_t mx = 0, arg = 0;
    for (uint32_t s = 0; s < S; s++) {
        const uint32_t v = ctr[(size_t)pu * S + s].x;
        if (v > mx) { mx = v; arg = s; }
    }
    out[4 * (size_t)pu] = ctr[(size_t)pu * S].x;
    out[4 * (size_t)pu + 1] = mx;
    out[4 * (size_t)pu + 2] = arg;
    out[4 * (size_t)order[pu] + 3] = pu;  // out[.3] of row r = the pixel at order rank r
}
hipError_t spec_pixels(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *order, uint32_t *d_out,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_spec_pixels, dim3((P + 255) / 256), dim3(256), 0, s, ctr, P, S, order, d_out);
    return hipGetLastError();
}
// diagnostics: where re-executed samples first read a stale entry (RT_DEBUG_FIRST_STALE runs):
// out[b] = samples, out[16 + b] = their rays, bucket b = 16 * first_stale_segment / rays
__global__ void k_spec_list_stale(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *list, const unsigned *count,
                                  unsigned long long *out) {
    const unsigned n = *count;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 c = ctr[spec_rec_ix(list[i], P, S)];
        if (!(c.y & 0x80000000u) || c.x == 0) continue;
        const unsigned b = min(15u, (unsigned)(((unsigned long long)(c.y & 0x7fffffffu) * 16ull) / c.x));
        atomicAdd(out + b, 1ull);
        atomicAdd(out + 16 + b, (unsigned long long)c.x);
    }
}
hipError_t spec_list_stale(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *list, const unsigned *count,
                           unsigned long long *d_out, hipStream_t s) {
    hipLaunchKernelGGL(k_spec_list_stale, dim3(1024), dim3(256), 0, s, ctr, P, S, list, count, d_out);
    return hipGetLastError();
}
// diagnostics: log2 histogram of the rays of the samples on the (first) re-execution list
__global__ void k_spec_list_hist(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *list, const unsigned *count,
                                 unsigned long long *out) {
    const unsigned n = *count;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const unsigned v = ctr[spec_rec_ix(list[i], P, S)].x;
        if (v == 0) continue;
        const int b = 31 - __clz(v);
        atomicAdd(out + 2 + b, 1ull);
        atomicAdd(out + 34 + b, (unsigned long long)v);
        atomicMax(out, (unsigned long long)v);
        atomicAdd(out + 1, 1ull);
    }
}
hipError_t spec_list_hist(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *list, const unsigned *count,
                          unsigned long long *d_out, hipStream_t s) {
    hipLaunchKernelGGL(k_spec_list_hist, dim3(1024), dim3(256), 0, s, ctr, P, S, list, count, d_out);
    return hipGetLastError();
}
hipError_t spec_hist(const uint4 *ctr, size_t n, unsigned long long *d_out, hipStream_t s) {
    hipLaunchKernelGGL(k_spec_hist, dim3(2048), dim3(256), 0, s, ctr, n, d_out);
    return hipGetLastError();
}
__global__ void k_spec_list_keys(SpecRecs R, unsigned *keys, size_t n) {
    const unsigned cnt = *R.list_count;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        keys[i] = i < cnt ? min(R.ctr[R.ix(R.list[i])].x, 0xffffffu) : 0u;
}
hipError_t spec_list_keys(const SpecRecs &R, unsigned *keys, size_t n, hipStream_t s) {
    hipLaunchKernelGGL(k_spec_list_keys, dim3(4096), dim3(256), 0, s, R, keys, n);
    return hipGetLastError();
}
// ---------------------------------------------------------------- heavy-first enumeration
// cost of sample index s (1..S-1) over the probe pixels: finished records (block s-1)
__global__ __launch_bounds__(kBlock) void k_sample_cost(SpecRecs R, unsigned long long *fcost) {
    __shared__ unsigned long long part[kBlock / 64];
    const uint32_t s = blockIdx.x + 1u;
    const uint32_t n_px = R.order_n ? R.order_n : R.P;
    const unsigned done_tag = (1u << 8) | ((R.epoch & 0xffffu) << 16);
    unsigned long long acc = 0;
    for (uint32_t i = threadIdx.x; (size_t)i * R.probe_stride < n_px; i += kBlock) {
        const size_t u = (size_t)s * R.P + R.order[R.order_base + i * R.probe_stride];
        if ((__float_as_uint(R.col[R.ix(u)].w) & 0xffff0100u) == done_tag) acc += R.ctr[R.ix(u)].x;
    }
    acc = wave_sum(acc);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < kBlock / 64; w++) t += part[w];
        atomicAdd(fcost + s, t);
    }
}
// progress of the parked lanes (the long samples still running) counts toward their index
__global__ __launch_bounds__(kBlock) void k_sample_cost_parked(SpecRecs R, const float4 *cont, const unsigned *count,
                                                               unsigned long long *fcost) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= *count) return;  // no cross-lane work in this kernel
    const float4 *p = cont + (size_t)i * kContSlots;
    if (p[12].y != 0.0f) return;
    const uint32_t u = __float_as_uint(p[0].x);
    atomicAdd(fcost + u / R.P, (unsigned long long)__float_as_uint(p[2].x));
}
// rank the indices 1..S-1 by cost, most expensive first (ties: lower index first)
__global__ __launch_bounds__(1024) void k_sample_rank(SpecRecs R, const unsigned long long *fcost, uint32_t *sorder) {
    for (uint32_t s = 1u + threadIdx.x; s < R.S; s += 1024u) {
        const unsigned long long c = fcost[s];
        uint32_t rank = 0;
        for (uint32_t t = 1; t < R.S; t++) rank += (fcost[t] > c || (fcost[t] == c && t < s)) ? 1u : 0u;
        sorder[rank] = s;
    }
}
// per pixel: the most rays among its heavy samples (finished records), for the re-sort
__global__ __launch_bounds__(kBlock) void k_pixel_key(Frame f, SpecRecs R, unsigned *key) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    const uint32_t n_px = R.order_n ? R.order_n : R.P;
    if (i >= n_px) return;  // no cross-lane work in this kernel
    const uint32_t pu = R.order[R.order_base + i];
    const unsigned done_tag = (1u << 8) | ((R.epoch & 0xffffu) << 16);
    unsigned k = R.ctr[R.ix(pu)].x;  // sample 0
    for (uint32_t j = 0; j < R.n_heavy; j++) {
        const size_t u = (size_t)R.sorder[j] * R.P + pu;
        if ((__float_as_uint(R.col[R.ix(u)].w) & 0xffff0100u) == done_tag) k = max(k, R.ctr[R.ix(u)].x);
    }
    key[pu] = unit_pixel(f, pu).in_image ? k : 0u;
}
__global__ __launch_bounds__(kBlock) void k_pixel_key_parked(SpecRecs R, const float4 *cont, const unsigned *count,
                                                             unsigned *key) {
    const uint32_t i = blockIdx.x * kBlock + threadIdx.x;
    if (i >= *count) return;  // no cross-lane work in this kernel
    const float4 *p = cont + (size_t)i * kContSlots;
    if (p[12].y != 0.0f) return;
    const uint32_t u = __float_as_uint(p[0].x);
    atomicMax(key + u % R.P, __float_as_uint(p[2].x));
}
hipError_t launch_iow03_sample_order(const Frame &f, const SpecRecs &R, const float4 *cont, const unsigned *count,
                                     int max_lanes, unsigned long long *fcost, uint32_t *sorder, hipStream_t s) {
    hipError_t e = hipMemsetAsync(fcost, 0, sizeof(unsigned long long) * R.S, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sample_cost, dim3(R.S - 1u), dim3(kBlock), 0, s, R, fcost);
    const unsigned blocks = (unsigned)((max_lanes + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_sample_cost_parked, dim3(blocks ? blocks : 1), dim3(kBlock), 0, s, R, cont, count, fcost);
    hipLaunchKernelGGL(k_sample_rank, dim3(1), dim3(1024), 0, s, R, fcost, sorder);
    return hipGetLastError();
}
hipError_t launch_iow03_pixel_key(const Frame &f, const SpecRecs &R, const float4 *cont, const unsigned *count,
                                  int max_lanes, unsigned *key, hipStream_t s) {
    const uint32_t n_px = R.order_n ? R.order_n : R.P;
    hipLaunchKernelGGL(k_pixel_key, dim3((n_px + kBlock - 1) / kBlock), dim3(kBlock), 0, s, f, R, key);
    const unsigned blocks = (unsigned)((max_lanes + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_pixel_key_parked, dim3(blocks ? blocks : 1), dim3(kBlock), 0, s, R, cont, count, key);
    return hipGetLastError();
}
hipError_t launch_iow03_frontier(const Frame &f, const SpecRecs &R, float4 *cont, unsigned *count, uint32_t cap,
                                 hipStream_t s) {
    const uint32_t n = R.order_n ? R.order_n : R.P;
    hipLaunchKernelGGL(k_iow03_frontier, dim3((n + kBlock - 1) / kBlock), dim3(kBlock), 0, s, f, R, cont, count, cap);
    return hipGetLastError();
}
hipError_t launch_iow03_altspawn(const Frame &f, const SpecRecs &R, float4 *cont, unsigned *count, uint32_t cap,
                                 hipStream_t s) {
    const uint32_t n = R.order_n ? R.order_n : R.P;
    const unsigned blocks = (n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_iow03_altspawn, dim3(blocks ? blocks : 1), dim3(kBlock), 0, s, f, R, cont, count, cap);
    return hipGetLastError();
}
hipError_t launch_iow03_fixf(const Frame &f, const SpecRecs &R, float4 *cont, const unsigned *count, int max_lanes,
                             hipStream_t s) {
    const unsigned blocks = (unsigned)((max_lanes + kBlock - 1) / kBlock);
    hipLaunchKernelGGL(k_iow03_fixf, dim3(blocks ? blocks : 1), dim3(kBlock), 0, s, f, R, cont, count);
    return hipGetLastError();
}
hipError_t launch_iow03_prep(const Frame &f, const SpecRecs &R, unsigned *key, float prior, uint32_t prior_from,
                             hipStream_t s) {
    const unsigned blocks = (R.P + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_iow03_prep, dim3(blocks ? blocks : 1), dim3(kBlock), 0, s, f, R, key, prior, prior_from);
    return hipGetLastError();
}
hipError_t launch_iow03_resolve(const Frame &f, const SpecRecs &R, bool final_pass, float4 *state, hipStream_t s) {
    const unsigned blocks = ((R.order_n ? R.order_n : R.P) + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(k_iow03_resolve, dim3(blocks ? blocks : 1), dim3(kBlock), 0, s, f, R, final_pass ? 1 : 0, state);
    return hipGetLastError();
}
hipError_t launch_inw_beam(const Frame &f, const InwScene &sc, const uint32_t *mode, uint32_t force, hipStream_t s) {
    const uint32_t n = units_of(f);
    const uint32_t nb = sc.beam_bins > 1u ? sc.beam_bins : 1u;
    hipLaunchKernelGGL(k_inw_beam, dim3((n + kBeamBlock - 1) / kBeamBlock, nb), dim3(kBeamBlock), 0, s, f, sc, mode, force);
    return hipGetLastError();
}
// One frame of the on-chip-fold INW kernels: the probe (unless forced), then k_inw_pm and
// k_inw_sm, of which the one the probe did not pick exits at once.  ring: blocks * 4 waves *
// max(ring_pm, ring_sm) float4; mode: 2 uints (zeroed here).  force: 0 = probe, 1 = pm, 2 = sm.
hipError_t launch_inw_fold(const Frame &f, const InwScene &sc, float4 *ring, uint32_t ring_pm, uint32_t ring_sm,
                           unsigned *counter, uint32_t *mode, uint32_t force, int blocks, int blocks_ln,
                           uint32_t *cost, hipStream_t s) {
    for (uint32_t r : {ring_pm, ring_sm})
        if (r < 64 || (r & (r - 1))) return hipErrorInvalidValue;
    hipError_t e = hipMemsetAsync(mode, 0, 2 * sizeof(uint32_t), s);
    if (e != hipSuccess) return e;
    // the probe first: the claim-order and beam kernels below read its verdict and exit at once
    // on a sample-major frame
    if (force == 0) {
        const uint32_t nblk = units_of(f) / 64u, waves = 1024u;  // ~1024 probe blocks of 8x8 pixels
        const uint32_t stride = nblk > waves ? nblk / waves : 1u, nw = (nblk + stride - 1u) / stride;
        const dim3 g((nw + 3u) / 4u);
        if (sc.layout == 4) hipLaunchKernelGGL(k_inw_probe<true>, g, dim3(kBlock), 0, s, f, sc, stride, mode);
        else hipLaunchKernelGGL(k_inw_probe<false>, g, dim3(kBlock), 0, s, f, sc, stride, mode);
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    // claim order of k_inw_pm (cost: 2 * nblk + 256 uints, or null = unit order)
    const uint32_t *border = nullptr;
    if (cost && units_of(f) >= 64u) {
        const uint32_t nblk = units_of(f) / 64u;
        uint32_t *key = cost, *order = cost + nblk, *hist = cost + 2 * nblk;
        if ((e = hipMemsetAsync(hist, 0, 256 * sizeof(uint32_t), s)) != hipSuccess) return e;
        const dim3 g((nblk + 3u) / 4u);  // 4 blocks of 8x8 pixels per 256-lane block
        if (sc.layout == 4) hipLaunchKernelGGL(k_inw_cost<true>, g, dim3(kBlock), 0, s, f, sc, key, hist, mode, force);
        else hipLaunchKernelGGL(k_inw_cost<false>, g, dim3(kBlock), 0, s, f, sc, key, hist, mode, force);
        hipLaunchKernelGGL(k_inw_order_scan, dim3(1), dim3(256), 0, s, hist, mode, force);
        hipLaunchKernelGGL(k_inw_order_scatter, dim3((nblk + kBlock - 1) / kBlock), dim3(kBlock), 0, s, key, hist,
                           order, nblk, mode, force);
        if ((e = hipGetLastError()) != hipSuccess) return e;
        border = order;
    }
    if (sc.beam && (e = launch_inw_beam(f, sc, mode, force, s)) != hipSuccess) return e;
    for (int k = 0; k < 2; k++) {  // (pm, then sm) each with its own queue counter
        if ((e = hipMemsetAsync(counter + 16 * k, 0, sizeof(unsigned), s)) != hipSuccess) return e;
        if (k == 0 && sc.xcdq && (e = hipMemsetAsync(counter + 64, 0, 8 * 16 * sizeof(unsigned), s)) != hipSuccess)
            return e;  // k_inw_pm's per-XCD queues
        const uint32_t rm = (k == 0 ? ring_pm : ring_sm) - 1u;
        unsigned *ctr = counter + 16 * k;
        if (blocks_ln > 0) {  // the LDS-staged BVH top (768-lane blocks); FU: the fused-fma cull
            const dim3 g(blocks_ln), b(3 * kBlock);
#define RT_INW_LN_LAUNCH(L, F)                                                                              \
    do {                                                                                                    \
        if (k == 0 && sc.lring) hipLaunchKernelGGL((k_inw_pm<L, true, F, true>), g, b, 0, s, f, sc, ring, rm, ctr, mode, force, border); \
        else if (k == 0) hipLaunchKernelGGL((k_inw_pm<L, true, F>), g, b, 0, s, f, sc, ring, rm, ctr, mode, force, border); \
        else if (sc.lring_sm) hipLaunchKernelGGL((k_inw_sm<L, true, F, true>), g, b, 0, s, f, sc, ring, rm, ctr, mode, force, border); \
        else hipLaunchKernelGGL((k_inw_sm<L, true, F>), g, b, 0, s, f, sc, ring, rm, ctr, mode, force, border);        \
    } while (0)
            if (k == 0 && sc.layout != 4 && sc.fused && sc.lring && sc.gstk && sc.gq_blocks)  // GQ
                hipLaunchKernelGGL((k_inw_pm<false, true, true, true, true>), dim3(sc.gq_blocks),
                                   dim3(pm_sub<true, true>() * kBlock), 0, s, f, sc, ring, rm, ctr, mode, force, border);
            else if (sc.layout == 4) {
                if (sc.fused) RT_INW_LN_LAUNCH(true, true);
                else RT_INW_LN_LAUNCH(true, false);
            } else {
                if (sc.fused) RT_INW_LN_LAUNCH(false, true);
                else RT_INW_LN_LAUNCH(false, false);
            }
#undef RT_INW_LN_LAUNCH
        } else if (sc.layout == 4) {
            if (k == 0) hipLaunchKernelGGL(k_inw_pm<true>, dim3(blocks), dim3(kBlock), 0, s, f, sc, ring, rm, counter, mode, force, border);
            else hipLaunchKernelGGL(k_inw_sm<true>, dim3(blocks), dim3(kBlock), 0, s, f, sc, ring, rm, counter + 16, mode, force, border);
        } else {
            if (k == 0) hipLaunchKernelGGL(k_inw_pm<false>, dim3(blocks), dim3(kBlock), 0, s, f, sc, ring, rm, counter, mode, force, border);
            else hipLaunchKernelGGL(k_inw_sm<false>, dim3(blocks), dim3(kBlock), 0, s, f, sc, ring, rm, counter + 16, mode, force, border);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}
hipError_t launch_inw(const Frame &f, const InwScene &sc, const Chunk &ch, const Cont &ct, uint32_t n_units,
                      unsigned *counter, int blocks_cap, hipStream_t s) {
    hipError_t e = hipMemsetAsync(counter, 0, sizeof(unsigned), s);
    if (e != hipSuccess) return e;
    const dim3 g(grid_of(n_units, blocks_cap));
    if (sc.layout == 4) hipLaunchKernelGGL(k_inw<true>, g, dim3(kBlock), 0, s, f, sc, ch, ct, counter);
    else hipLaunchKernelGGL(k_inw<false>, g, dim3(kBlock), 0, s, f, sc, ch, ct, counter);
    return hipGetLastError();
}

}  // namespace rtk

namespace rtk {
// The shortened sequences of rt_math.hpp against the compiler's correctly rounded ones over
// every bit pattern x (NaN == NaN): which 0 = rcp_sqrt_domain(sqrt(x)) vs 1.0f / sqrt(x).
// (An unscaled sqrt candidate failed here for 20.7M inputs, the denormal and tiny ones.)
__global__ __launch_bounds__(kBlock) void k_check_fastmath(int which, unsigned long long *bad, unsigned *first) {
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < (1ull << 32); i += stride) {
        const float xi = __uint_as_float((uint32_t)i);
        (void)which;
        const float b = __builtin_sqrtf(xi);
        const float x = rcp_sqrt_domain(b), y = 1.0f / b;
        if (__float_as_uint(x) != __float_as_uint(y) && !(x != x && y != y)) {
            atomicAdd(bad, 1ull);
            atomicMin(first, (uint32_t)i);
        }
    }
}
hipError_t launch_check_fastmath(int which, unsigned long long *bad, unsigned *first, hipStream_t s) {
    hipLaunchKernelGGL(k_check_fastmath, dim3(4096), dim3(kBlock), 0, s, which, bad, first);
    return hipGetLastError();
}
}  // namespace rtk
