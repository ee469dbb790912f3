// rt_capi.hip -- implementation of include/rt_hip.h and include/rt_scene.h.
//
// Owns device memory, converts the reference's record layouts into the kernels' device
// layouts (hot/cold split, per-object reciprocals hoisted under the numerics contract),
// builds the sample tables and launches.  No exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <algorithm>
#include <atomic>
#include <chrono>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/rt_hip.h"
#include "../../include/rt_scene.h"
#include "rt_host.hpp"
#include "rt_kernels.hpp"

namespace {

unsigned long long *g_dbg = nullptr;  // rt_debug_counters(): lane-occupancy diagnostics

// rt_options (include/rt_hip.h): the library-wide options; scenes copy them at creation
rt_options default_options() {
    rt_options o;
    std::memset(&o, 0, sizeof(o));
    o.size = sizeof(rt_options);
    o.inw_wide_walk = 1; o.inw_order = 0; o.inw_beams = 1; o.inw_ri_grid = 1; o.inw_lds_nodes = 1;
    o.inw_fused_cull = 1; o.inw_claim_order = 1; o.inw_ring_pm = 0; o.inw_ring_sm = 0; o.inw_stackless = 1;
    o.inw_device_build = 1; o.inw_claim_xcd = 1; o.inw_qnodes = 0; o.inw_time_bins = 2;
    o.inw_walk_bins = 1; o.inw_beam_bins = 1; o.inw_sphere_records = 1; o.inw_compact_nodes = 1;
    o.iow_spec = 1; o.iow_linear = 0; o.iow_narrow = 0; o.iow_lds_bvh = 1;
    o.iow_leaf_batch = 32;  // 32 measured 2.5% faster on the bench frame than 65 (round 2)
    o.iow_coop_max = 4; o.iow_chunks_lpt = 0;
    o.rounds_seq = 6; o.rounds_spec = 1; o.park_min = -1;
    o.spec_iters = 1; o.spec_probe = 64; o.spec_heavy = -1; o.spec_rounds = 24; o.spec_tail_rounds = 60;
    o.spec_tail_budget = 3072; o.spec_scan = 128; o.spec_chain = 1; o.spec_alt = 1; o.spec_alt_cap = 1 << 17;
    o.spec_alt_seg = 0; o.spec_alt_every = 0; o.spec_spread = 1; o.spec_prior_from = 2; o.spec_sort = 1;
    o.spec_solo = 4096; o.spec_validate = 1; o.spec_max_gb = 96.0;
    return o;
}
bool options_ok(const rt_options *o) {
    auto pow2 = [](int r) { return r >= 64 && r <= (1 << 16) && (r & (r - 1)) == 0; };
    return o && o->size == sizeof(rt_options) && o->inw_order >= -1 && o->inw_order <= 2 && (o->inw_ring_pm == 0 || pow2(o->inw_ring_pm)) &&
           (o->inw_ring_sm == 0 || pow2(o->inw_ring_sm)) && o->iow_leaf_batch >= 1 && o->iow_leaf_batch <= 65 && o->iow_coop_max >= 0 &&
           o->rounds_seq >= 0 && o->rounds_seq <= 14 && o->rounds_spec >= 0 && o->rounds_spec <= 14 &&
           o->park_min >= -1 && o->spec_iters >= 0 && o->spec_probe >= 1 && o->spec_heavy >= -1 &&
           o->spec_rounds >= 0 && o->spec_tail_rounds >= 0 && o->spec_tail_budget >= 1 && o->spec_scan >= 0 &&
           o->spec_alt_cap >= 1024 && o->spec_alt_cap <= (1 << 24) && o->spec_alt_seg >= 0 && o->spec_alt_every >= 0 &&
           o->spec_prior_from >= 1 && o->spec_solo >= 0 && o->spec_max_gb > 0.0 && o->inw_time_bins >= 0 &&
           o->inw_time_bins <= 16;
}
rt_options g_opt = default_options();
unsigned *g_px_rays = nullptr;        // rt_debug_pixel_rays(): rays per work unit
int g_build_levels = 0;               // rt_debug_build_level_cap(): the device build's level cap (0 = 256)

#define HIP_OK(expr)                                             \
    do {                                                         \
        hipError_t e_ = (expr);                                  \
        if (e_ != hipSuccess) {                                  \
            std::fprintf(stderr, "[rt_hip] %s failed: %s\n", #expr, hipGetErrorString(e_)); \
            return RT_E_HIP;                                     \
        }                                                        \
    } while (0)

struct DevBuf {  // RAII device allocation
    void *p = nullptr;
    size_t bytes = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    ~DevBuf() { if (p) (void)hipFree(p); }
    hipError_t alloc(size_t b) { bytes = b; return hipMalloc(&p, b ? b : 16); }
    hipError_t upload(const void *src, size_t b) {
        hipError_t e = alloc(b);
        if (e != hipSuccess || !b) return e;
        return hipMemcpy(p, src, b, hipMemcpyHostToDevice);
    }
    // at least b bytes of capacity (contents undefined; `bytes` stays the capacity)
    hipError_t reserve(size_t b) {
        if (p && bytes >= b) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; }
        return alloc(b);
    }
    // copy b bytes in, reusing the allocation when it is large enough (a scene update); `bytes`
    // stays the capacity
    hipError_t store(const void *src, size_t b) {
        if (!p || b > bytes) {
            if (p) { (void)hipFree(p); p = nullptr; }
            hipError_t e = alloc(b);
            if (e != hipSuccess) return e;
        }
        return b ? hipMemcpy(p, src, b, hipMemcpyHostToDevice) : hipSuccess;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

int check_device(int device) {
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || count <= 0) return RT_E_NODEVICE;
    if (device >= 0) {
        if (device >= count) return RT_E_NODEVICE;
        if (hipSetDevice(device) != hipSuccess) return RT_E_HIP;
    }
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return RT_E_HIP;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, cur) != hipSuccess) return RT_E_HIP;
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return RT_E_NODEVICE;
    return RT_OK;
}

bool params_ok(const rt_params *p) {
    return p && p->width > 0 && p->height > 0 && p->spp >= 1 && p->max_bounces >= 0;
}

// Uniforms of one dispatch.  screen_dist = 1/(2 tan(FOV/2)) is evaluated on the host in
// double and rounded (contract: transcendentals only on the host).
rtk::Frame make_frame(const rt_camera *cam, const rt_params *p) {
    rtk::Frame f;
    std::memset(&f, 0, sizeof(f));
    f.W = p->width; f.H = p->height; f.spp = p->spp; f.max_bounces = p->max_bounces;
    f.show_normal = p->show_normal;
    if (p->tile_w > 0 && p->tile_h > 0) { f.x0 = p->tile_x0; f.y0 = p->tile_y0; f.tw = p->tile_w; f.th = p->tile_h; }
    else { f.x0 = 0; f.y0 = 0; f.tw = p->width; f.th = p->height; }
    if (cam) {
        std::memcpy(f.pos, cam->pos, sizeof(f.pos));
        std::memcpy(f.dir, cam->dir, sizeof(f.dir));
        f.aperture = cam->aperture;
        f.focus = cam->focus_dist;
        f.screen_dist = 1.0f / (2.0f * (float)std::tan((double)(cam->fov_y_rad * 0.5f)));
    }
    f.inv_spp = 1.0f / (float)p->spp;
    f.dbg = g_dbg;
    f.px_rays = g_px_rays;
    // leaf_batch / coop_max / narrow come from the scene's options (launch_scene)
#ifdef RT_DIAG  // diagnostic builds only (make variant VDEFS=-DRT_DIAG)
    const char *fs = std::getenv("RT_DEBUG_FIRST_STALE");
    f.dbg_first_stale = (fs && fs[0] == '1') ? 1 : 0;
#endif
    return f;
}

}  // namespace

// A prepared scene: device-resident records, LBVH nodes, lights and sample tables.
struct rt_dev_scene {
    rt_options opt = g_opt;  // the options current when the scene was created (rt_dev_scene_set_options)
    int kind = 0;  // 3 = IOW-03, 11/14 = INW layout 1/4
    int device = 0;
    int spp = 0;
    uint32_t n = 0, n_lights = 0;
    int layout = 0;
    int s_stop = 0;      // IOW-03: samples before the ring schedule's early return (== spp in practice)
    int blocks_cap = 0;  // persistent grid size: resident blocks the device can hold (max over variants)
    int cus = 0;
    int root_link = 0;   // IOW-03 culling BVH: leftData of the root
    uint32_t n_wide = 0; // IOW-03 culling BVH: 4-wide nodes
    float ri_prior = 1.0f;  // IOW-03: most common refractive index (sample-parallel guess)
    // IOW-03 alternative runs: the values a stale ray-stack RI can hold (0 for a never-written
    // entry, 1 for the camera ray, every material RI; 03...glsl:285-356), up to 8, else none
    float alt_vals[8] = {};
    int n_alt_vals = 0;
    DevBuf sp_alt, sp_alt_hash, sp_alt_count;
    uint32_t alt_cap = 0;
    int n_focus = 0;        // INW-01 MULTIFOCUS lens chain (0 = the reference's single focus)
    float focus[9] = {};
    DevBuf hot, cold, nodes, lights, sunflower, fib, ring, counter;
    DevBuf sph;           // INW sphere scenes: 2 float4 per object (rtk::InwScene::sph)
    bool sph_ok = false;
    DevBuf obox;  // IOW-03: per-object culling boxes (2 float4 each) for wave-cooperative queries
    DevBuf tex, tex_info;  // INW-04 material textures (float4 texels, (first, w, h, 0) per texture)
    DevBuf wnodes, wrank, wleaf;  // INW wide walk: culling BVH, depth-first ranks, LBVH leaf boxes
    DevBuf qnodes;                // ... the culling BVH quantised (4 float4 per node, rtk::inw_quantize_wnodes)
    DevBuf cnodes;                // ... without the repeated low planes (7 float4 per node, rtk::inw_compact_wnodes)
    DevBuf gstk;                  // k_inw_pm's GQ instance: the reference's 40-float stacks, 160 B per lane
    DevBuf walk_ctr;              // the last frame's closest-hit queries handed to the LBVH walks (u64)
    DevBuf ri_cells, ri_ids;      // INW surrounding-RI grid (cell offsets, object ids)
    float ri_lo[3] = {}, ri_hi[3] = {}, ri_inv[3] = {};
    int ri_dim[3] = {};
    int wdepth = 0;               // levels of the 4-wide culling BVH
    uint32_t n_wnodes = 0;        // its nodes (every tree)
    uint32_t n_wtree0 = 0;        // ... of the tree over the swept boxes (the first ones)
    uint32_t wbins = 1, wbin_stride = 0;  // time-bin trees after it (rtamd::InwWide::bins)
    bool ri_ok = false;           // the RI grid applies (ri_cells / ri_ids hold it)
    DevBuf lbvh_ws, aabb, lcnt;   // rt_dev_scene_inw_update: device LBVH workspace, object boxes, leaf counts
    DevBuf build_ws, ri_fill, ri_tmp;  // ... and the device build of the wide walk and RI grid (rt_build.hip)
    bool last_ln = false;         // the last INW fold launch used the LDS-staged kernels
    bool last_fu = false;         // ... their fused-fma cull instances
    uint32_t last_force = 0;      // ... its forced order (0: the probe's pick, read back from inw_mode)
    bool last_lring = false;      // ... k_inw_pm's fold ring was in LDS
    bool last_lring_sm = false;   // ... k_inw_sm's
    bool last_gq = false;         // ... k_inw_pm's GQ instance (quantised nodes, global stacks)
    char kname[64] = {0};         // the fold kernel's instance name (rt_debug_launches)
    uint32_t last_ring[2] = {0, 0};  // ... its fold windows (pixel-major, sample-major)
    uint32_t ring_frame = 0;         // frames rendered with the current fold rings (their tag epoch)
    bool broken = false;             // a failed rt_dev_scene_inw_update left the buffers inconsistent: no renders
    rt_path_info last_path{};     // rt_debug_path: what the last render ran
    float wbound = 0.0f;          // largest |coordinate| of the INW culling boxes (the fused cull's condition)
    uint32_t dfs_high = 0;        // the reference walk's stack high-water mark (0: no walkable LBVH)
    bool sl_ok = false;           // the node buffer has the stackless walks' layout (lbvh_walk_info)
    uint32_t wbuild = 0;          // where the walk structures were built: 0 host, 1 device, 2 host after the
                                  // device build ran past its level cap (rt_debug_wide_info info[7])
    uint32_t n_tex = 0;
    // chunked-render workspace, sized for `ws_units` pixel units (grown on demand)
    uint32_t ws_units = 0;
    size_t ws_temp_bytes = 0;
    DevBuf ws_state, ws_cost, ws_keys, ws_iota, ws_order, ws_temp;
    // tail-compaction continuation buffers (ping-pong), blocks_cap*kBlock slots each
    DevBuf cont[2], cont_count;
    // sample-parallel IOW-03 records, sized for spec_cap (pixel units x samples)
    size_t spec_cap = 0, spec_units = 0;
    uint32_t spec_P = 0, spec_S = 0;  // the last sample-parallel render's P and S (its record layout, SpecRecs::ix)
    DevBuf sp_col, sp_fin, sp_ctr, sp_assume, sp_list, sp_fb, sp_counts;
    DevBuf sp_keys, sp_keys2, sp_list2, sp_temp;  // longest-first ordering of the re-execution list
    DevBuf sp_pstate;  // asynchronous windows: per-pixel frontier state
    DevBuf sp_front;   // checkpoint rounds: per-pixel frontier (uint4)
    DevBuf sp_sorder, sp_fcost;  // heavy-first enumeration: sample indices by cost, their costs
    DevBuf inw_ring;             // k_inw_pm / k_inw_sm: the waves' fold rings
    DevBuf inw_park;             // RT_INW_PARK builds: parked walk state per lane
    DevBuf inw_mode;             // k_inw_probe's verdict (2 uints)
    DevBuf inw_cost;             // claim order: block cost keys, the order, 256 bucket offsets
    DevBuf inw_beam, inw_beam_n;  // pixel beams: beam_cap (id, entry t) per unit; count + cut per unit
    float sf_max = 0.0f;          // largest |x| + |y| of the sunflower lens table
    DevBuf sp_dbg_t;             // RT_DEBUG_TIMES diagnostics: per unit start / end launch
    size_t sp_dbg_n = 0;         // units (P * S) of the render that last wrote sp_dbg_t
    uint32_t launch_seq = 0;
    DevBuf sp_exact;             // RT_SPEC_ORACLE diagnostics: exact incoming state per sample
    size_t sp_exact_n = 0;
    bool sp_exact_valid = false;
    size_t sp_temp_bytes = 0;
    // launches of the render's main kernel in the last render (rt_debug_launches)
    int last_launches = 0;
    const char *last_kernel = "";
    int last_chunks = 0;  // sample chunks of the last render (rt_debug_chunks)
    // sample-parallel pipelines: one stream per pixel group, each with its own queue counter,
    // continuation buffers and sort scratch (rt_render_* calls on one scene must not overlap)
    struct GroupLane {
        hipStream_t st = nullptr;
        hipEvent_t done = nullptr;
        DevBuf counter, cont[2], cont_count, temp;
        size_t temp_bytes = 0;
        ~GroupLane() {
            if (done) (void)hipEventDestroy(done);
            if (st) (void)hipStreamDestroy(st);
        }
    };
    std::vector<std::unique_ptr<GroupLane>> lanes;
    hipEvent_t ev_start = nullptr;
    // rt_debug_time_kernels: HIP events around every launch of the main sample-parallel kernel
    std::vector<std::pair<hipEvent_t, hipEvent_t>> kt_ev;
    size_t kt_used = 0;
    unsigned epoch = 0;  // frame tag of the sample records (16 bits in their flags; next_spec_epoch)
    ~rt_dev_scene() {
        if (ev_start) (void)hipEventDestroy(ev_start);
    }
};

namespace {

int build_tables(rt_dev_scene *s, int spp) {
    std::vector<float> sf(size_t(spp) * 2), fib3(size_t(spp) * 3), fib4(size_t(spp) * 4, 0.0f);
    std::vector<int> ring(size_t(spp) * 2);
    rtamd::sample_tables(spp, sf.data(), fib3.data(), ring.data());
    for (int i = 0; i < spp; i++)
        for (int k = 0; k < 3; k++) fib4[size_t(i) * 4 + k] = fib3[size_t(i) * 3 + k];
    HIP_OK(s->sunflower.upload(sf.data(), sf.size() * sizeof(float)));
    s->sf_max = 0.0f;
    for (int i = 0; i < spp; i++)
        s->sf_max = std::fmax(s->sf_max, std::fabs(sf[size_t(i) * 2]) + std::fabs(sf[size_t(i) * 2 + 1]));
    HIP_OK(s->fib.upload(fib4.data(), fib4.size() * sizeof(float)));
    HIP_OK(s->ring.upload(ring.data(), ring.size() * sizeof(int)));
    s->spp = spp;
    s->s_stop = spp;
    for (int i = 0; i < spp; i++)
        if (ring[size_t(i) * 2] < 0) { s->s_stop = i; break; }
    HIP_OK(s->counter.alloc(1024));  // queue counters 64 B apart (the INW fold launches: two, + 8 XCD queues)
    HIP_OK(s->inw_mode.alloc(64));
    return RT_OK;
}

// Persistent grid = the blocks the device keeps resident (a work-queue kernel gains nothing
// from more: extra blocks would only start after the queue ran dry).
void set_residency(rt_dev_scene *s) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    s->cus = cus;
    s->blocks_cap = cus * rtk::resident_blocks_per_cu(s->kind);
    if (s->kind == 3)  // continuation buffers serve every IOW-03 variant
        s->blocks_cap = std::max({s->blocks_cap, cus * rtk::resident_blocks_per_cu(4), cus * rtk::resident_blocks_per_cu(5)});
    else  // and every INW variant
        s->blocks_cap = std::max(s->blocks_cap, cus * rtk::resident_blocks_per_cu(s->kind == 14 ? 7 : 6));
}

int make_iow03(rt_dev_scene *s, const float *types, const float *rec, uint32_t n, int spp) {
    std::vector<float> hot(size_t(n) * rtk::kIowHot, 0.0f), cold(size_t(n) * rtk::kIowCold, 0.0f);
    for (uint32_t j = 0; j < n; j++) {
        const float *r = rec + size_t(j) * 24;
        float *h = hot.data() + size_t(j) * rtk::kIowHot;
        float *c = cold.data() + size_t(j) * rtk::kIowCold;
        h[0] = r[0]; h[1] = r[1]; h[2] = r[2];
        h[3] = types[j];
        for (int k = 0; k < 9; k++) h[4 + k] = r[3 + k];
        for (int k = 0; k < 3; k++) { h[13 + k] = r[12 + k]; h[16 + k] = 1.0f / r[12 + k]; }
        for (int k = 0; k < 3; k++) { c[k] = r[15 + k]; c[3 + k] = r[18 + k]; }
        c[6] = r[21]; c[7] = r[22];
        // glm::mat3(1) bit pattern (+0 off-diagonal): the kernel may reuse the ray's
        // identity-transformed direction, which is bit-identical to transforming it here
        static const float kI[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        h[19] = std::memcmp(r + 3, kI, sizeof(kI)) == 0 ? 1.0f : 0.0f;
    }
    s->kind = 3; s->n = n;
    {  // most common RefractiveIndex (record float 20, Geometry::FillBuffer materials.h:48-76)
        std::vector<float> ri(n);
        for (uint32_t j = 0; j < n; j++) ri[j] = rec[size_t(j) * 24 + 20];
        std::sort(ri.begin(), ri.end());
        size_t best = 0;
        for (size_t i = 0; i < ri.size();) {
            size_t k = i;
            while (k < ri.size() && ri[k] == ri[i]) k++;
            if (k - i > best) { best = k - i; s->ri_prior = ri[i]; }
            i = k;
        }
        std::vector<float> vals{0.0f, 1.0f};
        vals.insert(vals.end(), ri.begin(), ri.end());
        std::sort(vals.begin(), vals.end());
        vals.erase(std::unique(vals.begin(), vals.end(), [](float a, float b) {
            return std::memcmp(&a, &b, sizeof(a)) == 0; }), vals.end());
        s->n_alt_vals = 0;
        if (vals.size() <= 8) {
            for (size_t v = 0; v < vals.size(); v++) s->alt_vals[v] = vals[v];
            s->n_alt_vals = int(vals.size());
        }
    }
    HIP_OK(s->hot.upload(hot.data(), hot.size() * sizeof(float)));
    HIP_OK(s->cold.upload(cold.data(), cold.size() * sizeof(float)));
    // Culling BVH over the objects (the reference loops linearly; rtk::iow_launch_ray keeps its
    // exact result); iow_linear: the reference's linear loop (A/B)
    rtamd::IowCull cull;
    if (!s->opt.iow_linear && rtamd::iow_cull_build(types, rec, n, cull)) {
        HIP_OK(s->nodes.upload(cull.wide.data(), cull.wide.size() * sizeof(float)));
        s->root_link = 1;
        s->n_wide = cull.n_wide;
        HIP_OK(s->obox.upload(cull.obox.data(), cull.obox.size() * sizeof(float)));
    }
    set_residency(s);
    return build_tables(s, spp);
}

int upload_textures(rt_dev_scene *s, const rt_texture *tex, int n_tex);

// INW wide walk (DESIGN.md "INW wide walk").  The reference finds the closest hit by a
// depth-first walk of its LBVH (01_BVH...glsl:431-473); the result is the nearest hit, ties to
// the object the walk meets first, among the objects whose LBVH leaf box the ray crosses.  The
// kernels find the same object with an ordered walk of a 4-wide culling BVH over the leaf boxes
// (inflated to stay conservative), the reference's exact test on the leaf box, and a (t, rank)
// rule with each object's rank in the reference's depth-first order.  That equivalence needs
// the reference walk to drop no push on its shared 40-float stack: dfs_high is the walk's
// stack high-water mark, and the kernels use the wide walk only while size + dfs_high <= 40.
void set_wide(const rt_dev_scene *s, rtk::InwScene &sc) {
    if (!s->dfs_high) return;
    sc.dfs_high = s->dfs_high;
    sc.sl = s->sl_ok && s->opt.inw_stackless ? 1u : 0u;  // stackless LBVH walks (rt_options.inw_stackless)
    if (!s->n_wnodes) return;  // no wide walk
    sc.wnodes = s->wnodes.as<float4>();
    sc.wroot = 1;
    if (s->wbins > 1 && s->opt.inw_time_bins > 1) {  // (built at scene creation; 0 / 1 later: unused)
        sc.wbin_base = s->n_wtree0; sc.wbin_stride = s->wbin_stride;
        if (s->opt.inw_walk_bins) sc.wbins = s->wbins;  // the wide closest-hit walks (set_beam: the beam lists)
    }
    sc.rank = s->wrank.as<uint32_t>();
    sc.leafbox = s->wleaf.as<float4>();
    if (s->sph_ok && s->opt.inw_sphere_records) sc.sph = s->sph.as<float4>();
    if (s->opt.inw_compact_nodes) sc.cnodes = s->cnodes.as<float4>();
    sc.dfs_high = s->dfs_high;
    sc.n_wnodes = s->n_wnodes;
    if (s->ri_ok && s->opt.inw_ri_grid) {
        sc.ri_cells = s->ri_cells.as<uint32_t>();
        sc.ri_ids = s->ri_ids.as<uint32_t>();
        for (int a = 0; a < 3; a++) {
            sc.ri_lo[a] = s->ri_lo[a]; sc.ri_hi[a] = s->ri_hi[a]; sc.ri_inv[a] = s->ri_inv[a]; sc.ri_dim[a] = s->ri_dim[a];
        }
    }
}

// The quantised culling BVH (DESIGN.md §5.2 "Quantised nodes") from the scene's wide nodes, on the
// device: planes rounded outward by kQMargin beyond the wide nodes' own (the error bound of the
// walk's decode is below it while every coordinate lies within 1000 of the origin, the fused
// cull's condition, which the launch checks per frame)
constexpr float kQMargin = 2e-3f;
int make_qnodes(rt_dev_scene *s) {
    if (!s->n_wnodes) return RT_OK;
    HIP_OK(s->cnodes.reserve(size_t(s->n_wnodes) * 7 * sizeof(float4)));
    HIP_OK(rtk::inw_compact_wnodes(s->wnodes.as<float4>(), s->n_wnodes, s->cnodes.as<float4>(), nullptr));
    HIP_OK(s->qnodes.reserve(size_t(s->n_wnodes) * rtk::kQNodeF4 * sizeof(float4)));
    HIP_OK(rtk::inw_quantize_wnodes(s->wnodes.as<float4>(), s->n_wnodes, s->qnodes.as<float4>(), kQMargin, nullptr));
    return RT_OK;
}

// The wide walk's structures and the RI grid, built on the host (rtamd::inw_wide_build,
// rtamd::ri_grid_build) and uploaded.
// ms (may be null): host time of the builds, then of the uploads
// geom (may be null): the reference's GeometryBuff records, for the time-bin trees
int make_inw_wide(rt_dev_scene *s, const float *nodes, uint32_t n, double *ms = nullptr, const float *geom = nullptr) {
    s->dfs_high = 0;
    s->sl_ok = false;
    s->n_wnodes = s->n_wtree0 = 0;
    s->wbins = 1;
    s->wbin_stride = 0;
    s->ri_ok = false;
    const auto t0 = std::chrono::steady_clock::now();
    uint32_t high = 0;
    bool sl = false;
    const bool walkable = rtamd::lbvh_walk_info(nodes, n, high, sl);
    rtamd::InwWide w;
    rtamd::RiGrid g;
    const bool ok = walkable && s->opt.inw_wide_walk && rtamd::inw_wide_build(nodes, n, w);
    if (ok) g = rtamd::ri_grid_build(w.leafbox.data(), n);
    if (ok && geom && s->opt.inw_time_bins > 1) rtamd::inw_wide_add_bins(geom, n, uint32_t(s->opt.inw_time_bins), w);
    const auto t1 = std::chrono::steady_clock::now();
    if (ms) ms[0] = std::chrono::duration<double, std::milli>(t1 - t0).count();
    if (!ok) {  // the reference walk only (stackless where it cannot drop a push)
        if (walkable) { s->dfs_high = high; s->sl_ok = sl; }
        return RT_OK;
    }
    HIP_OK(s->wnodes.store(w.wnodes.data(), w.wnodes.size() * sizeof(float)));
    HIP_OK(s->wrank.store(w.rank.data(), w.rank.size() * sizeof(uint32_t)));
    HIP_OK(s->wleaf.store(w.leafbox.data(), w.leafbox.size() * sizeof(float)));
    if (g.ok) {
        HIP_OK(s->ri_cells.store(g.cells.data(), g.cells.size() * sizeof(uint32_t)));
        HIP_OK(s->ri_ids.store(g.ids.data(), std::max<size_t>(1, g.ids.size()) * sizeof(uint32_t)));
        s->ri_ok = true;
        for (int a = 0; a < 3; a++) {
            s->ri_lo[a] = g.lo[a]; s->ri_hi[a] = g.hi[a]; s->ri_inv[a] = g.inv[a]; s->ri_dim[a] = g.dim[a];
        }
    }
    s->n_wnodes = uint32_t(w.wnodes.size() / 40);
    s->n_wtree0 = w.n_tree0;
    s->wbins = w.bins;
    s->wbin_stride = w.bin_stride;
    s->dfs_high = w.dfs_high;
    s->sl_ok = sl;
    s->wdepth = w.depth;
    s->wbound = w.wbound;
    if (int rc = make_qnodes(s); rc != RT_OK) return rc;
    if (ms) ms[1] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t1).count();
    return RT_OK;
}

// Sphere records (rtk::InwScene::sph) when every object is an ellipsoid with equal scales and the
// identity rotation (entries exactly 1 and +-0): (position, RN(1/scale)), (position - last_position,
// RI), (RN(1/RN(scale^2)) per axis, extra).  false: some object is not.
bool inw_sphere_records(const float *geom, uint32_t n, int layout, std::vector<float> &out) {
    out.assign(size_t(n) * 12, 0.0f);
    for (uint32_t j = 0; j < n; j++) {
        const float *f = geom + size_t(j) * 28;
        if (int(f[18] + 0.1f) != 1 || !(f[12] == f[13] && f[13] == f[14]) || !std::isfinite(f[12])) return false;
        for (int k = 0; k < 9; k++)
            if (f[3 + k] != ((k % 4) == 0 ? 1.0f : 0.0f)) return false;
        float *o = out.data() + size_t(j) * 12;
        o[0] = f[0]; o[1] = f[1]; o[2] = f[2]; o[3] = 1.0f / f[12];  // the hot record's is (RN(1/scale))
        o[4] = f[15]; o[5] = f[16]; o[6] = f[17];
        o[7] = layout == 4 ? f[19] : f[20];  // the RI the surrounding-RI walk adds (the hot record's)
        for (int k = 0; k < 3; k++) o[8 + k] = 1.0f / (f[12 + k] * f[12 + k]);  // the hot record's is2
        o[11] = f[19];  // its extra data
    }
    return n > 0;
}

// The kernels' hot / cold records from the reference's GeometryBuff(_04) records (28 floats).
void inw_records(const float *geom, uint32_t n, int layout, std::vector<float> &hot, std::vector<float> &cold) {
    hot.assign(size_t(n) * rtk::kInwHot, 0.0f);
    cold.assign(size_t(n) * rtk::kInwCold, 0.0f);
    for (uint32_t j = 0; j < n; j++) {
        const float *f = geom + size_t(j) * 28;
        float *h = hot.data() + size_t(j) * rtk::kInwHot;
        float *c = cold.data() + size_t(j) * rtk::kInwCold;
        for (int k = 0; k < 20; k++) h[k] = f[k];  // pos R scale delta type extra
        bool ident = true;  // the rotation exactly the identity (entries 1 and +-0): type + 0.5 (rtk::Xf::ident)
        for (int k = 0; k < 9; k++) ident = ident && f[3 + k] == ((k % 4) == 0 ? 1.0f : 0.0f);
        if (ident && (f[18] == 1.0f || f[18] == 2.0f)) h[18] = f[18] + 0.5f;
        for (int k = 0; k < 3; k++) {
            h[20 + k] = 1.0f / f[12 + k];                  // a / scale  -> a * RN(1/scale)
            h[23 + k] = 1.0f / (f[12 + k] * f[12 + k]);    // a / (s*s)  -> a * RN(1/RN(s*s))
        }
        h[26] = layout == 4 ? f[19] : f[20];  // RI accumulated by the surrounding-RI walk
        if (layout == 1) {  // BVH.h:6-19
            c[0] = f[21]; c[1] = f[22]; c[2] = f[23]; c[3] = f[24];
            c[4] = f[25]; c[5] = f[26]; c[6] = f[27]; c[7] = f[20];
        } else {            // lights.h:6-21
            c[0] = f[20]; c[1] = f[21]; c[2] = f[22]; c[3] = f[23];
            c[4] = f[24]; c[5] = f[25]; c[6] = f[26];
            // TextureIndex = uint(texel 6.w + 0.1) (04...glsl:414), as uint bits; the RI (f[19])
            // reaches the kernel as IntersectRay's extra data instead
            const float ti = f[27] + 0.1f;
            const uint32_t tu = ti <= 0.0f ? 0u : (ti >= 4294967040.0f ? 0xffffffffu : uint32_t(ti));
            std::memcpy(&c[7], &tu, 4);
        }
    }
}

int make_inw(rt_dev_scene *s, const float *geom, uint32_t n, int layout, const float *nodes,
             const float *lights, uint32_t n_lights, const rt_texture *tex, int n_tex, int spp) {
    if (int rc = upload_textures(s, layout == 4 ? tex : nullptr, layout == 4 ? n_tex : 0); rc != RT_OK) return rc;
    std::vector<float> hot, cold;
    inw_records(geom, n, layout, hot, cold);
    s->kind = layout == 4 ? 14 : 11;
    s->n = n; s->layout = layout; s->n_lights = layout == 4 ? n_lights : 0;
    HIP_OK(s->hot.store(hot.data(), hot.size() * sizeof(float)));
    HIP_OK(s->cold.store(cold.data(), cold.size() * sizeof(float)));
    {
        std::vector<float> sph;
        s->sph_ok = inw_sphere_records(geom, n, layout, sph);
        if (s->sph_ok) HIP_OK(s->sph.store(sph.data(), sph.size() * sizeof(float)));
    }
    HIP_OK(s->nodes.store(nodes, size_t(2 * n - 1) * 8 * sizeof(float)));
    if (int rc = make_inw_wide(s, nodes, n, nullptr, geom); rc != RT_OK) return rc;
    if (s->n_lights) HIP_OK(s->lights.store(lights, size_t(s->n_lights) * 7 * sizeof(float)));
    else HIP_OK(s->lights.store(nullptr, 0));
    set_residency(s);
    return build_tables(s, spp);
}

// The same structures built on the device from the scene's device LBVH (rt_build.hip, DESIGN.md
// "Device build"; rt_options.inw_device_build): no host build, no upload.  ms: host wall time of
// the build (its level loop and the RI grid read counts back) in ms[0], 0 in ms[1].
int make_inw_wide_device(rt_dev_scene *s, uint32_t n, double *ms) {
    s->dfs_high = 0;
    s->sl_ok = false;
    s->n_wnodes = s->n_wtree0 = 0;
    s->wbins = 1;
    s->wbin_stride = 0;
    s->ri_ok = false;
    const auto t0 = std::chrono::steady_clock::now();
    HIP_OK(s->wnodes.reserve(size_t(n) * 40 * sizeof(float)));
    HIP_OK(s->wrank.reserve(size_t(n) * 2 * sizeof(uint32_t)));
    HIP_OK(s->wleaf.reserve(size_t(n) * 8 * sizeof(float)));
    const size_t wsb = rtk::inw_build_workspace_bytes(n);
    HIP_OK(s->build_ws.reserve(wsb));
    rtk::InwWideDev out{s->wnodes.as<float4>(), s->wrank.as<uint32_t>(), s->wleaf.as<float4>(), 0, 0, 0, 0.0f, {}, {}};
    {
        const hipError_t be = rtk::inw_wide_build_device(s->nodes.as<float4>(), s->lcnt.as<uint32_t>(), n,
                                                         s->build_ws.p, s->build_ws.bytes, out, nullptr, g_build_levels);
        if (be == hipErrorNotSupported) return RT_E_UNSUPPORTED;  // deeper than its level cap: the caller builds on the host
        HIP_OK(be);
    }
    if (s->opt.inw_wide_walk) {
        double dlo[3], dhi[3], inv[3];
        int dim[3];
        for (int a = 0; a < 3; a++) { dlo[a] = out.ri_lo[a]; dhi[a] = out.ri_hi[a]; }
        if (rtamd::ri_grid_dims(dlo, dhi, n, dim, inv)) {
            const size_t nc = size_t(dim[0]) * dim[1] * dim[2];
            HIP_OK(s->ri_cells.reserve((nc + 1) * sizeof(uint32_t)));
            const size_t tb = rtk::ri_scan_temp_bytes(nc + 1);
            HIP_OK(s->ri_tmp.reserve(tb));
            uint32_t total = 0, over = 0;
            HIP_OK(rtk::ri_count_device(s->wleaf.as<float4>(), n, s->build_ws.p, dlo, inv, dim, s->ri_cells.as<uint32_t>(),
                                        s->ri_tmp.p, tb, &total, &over, nullptr));
            if (!over) {
                HIP_OK(s->ri_ids.reserve(std::max<size_t>(1, total) * sizeof(uint32_t)));
                HIP_OK(s->ri_fill.reserve(std::max<size_t>(1, nc) * sizeof(uint32_t)));
                HIP_OK(rtk::ri_fill_device(s->wleaf.as<float4>(), n, dlo, inv, dim, s->ri_cells.as<uint32_t>(),
                                           s->ri_fill.as<uint32_t>(), s->ri_ids.as<uint32_t>(), nullptr));
                for (int a = 0; a < 3; a++) {
                    s->ri_lo[a] = float(dlo[a]); s->ri_hi[a] = float(dhi[a]); s->ri_inv[a] = float(inv[a]);
                    s->ri_dim[a] = dim[a];
                }
                s->ri_ok = true;
            }
        }
        s->n_wnodes = s->n_wtree0 = out.n_wnodes;
        s->wdepth = out.depth;
        s->wbound = out.wbound;
        if (int rc = make_qnodes(s); rc != RT_OK) return rc;
    }
    HIP_OK(hipDeviceSynchronize());
    s->dfs_high = out.dfs_high;
    s->sl_ok = true;  // the device LBVH has the stackless layout by construction (rt_lbvh.hip)
    if (ms) {
        ms[0] = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        ms[1] = 0.0;
    }
    return RT_OK;
}

// RT_Base<>::OnUpdateBase's per-redraw work on an existing device scene (In-Next-Week/base.h:
// 96-175): new records, the LBVH (the caller's, or built on the device from the boxes), the wide
// walk and RI grid rebuilt on the host, every upload into the scene's buffers.  ms[4]: host time
// of the records, the LBVH (upload + device build + read-back), the host structures, their upload.
int update_inw(rt_dev_scene *s, const float *geom, uint32_t n, const float *nodes, const float *aabbs,
               const float *lights, uint32_t n_lights, double *ms) {
    using clk = std::chrono::steady_clock;
    auto t = clk::now();
    auto lap = [&](int k) {
        const auto now = clk::now();
        if (ms) ms[k] = std::chrono::duration<double, std::milli>(now - t).count();
        t = now;
    };
    if (n > (1u << 24)) return RT_E_UNSUPPORTED;  // node / object ids are stored as floats (exact to 2^24)
    // the wide walk's structures and the RI grid built on the device from the device LBVH
    // (rt_options.inw_device_build; a caller's host LBVH keeps the host builders)
    const bool device_build = s->opt.inw_device_build && !nodes && n >= 2;
    // Until every step below has succeeded the buffers may hold a mix of the old and the new
    // scene (sizes included): the scene refuses renders (launch_scene) and keeps its old n and
    // counts, so nothing indexes past a buffer.  The new sizes are committed at the end.
    s->broken = true;
    std::vector<float> hot, cold;
    inw_records(geom, n, s->layout, hot, cold);
    const uint32_t nl = s->layout == 4 ? n_lights : 0;
    HIP_OK(s->hot.store(hot.data(), hot.size() * sizeof(float)));
    HIP_OK(s->cold.store(cold.data(), cold.size() * sizeof(float)));
    {
        std::vector<float> sph;
        s->sph_ok = false;  // (the scene is marked broken until the update completes)
        if (inw_sphere_records(geom, n, s->layout, sph)) {
            HIP_OK(s->sph.store(sph.data(), sph.size() * sizeof(float)));
            s->sph_ok = true;
        }
    }
    if (nl) HIP_OK(s->lights.store(lights, size_t(nl) * 7 * sizeof(float)));
    lap(0);
    const size_t nbytes = size_t(2 * n - 1) * 8 * sizeof(float);
    std::vector<float> host_nodes;
    if (!nodes) {  // ConstructLBVH_Buff on the device (rt_lbvh_build_async), read back for the host builders
        if (s->nodes.bytes < nbytes) {
            s->nodes.~DevBuf();
            new (&s->nodes) DevBuf();
            HIP_OK(s->nodes.alloc(nbytes));
        }
        HIP_OK(s->aabb.store(aabbs, size_t(n) * 6 * sizeof(float)));
        const size_t ws = rtk::lbvh_workspace_bytes(n);
        HIP_OK(s->lbvh_ws.reserve(ws));
        if (device_build) HIP_OK(s->lcnt.reserve(size_t(2 * n - 1) * sizeof(uint32_t)));
        HIP_OK(rtk::lbvh_build_device(s->aabb.as<float>(), n, s->nodes.as<float>(), s->lbvh_ws.p, ws, nullptr,
                                      device_build ? s->lcnt.as<uint32_t>() : nullptr));
        if (!device_build) {  // the host builders read it
            host_nodes.resize(nbytes / sizeof(float));
            HIP_OK(hipMemcpy(host_nodes.data(), s->nodes.p, nbytes, hipMemcpyDeviceToHost));
            nodes = host_nodes.data();
        }
    } else {
        HIP_OK(s->nodes.store(nodes, nbytes));
    }
    lap(1);
    double w[2] = {0.0, 0.0};
    if (device_build) {
        int rc = make_inw_wide_device(s, n, w);
        s->wbuild = 1;
        if (rc == RT_E_UNSUPPORTED) {
            // the binned SAH tree ran past the device build's level cap (a chain-like scene: a split
            // can peel one object off per level); the host builders have no such limit, so read the
            // device LBVH back and build the walk structures there, as rt_dev_scene_inw does
            host_nodes.resize(nbytes / sizeof(float));
            HIP_OK(hipMemcpy(host_nodes.data(), s->nodes.p, nbytes, hipMemcpyDeviceToHost));
            rc = make_inw_wide(s, host_nodes.data(), n, w, geom);
            s->wbuild = 2;
        }
        if (rc != RT_OK) return rc;
    } else {
        if (int rc = make_inw_wide(s, nodes, n, w, geom); rc != RT_OK) return rc;
        s->wbuild = 0;
    }
    if (ms) { ms[2] = w[0]; ms[3] = w[1]; }
    s->n = n;
    s->n_lights = nl;
    s->broken = false;
    return RT_OK;
}

// Sample ranges of the render.  Default: one range (tail compaction keeps the SIMDs full).
// rt_options.iow_chunks_lpt: a short first chunk measures every pixel's cost and the rest run
// longest-first (LPT) -- kept as an A/B switch; with compaction it measured slower.
std::vector<std::pair<int, int>> chunk_plan(int spp, bool lpt) {
    std::vector<std::pair<int, int>> plan;
    if (spp <= 2 || !lpt) { plan.push_back({0, spp}); return plan; }
    const int first = std::max(1, spp / 20);
    const int step = std::max(1, (spp - first + 7) / 8);
    plan.push_back({0, first});
    for (int b = first; b < spp; b += step) plan.push_back({b, std::min(spp, b + step)});
    return plan;
}

int ensure_workspace(rt_dev_scene *s, uint32_t units) {
    if (units <= s->ws_units) return RT_OK;
    s->ws_state.~DevBuf(); new (&s->ws_state) DevBuf();
    s->ws_cost.~DevBuf(); new (&s->ws_cost) DevBuf();
    s->ws_keys.~DevBuf(); new (&s->ws_keys) DevBuf();
    s->ws_iota.~DevBuf(); new (&s->ws_iota) DevBuf();
    s->ws_order.~DevBuf(); new (&s->ws_order) DevBuf();
    s->ws_temp.~DevBuf(); new (&s->ws_temp) DevBuf();
    HIP_OK(s->ws_state.alloc(size_t(units) * 32));
    HIP_OK(s->ws_cost.alloc(size_t(units) * 4));
    HIP_OK(s->ws_keys.alloc(size_t(units) * 4));
    HIP_OK(s->ws_order.alloc(size_t(units) * 4));
    std::vector<unsigned> iota(units);
    for (uint32_t i = 0; i < units; i++) iota[i] = i;
    HIP_OK(s->ws_iota.upload(iota.data(), size_t(units) * 4));
    s->ws_temp_bytes = rtk::sort_temp_bytes(units);
    HIP_OK(s->ws_temp.alloc(s->ws_temp_bytes));
    s->ws_units = units;
    return RT_OK;
}

#ifdef RT_DIAG  // diagnostic builds only: switches of the diagnostics (never of the render path)
int env_int(const char *name, int dflt) {
    const char *v = std::getenv(name);
    return (v && *v) ? std::atoi(v) : dflt;
}
#endif
// park lanes only while at least this many units remain (rt_options.park_min; -1: cap / 8 waves)
uint32_t park_min_of(const rt_dev_scene *s, int cap) {
    return uint32_t(s->opt.park_min >= 0 ? s->opt.park_min : cap * rtk::kBlock / 8);
}

int ensure_cont(rt_dev_scene *s) {
    if (s->cont_count.p) return RT_OK;
    const size_t slots = size_t(s->blocks_cap) * rtk::kBlock;
    for (auto &b : s->cont) HIP_OK(b.alloc(slots * rtk::kContSlots * sizeof(float4)));
    HIP_OK(s->cont_count.alloc(64 * 16));  // one count per round, 64 B apart (rt_debug_rounds)
    return RT_OK;
}

constexpr int kCountSlots = 160;  // round counts per group lane, 64 B apart

// group lanes of the sample-parallel pipeline; temp_bytes = sort scratch each lane needs
int ensure_lanes(rt_dev_scene *s, int groups, size_t temp_bytes) {
    if (!s->ev_start) HIP_OK(hipEventCreateWithFlags(&s->ev_start, hipEventDisableTiming));
    const size_t slots = size_t(s->blocks_cap) * rtk::kBlock;
    while (s->lanes.size() < size_t(groups)) {
        auto L = std::make_unique<rt_dev_scene::GroupLane>();
        HIP_OK(hipStreamCreateWithFlags(&L->st, hipStreamNonBlocking));
        HIP_OK(hipEventCreateWithFlags(&L->done, hipEventDisableTiming));
        HIP_OK(L->counter.alloc(64));
        // 2x: parked lanes (<= resident lanes) plus restarts queued between checkpoint rounds
        for (auto &b : L->cont) HIP_OK(b.alloc(2 * slots * rtk::kContSlots * sizeof(float4)));
        HIP_OK(L->cont_count.alloc(kCountSlots * 64));
        s->lanes.push_back(std::move(L));
    }
    for (int g = 0; g < groups; g++) {
        auto &L = *s->lanes[size_t(g)];
        if (L.temp_bytes < temp_bytes) {
            L.temp.~DevBuf();
            new (&L.temp) DevBuf();
            HIP_OK(L.temp.alloc(temp_bytes));
            L.temp_bytes = temp_bytes;
        }
    }
    return RT_OK;
}

// Frame tag of the sample-parallel records: a record is "done" for a frame when its flags carry
// the frame's tag (16 bits).  The tags are process-wide, so a new scene whose record buffers
// reuse a freed scene's memory never takes that scene's records for its own (the same render of
// the full frame, then of one tile alone, found the full frame's records at its own indices and
// returned their colours), and a scene clears its flags when its tag comes round again.
// The clear goes on the render's stream st, ordered after the scene's earlier frames on that stream
// (a null-stream memset would not wait for a non-blocking caller stream).
unsigned next_spec_epoch(rt_dev_scene *s, hipStream_t st) {
    static std::atomic<unsigned> g{0};
    unsigned v;
    do v = (g.fetch_add(1u) + 1u) & 0xffffu; while (v == 0u);
    if (v <= s->epoch && s->sp_col.p)  // wrapped since this scene's last frame: forget its tags
        (void)hipMemsetAsync(s->sp_col.p, 0, s->sp_col.bytes, st);
    s->epoch = v;
    return v;
}

// Sample-parallel records for P pixel units x S samples; false if they do not fit.
bool ensure_spec(rt_dev_scene *s, uint32_t P, uint32_t S) {
    const size_t n = size_t(P) * S;
    const size_t bytes = n * (4 * sizeof(float4) + 4 * sizeof(uint32_t)) + size_t(P) * (4 + 32);
    if (double(bytes) > s->opt.spec_max_gb * 1e9) return false;
    if (n <= s->spec_cap && P <= s->spec_units) return true;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess || bytes > free_b / 2) return false;
    for (DevBuf *b : {&s->sp_col, &s->sp_fin, &s->sp_ctr, &s->sp_assume, &s->sp_list, &s->sp_fb, &s->sp_counts,
                      &s->sp_keys, &s->sp_keys2, &s->sp_list2, &s->sp_temp, &s->sp_pstate, &s->sp_front,
                      &s->sp_sorder, &s->sp_fcost}) {
        b->~DevBuf();
        new (b) DevBuf();
    }
    if (s->sp_col.alloc(n * sizeof(float4)) != hipSuccess || s->sp_fin.alloc(n * sizeof(float4)) != hipSuccess ||
        s->sp_ctr.alloc(n * sizeof(uint4)) != hipSuccess || s->sp_assume.alloc(n * sizeof(float4)) != hipSuccess ||
        s->sp_list.alloc(n * sizeof(uint32_t)) != hipSuccess || s->sp_fb.alloc(size_t(P) * 4) != hipSuccess ||
        s->sp_counts.alloc(64 * 64) != hipSuccess || s->sp_keys.alloc(n * 4) != hipSuccess ||
        s->sp_keys2.alloc(n * 4) != hipSuccess || s->sp_list2.alloc(n * 4) != hipSuccess ||
        s->sp_pstate.alloc(size_t(P) * 3 * sizeof(uint4)) != hipSuccess ||
        s->sp_front.alloc(size_t(P) * 2 * sizeof(uint4)) != hipSuccess ||
        s->sp_sorder.alloc(size_t(S) * sizeof(uint32_t)) != hipSuccess ||
        s->sp_fcost.alloc(size_t(S) * sizeof(unsigned long long)) != hipSuccess ||
        s->sp_temp.alloc(s->sp_temp_bytes = rtk::sort_pairs_temp_bytes(n, 24)) != hipSuccess) {
        s->spec_cap = s->spec_units = 0;
        return false;
    }
    if (hipMemset(s->sp_col.p, 0, s->sp_col.bytes) != hipSuccess) {  // no flags: no record is done
        s->spec_cap = s->spec_units = 0;
        return false;
    }
    s->spec_cap = n;
    s->spec_units = P;
    return true;
}


int launch_scene_inw_fold(rt_dev_scene *s, rtk::Frame &f, hipStream_t st);

// Enqueue a whole render (all chunks) on `st`.  The first call for a given frame size
// allocates the chunk workspace; later calls allocate nothing.
int launch_scene_spec(rt_dev_scene *s, rtk::Frame &f, hipStream_t st);

int launch_scene(rt_dev_scene *s, rtk::Frame &f, hipStream_t st) {
    if (s->broken) return RT_E_ARG;  // a failed rt_dev_scene_inw_update (update_inw)
    f.n_focus = (s->kind != 3 && s->layout == 1) ? s->n_focus : 0;
    std::memcpy(f.focus_list, s->focus, sizeof(f.focus_list));
    f.leaf_batch = s->opt.iow_leaf_batch;
    f.coop_max = s->opt.iow_coop_max;
    f.narrow = s->opt.iow_narrow;
    s->last_path = rt_path_info{};
    if (s->kind != 3) {  // the frame's closest-hit queries that fell back to the LBVH walks (rt_debug_path)
        HIP_OK(s->walk_ctr.reserve(sizeof(unsigned long long)));
        HIP_OK(hipMemsetAsync(s->walk_ctr.p, 0, sizeof(unsigned long long), st));
        f.walk_ctr = s->walk_ctr.as<unsigned long long>();
    }
    if (s->kind == 3 && s->opt.iow_spec && !rtk::iow_narrow(f) && s->s_stop > 0 &&
        ensure_spec(s, rtk::units_of(f), uint32_t(s->s_stop)))
        return launch_scene_spec(s, f, st);
    // INW: the on-chip fold kernels; inw_order = -1 runs the per-pixel sequential kernel k_inw
    // (a second restatement of End()'s loop, kept for the strategy-exactness tests)
    if (s->kind != 3 && s->opt.inw_order >= 0) return launch_scene_inw_fold(s, f, st);
    const std::vector<std::pair<int, int>> plan = chunk_plan(f.spp, s->opt.iow_chunks_lpt != 0);
    const uint32_t units = rtk::units_of(f);
    s->last_kernel = s->kind == 3 ? (rtk::iow_narrow(f) ? "k_iow03n" : "k_iow03") : (s->layout == 4 ? "k_inw<true>" : "k_inw<false>");
    s->last_launches = int(plan.size()) * (1 + s->opt.rounds_seq);
    s->last_path.order = s->kind == 3 ? 5 : 3;
    s->last_path.wide_walk = s->kind != 3 && s->n_wnodes != 0;
    s->last_path.stackless = s->kind != 3 && s->dfs_high != 0 && s->sl_ok && s->opt.inw_stackless;
    s->last_chunks = int(plan.size());
    if (plan.size() > 1) {
        int rc = ensure_workspace(s, units);
        if (rc != RT_OK) return rc;
    }
    // Each chunk runs as 1 + `rounds` launches: the pixel launch, then launches that resume the
    // lanes the previous one parked.  Counts stay on the device (no host round trip): a resume
    // launch with nothing parked exits at once.  Parking stops below ~one wave per SIMD, where
    // compaction can no longer shorten the critical path; the last round never parks.
    const int rounds = s->opt.rounds_seq;  // <= 14: one count slot per round
    // grid of this frame's kernel variant
    int cap = s->kind == 3 ? s->cus * rtk::resident_blocks_per_cu(rtk::iow_narrow(f) ? 4 : 3) : s->blocks_cap;
    if (s->kind == 3 && !rtk::iow_narrow(f)) {
        rtk::IowScene probe{};
        probe.nodes = s->nodes.as<float4>();
        probe.n_nodes = s->n_wide;
        probe.lds_on = s->opt.iow_lds_bvh;
        if (rtk::iow_lds(probe)) {
            cap = s->cus * 3 * rtk::resident_blocks_per_cu(9);  // 256-lane slots of the 768-lane blocks
            s->last_kernel = "k_iow03L";
        }
        s->last_path.iow_bvh = s->root_link ? (rtk::iow_lds(probe) ? 2 : 1) : 0;
    }
    const uint32_t park_min = park_min_of(s, cap);
    if (rounds > 0) {
        int rc = ensure_cont(s);
        if (rc != RT_OK) return rc;
    }
    unsigned *cnt = s->cont_count.as<unsigned>();  // cnt[16*r]: lanes parked by round r (separate cache lines)
    hipError_t e = hipSuccess;
    for (size_t k = 0; k < plan.size() && e == hipSuccess; k++) {
        rtk::Chunk ch{};
        ch.s_begin = plan[k].first;
        ch.s_end = plan[k].second;
        ch.final_chunk = k + 1 == plan.size();
        ch.state = plan.size() > 1 ? s->ws_state.as<float4>() : nullptr;
        ch.order = k > 0 ? s->ws_order.as<unsigned>() : nullptr;
        ch.cost = ch.final_chunk ? nullptr : s->ws_cost.as<unsigned>();
        for (int r = 0; r <= rounds && e == hipSuccess; r++) {
            rtk::Cont ct{};
            uint32_t n_units = units;
            if (r > 0) {
                ct.in = s->cont[(r - 1) & 1].as<float4>();
                ct.in_count = cnt + 16 * std::min(r - 1, 15);
                n_units = uint32_t(cap) * rtk::kBlock;
            }
            if (r < rounds) {
                ct.out = s->cont[r & 1].as<float4>();
                ct.out_count = cnt + 16 * std::min(r, 15);
                ct.park_min = park_min;
                e = hipMemsetAsync(ct.out_count, 0, sizeof(unsigned), st);
                if (e != hipSuccess) break;
            }
            if (s->kind == 3) {
                rtk::IowScene sc{s->hot.as<float>(), s->cold.as<float>(), s->n, s->nodes.as<float4>(),
                                 s->sunflower.as<float>(), s->fib.as<float>(), s->ring.as<int>(), s->root_link,
                                 s->obox.as<float4>(), s->n_wide, s->opt.iow_lds_bvh};
                e = rtk::launch_iow03(f, sc, ch, ct, n_units, s->counter.as<unsigned>(), s->s_stop, cap, st);
            } else {
                rtk::InwScene sc{s->hot.as<float4>(), s->cold.as<float4>(), s->nodes.as<float4>(),
                                 s->lights.as<float>(), s->n, s->n_lights, s->layout, s->sunflower.as<float>(),
                                 s->tex.as<float4>(), s->tex_info.as<int4>(), s->n_tex};
    set_wide(s, sc);
                e = rtk::launch_inw(f, sc, ch, ct, n_units, s->counter.as<unsigned>(), s->blocks_cap, st);
            }
        }
        if (e == hipSuccess && !ch.final_chunk)
            e = rtk::sort_units_by_cost(s->ws_cost.as<unsigned>(), s->ws_keys.as<unsigned>(),
                                        s->ws_iota.as<unsigned>(), s->ws_order.as<unsigned>(), units,
                                        s->ws_temp.p, s->ws_temp_bytes, st);
    }
    if (e != hipSuccess) {
        std::fprintf(stderr, "[rt_hip] launch failed: %s\n", hipGetErrorString(e));
        return RT_E_HIP;
    }
    return RT_OK;
}

// Sample-parallel IOW-03: speculate every (pixel, sample) at once, then resolve / re-run the
// samples whose assumed incoming stack state was wrong (RT_SPEC_ITERS passes), and hand any
// pixel still unresolved to the sequential kernel from its first unresolved sample.  All
// launches are enqueued on `st`; counts stay on the device.
bool g_time_kernels = false;  // rt_debug_time_kernels

// k_iow03s(L) launch, bracketed by events on its stream when kernel timing is on
hipError_t spec_launch(rt_dev_scene *s, const rtk::Frame &f, const rtk::IowScene &sc, const rtk::SpecRecs &R, int mode,
                       const rtk::Cont &ct, uint32_t n, unsigned *counter, int cap, hipStream_t st) {
    std::pair<hipEvent_t, hipEvent_t> *ev = nullptr;
    if (g_time_kernels) {
        if (s->kt_used == s->kt_ev.size()) {
            std::pair<hipEvent_t, hipEvent_t> p{nullptr, nullptr};
            if (hipEventCreate(&p.first) != hipSuccess || hipEventCreate(&p.second) != hipSuccess) return hipErrorUnknown;
            s->kt_ev.push_back(p);
        }
        ev = &s->kt_ev[s->kt_used++];
        hipError_t e = hipEventRecord(ev->first, st);
        if (e != hipSuccess) return e;
    }
    rtk::Cont c2 = ct;
    c2.launch_id = s->launch_seq++;
    hipError_t e = rtk::launch_iow03_spec(f, sc, R, mode, c2, n, counter, cap, st);
    if (e == hipSuccess && ev) e = hipEventRecord(ev->second, st);
    return e;
}

int launch_scene_spec(rt_dev_scene *s, rtk::Frame &f, hipStream_t st) {
    const uint32_t P = rtk::units_of(f), S = uint32_t(s->s_stop);
    s->kt_used = 0;
    int rc = ensure_workspace(s, P);
    if (rc != RT_OK) return rc;
    const rt_options &o = s->opt;
    const int rounds = o.rounds_spec;
    const int iters = o.spec_iters;
    const int groups = 1;  // one pipeline (per-group streams measured slower: 8.8 s with 4 groups)
    // A render of at most half the frame (one rank's tiles of a partition) has less parallel work
    // per sample chain, and its time becomes the longest dependent chain of its heaviest pixel
    // (north star): the automatic settings then spend more on the long samples,
    // twice the heavy-first indices and alternative runs from 2048 segments on (north-star 8-way
    // shares 5.87x -> 6.09x; whole frames keep (S - 1) / 20 and 16384: C2 +2.3% otherwise).
    const bool partial = uint64_t(P) * 2u <= uint64_t((f.W + 7) / 8 * 8) * uint64_t((f.H + 7) / 8 * 8);
    const int heavy_auto = int(S - 1) / (partial ? 10 : 20);
    const int alt_seg = o.spec_alt_seg > 0 ? o.spec_alt_seg : (partial ? 2048 : 16384);
    const size_t gmax = size_t(P + groups - 1) / groups + 1;  // pixels in the largest group
    if ((rc = ensure_cont(s)) != RT_OK) return rc;
    if ((rc = ensure_lanes(s, groups, rtk::sort_pairs_temp_bytes(gmax * S, 24))) != RT_OK) return rc;
    unsigned *sc = s->sp_counts.as<unsigned>();  // group g: [32g] list count, [32g+16] fallback count
    rtk::SpecRecs R{s->sp_col.as<float4>(), s->sp_fin.as<float4>(), s->sp_ctr.as<uint4>(),
                          s->sp_assume.as<float4>(), P, S, s->sp_list.as<uint32_t>(), sc, s->sp_fb.as<uint32_t>(),
                          sc + 16, s->ws_order.as<uint32_t>(), 0, 0, s->sp_pstate.as<uint4>(), next_spec_epoch(s, st),
                          s->sp_front.as<uint4>(), s->sp_sorder.as<uint32_t>(),
                          uint32_t(o.spec_probe),
                          S > 2 && groups == 1 ? uint32_t(std::min(int(S) - 2, o.spec_heavy >= 0 ? o.spec_heavy
                                                                                                : heavy_auto))
                                               : 0u};
    R.pmag = rtk::spec_pmag(P);
    s->spec_P = P;
    s->spec_S = S;
    s->launch_seq = 0;
#ifdef RT_DIAG
    if (env_int("RT_DEBUG_TIMES", 0) != 0) {  // diagnostic builds only (rt_debug_spec_times)
        const size_t n = size_t(P) * S * 2 * sizeof(uint32_t);
        if (s->sp_dbg_t.bytes < n) {
            s->sp_dbg_t.~DevBuf();
            new (&s->sp_dbg_t) DevBuf();
            HIP_OK(s->sp_dbg_t.alloc(n));
        }
        HIP_OK(hipMemsetAsync(s->sp_dbg_t.p, 0, n, st));
        R.dbg_start = s->sp_dbg_t.as<uint32_t>();
        R.dbg_end = R.dbg_start + size_t(P) * S;
        s->sp_dbg_n = size_t(P) * S;
    }
#endif
    const bool alt_on = o.spec_alt != 0 && s->n_alt_vals > 1 && S > 1;
    if (alt_on) {  // alternative runs (DESIGN.md "Alternative runs")
        // slots pack as first | count << 24 in the hash (alt_find): the cap stays below 2^24
        const uint32_t cap = uint32_t(o.spec_alt_cap);
        if (s->alt_cap != cap) {
            for (DevBuf *b : {&s->sp_alt, &s->sp_alt_hash, &s->sp_alt_count}) { b->~DevBuf(); new (b) DevBuf(); }
            HIP_OK(s->sp_alt.alloc(size_t(cap) * sizeof(rtk::AltRec)));
            HIP_OK(s->sp_alt_hash.alloc(size_t(cap) * 2 * sizeof(uint2)));
            HIP_OK(s->sp_alt_count.alloc(64));
            s->alt_cap = cap;
        }
        HIP_OK(hipMemsetAsync(s->sp_alt_hash.p, 0, size_t(cap) * 2 * sizeof(uint2), st));
        HIP_OK(hipMemsetAsync(s->sp_alt_count.p, 0, 64, st));
        R.alt = s->sp_alt.as<rtk::AltRec>();
        R.alt_hash = s->sp_alt_hash.as<uint2>();
        R.alt_count = s->sp_alt_count.as<unsigned>();
        R.alt_cap = cap;
        R.alt_hcap = cap * 2;
        R.alt_min_seg = uint32_t(alt_seg);
        for (int v = 0; v < 8; v++) R.alt_vals[v] = s->alt_vals[v];
        R.n_alt_vals = s->n_alt_vals;
    }
    // alternatives are spawned after the checkpoint rounds and, with spec_alt_every = k > 0,
    // after every k-th budgeted tail round too (measured: once is best on the bench frame)
    const int alt_every = o.spec_alt_every;
    R.front2 = s->sp_front.as<uint4>() + P;  // the anchored scan's secondary frontier
    R.scan_max = uint32_t(o.spec_scan);
    if (R.scan_max == 0) R.front2 = nullptr;
#ifdef RT_DIAG  // diagnostic builds only: copy one render's exact per-sample state into the next
    if (env_int("RT_SPEC_ORACLE", 0) != 0) {  // (see SpecRecs::exact)
        const size_t n = size_t(P) * S;
        if (s->sp_exact_n != n) {
            s->sp_exact.~DevBuf();
            new (&s->sp_exact) DevBuf();
            HIP_OK(s->sp_exact.alloc(n * sizeof(float4)));
            s->sp_exact_n = n;
            s->sp_exact_valid = false;
        }
        R.exact = s->sp_exact.as<float4>();
        R.exact_mode = 1 | (s->sp_exact_valid ? 2 : 0);
        s->sp_exact_valid = true;
    }
#endif
    rtk::IowScene scene{s->hot.as<float>(), s->cold.as<float>(), s->n, s->nodes.as<float4>(),
                        s->sunflower.as<float>(), s->fib.as<float>(), s->ring.as<int>(), s->root_link,
                        s->obox.as<float4>(), s->n_wide, o.iow_lds_bvh};
    // caps in 256-lane slots; the LDS-BVH kernels run 768-lane blocks
    const bool lds = rtk::iow_lds(scene);
    const int cap_s = s->cus * (lds ? 3 * rtk::resident_blocks_per_cu(10) : rtk::resident_blocks_per_cu(5));
    const int cap_q = s->cus * (lds ? 3 * rtk::resident_blocks_per_cu(9) : rtk::resident_blocks_per_cu(3));
    hipError_t e = hipSuccess;
    // one compacted pass on a stream with its own queue counter and continuation buffers: the
    // first launch takes `n0` units, resume launches take the parked lanes
    struct Lane { hipStream_t st; unsigned *counter; const DevBuf *cont; unsigned *cnt; };
    const bool spread_last = o.spec_spread != 0;
    // the first launch of the next pass takes its sorted head one unit per wave (Cont.solo_n)
    uint32_t solo_first = 0;
    auto pass = [&](const Lane &q, auto &&launch, uint32_t n0, int cap) {
        const uint32_t park_min = park_min_of(s, cap);
        for (int r = 0; r <= rounds && e == hipSuccess; r++) {
            rtk::Cont ct{};
            uint32_t n_units = n0;
            if (r > 0) {
                ct.in = q.cont[(r - 1) & 1].as<float4>();
                ct.in_count = q.cnt + 16 * std::min(r - 1, 15);
                n_units = uint32_t(cap) * rtk::kBlock;
            }
            if (r < rounds) {
                ct.out = q.cont[r & 1].as<float4>();
                ct.out_count = q.cnt + 16 * std::min(r, 15);
                ct.park_min = park_min;
                e = hipMemsetAsync(ct.out_count, 0, sizeof(unsigned), q.st);
                if (e != hipSuccess) break;
            } else if (r > 0 && spread_last) ct.spread = 1;  // the last round: long samples get a wave each
            if (r == 0) ct.solo_n = solo_first;
            e = launch(q, ct, n_units);
        }
    };
    auto spec = [&](const rtk::SpecRecs &RR, int mode) {
        return [&, RR, mode](const Lane &q, const rtk::Cont &ct, uint32_t n) {
            return spec_launch(s, f, scene, RR, mode, ct, n, q.counter, cap_s, q.st);
        };
    };
    // Checkpoint rounds (spec_rounds = k > 0): the speculative pass over samples 1.. runs as k
    // launches, each taking the lanes the previous one parked plus the next slice of fresh units
    // and parking every lane once its queue drains; between launches the pixel frontiers advance
    // and mispredicted samples at a frontier are re-run at once (k_iow03_frontier,
    // k_iow03_fixf).  The tail then runs as before (compaction rounds).
    const int ckpt = S > 1 ? std::min(kCountSlots - 16, o.spec_rounds) : 0;
    // Heavy-first (R.n_heavy = K > 0): round 0 runs every sample of every R.probe_stride-th pixel;
    // the measured cost per sample index orders the indices (k_sample_rank); the next rounds run
    // the K costliest indices for every pixel (sample-major, so the long samples start first);
    // the pixels are then re-sorted by the rays of those samples and the remaining indices run
    // pixel-major (so each heavy pixel's frontier reaches its long samples early).
    // Budgeted tail rounds (spec_tail_rounds, spec_tail_budget segments each; DESIGN.md
    // "Budgeted tail"): the frontier advances between them, so mispredicted samples re-run while
    // the long ones still run instead of in a re-run pass after them.
    // exact restarts go on down their pixel's chain of mispredicted samples (spec_chain)
    const int chain = o.spec_chain != 0 ? 1 : 0;
    const int tail_budgeted = ckpt > 0 ? std::max(0, std::min(kCountSlots - 16 - ckpt - rounds, o.spec_tail_rounds)) : 0;
    auto ckpt_pass = [&](const Lane &q, const rtk::SpecRecs &RG, uint32_t n_fresh) {
        const uint32_t slots = uint32_t(s->blocks_cap) * rtk::kBlock, cap_cont = 2 * slots;
        struct Rnd { int mode; uint32_t lo, hi; };
        std::vector<Rnd> plan;
        const uint32_t n_px = RG.order_n ? RG.order_n : RG.P, K = RG.n_heavy;
        int r_heavy_end = -1;  // last round of the heavy phase
        if (K > 0 && ckpt >= 3) {
            const uint32_t n_probe = (n_px + RG.probe_stride - 1) / RG.probe_stride * (S - 1);
            plan.push_back({1, 0, n_probe});
            const int rest = ckpt - 1;
            const int ra = std::max(1, std::min(rest - 1, int(std::lround(double(rest) * K / (S - 1)))));
            const uint64_t nh = uint64_t(K) * n_px, nr = uint64_t(S - 1 - K) * n_px;
            for (int r = 0; r < ra; r++) plan.push_back({2, uint32_t(nh * r / ra), uint32_t(nh * (r + 1) / ra)});
            r_heavy_end = ra;
            for (int r = 0; r < rest - ra; r++)
                plan.push_back({3, uint32_t(nr * r / (rest - ra)), uint32_t(nr * (r + 1) / (rest - ra))});
        } else {
            for (int r = 0; r < ckpt; r++)
                plan.push_back({0, uint32_t(uint64_t(n_fresh) * r / ckpt), uint32_t(uint64_t(n_fresh) * (r + 1) / ckpt)});
        }
        int b = 0;  // continuation buffer written last
        for (int r = 0; r < ckpt && e == hipSuccess; r++) {
            rtk::Cont ct{};
            if (r > 0) { ct.in = q.cont[(r - 1) & 1].as<float4>(); ct.in_count = q.cnt + 16 * (r - 1); }
            ct.out = q.cont[r & 1].as<float4>();
            ct.out_count = q.cnt + 16 * r;
            ct.mixed = 1;
            ct.chain = chain;
            ct.park_below = 65;  // park every busy lane once the queue drains
            ct.fresh_mode = plan[size_t(r)].mode;
            ct.fresh_lo = plan[size_t(r)].lo;
            ct.fresh_hi = plan[size_t(r)].hi;
            if (r == ckpt - 1) ct.park_below = 0;  // the last round compacts as the tail rounds do
            ct.park_min = r == ckpt - 1 ? park_min_of(s, cap_s) : 0u;
            e = hipMemsetAsync(ct.out_count, 0, sizeof(unsigned), q.st);
            if (e == hipSuccess) e = spec_launch(s, f, scene, RG, rtk::kSpecRest, ct, uint32_t(cap_s) * rtk::kBlock,
                                                 q.counter, cap_s, q.st);
            if (e == hipSuccess) e = rtk::launch_iow03_frontier(f, RG, ct.out, ct.out_count, cap_cont, q.st);
            if (e == hipSuccess) e = rtk::launch_iow03_fixf(f, RG, ct.out, ct.out_count, int(cap_cont), q.st);
            if (e == hipSuccess && RG.alt && r == ckpt - 1)
                e = rtk::launch_iow03_altspawn(f, RG, ct.out, ct.out_count, cap_cont, q.st);
            if (e == hipSuccess && r == 0 && r_heavy_end > 0)
                e = rtk::launch_iow03_sample_order(f, RG, ct.out, ct.out_count, int(cap_cont),
                                                   s->sp_fcost.as<unsigned long long>(), s->sp_sorder.as<uint32_t>(),
                                                   q.st);
            if (e == hipSuccess && r == r_heavy_end) {
                e = rtk::launch_iow03_pixel_key(f, RG, ct.out, ct.out_count, int(cap_cont), s->ws_cost.as<unsigned>(),
                                                q.st);
                if (e == hipSuccess)
                    e = rtk::sort_units_by_cost(s->ws_cost.as<unsigned>(), s->ws_keys.as<unsigned>(),
                                                s->ws_iota.as<unsigned>(), s->ws_order.as<unsigned>(), P,
                                                s->ws_temp.p, s->ws_temp_bytes, q.st);
            }
            b = r & 1;
        }
        // tail: resume rounds with compaction; the first `tb` of them are budgeted (every unit
        // parks after spec_tail_budget segments) and followed by the frontier, so a sample found
        // mispredicted re-runs while the long samples are still running; the last round runs to
        // completion
        const uint32_t park_min = park_min_of(s, cap_s);
        const int tb = tail_budgeted;
        const uint32_t budget = uint32_t(o.spec_tail_budget);
        const int n_tail = tb + rounds;
        const bool spread = spread_last;
        for (int t = 0; t <= n_tail && e == hipSuccess; t++) {
            const int r = ckpt + t;
            rtk::Cont ct{};
            ct.chain = chain;
            ct.in = q.cont[b].as<float4>();
            ct.in_count = q.cnt + 16 * (r - 1);
            if (t < n_tail) {
                ct.out = q.cont[b ^ 1].as<float4>();
                ct.out_count = q.cnt + 16 * r;
                ct.park_min = park_min;
                if (t < tb) {
                    ct.seg_budget = budget;
                    if (spread) { ct.spread = 1; ct.park_min = 0xffffffffu; }  // no compaction parking
                }
                e = hipMemsetAsync(ct.out_count, 0, sizeof(unsigned), q.st);
            }
            if (t == n_tail && spread) ct.spread = 1;  // the last round: long samples get a wave each
            if (e == hipSuccess) e = spec_launch(s, f, scene, RG, rtk::kSpecRest, ct, uint32_t(cap_s) * rtk::kBlock,
                                                 q.counter, cap_s, q.st);
            if (e == hipSuccess && t < tb) {
                e = rtk::launch_iow03_frontier(f, RG, ct.out, ct.out_count, cap_cont, q.st);
                if (e == hipSuccess) e = rtk::launch_iow03_fixf(f, RG, ct.out, ct.out_count, int(cap_cont), q.st);
                if (e == hipSuccess && RG.alt && alt_every > 0 && t % alt_every == alt_every - 1)
                    e = rtk::launch_iow03_altspawn(f, RG, ct.out, ct.out_count, cap_cont, q.st);
            }
            b ^= 1;
        }
    };
    s->last_kernel = lds ? "k_iow03sL" : "k_iow03s";
    s->last_path.order = 4;
    s->last_path.iow_bvh = s->root_link ? (lds ? 2 : 1) : 0;
    s->last_launches = (1 + rounds) * (1 + groups * ((S > 1 ? 1 : 0) + iters)) +
                       (ckpt > 0 ? groups * (ckpt + tail_budgeted) : 0);
    s->last_chunks = 1;
    // (1) on the caller's stream: sample 0 of every pixel (exact), the guesses for the other
    // samples, and the pixel order (heaviest sample 0 first)
    const Lane L0{st, s->counter.as<unsigned>(), s->cont, s->cont_count.as<unsigned>()};
    e = hipMemsetAsync(R.assume, 0, size_t(P) * sizeof(float4), st);
    if (e == hipSuccess) pass(L0, spec(R, rtk::kSpecFirst), P, cap_s);
    if (S > 1) {
        // Sample 1 starts from sample 0's final stack (exact: its written entries, 0 elsewhere).
        // From spec_prior_from (2) on every entry is guessed as the scene's most common RI
        // The prior misses far less often (the re-run pass re-traces ~1% of the rays instead of
        // ~20% with zeros); the dependent chains it forms are cheap for the validating pass.
        const uint32_t prior_from = uint32_t(o.spec_prior_from);
        if (e == hipSuccess)
            e = rtk::launch_iow03_prep(f, R, s->ws_cost.as<unsigned>(), s->ri_prior, prior_from, st);
        if (e == hipSuccess)
            e = rtk::sort_units_by_cost(s->ws_cost.as<unsigned>(), s->ws_keys.as<unsigned>(), s->ws_iota.as<unsigned>(),
                                        s->ws_order.as<unsigned>(), P, s->ws_temp.p, s->ws_temp_bytes, st);
    }
    if (e == hipSuccess) e = hipEventRecord(s->ev_start, st);
    // (2) one independent pipeline per pixel group, each on its own stream, so one group's long
    // samples overlap the other groups' work: speculative pass over samples 1.., resolve and
    // re-run passes (the first list longest first), final resolve, sequential leftovers
    const bool sort_first = o.spec_sort != 0;
    for (int g = 0; g < groups && e == hipSuccess; g++) {
        auto &GL = *s->lanes[size_t(g)];
        const Lane L{GL.st, GL.counter.as<unsigned>(), GL.cont, GL.cont_count.as<unsigned>()};
        rtk::SpecRecs RG = R;
        const uint32_t base = uint32_t(uint64_t(P) * g / groups);
        const uint32_t cnt_g = uint32_t(uint64_t(P) * (g + 1) / groups) - base;
        if (S > 1) { RG.order_base = base; RG.order_n = cnt_g; }
        RG.list = R.list + size_t(base) * S;
        RG.list_count = sc + 32 * g;
        RG.fb_list = R.fb_list + base;
        RG.fb_count = sc + 32 * g + 16;
        const size_t nmax = size_t(cnt_g) * S;  // list bound for this group
        e = hipStreamWaitEvent(L.st, s->ev_start, 0);
        if (S > 1 && e == hipSuccess) {
            if (ckpt > 0) ckpt_pass(L, RG, cnt_g * (S - 1));
            else pass(L, spec(RG, rtk::kSpecRest), cnt_g * (S - 1), cap_s);
        }
        for (int it = 0; it < iters && e == hipSuccess; it++) {
            e = hipMemsetAsync(RG.list_count, 0, sizeof(unsigned), L.st);
            if (e == hipSuccess) e = rtk::launch_iow03_resolve(f, RG, false, nullptr, L.st);
            if (it == 0 && sort_first && e == hipSuccess) {
                // the first re-execution list holds the long samples: run it longest first (LPT),
                // keyed by each sample's ray count in its speculative run
                unsigned *k1 = s->sp_keys.as<unsigned>() + size_t(base) * S;
                unsigned *k2 = s->sp_keys2.as<unsigned>() + size_t(base) * S;
                uint32_t *l2 = s->sp_list2.as<uint32_t>() + size_t(base) * S;
                e = rtk::spec_list_keys(RG, k1, nmax, L.st);
                if (e == hipSuccess)
                    e = rtk::sort_pairs_desc(k1, k2, RG.list, l2, nmax, GL.temp.p, GL.temp_bytes, 24, L.st);
                rtk::SpecRecs R2 = RG;
                R2.list = l2;
                solo_first = uint32_t(o.spec_solo);
                if (e == hipSuccess) pass(L, spec(R2, rtk::kSpecList), uint32_t(nmax), cap_s);
                solo_first = 0;
            } else if (e == hipSuccess) pass(L, spec(RG, rtk::kSpecList), uint32_t(nmax), cap_s);
        }
        if (e == hipSuccess) e = hipMemsetAsync(RG.fb_count, 0, sizeof(unsigned), L.st);
        if (e == hipSuccess) e = rtk::launch_iow03_resolve(f, RG, true, s->ws_state.as<float4>(), L.st);
        // leftovers: the sequential kernel from each pixel's first unresolved sample
        rtk::Chunk ch{};
        ch.s_begin = 0;
        ch.s_end = int(S);
        ch.final_chunk = 1;
        ch.state = s->ws_state.as<float4>();
        ch.order = RG.fb_list;
        ch.order_count = RG.fb_count;
        ch.per_unit_begin = 1;
        if (o.spec_validate != 0) {  // reuse the records that are still exact
            ch.rec_col = R.col; ch.rec_fin = R.fin; ch.rec_assume = R.assume; ch.rec_ctr = R.ctr;
            ch.rec_P = P;
            ch.rec_S = S;
        }
        if (e == hipSuccess)
            pass(L, [&, ch](const Lane &q, const rtk::Cont &ct, uint32_t n) {
                return rtk::launch_iow03(f, scene, ch, ct, n, q.counter, s->s_stop, cap_q, q.st);
            }, cnt_g, cap_q);
        if (e == hipSuccess) e = hipEventRecord(GL.done, L.st);
        if (e == hipSuccess) e = hipStreamWaitEvent(st, GL.done, 0);  // join
    }
    if (e != hipSuccess) {
        std::fprintf(stderr, "[rt_hip] launch failed: %s\n", hipGetErrorString(e));
        return RT_E_HIP;
    }
    return RT_OK;
}

// Pixel beams (DESIGN.md §5 "Pixel beams"; rt_options.inw_beams = 0 turns them off).  Sample s of a pixel
// starts its primary ray one unit behind tip = C0 + rr * ox + ru * oy (C0 = co + cd, |rr|, |ru|
// <= 1, |ox| + |oy| <= aperture / 2 * sf_max) and aims it at F = co + cd * focus.  With
// L = |F - C0| = focus - 1, the point of that ray at fraction u of the way from tip to F is
// within delta0 * |1 - u| of the point C0 + u * L * cd of the central ray, so over the central
// parameter range [tmin, tfar] that covers the scene, every primary ray lies within
// R = delta0 * max |1 - t / L| (+ rounding slack) of the central ray.  A sample ray's hit at t
// has central parameter <= t * kappa, kappa = L / (L - delta0).
int set_beam(rt_dev_scene *s, const rtk::Frame &f, rtk::InwScene &sc) {
    const uint32_t cap = 32;
    const double units = double(rtk::units_of(f));
    const double ap = std::fabs(double(f.aperture)), L = double(f.focus) - 1.0;
    const double d0 = 0.5 * ap * double(s->sf_max) * (1.0 + 1e-4) + 1e-6;
    if (!s->opt.inw_beams || !sc.wnodes || f.n_focus > 0 || !(L > 8.0 * d0 + 1e-3) ||
        units * cap * 8.0 * std::max<uint32_t>(1u, s->wbins) > 8.0e9)  // list capacity; each list is packed
        return RT_OK;
    const double cam = std::sqrt(double(f.pos[0]) * f.pos[0] + double(f.pos[1]) * f.pos[1] + double(f.pos[2]) * f.pos[2]);
    const double Lh = L + 1e-3 * (1.0 + cam), Ll = L - 1e-3 * (1.0 + cam);
    if (!(Ll > 4.0 * d0)) return RT_OK;
    // every point of a culling box lies within sqrt(3) * wbound of the origin
    const double tfar = (cam + 1.0 + std::sqrt(3.0) * double(s->wbound) + 2.0) / (1.0 - d0 / Ll) * 1.001;
    const double tmin = -Lh / (Ll - d0) - 0.01;
    const double r = d0 * std::fmax(1.0 - tmin / Ll, std::fabs(1.0 - tfar / Ll));
    const double R = r + 2e-3 + 1e-5 * (cam + tfar);
    // object ids below 2^16: one uint32 per entry (the id, t's high half), else (id, t)
    const bool b16 = s->n <= 65536u && s->opt.inw_beams != 2;  // inw_beams = 2: the pairs (A/B)
    // one list per unit and time bin when the scene has time-bin trees (rt_options.inw_time_bins)
    const uint32_t nb = s->wbins > 1 && s->opt.inw_time_bins > 1 && s->opt.inw_beam_bins ? s->wbins : 1u;
    const size_t need = size_t(units) * nb * cap * (b16 ? sizeof(uint32_t) : sizeof(uint2)),
                 need_n = size_t(units) * nb * 2 * sizeof(uint32_t);
    // the lists are an optional speed-up: on a device short of memory the frame runs without them
    size_t free_b = 0, total_b = 0;
    const size_t grow = (s->inw_beam.bytes < need ? need : 0) + (s->inw_beam_n.bytes < need_n ? need_n : 0);
    if (grow && (hipMemGetInfo(&free_b, &total_b) != hipSuccess || grow > free_b / 2)) return RT_OK;
    if (s->inw_beam.bytes < need) {
        s->inw_beam.~DevBuf();
        new (&s->inw_beam) DevBuf();
        if (s->inw_beam.alloc(need) != hipSuccess) { (void)hipGetLastError(); s->inw_beam.bytes = 0; return RT_OK; }
    }
    if (s->inw_beam_n.bytes < need_n) {
        s->inw_beam_n.~DevBuf();
        new (&s->inw_beam_n) DevBuf();
        if (s->inw_beam_n.alloc(need_n) != hipSuccess) { (void)hipGetLastError(); s->inw_beam_n.bytes = 0; return RT_OK; }
    }
    sc.beam = s->inw_beam.as<uint2>();
    sc.beam_n = s->inw_beam_n.as<uint32_t>();
    sc.beam_cut = reinterpret_cast<const float *>(s->inw_beam_n.as<uint32_t>() + size_t(units) * nb);
    sc.beam_cap = cap;
    sc.beam_bins = nb > 1 ? nb : 0u;
    sc.beam_units = uint32_t(units);
    if (nb > 1) { sc.wbin_base = s->n_wtree0; sc.wbin_stride = s->wbin_stride; }
    sc.beam16 = b16 ? 1u : 0u;
    sc.beam_R = float(R);
    sc.beam_tmin = float(tmin);
    sc.beam_tfar = float(tfar);
    sc.beam_kappa = float(Lh / (Ll - d0) * (1.0 + 1e-5));
    return RT_OK;
}

// INW with on-chip End() folds (DESIGN.md §5 "INW: on-chip End() folds"): the probe, then
// k_inw_pm and k_inw_sm (one of them exits at once), persistent launches of one frame.  The
// launches are bracketed by HIP events on their stream when kernel timing is on
// (rt_debug_kernel_time).  rt_options.inw_order = 1 / 2 forces pixel- / sample-major (tests, A/B);
// inw_ring_pm / inw_ring_sm set the fold windows (samples per wave, powers of two).
int launch_scene_inw_fold(rt_dev_scene *s, rtk::Frame &f, hipStream_t st) {
    const rt_options &o = s->opt;
    const int blocks = s->cus * rtk::resident_blocks_per_cu(s->layout == 4 ? 16 : 15);
    // the top of the wide BVH staged in LDS (768-lane blocks, 3 waves per SIMD);
    // inw_lds_nodes = 0: 256-lane blocks reading every node from L1 / L2 (A/B)
    // (without the wide walk the stackless LBVH walks read the top of the LBVH from that LDS; the
    // stack walks run in the same 768-lane instances, with nothing staged)
    const int blocks_ln = o.inw_lds_nodes && (s->n_wnodes || s->dfs_high)
                              ? s->cus * rtk::resident_blocks_per_cu(s->layout == 4 ? 18 : 17) : 0;
    // inw_ring_pm = 0: k_inw_pm's fold ring in LDS (768-lane blocks), else a global
    // ring of that many entries per wave (1024 for the 256-lane blocks)
    const bool lring = o.inw_ring_pm == 0 && blocks_ln > 0;
    const uint32_t ring_pm = lring ? rtk::kPmLdsRing : uint32_t(o.inw_ring_pm ? o.inw_ring_pm : 1024);
    // inw_ring_sm = 0: k_inw_sm's ring in LDS too when the staging keeps every node it would stage
    // anyway (a BVH top of at most kPmLdsNodes wide nodes: INW-04's rooms), else a global ring of
    // 256 entries; a power of two: the global ring of that size
    const bool fits5 = s->n_wnodes ? s->n_wtree0 <= rtk::kPmLdsNodes
                                   : (s->sl_ok && 2 * size_t(s->n) - 1 <= size_t(rtk::kPmLdsNodes) * 10 / 2);
    const bool lring_sm = o.inw_ring_sm == 0 && blocks_ln > 0 && fits5;
    const uint32_t ring_sm = lring_sm ? rtk::kPmLdsRing : uint32_t(o.inw_ring_sm ? o.inw_ring_sm : 256);
    const size_t waves = std::max(size_t(blocks) * (rtk::kBlock / 64), size_t(blocks_ln) * (3 * rtk::kBlock / 64));
    const size_t ring_bytes = waves * std::max(lring ? 0u : ring_pm, lring_sm ? 0u : ring_sm) * sizeof(float4);
    if (s->inw_ring.bytes < ring_bytes) {
        s->inw_ring.~DevBuf();
        new (&s->inw_ring) DevBuf();
        if (s->inw_ring.alloc(ring_bytes) != hipSuccess) return RT_E_HIP;
        s->ring_frame = 0;  // fresh memory: clear it before the first frame
    }
    // ring tags carry the frame's epoch (rtk::ring_tag); the rings are cleared only when it wraps.
    // ring_frame advances only once this frame's clear (epoch 0) is enqueued, and any failure
    // below resets it, so the next frame clears the rings before it uses them
    const uint32_t epoch = s->ring_frame % 63u;
    s->ring_frame = 0;
    rtk::InwScene sc{s->hot.as<float4>(), s->cold.as<float4>(), s->nodes.as<float4>(),
                     s->lights.as<float>(), s->n, s->n_lights, s->layout, s->sunflower.as<float>(),
                     s->tex.as<float4>(), s->tex_info.as<int4>(), s->n_tex};
    set_wide(s, sc);
    sc.ring_epoch = epoch << 26;
    sc.lring = lring ? 1u : 0u;
    sc.lring_sm = lring_sm ? 1u : 0u;
    sc.xcdq = o.inw_claim_xcd ? 1u : 0u;
#ifdef RT_INW_PARK  // walk parking (experiment): 2 float4 per lane of the fold grid
    {
        const size_t need = waves * 64 * 2 * sizeof(float4);
        if (s->inw_park.bytes < need) {
            s->inw_park.~DevBuf();
            new (&s->inw_park) DevBuf();
            if (s->inw_park.alloc(need) != hipSuccess) return RT_E_HIP;
        }
        sc.park = s->inw_park.as<float4>();
    }
#endif
    // the fused cull (cull4nf<true>: one fma per plane) while every ray origin -- the camera (+ lens and the unit step
    // of the primary ray), hit points inside the scene's boxes -- lies within 1000 of the origin
    // (DESIGN.md §2); not with the MULTIFOCUS lens chain, whose lens points are farther out
    {
        const float cam = std::fmax(std::fabs(f.pos[0]), std::fmax(std::fabs(f.pos[1]), std::fabs(f.pos[2]))) +
                          2.0f + std::fabs(f.aperture);
        sc.fused = (o.inw_fused_cull && f.n_focus == 0 && std::fmax(cam, s->wbound) <= 1000.0f) ? 1 : 0;
    }
    // GQ: k_inw_pm over the quantised nodes with the reference's stacks in global
    // memory -- INW-01, the LDS ring instances, the fused cull's error bound (the quantised decode
    // is argued under it)
    if (o.inw_qnodes && s->layout != 4 && lring && sc.fused && sc.wnodes && s->qnodes.p) {
        const uint32_t gb = uint32_t(s->cus * rtk::resident_blocks_per_cu(19));
        const size_t need = size_t(gb) * rtk::kGqSub * rtk::kBlock * (rtk::kFStack / 4) * sizeof(float4);
        if (s->gstk.bytes < need) {
            s->gstk.~DevBuf();
            new (&s->gstk) DevBuf();
            if (s->gstk.alloc(need) != hipSuccess) { s->gstk.bytes = 0; return RT_E_HIP; }
        }
        if (rtk::kGqQn) sc.qnodes = s->qnodes.as<float4>();
        sc.gstk = s->gstk.as<float4>();
        sc.gq_blocks = gb;
    }
    s->last_gq = sc.gstk != nullptr;
    const uint32_t force = (o.inw_order == 1 || o.inw_order == 2) ? uint32_t(o.inw_order) : 0u;
    s->last_force = force;
    s->last_ring[0] = ring_pm;
    s->last_lring = lring;
    s->last_lring_sm = lring_sm;
    s->last_ring[1] = ring_sm;
    s->last_kernel = s->layout == 4 ? "k_inw_fold<true>" : "k_inw_fold<false>";
    s->last_ln = blocks_ln > 0;
    s->last_fu = s->last_ln && sc.fused;
    s->last_launches = 1;
    s->last_chunks = 1;
    s->kt_used = 0;
    std::pair<hipEvent_t, hipEvent_t> *ev = nullptr;
    hipError_t e = hipSuccess;
    if (g_time_kernels) {
        if (s->kt_ev.empty()) {
            std::pair<hipEvent_t, hipEvent_t> p{nullptr, nullptr};
            if (hipEventCreate(&p.first) != hipSuccess || hipEventCreate(&p.second) != hipSuccess) return RT_E_HIP;
            s->kt_ev.push_back(p);
        }
        ev = &s->kt_ev[0];
        s->kt_used = 1;
    }
    // the rings are cleared first (when the epoch wraps), so the events bracket the probe and the
    // two fold kernels
    // claim order, costliest blocks first (inw_claim_order = 0: unit order)
    uint32_t *cost = nullptr;
    if (o.inw_claim_order) {
        const size_t need = (2 * size_t(rtk::units_of(f) / 64) + 256) * sizeof(uint32_t);
        if (s->inw_cost.bytes < need) {
            s->inw_cost.~DevBuf();
            new (&s->inw_cost) DevBuf();
            if (s->inw_cost.alloc(need) != hipSuccess) return RT_E_HIP;
        }
        cost = s->inw_cost.as<uint32_t>();
    }
    if (int rc = set_beam(s, f, sc); rc != RT_OK) return rc;
    {  // the path this frame takes (rt_debug_path; the order is resolved at query time)
        rt_path_info &P = s->last_path;
        P.launches = 1;
        P.order_forced = force != 0;
        P.order = int(force);
        P.wide_walk = sc.wnodes != nullptr;
        P.beams = sc.beam != nullptr;
        P.ri_grid = sc.ri_cells != nullptr;
        P.fused_cull = s->last_fu && sc.wnodes ? 1 : 0;  // the fused cull is the wide walk's
        P.lds_nodes = s->last_ln ? int(std::min<uint32_t>(s->n_wtree0, uint32_t(rtk::kInwLdsNodes))) : 0;
        P.stackless = sc.sl ? 1 : 0;
        // the LBVH nodes the stackless walks read from LDS (LN kernels without the wide walk)
        P.lbvh_lds_nodes = s->last_ln && sc.sl && !sc.wnodes
                               ? int(std::min<uint32_t>(2 * s->n - 1, uint32_t(rtk::kInwLdsNodes * 10 / 2))) : 0;
        P.claim_order = cost != nullptr;
        P.qnodes = sc.qnodes != nullptr;
        P.global_stack = sc.gstk != nullptr;
        P.walk_stack = sc.gstk ? rtk::kWStack : rtk::kFStack - 3;
        if (sc.gstk)
            P.lds_nodes = int(std::min<uint32_t>(s->n_wtree0, uint32_t(rtk::kGqQn ? rtk::kQLdsNodes : rtk::kInwLdsNodes)));
        P.time_bins = sc.wnodes && !sc.gstk ? int(sc.wbins) : 0;  // the GQ walks read the staged (swept) tree
        P.beam_bins = sc.beam ? int(sc.beam_bins) : 0;
        P.sphere_records = sc.sph ? 1 : 0;
    }
    if (epoch == 0) e = hipMemsetAsync(s->inw_ring.p, 0xff, s->inw_ring.bytes, st);
    if (e == hipSuccess) s->ring_frame = epoch + 1;
    if (e == hipSuccess && ev) e = hipEventRecord(ev->first, st);
    if (e == hipSuccess)
        e = rtk::launch_inw_fold(f, sc, s->inw_ring.as<float4>(), ring_pm, ring_sm, s->counter.as<unsigned>(),
                                 s->inw_mode.as<uint32_t>(), force, blocks, blocks_ln, cost, st);
    if (e == hipSuccess && ev) e = hipEventRecord(ev->second, st);
    if (e != hipSuccess) {
        s->ring_frame = 0;
        std::fprintf(stderr, "[rt_hip] launch failed: %s\n", hipGetErrorString(e));
        return RT_E_HIP;
    }
    return RT_OK;
}


// blocking render of one scene into host buffers
int render_blocking(rt_dev_scene *s, const rt_camera *cam, const rt_params *p, float *rgba, float *depth,
                    rt_stats *st) {
    rtk::Frame f = make_frame(cam, p);
    const size_t npx = size_t(p->width) * p->height;
    DevBuf d_rgba, d_depth, d_ctr;
    HIP_OK(d_rgba.alloc(npx * 16));
    HIP_OK(hipMemcpy(d_rgba.p, rgba, npx * 16, hipMemcpyHostToDevice));  // untouched pixels keep their value
    if (depth) {
        HIP_OK(d_depth.alloc(npx * 4));
        HIP_OK(hipMemcpy(d_depth.p, depth, npx * 4, hipMemcpyHostToDevice));
    }
    HIP_OK(d_ctr.alloc(6 * sizeof(unsigned long long)));
    HIP_OK(hipMemset(d_ctr.p, 0, 6 * sizeof(unsigned long long)));
    f.out_rgba = d_rgba.as<float>();
    f.out_depth = depth ? d_depth.as<float>() : nullptr;
    f.counters = d_ctr.as<unsigned long long>();
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, nullptr));
    int rc = launch_scene(s, f, nullptr);
    HIP_OK(hipEventRecord(e1, nullptr));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc != RT_OK) return rc;
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(rgba, d_rgba.p, npx * 16, hipMemcpyDeviceToHost));
    if (depth) HIP_OK(hipMemcpy(depth, d_depth.p, npx * 4, hipMemcpyDeviceToHost));
    if (st) {
        unsigned long long c[6];
        HIP_OK(hipMemcpy(c, d_ctr.p, sizeof(c), hipMemcpyDeviceToHost));
        st->segments = c[0]; st->node_visits = c[1]; st->prim_tests = c[2];
        st->shadow_queries = c[3]; st->stack_drops = c[4]; st->nan_drops = c[5];
        st->ms = ms;
    }
    return RT_OK;
}

bool inw_textured(const float *geom, uint32_t n, int layout) {
    if (layout != 4) return false;
    for (uint32_t g = 0; g < n; g++)
        if (geom[size_t(g) * 28 + 27] + 0.1f >= 1.0f) return true;
    return false;
}

bool textures_ok(const rt_texture *tex, int n_tex) {
    if (n_tex < 0 || (n_tex > 0 && !tex)) return false;
    for (int k = 0; k < n_tex; k++)
        if (!tex[k].texels || tex[k].width <= 0 || tex[k].height <= 0 || (tex[k].channels != 3 && tex[k].channels != 4) ||
            size_t(tex[k].width) * size_t(tex[k].height) > (size_t(1) << 31))
            return false;
    return true;
}

// u_MaterialTextures[0..n_tex) (04...glsl:10; bound by GeometryData_04::BindExtraData,
// lights.cpp:22): unorm8 texels -> float (c / 255, the GL conversion) once, on the host
int upload_textures(rt_dev_scene *s, const rt_texture *tex, int n_tex) {
    s->n_tex = 0;
    if (n_tex == 0) {
        HIP_OK(s->tex.alloc(16));
        HIP_OK(s->tex_info.alloc(16));
        return RT_OK;
    }
    size_t total = 0;
    std::vector<int> info(size_t(n_tex) * 4, 0);
    for (int k = 0; k < n_tex; k++) {
        info[4 * k] = int(total);
        info[4 * k + 1] = tex[k].width;
        info[4 * k + 2] = tex[k].height;
        total += size_t(tex[k].width) * size_t(tex[k].height);
    }
    if (total > (size_t(1) << 31)) return RT_E_ARG;
    std::vector<float> texels(total * 4, 0.0f);
    for (int k = 0; k < n_tex; k++) {
        const size_t m = size_t(tex[k].width) * size_t(tex[k].height);
        const int ch = tex[k].channels;
        float *o = texels.data() + size_t(info[4 * k]) * 4;
        for (size_t i = 0; i < m; i++) {
            for (int c = 0; c < 3; c++) o[4 * i + c] = float(tex[k].texels[i * ch + c]) / 255.0f;
            o[4 * i + 3] = ch == 4 ? float(tex[k].texels[i * ch + 3]) / 255.0f : 1.0f;
        }
    }
    HIP_OK(s->tex.upload(texels.data(), texels.size() * sizeof(float)));
    HIP_OK(s->tex_info.upload(info.data(), info.size() * sizeof(int)));
    s->n_tex = uint32_t(n_tex);
    return RT_OK;
}

bool noise_args_ok(int width, int height, int type, const float *gradient, int n_grad, int octaves) {
    return width > 0 && height > 0 && size_t(width) * size_t(height) < (size_t(1) << 31) && type >= 0 && type <= 2 &&
           octaves >= 0 && n_grad >= 0 && n_grad <= 64 && (n_grad == 0 || gradient) &&
           rtk::noise_batches_exact(uint32_t(width));
}
bool remap_args_ok(int width, int height, int channels, int load_as, int map_to) {
    return width > 0 && height > 0 && size_t(width) * size_t(height) < (size_t(1) << 31) &&
           (channels == 3 || channels == 4) && load_as >= 0 && load_as <= 1 && map_to >= 0 && map_to <= 1 &&
           (load_as == map_to || rtk::noise_batches_exact(uint32_t(width)));
}
// device time of the work enqueued by `fn` on the null stream
template <class F> int timed(F &&fn, double *ms) {
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, nullptr));
    const int rc = fn();
    HIP_OK(hipEventRecord(e1, nullptr));
    HIP_OK(hipEventSynchronize(e1));
    float t = 0.0f;
    (void)hipEventElapsedTime(&t, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (ms) *ms = t;
    return rc;
}

}  // namespace

extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
}  // extern "C"
int rtamd::scene_device(const rt_dev_scene *s) { return s ? s->device : -1; }
extern "C" {

void rt_options_default(rt_options *o) {
    if (o) *o = default_options();
}

int rt_options_set(const rt_options *o) {
    if (!options_ok(o)) return RT_E_ARG;
    g_opt = *o;
    return RT_OK;
}

int rt_options_get(rt_options *o) {
    if (!o) return RT_E_ARG;
    *o = g_opt;
    return RT_OK;
}

int rt_dev_scene_inw_update(rt_dev_scene *s, const float *geom, uint32_t n, const float *nodes, const float *aabbs,
                            const float *lights, uint32_t n_lights, double timing_ms[4]) {
    if (!s || s->kind == 3 || !geom || n == 0 || (!nodes && !aabbs)) return RT_E_ARG;
    if (s->layout == 4 && n_lights > 0 && !lights) return RT_E_ARG;
    if (s->n_tex == 0 && inw_textured(geom, n, s->layout)) return RT_E_UNSUPPORTED;
    HIP_OK(hipSetDevice(s->device));
    HIP_OK(hipDeviceSynchronize());  // the scene's last frame may still read the buffers being replaced
    try {  // the host builders allocate: no exception crosses the ABI
        return update_inw(s, geom, n, nodes, aabbs, lights, n_lights, timing_ms);
    } catch (...) {
        s->broken = true;
        return RT_E_ARG;
    }
}

int rt_dev_scene_set_options(rt_dev_scene *s, const rt_options *o) {
    if (!s || !options_ok(o)) return RT_E_ARG;
    const int wide = s->opt.inw_wide_walk, linear = s->opt.iow_linear;  // [build] options stay
    s->opt = *o;
    s->opt.inw_wide_walk = wide;
    s->opt.iow_linear = linear;
    return RT_OK;
}

int rt_debug_build_level_cap(int levels) {
    if (levels < 0) return RT_E_ARG;
    g_build_levels = levels;
    return RT_OK;
}

int rt_debug_wide_info(rt_dev_scene *s, uint32_t info[8], uint32_t *rank_out) {
    if (!s || s->kind == 3 || !info) return RT_E_ARG;
    HIP_OK(hipSetDevice(s->device));
    HIP_OK(hipDeviceSynchronize());
    const uint32_t cells = s->ri_ok ? uint32_t(s->ri_dim[0]) * uint32_t(s->ri_dim[1]) * uint32_t(s->ri_dim[2]) : 0u;
    const uint32_t v[8] = {s->n_wtree0, s->dfs_high, uint32_t(s->wdepth), s->ri_ok ? 1u : 0u, cells,
                           s->sl_ok ? 1u : 0u, s->n, s->wbuild};
    std::memcpy(info, v, sizeof(v));
    if (rank_out && s->n_wnodes)
        HIP_OK(hipMemcpy(rank_out, s->wrank.p, size_t(s->n) * 2 * sizeof(uint32_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_path(rt_dev_scene *s, rt_path_info *out) {
    if (!s || !out) return RT_E_ARG;
    char name[64] = {0};
    const int n = rt_debug_launches(s, name, int(sizeof(name)));  // resolves the fold kernel (synchronises)
    if (n < 0) return n;
    rt_path_info P = s->last_path;
    std::memcpy(P.kernel, name, sizeof(P.kernel));
    P.launches = n;
    P.ref_walks = 0;
    if (s->kind != 3 && s->walk_ctr.p) {
        unsigned long long v = 0;
        HIP_OK(hipMemcpy(&v, s->walk_ctr.p, sizeof(v), hipMemcpyDeviceToHost));
        P.ref_walks = v;
    }
    if (std::strncmp(name, "k_inw_pm", 8) == 0) {
        P.order = 1;
        P.ring_entries = int(s->last_ring[0]);
        P.ring_lds = s->last_lring ? 1 : 0;
        if (s->last_lring && !s->last_gq) { P.lds_nodes = 0; P.lbvh_lds_nodes = 0; }  // the FStack ring instances stage no nodes
        if (s->last_ln && !s->last_lring) P.time_bins = 0;  // the global-ring LN instance walks the staged swept tree
    }
    else if (std::strncmp(name, "k_inw_sm", 8) == 0) {
        P.order = 2;
        P.ring_entries = int(s->last_ring[1]);
        P.ring_lds = s->last_lring_sm ? 1 : 0;
        if (s->last_lring_sm) P.lds_nodes = std::min(P.lds_nodes, int(rtk::kPmLdsNodes));
        if (s->last_lring_sm) P.lbvh_lds_nodes = std::min(P.lbvh_lds_nodes, int(rtk::kPmLdsNodes * 10 / 2));
        if (s->last_ln) P.time_bins = 0;  // its walks read the staged top of the swept tree
        if (s->last_gq) {  // the GQ instance is pixel-major only: k_inw_sm ran the 236-node FStack kernel
            P.qnodes = 0; P.global_stack = 0; P.walk_stack = rtk::kFStack - 3;
            P.lds_nodes = s->last_lring_sm ? std::min(s->n_wtree0, rtk::kPmLdsNodes) : std::min(s->n_wtree0, uint32_t(rtk::kInwLdsNodes));
        }
    }
    if (P.order != 1) { P.beams = 0; P.claim_order = 0; P.beam_bins = 0; }  // both serve the pixel-major kernel only
    *out = P;
    return RT_OK;
}

// Diagnostics (not part of the reference's surface): pass a device buffer of 8 u64 to make
// the kernels tally lane occupancy per phase; NULL turns it off.
int rt_debug_pixel_rays(uint32_t *d_buf) {
    g_px_rays = d_buf;
    return RT_OK;
}

int rt_debug_rounds(rt_dev_scene *s, uint32_t *out, int cap) {
    if (!s || !out || cap <= 0) return RT_E_ARG;
    if (!s->cont_count.p) return 0;
    std::vector<unsigned> v(16 * 16);
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(v.data(), s->cont_count.p, v.size() * sizeof(unsigned), hipMemcpyDeviceToHost));
    const int n = std::min(cap, 16);
    for (int r = 0; r < n; r++) out[r] = v[size_t(16) * r];
    return n;
}

int rt_debug_spec_hist(rt_dev_scene *s, uint64_t *out) {
    if (!s || !out) return RT_E_ARG;
    std::memset(out, 0, 66 * sizeof(uint64_t));
    if (!s->spec_cap) return RT_OK;
    DevBuf d;
    HIP_OK(d.alloc(66 * sizeof(uint64_t)));
    HIP_OK(hipMemset(d.p, 0, 66 * sizeof(uint64_t)));
    HIP_OK(rtk::spec_hist(s->sp_ctr.as<uint4>(), s->spec_cap, d.as<unsigned long long>(), nullptr));
    HIP_OK(hipMemcpy(out, d.p, 66 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_spec_list_hist(rt_dev_scene *s, uint64_t *out) {
    if (!s || !out) return RT_E_ARG;
    std::memset(out, 0, 66 * sizeof(uint64_t));
    if (!s->spec_cap) return RT_OK;
    DevBuf d;
    HIP_OK(d.alloc(66 * sizeof(uint64_t)));
    HIP_OK(hipMemset(d.p, 0, 66 * sizeof(uint64_t)));
    HIP_OK(rtk::spec_list_hist(s->sp_ctr.as<uint4>(), s->spec_P, s->spec_S, s->sp_list.as<uint32_t>(),
                               s->sp_counts.as<unsigned>(), d.as<unsigned long long>(), nullptr));
    HIP_OK(hipMemcpy(out, d.p, 66 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_spec_list_stale(rt_dev_scene *s, uint64_t *out) {
    if (!s || !out) return RT_E_ARG;
    std::memset(out, 0, 32 * sizeof(uint64_t));
    if (!s->spec_cap) return RT_OK;
    DevBuf d;
    HIP_OK(d.alloc(32 * sizeof(uint64_t)));
    HIP_OK(hipMemset(d.p, 0, 32 * sizeof(uint64_t)));
    HIP_OK(rtk::spec_list_stale(s->sp_ctr.as<uint4>(), s->spec_P, s->spec_S, s->sp_list.as<uint32_t>(),
                                s->sp_counts.as<unsigned>(), d.as<unsigned long long>(), nullptr));
    HIP_OK(hipMemcpy(out, d.p, 32 * sizeof(uint64_t), hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_spec_pixels(rt_dev_scene *s, uint32_t *out, uint32_t cap_units) {
    if (!s || !out) return RT_E_ARG;
    if (!s->spec_cap || !s->spec_P || s->spec_P > cap_units) return RT_E_ARG;
    const uint32_t P = s->spec_P, S = s->spec_S;  // the last render's record layout
    DevBuf d;
    HIP_OK(d.alloc(size_t(P) * 16));
    HIP_OK(rtk::spec_pixels(s->sp_ctr.as<uint4>(), P, S, s->ws_order.as<uint32_t>(), d.as<uint32_t>(), nullptr));
    HIP_OK(hipMemcpy(out, d.p, size_t(P) * 16, hipMemcpyDeviceToHost));
    return int(P);
}

int rt_debug_spec_dump(rt_dev_scene *s, uint32_t *rays_out, size_t cap, uint32_t *list_out, uint32_t list_cap,
                       uint32_t *dims) {
    if (!s || !rays_out || !dims) return RT_E_ARG;
    if (!s->spec_cap || !s->spec_P) return RT_E_ARG;
    const uint32_t P = s->spec_P, S = s->spec_S;  // the last render's record layout (SpecRecs::ix)
    if (size_t(P) * S > cap) return RT_E_ARG;
    std::vector<uint4> h(size_t(P) * S);
    HIP_OK(hipMemcpy(h.data(), s->sp_ctr.p, h.size() * sizeof(uint4), hipMemcpyDeviceToHost));
    for (size_t u = 0; u < h.size(); u++) rays_out[u] = h[rtk::spec_rec_ix(u, P, S)].x;  // in unit order s * P + pu
    unsigned cnt[32] = {};
    HIP_OK(hipMemcpy(cnt, s->sp_counts.p, sizeof(cnt), hipMemcpyDeviceToHost));
    const uint32_t nl = std::min(cnt[0], list_cap);
    if (list_out && nl) HIP_OK(hipMemcpy(list_out, s->sp_list.p, size_t(nl) * 4, hipMemcpyDeviceToHost));
    dims[0] = P; dims[1] = S; dims[2] = cnt[0]; dims[3] = cnt[16];
    return RT_OK;
}

int rt_debug_spec_times(rt_dev_scene *s, uint32_t *start_out, uint32_t *end_out, size_t cap) {
    if (!s || !start_out || !end_out || !s->sp_dbg_n || !s->sp_dbg_t.p) return RT_E_ARG;
    const size_t n = s->sp_dbg_n;  // the last render's P * S: its end times start at offset n
    if (n > cap || s->sp_dbg_t.bytes < 2 * n * sizeof(uint32_t)) return RT_E_ARG;
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(start_out, s->sp_dbg_t.p, n * 4, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(end_out, static_cast<char *>(s->sp_dbg_t.p) + n * 4, n * 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_launches(rt_dev_scene *s, char *name_out, int name_cap) {
    if (!s) return RT_E_ARG;
    if (s->last_kernel == std::string("k_inw_fold<true>") || s->last_kernel == std::string("k_inw_fold<false>")) {
        // the probe picked the fold kernel on the device: read its verdict (synchronises)
        uint32_t m[2] = {0, 0};
        HIP_OK(hipDeviceSynchronize());
        HIP_OK(hipMemcpy(m, s->inw_mode.p, sizeof(m), hipMemcpyDeviceToHost));
        const uint32_t ord = s->last_force;  // the order the launch used (0: the probe's verdict)
        const bool sm = ord == 2 || (ord != 1 && m[0] > 0 && 2 * m[1] >= m[0]);
        // the template instance's name as rocprofv3 prints it, every template argument:
        // <LIGHTS, LN (LDS-staged BVH top), FU (fused cull), LRING (the fold ring in LDS)[, GQ (k_inw_pm)]>
        auto tf = [](bool b) { return b ? "true" : "false"; };
        const bool fu = s->last_fu, ln = s->last_ln, lights = s->layout == 4;
        if (sm)
            std::snprintf(s->kname, sizeof(s->kname), "k_inw_sm<%s, %s, %s, %s>", tf(lights), tf(ln), tf(fu),
                          tf(s->last_lring_sm));
        else
            std::snprintf(s->kname, sizeof(s->kname), "k_inw_pm<%s, %s, %s, %s, %s>", tf(lights), tf(ln), tf(fu),
                          tf(s->last_lring || s->last_gq), tf(s->last_gq));
        s->last_kernel = s->kname;
    }
    if (name_out && name_cap > 0) {
        std::strncpy(name_out, s->last_kernel, size_t(name_cap) - 1);
        name_out[name_cap - 1] = 0;
    }
    return s->last_launches;
}

int rt_debug_chunks(rt_dev_scene *s) {
    if (!s) return RT_E_ARG;
    return s->last_chunks;
}

int rt_debug_check_fastmath(int which, uint64_t *mismatches, uint32_t *first_bad) {
    if (!mismatches || !first_bad || which != 0) return RT_E_ARG;
    DevBuf d;
    HIP_OK(d.alloc(16));
    HIP_OK(hipMemset(d.p, 0, 8));
    HIP_OK(hipMemset(static_cast<char *>(d.p) + 8, 0xff, 4));
    HIP_OK(rtk::launch_check_fastmath(which, d.as<unsigned long long>(), reinterpret_cast<unsigned *>(static_cast<char *>(d.p) + 8),
                                 nullptr));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(mismatches, d.p, 8, hipMemcpyDeviceToHost));
    HIP_OK(hipMemcpy(first_bad, static_cast<char *>(d.p) + 8, 4, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_debug_time_kernels(int on) {
    g_time_kernels = on != 0;
    return RT_OK;
}

int rt_debug_kernel_time(rt_dev_scene *s, double *ms_total, int *launches) {
    if (!s || !ms_total || !launches) return RT_E_ARG;
    double t = 0.0;
    for (size_t i = 0; i < s->kt_used; i++) {
        HIP_OK(hipEventSynchronize(s->kt_ev[i].second));
        float ms = 0.0f;
        HIP_OK(hipEventElapsedTime(&ms, s->kt_ev[i].first, s->kt_ev[i].second));
        t += ms;
    }
    *ms_total = t;
    *launches = int(s->kt_used);
    return RT_OK;
}

int rt_debug_counters(uint64_t *d_buf) {
    g_dbg = reinterpret_cast<unsigned long long *>(d_buf);
    return RT_OK;
}

int rt_device_info(int device, char *name_out, int name_cap, int *cu_count) {
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    int cur = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&cur) != hipSuccess || hipGetDeviceProperties(&prop, cur) != hipSuccess) return RT_E_HIP;
    if (name_out && name_cap > 0) std::snprintf(name_out, size_t(name_cap), "%s (%s)", prop.name, prop.gcnArchName);
    if (cu_count) *cu_count = prop.multiProcessorCount;
    return RT_OK;
}

int rt_render_iow01(const rt_camera *cam, const float sphere[4], const rt_params *p, float *rgba, rt_stats *st) {
    if (!cam || !sphere || !params_ok(p) || !rgba) return RT_E_ARG;
    int rc = check_device(p->device);
    if (rc != RT_OK) return rc;
    rtk::Frame f = make_frame(cam, p);
    std::memcpy(f.sphere, sphere, sizeof(f.sphere));
    const size_t npx = size_t(p->width) * p->height;
    DevBuf d_rgba;
    HIP_OK(d_rgba.alloc(npx * 16));
    HIP_OK(hipMemcpy(d_rgba.p, rgba, npx * 16, hipMemcpyHostToDevice));
    f.out_rgba = d_rgba.as<float>();
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, nullptr));
    hipError_t e = rtk::launch_iow01(f, nullptr);
    HIP_OK(hipEventRecord(e1, nullptr));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    HIP_OK(e);
    HIP_OK(hipMemcpy(rgba, d_rgba.p, npx * 16, hipMemcpyDeviceToHost));
    if (st) {
        std::memset(st, 0, sizeof(*st));
        st->segments = uint64_t(f.tw) * uint64_t(f.th);
        st->ms = ms;
    }
    return RT_OK;
}

int rt_render_iow03(const float *types, const float *records, uint32_t n, const rt_camera *cam,
                    const rt_params *p, float *rgba, rt_stats *st) {
    if (!types || !records || !cam || !params_ok(p) || !rgba) return RT_E_ARG;
    int rc = check_device(p->device);
    if (rc != RT_OK) return rc;
    std::unique_ptr<rt_dev_scene> s(new (std::nothrow) rt_dev_scene());
    if (!s) return RT_E_ARG;
    rc = make_iow03(s.get(), types, records, n, p->spp);
    if (rc != RT_OK) return rc;
    return render_blocking(s.get(), cam, p, rgba, nullptr, st);
}

int rt_render_inw(const float *geom, uint32_t n, int layout, const float *nodes, const float *lights,
                  uint32_t n_lights, const rt_camera *cam, const rt_params *p, float *rgba, float *depth,
                  rt_stats *st) {
    return rt_render_inw_tex(geom, n, layout, nodes, lights, n_lights, nullptr, 0, cam, p, rgba, depth, st);
}

int rt_render_inw_tex(const float *geom, uint32_t n, int layout, const float *nodes, const float *lights,
                      uint32_t n_lights, const rt_texture *tex, int n_tex, const rt_camera *cam, const rt_params *p,
                      float *rgba, float *depth, rt_stats *st) {
    if (!geom || !nodes || n == 0 || !cam || !params_ok(p) || !rgba) return RT_E_ARG;
    if (layout != 1 && layout != 4) return RT_E_ARG;
    if (layout == 4 && n_lights > 0 && !lights) return RT_E_ARG;
    if (!textures_ok(tex, n_tex)) return RT_E_ARG;
    if (n_tex == 0 && inw_textured(geom, n, layout)) return RT_E_UNSUPPORTED;  // no texture bound
    int rc = check_device(p->device);
    if (rc != RT_OK) return rc;
    std::unique_ptr<rt_dev_scene> s(new (std::nothrow) rt_dev_scene());
    if (!s) return RT_E_ARG;
    rc = make_inw(s.get(), geom, n, layout, nodes, lights, n_lights, tex, n_tex, p->spp);
    if (rc != RT_OK) return rc;
    return render_blocking(s.get(), cam, p, rgba, depth, st);
}

int rt_inw_host_build(const float *nodes, uint32_t n, uint32_t info[8], double *ms) {
    if (!nodes || n == 0) return RT_E_ARG;
    try {
        const auto t0 = std::chrono::steady_clock::now();
        rtamd::InwWide w;
        rtamd::RiGrid g;
        const bool ok = rtamd::inw_wide_build(nodes, n, w);
        if (ok) g = rtamd::ri_grid_build(w.leafbox.data(), n);
        const auto t1 = std::chrono::steady_clock::now();
        if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (info) {
            const uint32_t v[8] = {uint32_t(w.wnodes.size() / 40), w.dfs_high, uint32_t(w.depth), g.ok ? 1u : 0u,
                                   g.ok ? uint32_t(g.cells.size() - 1) : 0u, uint32_t(g.ids.size()), 0u, 0u};
            std::memcpy(info, v, sizeof(v));
        }
    } catch (...) {
        return RT_E_ARG;
    }
    return RT_OK;
}

int rt_debug_time_bins(const float *nodes, const float *geom, uint32_t n, uint32_t bins, float *wnodes_out,
                       uint32_t wnodes_cap, uint32_t info[4]) {
    if (!nodes || !geom || n == 0 || !info) return RT_E_ARG;
    try {
        rtamd::InwWide w;
        if (!rtamd::inw_wide_build(nodes, n, w)) { std::memset(info, 0, 4 * sizeof(uint32_t)); return RT_OK; }
        rtamd::inw_wide_add_bins(geom, n, bins, w);
        const uint32_t total = uint32_t(w.wnodes.size() / 40);
        const uint32_t v[4] = {w.n_tree0, w.bins, w.bin_stride, total};
        std::memcpy(info, v, sizeof(v));
        if (wnodes_out && wnodes_cap >= total) std::memcpy(wnodes_out, w.wnodes.data(), w.wnodes.size() * sizeof(float));
    } catch (...) {
        return RT_E_ARG;
    }
    return RT_OK;
}

int rt_debug_bin_boxes(const float *geom, uint32_t n, uint32_t bins, uint32_t b, float *boxes_out) {
    if (!geom || !boxes_out || n == 0 || bins == 0 || b >= bins) return RT_E_ARG;
    try {
        std::vector<float> boxes;
        float wb = 0.0f;
        if (!rtamd::inw_bin_boxes(geom, n, bins, b, boxes, wb)) return RT_E_ARG;
        std::memcpy(boxes_out, boxes.data(), boxes.size() * sizeof(float));
    } catch (...) {
        return RT_E_ARG;
    }
    return RT_OK;
}

int rt_debug_sphere_records(const float *geom, uint32_t n, int layout, float *out) {
    if (!geom || !out || n == 0 || (layout != 1 && layout != 4)) return RT_E_ARG;
    try {
        std::vector<float> r;
        if (!inw_sphere_records(geom, n, layout, r)) return 0;
        std::memcpy(out, r.data(), r.size() * sizeof(float));
    } catch (...) {
        return RT_E_ARG;
    }
    return 1;
}

int rt_iow_host_build(const float *types, const float *records, uint32_t n, uint32_t info[4], double *ms) {
    if (!types || !records || n == 0) return RT_E_ARG;
    try {
        const auto t0 = std::chrono::steady_clock::now();
        rtamd::IowCull c;
        const bool ok = rtamd::iow_cull_build(types, records, n, c);
        const auto t1 = std::chrono::steady_clock::now();
        if (ms) *ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        if (info) {
            const uint32_t v[4] = {ok ? c.n_wide : 0u, 0u, 0u, 0u};
            std::memcpy(info, v, sizeof(v));
        }
    } catch (...) {
        return RT_E_ARG;
    }
    return RT_OK;
}

int rt_lbvh_build(const float *aabbs, uint32_t n, float *nodes_out) {
    if (!aabbs || !nodes_out || n == 0) return RT_E_ARG;
    try {
        std::vector<float> v = rtamd::lbvh_build(aabbs, n);
        std::memcpy(nodes_out, v.data(), v.size() * sizeof(float));
    } catch (...) {
        return RT_E_ARG;
    }
    return RT_OK;
}

size_t rt_lbvh_workspace_bytes(uint32_t n) { return rtk::lbvh_workspace_bytes(n); }

int rt_lbvh_build_async(const float *d_aabbs, uint32_t n, float *d_nodes_out, void *d_ws, size_t ws_bytes,
                        void *stream) {
    if (!d_aabbs || !d_nodes_out || n == 0 || (n > 1 && (!d_ws || ws_bytes < rtk::lbvh_workspace_bytes(n))))
        return RT_E_ARG;
    if (n > (1u << 24)) return RT_E_UNSUPPORTED;  // node / object ids are stored as floats (exact to 2^24)
    const hipError_t e = rtk::lbvh_build_device(d_aabbs, n, d_nodes_out, d_ws, ws_bytes, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        std::fprintf(stderr, "[rt_hip] lbvh build failed: %s\n", hipGetErrorString(e));
        return RT_E_HIP;
    }
    return RT_OK;
}

int rt_lbvh_build_gpu(const float *aabbs, uint32_t n, float *nodes_out, int device, double *ms) {
    if (!aabbs || !nodes_out || n == 0) return RT_E_ARG;
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    const size_t total = 2 * size_t(n) - 1;
    DevBuf d_in, d_out, d_ws;
    HIP_OK(d_in.upload(aabbs, size_t(n) * 6 * sizeof(float)));
    HIP_OK(d_out.alloc(total * 8 * sizeof(float)));
    HIP_OK(d_ws.alloc(rtk::lbvh_workspace_bytes(n)));
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, nullptr));
    rc = rt_lbvh_build_async(d_in.as<float>(), n, d_out.as<float>(), d_ws.p, d_ws.bytes, nullptr);
    HIP_OK(hipEventRecord(e1, nullptr));
    HIP_OK(hipEventSynchronize(e1));
    float t = 0.0f;
    (void)hipEventElapsedTime(&t, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (ms) *ms = t;
    if (rc != RT_OK) return rc;
    HIP_OK(hipMemcpy(nodes_out, d_out.p, total * 8 * sizeof(float), hipMemcpyDeviceToHost));
    return RT_OK;
}

size_t rt_noise_workspace_bytes(int width, int height) {
    return width > 0 && height > 0 ? rtk::noise_workspace_bytes(width, height) : 0;
}


int rt_noise_texture_async(int width, int height, int type, const float *gradient, int n_grad, float freq,
                           float lac, float gain, int octaves, uint8_t *d_rgb_out, void *d_ws, size_t ws_bytes,
                           void *stream) {
    if (!noise_args_ok(width, height, type, gradient, n_grad, octaves) || !d_rgb_out || !d_ws ||
        ws_bytes < rtk::noise_workspace_bytes(width, height))
        return RT_E_ARG;
    const hipError_t e = rtk::noise_texture(width, height, type, gradient, n_grad, freq, lac, gain, octaves, d_rgb_out,
                                            d_ws, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        std::fprintf(stderr, "[rt_hip] noise texture failed: %s\n", hipGetErrorString(e));
        return RT_E_HIP;
    }
    return RT_OK;
}

int rt_noise_texture(int width, int height, int type, const float *gradient, int n_grad, float freq, float lac,
                     float gain, int octaves, uint8_t *rgb_out, int device, double *ms) {
    if (!noise_args_ok(width, height, type, gradient, n_grad, octaves) || !rgb_out) return RT_E_ARG;
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    const size_t bytes = size_t(width) * size_t(height) * 3;
    DevBuf d_out, d_ws;
    HIP_OK(d_out.alloc(bytes));
    HIP_OK(d_ws.alloc(rtk::noise_workspace_bytes(width, height)));
    rc = timed([&] {
        return rt_noise_texture_async(width, height, type, gradient, n_grad, freq, lac, gain, octaves,
                                      d_out.as<uint8_t>(), d_ws.p, d_ws.bytes, nullptr);
    }, ms);
    if (rc != RT_OK) return rc;
    uint32_t status = 0;
    HIP_OK(hipMemcpy(&status, d_ws.as<uint32_t>() + 2, sizeof(status), hipMemcpyDeviceToHost));
    if (status) return RT_E_ARG;  // degenerate value range (the reference divides by zero)
    HIP_OK(hipMemcpy(rgb_out, d_out.p, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
}

size_t rt_remap_workspace_bytes(int width, int height) {
    return width > 0 && height > 0 ? rtk::remap_workspace_bytes(width, height) : 0;
}

int rt_texture_remap_async(const uint8_t *d_in, int width, int height, int channels, int load_as, int map_to,
                           uint8_t *d_out, void *d_ws, size_t ws_bytes, void *stream) {
    if (!remap_args_ok(width, height, channels, load_as, map_to) || !d_in || !d_out) return RT_E_ARG;
    const hipStream_t st = static_cast<hipStream_t>(stream);
    hipError_t e;
    if (load_as == map_to) {
        e = hipMemcpyAsync(d_out, d_in, size_t(width) * height * channels, hipMemcpyDeviceToDevice, st);
    } else {
        if (!d_ws || ws_bytes < rtk::remap_workspace_bytes(width, height)) return RT_E_ARG;
        e = rtk::texture_remap(d_in, width, height, channels, load_as, d_out, d_ws, st);
    }
    if (e != hipSuccess) {
        std::fprintf(stderr, "[rt_hip] texture remap failed: %s\n", hipGetErrorString(e));
        return RT_E_HIP;
    }
    return RT_OK;
}

int rt_texture_remap(const uint8_t *in, int width, int height, int channels, int load_as, int map_to, uint8_t *out,
                     int device, double *ms) {
    if (!remap_args_ok(width, height, channels, load_as, map_to) || !in || !out) return RT_E_ARG;
    int rc = check_device(device);
    if (rc != RT_OK) return rc;
    const size_t bytes = size_t(width) * size_t(height) * channels;
    DevBuf d_in, d_out, d_ws;
    HIP_OK(d_in.upload(in, bytes));
    HIP_OK(d_out.alloc(bytes));
    HIP_OK(d_ws.alloc(rtk::remap_workspace_bytes(width, height)));
    rc = timed([&] {
        return rt_texture_remap_async(d_in.as<uint8_t>(), width, height, channels, load_as, map_to,
                                      d_out.as<uint8_t>(), d_ws.p, d_ws.bytes, nullptr);
    }, ms);
    if (rc != RT_OK) return rc;
    HIP_OK(hipMemcpy(out, d_out.p, bytes, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_tile_spiral(int width, int height, int tile_w, int tile_h, int *out, int cap) {
    if (width <= 0 || height <= 0 || tile_w <= 0 || tile_h <= 0 || cap < 0 || (cap > 0 && !out)) return RT_E_ARG;
    if (width / tile_w > 32766 || height / tile_h > 32766) return RT_E_ARG;  // int16 tile indices
    const std::vector<rtamd::SpiralTile> t = rtamd::tile_spiral(width, height, tile_w, tile_h);
    for (size_t i = 0; i < t.size() && int(i) < cap; i++) {
        out[4 * i] = t[i].tx; out[4 * i + 1] = t[i].ty; out[4 * i + 2] = t[i].w; out[4 * i + 3] = t[i].h;
    }
    return int(t.size());
}

int rt_render_spiral_async(rt_dev_scene *s, const rt_camera *cam, const rt_params *p, int tile_w, int tile_h,
                           int first, int count, float *d_rgba, float *d_depth, uint64_t *d_counters,
                           void *stream) {
    if (!s || !cam || !params_ok(p) || !d_rgba || tile_w <= 0 || tile_h <= 0 || first < 0 || count < 0)
        return RT_E_ARG;
    if (p->width / tile_w > 32766 || p->height / tile_h > 32766) return RT_E_ARG;
    const std::vector<rtamd::SpiralTile> t = rtamd::tile_spiral(p->width, p->height, tile_w, tile_h);
    int i = std::min(first, int(t.size()));
    const int end = int(std::min<size_t>(t.size(), size_t(i) + size_t(count)));
    for (; i < end; i++) {
        if (t[size_t(i)].w <= 0 || t[size_t(i)].h <= 0) continue;  // a zero-size dispatch draws nothing
        rt_params q = *p;
        q.tile_x0 = t[size_t(i)].tx * tile_w;
        q.tile_y0 = t[size_t(i)].ty * tile_h;
        q.tile_w = t[size_t(i)].w;
        q.tile_h = t[size_t(i)].h;
        const int rc = rt_render_image_async(s, cam, &q, d_rgba, d_depth, d_counters, stream);
        if (rc != RT_OK) return rc;
    }
    return end;
}

int rt_display_rgba8_async(const float *d_rgba, const float *d_depth, int width, int height, int use_depth,
                           uint8_t *d_out, void *stream) {
    if (width <= 0 || height <= 0 || !d_out || (use_depth ? !d_depth : !d_rgba)) return RT_E_ARG;
    const hipError_t e = rtk::display_rgba8(d_rgba, d_depth, uint32_t(size_t(width) * size_t(height)), use_depth,
                                            d_out, static_cast<hipStream_t>(stream));
    if (e != hipSuccess) {
        std::fprintf(stderr, "[rt_hip] display pass failed: %s\n", hipGetErrorString(e));
        return RT_E_HIP;
    }
    return RT_OK;
}

rt_dev_scene *rt_dev_scene_iow03(const float *types, const float *records, uint32_t n, int spp, int device) {
    if (!types || !records || spp < 1) return nullptr;
    if (check_device(device) != RT_OK) return nullptr;
    rt_dev_scene *s = new (std::nothrow) rt_dev_scene();
    if (!s) return nullptr;
    (void)hipGetDevice(&s->device);
    if (make_iow03(s, types, records, n, spp) != RT_OK) { delete s; return nullptr; }
    return s;
}

rt_dev_scene *rt_dev_scene_inw(const float *geom, uint32_t n, int layout, const float *nodes, const float *lights,
                               uint32_t n_lights, int spp, int device) {
    return rt_dev_scene_inw_tex(geom, n, layout, nodes, lights, n_lights, nullptr, 0, spp, device);
}

rt_dev_scene *rt_dev_scene_inw_tex(const float *geom, uint32_t n, int layout, const float *nodes,
                                   const float *lights, uint32_t n_lights, const rt_texture *tex, int n_tex,
                                   int spp, int device) {
    if (!geom || !nodes || n == 0 || spp < 1 || (layout != 1 && layout != 4)) return nullptr;
    if (layout == 4 && n_lights > 0 && !lights) return nullptr;
    if (!textures_ok(tex, n_tex)) return nullptr;
    if (n_tex == 0 && inw_textured(geom, n, layout)) return nullptr;
    if (check_device(device) != RT_OK) return nullptr;
    rt_dev_scene *s = new (std::nothrow) rt_dev_scene();
    if (!s) return nullptr;
    (void)hipGetDevice(&s->device);
    if (make_inw(s, geom, n, layout, nodes, lights, n_lights, tex, n_tex, spp) != RT_OK) { delete s; return nullptr; }
    return s;
}

void rt_dev_scene_free(rt_dev_scene *s) {
    if (!s) return;
    (void)hipDeviceSynchronize();  // the scene's internal stream may still run its last frame
    delete s;
}

int rt_render_tiles_async(rt_dev_scene *s, const rt_camera *cam, const rt_params *p, const int *d_tiles,
                          int n_tiles, int tile_size, float *d_out_packed, float *d_out_depth_packed,
                          uint64_t *d_counters, void *stream) {
    if (!s || !cam || !params_ok(p) || !d_tiles || n_tiles <= 0 || !d_out_packed) return RT_E_ARG;
    if (tile_size <= 0 || tile_size % 16 != 0) return RT_E_ARG;
    if (p->spp != s->spp) return RT_E_ARG;  // tables are built for the scene's spp
    rtk::Frame f = make_frame(cam, p);
    f.tiles = d_tiles; f.n_tiles = n_tiles; f.tile_size = tile_size;
    f.out_rgba = d_out_packed; f.out_depth = d_out_depth_packed;
    f.counters = reinterpret_cast<unsigned long long *>(d_counters);
    return launch_scene(s, f, static_cast<hipStream_t>(stream));
}

int rt_render_image_async(rt_dev_scene *s, const rt_camera *cam, const rt_params *p, float *d_rgba, float *d_depth,
                          uint64_t *d_counters, void *stream) {
    if (!s || !cam || !params_ok(p) || !d_rgba) return RT_E_ARG;
    if (p->spp != s->spp) return RT_E_ARG;
    rtk::Frame f = make_frame(cam, p);
    f.out_rgba = d_rgba; f.out_depth = d_depth;
    f.counters = reinterpret_cast<unsigned long long *>(d_counters);
    return launch_scene(s, f, static_cast<hipStream_t>(stream));
}

// ------------------------------------------------------------------------ rt_scene.h
int rt_scene_preset(int preset, uint32_t seed, int n_hint, rt_geom_desc *out, int cap, rt_cam_desc *cam,
                    rt_params *params) {
    try {
        std::vector<rt_geom_desc> v;
        rt_cam_desc c;
        rt_params p;
        int n = rtamd::scene_preset(preset, seed, n_hint, v, c, p);
        if (n < 0) return n;
        if (out) {
            if (cap < n) return RT_E_ARG;
            std::memcpy(out, v.data(), v.size() * sizeof(rt_geom_desc));
        }
        if (cam) *cam = c;
        if (params) *params = p;
        return n;
    } catch (...) {
        return RT_E_ARG;
    }
}

int rt_camera_from_desc(const rt_cam_desc *d, int stage, rt_camera *out) {
    if (!d || !out) return RT_E_ARG;
    const bool iow = stage == RT_STAGE_IOW01 || stage == RT_STAGE_IOW02 || stage == RT_STAGE_IOW03;
    if (!iow && stage != RT_STAGE_INW01 && stage != RT_STAGE_INW04) return RT_E_ARG;
    rtamd::Vec3 fr = rtamd::front_from_pitch_yaw(d->pitch_deg, d->yaw_deg, iow);
    std::memcpy(out->pos, d->position, sizeof(out->pos));
    out->dir[0] = fr.x; out->dir[1] = fr.y; out->dir[2] = fr.z;
    out->fov_y_rad = rtamd::radians(d->fov_y_deg);
    out->aperture = d->aperture;
    out->focus_dist = d->focus_dist;
    return RT_OK;
}

int rt_pack_iow03(const rt_geom_desc *g, uint32_t n, float *types, float *records) {
    if (!g || !types || !records) return RT_E_ARG;
    for (uint32_t k = 0; k < n; k++) {
        rtamd::IowGeometry geo = rtamd::to_iow(g[k]);
        geo.fill_buffer(records + size_t(k) * 24);
        types[k] = float(geo.type);
    }
    return RT_OK;
}

// Groups::Geometry::FillBuffer (groups.h:45-64) packs the same position / inverse rotation /
// scale / colour as the IOW-03 Geometry::FillBuffer (materials.h:48-76): its first 18 floats.
int rt_pack_iow02(const rt_geom_desc *g, uint32_t n, float *types, float *records) {
    if (!g || !types || !records) return RT_E_ARG;
    float r24[24];
    for (uint32_t k = 0; k < n; k++) {
        rtamd::IowGeometry geo = rtamd::to_iow(g[k]);
        geo.fill_buffer(r24);
        std::memcpy(records + size_t(k) * 18, r24, 18 * sizeof(float));
        types[k] = float(geo.type);
    }
    return RT_OK;
}

int rt_pack_inw(const rt_geom_desc *g, uint32_t n, int layout, float *geom, float *aabbs, float *lights,
                uint32_t *n_lights) {
    if (!g || (layout != 1 && layout != 4)) return RT_E_ARG;
    uint32_t nl = 0;
    for (uint32_t k = 0; k < n; k++) {
        std::pair<rtamd::Vec3, rtamd::Vec3> bb;
        if (layout == 1) {
            rtamd::GeometryData d = rtamd::to_inw01(g[k]);
            if (geom) d.fill_buffer(geom + size_t(k) * 28);
            bb = d.bb_min_max();
        } else {
            rtamd::GeometryData04 d = rtamd::to_inw04(g[k]);
            if (geom) d.fill_buffer(geom + size_t(k) * 28);
            bb = d.bb_min_max();
            if (d.emissive) {  // Lights::FillBuffer, lights.cpp:261-264
                if (lights) {
                    float *L = lights + size_t(nl) * 7;
                    L[0] = bb.first.x; L[1] = bb.first.y; L[2] = bb.first.z;
                    L[3] = bb.second.x; L[4] = bb.second.y; L[5] = bb.second.z;
                    uint32_t idx = k;
                    std::memcpy(L + 6, &idx, 4);
                }
                nl++;
            }
        }
        if (aabbs) {
            float *b = aabbs + size_t(k) * 6;
            b[0] = bb.first.x; b[1] = bb.first.y; b[2] = bb.first.z;
            b[3] = bb.second.x; b[4] = bb.second.y; b[5] = bb.second.z;
        }
    }
    if (n_lights) *n_lights = nl;
    return RT_OK;
}

int rt_sample_tables(int spp, float *sunflower, float *fib, int *ring) {
    if (spp < 1) return RT_E_ARG;
    rtamd::sample_tables(spp, sunflower, fib, ring);
    return RT_OK;
}

int rt_render_iow00(const rt_params *p, float *rgba) {
    if (!p || p->width <= 0 || p->height <= 0 || !rgba) return RT_E_ARG;
    int rc = check_device(p->device);
    if (rc != RT_OK) return rc;
    const size_t npx = size_t(p->width) * p->height;
    DevBuf d_rgba;
    HIP_OK(d_rgba.alloc(npx * 16));
    HIP_OK(rtk::launch_iow00(p->width, p->height, d_rgba.as<float>(), nullptr));
    HIP_OK(hipDeviceSynchronize());
    HIP_OK(hipMemcpy(rgba, d_rgba.p, npx * 16, hipMemcpyDeviceToHost));
    return RT_OK;
}

int rt_render_iow02(const float *types, const float *records, uint32_t n, const rt_camera *cam, const rt_params *p,
                    int cull_front, int cull_back, float *rgba, rt_stats *st) {
    if ((n > 0 && (!types || !records)) || !cam || !params_ok(p) || !rgba) return RT_E_ARG;
    int rc = check_device(p->device);
    if (rc != RT_OK) return rc;
    rtk::Frame f = make_frame(cam, p);
    const size_t npx = size_t(p->width) * p->height;
    // host tables: the ring schedule (02.glsl:146-157) and pow(0.4, i) (02.glsl:206), double -> float
    std::vector<int> ring(size_t(p->spp) * 2);
    rtamd::sample_tables(p->spp, nullptr, nullptr, ring.data());
    std::vector<float> pw(size_t(std::max(1, p->max_bounces)));
    for (int i = 0; i < p->max_bounces; i++) pw[size_t(i)] = float(std::pow(double(0.4f), double(i)));
    DevBuf d_rgba, d_types, d_rec, d_ring, d_pw, d_ctr;
    HIP_OK(d_rgba.alloc(npx * 16));
    HIP_OK(hipMemcpy(d_rgba.p, rgba, npx * 16, hipMemcpyHostToDevice));  // untouched pixels keep their value
    if (n > 0) {
        HIP_OK(d_types.upload(types, size_t(n) * sizeof(float)));
        HIP_OK(d_rec.upload(records, size_t(n) * 18 * sizeof(float)));
    }
    HIP_OK(d_ring.upload(ring.data(), ring.size() * sizeof(int)));
    HIP_OK(d_pw.upload(pw.data(), pw.size() * sizeof(float)));
    HIP_OK(d_ctr.alloc(6 * sizeof(unsigned long long)));
    HIP_OK(hipMemset(d_ctr.p, 0, 6 * sizeof(unsigned long long)));
    f.out_rgba = d_rgba.as<float>();
    f.counters = d_ctr.as<unsigned long long>();
    hipEvent_t e0, e1;
    HIP_OK(hipEventCreate(&e0));
    HIP_OK(hipEventCreate(&e1));
    HIP_OK(hipEventRecord(e0, nullptr));
    hipError_t e = rtk::launch_iow02(f, d_types.as<float>(), d_rec.as<float>(), n, d_ring.as<int>(), d_pw.as<float>(),
                                     cull_front, cull_back, nullptr);
    HIP_OK(hipEventRecord(e1, nullptr));
    HIP_OK(hipEventSynchronize(e1));
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    HIP_OK(e);
    HIP_OK(hipMemcpy(rgba, d_rgba.p, npx * 16, hipMemcpyDeviceToHost));
    if (st) {
        unsigned long long c[6];
        HIP_OK(hipMemcpy(c, d_ctr.p, sizeof(c), hipMemcpyDeviceToHost));
        std::memset(st, 0, sizeof(*st));
        st->segments = c[0];
        st->prim_tests = c[2];
        st->ms = ms;
    }
    return RT_OK;
}

int rt_render_inw_mf(const float *geom, uint32_t n, const float *nodes, const rt_camera *cam, const float *focus,
                     int n_focus, const rt_params *p, float *rgba, float *depth, rt_stats *st) {
    if (!geom || !nodes || n == 0 || !cam || !params_ok(p) || !rgba || !focus || n_focus < 1 || n_focus > 9)
        return RT_E_ARG;
    int rc = check_device(p->device);
    if (rc != RT_OK) return rc;
    std::unique_ptr<rt_dev_scene> s(new (std::nothrow) rt_dev_scene());
    if (!s) return RT_E_ARG;
    rc = make_inw(s.get(), geom, n, 1, nodes, nullptr, 0, nullptr, 0, p->spp);
    if (rc != RT_OK) return rc;
    s->n_focus = n_focus;
    std::memcpy(s->focus, focus, sizeof(float) * size_t(n_focus));
    return render_blocking(s.get(), cam, p, rgba, depth, st);
}

}  // extern "C"
