// rt_kernels.hpp -- launch-side declarations shared by rt_kernels.hip and rt_capi.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace rtk {

// Per-launch uniforms, computed on the host exactly as the reference host + shader
// prologue would (camera vectors are derived on the device with the contract's ops).
struct Frame {
    int W, H, spp, max_bounces, show_normal;
    // pixel mapping: rect mode (tiles == nullptr) or tile-list mode
    int x0, y0, tw, th;
    const int *tiles;
    int n_tiles, tile_size;
    float *out_rgba;    // full image (rect mode) or packed tiles (tile mode)
    float *out_depth;   // may be null
    unsigned long long *counters;  // 6 x u64
    float pos[3], dir[3];
    float aperture, focus, screen_dist, inv_spp;
    float sphere[4];    // IOW-01 only
    unsigned long long *dbg;  // optional lane-occupancy counters (kDbg* slots), null in production
    int leaf_batch;           // IOW-03 walk: test postponed leaves once this many lanes hold one
    unsigned *px_rays;        // optional: rays cast per work unit, written when its pixel completes (IOW);
                              // INW fold kernels add one per segment at the output pixel's index
    int coop_max;             // IOW-03: wave-cooperative closest hits when at most this many lanes trace
    int dbg_first_stale;      // diagnostics: record the segment of a sample's first stale read (corrupts drops)
    // INW-01 MULTIFOCUS (01_BVH...glsl:388-404, 505-549; "#if MULTIFOCUS" in the reference):
    // n_focus = 0 is the single-focus camera the reference builds, 1..9 the lens chain
    int n_focus;
    float focus_list[9];
    int narrow;               // rt_options.iow_narrow (host side: iow_narrow)
    unsigned long long *walk_ctr;  // INW: closest-hit queries that fell back to the LBVH walks (added to; may be null)
};
// lane-occupancy counters (per wave-iteration: 1 and popcount of the participating lanes)
enum { kDbgOuter = 0, kDbgOuterLanes, kDbgTrav, kDbgTravLanes, kDbgLeaf, kDbgLeafLanes, kDbgSeg, kDbgSegLanes,
       // per-wave shader-clock cycles (IOW-03): camera-ray part of the work loop, closest-hit
       // queries, their BVH walk (incl. leaf tests), the leaf tests, ray segments (incl. query)
       kDbgCycCam, kDbgCycRay, kDbgCycTrav, kDbgCycLeaf, kDbgCycSeg, kDbgCycSpare0, kDbgCycSpare1, kDbgCycSpare2,
       kDbgSlots = 16 };

// IOW-03 device scene: "hot" records walked by the linear loop + "cold" hit attributes.
constexpr int kIowHot = 20;   // pos3 type M9 scale3 inv_scale3 pad
constexpr int kIowCold = 8;   // color3 material3 scat2
// INW device scene
constexpr int kInwHot = 28;   // pos3 R9 scale3 delta3 type extra inv_scale3 inv_s2_3 ri_acc pad
constexpr int kInwCold = 8;   // refr refl srfr srfl color3 ri

constexpr int kIowBvhStack = 32;  // IOW BVH traversal stack entries; a ray that overflows it also runs the linear loop
struct IowScene {
    const float *hot, *cold;
    uint32_t n;
    const float4 *nodes;     // conservative 4-wide BVH over the objects (8 float4 per node) or null = linear loop
    const float *sunflower;  // spp*2
    const float *fib;        // spp*4 (xyz + pad)
    const int *ring;         // spp*2
    int root_link;           // link of the BVH root (wide node 0 -> 1)
    const float4 *obox;      // the BVH leaves' conservative boxes: n float4 (lo.xyz, hi.x), n float2 (hi.yz); or null
    uint32_t n_nodes;        // 4-wide BVH nodes
    int lds_on;              // rt_options.iow_lds_bvh: the LDS-staged kernels may run (iow_lds)
};
struct InwScene {
    const float4 *hot;       // n * 7 float4
    const float4 *cold;      // n * 2 float4
    const float4 *nodes;     // (2n-1) * 2 float4
    const float *lights;     // L * 7
    uint32_t n, n_lights;
    int layout;
    const float *sunflower;  // spp*2
    // u_MaterialTextures (04...glsl:10): texels as float4 (unorm8 / 255, converted on the
    // host), tex_info[k] = (first texel, width, height, 0); n_tex = 0: none bound
    const float4 *tex;
    const int4 *tex_info;
    uint32_t n_tex;
    // Wide walk (DESIGN.md "INW wide walk"; null wnodes = off): a 4-wide culling BVH over the
    // LBVH leaf boxes, each object's rank in the reference's depth-first order for either child
    // order (rank[g] with invert false, rank[n + g] with invert true), its LBVH leaf node, and the
    // depth-first stack high-water mark (pushes can only drop when size + dfs_high > 40)
    const float4 *wnodes = nullptr;
    // the same nodes as 7 float4 (lx ly lz hx hy hz links; DESIGN.md §5.2 "Compact nodes"), read by
    // the buffer-load walk from global memory when set (the LDS staging and the other walks keep wnodes)
    const float4 *cnodes = nullptr;
    int wroot = 0;
    const uint32_t *rank = nullptr;
    const float4 *leafbox = nullptr;  // per object: its LBVH leaf node (2 float4: the reference's leaf box)
    // Sphere scenes (DESIGN.md §5.2 "Sphere records"; null = off): every object an ellipsoid of equal
    // scales with the identity rotation; per object 3 float4, (position, RN(1/scale)), (position -
    // last_position, its RI) and (RN(1/RN(scale^2)) per axis, extra: the hit normal's inputs).  The wide walk's, the beam lists' and the RI grid's object tests read
    // these instead of the 7-float4 record: R = I makes the object-space ray the world one, the same
    // floats (up to the signs of zero terms, which neither t nor the inside test can see); the
    // winner's normal still comes from the full record
    const float4 *sph = nullptr;
    uint32_t dfs_high = 0;
    uint32_t n_wnodes = 0;  // wide nodes
    uint32_t n_lnodes = 0;  // the first n_lnodes wide nodes are staged in LDS (LN kernels only)
    // Time-bin trees (wbins = 0: none): the wide closest-hit walk of a ray with time
    // ratio r starts at node 1 + wbin_base + b * wbin_stride, b = min(int(r * wbins), wbins - 1),
    // the root of the tree over the boxes the objects sweep in [b / wbins, (b + 1) / wbins]
    uint32_t wbins = 0, wbin_base = 0, wbin_stride = 0;
    // Stackless LBVH walks (rt_options.inw_stackless; DESIGN.md §5 "Stackless LBVH
    // walk"): the reference's depth-first walks without their stack, by parent links, wherever no
    // push of the reference walk could drop (size + dfs_high <= 40).  sl = 0: off (or the node
    // buffer lacks the layout: left children at odd indices, right = left + 1, rightData = parent)
    uint32_t sl = 0;
    uint32_t n_blds = 0;    // LN kernels without the wide walk: the first n_blds LBVH nodes staged in LDS
    int fused = 0;          // the wide walk culls with one fma per plane (cull4nf<true>; set per frame)
    uint32_t lring = 0;       // k_inw_pm (768-lane instances): the fold ring in LDS (kPmLdsRing entries per wave)
    uint32_t lring_sm = 0;    // k_inw_sm (768-lane instances): the same
    uint32_t xcdq = 0;        // k_inw_pm claims from per-XCD queues (rt_options.inw_claim_xcd)
    uint32_t ring_epoch = 0;  // fold-ring tags: the frame's epoch (0..62) << 26 (ring_tag, rt_kernels.hip)
    float4 *park = nullptr;   // RT_INW_PARK builds: 2 float4 of parked walk state per lane of the fold grid
    // Quantised wide nodes (DESIGN.md §5.2 "Quantised nodes"; null = off): the culling BVH of
    // wnodes as 4 float4 per node -- origin.xyz, scale.x | scale.yz, low-plane bytes x, y | low z,
    // high x, y, z (byte k = child k) | links -- each plane rounded outward (rt_build.hip:
    // k_quantize_wnodes).  Read by the wide closest-hit walk of the k_inw_pm<..., GQ> instance, which
    // also stages the first n_lnodes of them in LDS and keeps the reference's 40-float stack in
    // global memory (gstk: kFStack / 4 float4 per lane of the grid, [slot4][lane]).
    const float4 *qnodes = nullptr;
    float4 *gstk = nullptr;
    uint32_t gq_blocks = 0;  // the GQ instance's grid (kGqSub * kBlock lanes per block, resident blocks)
    // Pixel beams (DESIGN.md §5 "Pixel beams"; null beam = off): for each pixel unit, the objects
    // whose culling box the beam of its primary rays can cross, sorted by the entry t of the
    // central ray into the box inflated by beam_R (k_inw_beam).  The 64 lists of an 8x8 block are
    // packed in unit order in the block's region of 64 * beam_cap entries: beam_n[u] = offset in
    // the region << 8 | count (kBeamOff: use the wide walk), beam_cut[u] = every object with an
    // entry below it is listed.
    const uint2 *beam = nullptr;  // beam_cap entries per unit: object id, entry t (float bits); beam16:
                                  // one uint32 each, id in the low half, t's high half (t rounded down)
    uint32_t beam16 = 0;
    const uint32_t *beam_n = nullptr;
    const float *beam_cut = nullptr;
    uint32_t beam_cap = 0;
    // beam_bins > 1: one list per pixel unit and time bin (k_inw_beam walks bin b's tree, the one at
    // 1 + wbin_base + b * wbin_stride): the lists, counts and cuts of bin b follow those of bins < b
    // (beam_units units each); a primary ray reads its time bin's list
    uint32_t beam_bins = 0, beam_units = 0;
    float beam_R = 0.0f, beam_tmin = 0.0f, beam_tfar = 0.0f, beam_kappa = 0.0f;
    // Surrounding-RI grid (DESIGN.md §5 "RI grid"; null ri_cells = off): a uniform grid over the
    // LBVH leaf boxes; cell c lists (ri_ids[ri_cells[c] .. ri_cells[c + 1]]) every object whose
    // leaf box, widened by a margin above the rounding of the cell index, overlaps the cell.
    const uint32_t *ri_cells = nullptr, *ri_ids = nullptr;
    float ri_lo[3] = {0, 0, 0}, ri_hi[3] = {0, 0, 0}, ri_inv[3] = {0, 0, 0};
    int ri_dim[3] = {0, 0, 0};
};
constexpr uint32_t kBeamOff = 0xffffffffu;

// One launch of a chunked render: samples [s_begin, s_end) of every pixel unit.  A pixel's
// samples must run in order (IOW-03 reads stale stack slots of earlier samples), so the
// per-pixel state (accumulator + the IOW stack's RI slots) is parked in `state` between
// launches, `cost` records the rays each unit spent, and `order` (a permutation of unit ids,
// longest first) lets the next launch schedule the expensive pixels first.
struct Chunk {
    int s_begin, s_end;      // sample range of this launch
    int final_chunk;         // write the image (else park the state)
    float4 *state;           // 2 float4 per unit (may be null for a single-chunk render)
    const unsigned *order;   // unit permutation or null (natural order)
    unsigned *cost;          // rays per unit in this launch, or null
    const unsigned *order_count;  // device count of `order` entries (null: all units)
    int per_unit_begin;      // first sample of each unit = bits of state[2*unit].w (else s_begin)
    // sample-parallel records (SpecRecs, below) to validate before running a sample, or null:
    // a sample whose record assumed the exact incoming stack state is taken from the record
    const float4 *rec_col, *rec_fin, *rec_assume;
    const uint4 *rec_ctr;
    uint32_t rec_P, rec_S;  // their layout: unit s * rec_P + pu at pu * rec_S + s (SpecRecs::ix)
};

// Sample-parallel IOW-03 (DESIGN.md "Sample-parallel speculation").  A unit is one (pixel,
// sample) pair, u = s*P + pu.  Each sample runs with an assumed incoming stack state (the RI
// of entries 1..3 that earlier samples of the pixel left behind) and records what it read and
// wrote; a resolve pass replays the pixel's samples in order and re-queues every sample whose
// assumption was wrong.  Records are SoA over u.
struct AltRec {  // an alternative run of a speculative sample (RT_SPEC_ALT, DESIGN.md "Alternative runs")
    uint32_t u;      // unit (s * P + pu)
    uint32_t state;  // 0 queued / running, else 1 + the launch it finished in
    uint32_t pad0, pad1;
    float4 assume, col, fin;
    uint4 ctr;
};
struct SpecRecs {
    float4 *col;       // rgb of the sample, flags (bits: rmask 0-3, wmask 4-7)
    float4 *fin;       // RI of entries 1..3 after the sample, prim tests (bits)
    uint4 *ctr;        // segments, stack drops, NaN directions, node visits
    float4 *assume;    // assumed RI of entries 1..3 before the sample
    uint32_t P, S;     // pixel units, samples per pixel (s_stop)
    // The record of unit u = s * P + pu sits at pu * S + s: a pixel's samples are adjacent, so the
    // waves of the bulk pass (consecutive samples of one pixel) read and write whole lines, and the
    // per-pixel sample walks (chain following, the frontier rounds) stay in one line for 8 samples
    // (DESIGN.md §5.4).  u < 2^32; q = mulhi(u, pmag) is u / P or one more.
    __host__ __device__ __forceinline__ size_t ix(size_t u) const {
        const uint32_t uu = (uint32_t)u;
#ifdef __HIP_DEVICE_COMPILE__
        uint32_t q = __umulhi(uu, pmag);
#else
        uint32_t q = (uint32_t)(((uint64_t)uu * pmag) >> 32);
#endif
        int32_t r = (int32_t)(uu - q * P);
        if (r < 0) { q--; r += (int32_t)P; }
        return (size_t)(uint32_t)r * S + q;
    }
    uint32_t *list;    // re-execution list (units)
    unsigned *list_count;
    uint32_t *fb_list; // pixels left to the sequential kernel after the last resolve
    unsigned *fb_count;
    const uint32_t *order;  // pixel units, heaviest sample 0 first (kSpecRest)
    uint32_t order_base, order_n;  // this group's slice of `order` (order_n == 0: all P units)
    uint4 *pstate;     // asynchronous windows: per pixel unit 3 x uint4 of frontier state
    uint32_t epoch;    // frame tag: finished records carry it in their flags
    uint4 *front;      // checkpoint rounds: per pixel unit (first unvalidated sample, exact RI bits of entries 1..3)
    // heavy-first enumeration (fresh_mode 1..3): sample indices 1..S-1 by measured cost, most
    // expensive first; the first n_heavy of them run for every pixel before the rest
    const uint32_t *sorder;
    uint32_t probe_stride, n_heavy;
    // diagnostics (RT_SPEC_ORACLE=1): the final resolve stores every sample's exact incoming
    // RI of entries 1..3 (exact_mode bit 0) and the next render's guesses copy them (bit 1), so
    // a frame runs with no misprediction -- the bound any better guess could reach
    float4 *exact = nullptr;
    int exact_mode = 0;
    // checkpoint rounds: per pixel unit, the first unfinished sample past the main frontier whose
    // exact incoming state the anchored scan of k_iow03_frontier found, and that state (x =
    // 0xffffffff: none); k_iow03_fixf patches or restarts it like a sample at the frontier
    uint4 *front2 = nullptr;
    uint32_t scan_max = 0;  // samples the anchored scan may look past the main frontier (0 = off)
    // diagnostics (RT_DEBUG_TIMES=1): per unit, the launch of its last start (bits 0-15) and its
    // start count (bits 16-31), and the launch it finished in (rt_debug_spec_times)
    uint32_t *dbg_start = nullptr, *dbg_end = nullptr;
    // alternative runs: records, a hash u -> (first slot, count) with key u + 1 (0 = empty), the
    // slot counter, the values a stale entry can hold, and the segment count that makes a
    // sample long enough to get alternatives
    AltRec *alt = nullptr;
    uint2 *alt_hash = nullptr;
    unsigned *alt_count = nullptr;
    uint32_t alt_cap = 0, alt_hcap = 0, alt_min_seg = 0;
    float alt_vals[8] = {};
    int n_alt_vals = 0;
    uint32_t pmag = 0;  // ceil(2^32 / P) (spec_pmag): ix() divides a unit by P with one mulhi
};
// ceil(2^32 / P) for SpecRecs::pmag (P >= 2)
inline uint32_t spec_pmag(uint32_t P) { return (uint32_t)(((1ull << 32) + P - 1) / P); }
// the record index of unit u (SpecRecs::ix) by plain division (diagnostics, host reads)
__host__ __device__ inline size_t spec_rec_ix(size_t u, uint32_t P, uint32_t S) { return (u % P) * S + u / P; }
enum { kSpecFirst = 0, kSpecRest = 1, kSpecList = 2 };

// Tail compaction between launches.  Once the work queue is empty, a wave whose busy lanes
// fall below kParkBelow parks them (state at a ray-segment boundary) in `out`, slot ids from
// a wave-aggregated atomic on `out_count`, and exits; the next launch resumes the parked
// lanes from `in` in full waves.  in == null: the launch's units are pixels.  out == null or
// fewer than park_min units in the launch: lanes run to completion (the final round).
constexpr int kBlock = 256;      // threads per block of every render kernel
constexpr int kInwLdsNodes = 236;        // wide BVH nodes the INW fold kernels stage in LDS (rt_kernels.hip)
constexpr uint32_t kPmLdsRing = 256;     // k_inw_pm's LDS fold ring: entries per wave (InwScene::lring) ...
constexpr uint32_t kPmLdsNodes = 5;      // ... and the nodes it leaves staged
// k_inw_pm's GQ instance (DESIGN.md §5.1 "GQ": the reference's 40-float stacks in global memory):
// kGqSub 256-lane sub-blocks per block (= waves per SIMD; 1 block per CU), per block the wide walks'
// node stacks in LDS (kWStack entries per lane), the fold rings (3 KB per wave), the depth slots,
// and in the rest of the CU's 160 KB the top of the culling BVH: kQLdsNodes quantised nodes
// (kGqQn; 64 B each) or the 236 full ones of g_inw_lnodes
constexpr int kFStack = 40;  // stack_capacity (FLT_STACK, 01_BVH...glsl:80)
constexpr int kWStack = 16;
constexpr int kQNodeF4 = 4;
#ifndef RT_GQ_SUB
#define RT_GQ_SUB 3
#endif
#ifndef RT_GQ_QN
#define RT_GQ_QN 1
#endif
constexpr int kGqSub = RT_GQ_SUB;
constexpr bool kGqQn = RT_GQ_QN != 0;
constexpr int kGqLdsFree = 163840 - kGqSub * kWStack * kBlock * 4 - kGqSub * 4 * 3 * (int)kPmLdsRing * 4 -
                           kGqSub * kBlock * 4;
constexpr int kQLdsNodes = kGqLdsFree / 64;
constexpr int kParkBelow = 32;    // park when fewer than half the wave's lanes are busy
constexpr int kContSlots = 13;    // float4 per parked lane
struct Cont {
    const float4 *in;
    const unsigned *in_count;
    float4 *out;
    unsigned *out_count;
    uint32_t park_min;
    // sample-parallel checkpoint rounds: a launch takes the parked lanes of `in` first, then the
    // fresh units [fresh_lo, fresh_hi) of its mode (mixed != 0); park_below = 65 parks every
    // busy lane once the queue drains (0 = kParkBelow, the tail-compaction rule)
    int mixed, park_below;
    uint32_t fresh_lo, fresh_hi;
    // fresh units of kSpecRest: 0 = samples 1.. pixel-major in R.order; 1 = probe (every sample
    // of every probe_stride-th pixel of R.order); 2 = the n_heavy costliest sample indices,
    // sample-major; 3 = the other indices, pixel-major.  Modes 1-3 skip units already started.
    int fresh_mode;
    uint32_t seg_budget;  // > 0: a lane parks its unit after this many segments in the launch
    int spread;           // a wave takes at most ceil(units / waves) units at a time
    // units sorted longest first (the LPT re-execution list): while the queue head is below
    // min(solo_n, waves), an empty wave takes one unit and keeps it alone to the end, so
    // the longest samples run with the wave-cooperative closest hits instead of sharing a wave
    uint32_t solo_n;
    uint32_t launch_id;  // sequence number of the launch in the frame (diagnostics)
    int chain;           // exact restarts follow their pixel's chain of mispredicted samples
};

hipError_t launch_iow01(const Frame &f, hipStream_t s);
// rt_stages.hip: IOW-00 gradient, IOW-02 groups (records N x 18, ring = sample-table ring
// schedule, pw[i] = pow(0.4, i) for i < max_bounces)
hipError_t launch_iow00(int W, int H, float *out, hipStream_t s);
hipError_t launch_iow02(const Frame &f, const float *types, const float *rec, uint32_t n, const int *ring,
                        const float *pw, int cull_front, int cull_back, hipStream_t s);
// Persistent work-queue launches: `counter` (one u32, device) is zeroed on `s` before the
// kernel; at most `blocks_cap` blocks are launched (they pull pixels until none are left).
// n_units: pixel units (cont.in == null) or parked lanes to resume (host-known count)
hipError_t launch_iow03(const Frame &f, const IowScene &sc, const Chunk &ch, const Cont &ct, uint32_t n_units,
                        unsigned *counter, int s_stop, int blocks_cap, hipStream_t s);
hipError_t launch_inw(const Frame &f, const InwScene &sc, const Chunk &ch, const Cont &ct, uint32_t n_units,
                      unsigned *counter, int blocks_cap, hipStream_t s);
uint32_t units_of(const Frame &f);
// resident 256-thread blocks per CU for the persistent kernels (occupancy query)
// sample-parallel IOW-03 pass over the units of `mode` (kSpec*)
hipError_t launch_iow03_spec(const Frame &f, const IowScene &sc, const SpecRecs &R, int mode, const Cont &ct,
                             uint32_t n_units, unsigned *counter, int blocks_cap, hipStream_t s);
// LBVH build on the device (rt_lbvh.hip); ws = lbvh_workspace_bytes(n) of scratch; lcnt (optional,
// 2n - 1 entries): every node's leaf count, in the output's (breadth-first) numbering
size_t lbvh_workspace_bytes(uint32_t n);
hipError_t lbvh_build_device(const float *aabb, uint32_t n, float *out, void *ws, size_t ws_bytes, hipStream_t s,
                             uint32_t *lcnt = nullptr);
// INW wide walk structures built on the device from a device LBVH (rt_build.hip, DESIGN.md
// "Device build"): 4-wide culling BVH (10 float4 per node, <= n nodes), depth-first ranks (2n),
// leaf boxes (2n float4); out's scalars are filled in.  Synchronises the stream (level counts).
struct InwWideDev {
    float4 *wnodes;
    uint32_t *rank;
    float4 *leafbox;
    uint32_t n_wnodes, dfs_high;
    int depth;
    float wbound;
    float ri_lo[3], ri_hi[3];  // bounds of the leaf boxes (the RI grid's extent)
};
size_t inw_build_workspace_bytes(uint32_t n);
// nodes: the device LBVH (lbvh_build_device), lcnt: its leaf counts (lbvh_build_device's lcnt)
// max_levels (0 = 256): the binary SAH and collapse levels launched at most; a deeper tree returns
// hipErrorNotSupported (the caller then builds on the host)
hipError_t inw_wide_build_device(const float4 *nodes, const uint32_t *lcnt, uint32_t n, void *ws, size_t ws_bytes,
                                 InwWideDev &out, hipStream_t s, int max_levels = 0);
// the quantised form of nw wide nodes (InwScene::qnodes): 4 float4 per node, planes rounded
// outward by at least `margin` beyond the wide node's (rt_build.hip)
hipError_t inw_quantize_wnodes(const float4 *wnodes, uint32_t nw, float4 *qnodes, float margin, hipStream_t s);
// InwScene::cnodes from the wide nodes (rt_build.hip)
hipError_t inw_compact_wnodes(const float4 *wnodes, uint32_t nw, float4 *cnodes, hipStream_t s);
// the surrounding-RI grid on the device (rtamd::ri_grid_build's cells and ids) over the extent
// inw_wide_build_device returned: per-cell counts scanned into cells[0..nc] with the total and an
// over-64 flag read back (synchronises), then the ids
size_t ri_scan_temp_bytes(size_t cells);
hipError_t ri_count_device(const float4 *leafbox, uint32_t n, void *ws, const double lo[3], const double inv[3],
                           const int dim[3], uint32_t *cells, void *tmp, size_t tmp_bytes, uint32_t *total,
                           uint32_t *over, hipStream_t s);
hipError_t ri_fill_device(const float4 *leafbox, uint32_t n, const double lo[3], const double inv[3], const int dim[3],
                          const uint32_t *cells, uint32_t *fill, uint32_t *ids, hipStream_t s);
// Texture producers (rt_texture.hip): noise textures (MakeTexture, utility.h:69-192) and the
// Mercator <-> cubic re-projection (utility.cpp:266-463).  noise_batches_exact(W): the
// reference's 4 column batches tile [0, W) (other widths index out of bounds there).
bool noise_batches_exact(uint32_t W);
size_t noise_workspace_bytes(int W, int H);
hipError_t noise_texture(int W, int H, int type, const float *grad, int n_grad, float freq, float lac, float gain,
                         int octaves, uint8_t *d_rgb, void *d_ws, hipStream_t s);
// Display pass (rt_display.hip): RGBA32F colour or R32F depth -> RGBA8 framebuffer texels
hipError_t display_rgba8(const float *rgba, const float *depth, uint32_t n, int use_depth, uint8_t *out,
                         hipStream_t s);
size_t remap_workspace_bytes(int W, int H);
hipError_t texture_remap(const uint8_t *d_in, int W, int H, int C, int load_as, uint8_t *d_out, void *d_ws,
                         hipStream_t s);
hipError_t spec_hist(const uint4 *ctr, size_t n, unsigned long long *d_out, hipStream_t s);  // diagnostics
hipError_t spec_list_stale(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *list, const unsigned *count,
                           unsigned long long *d_out,
                           hipStream_t s);  // diagnostics
hipError_t spec_list_hist(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *list, const unsigned *count,
                          unsigned long long *d_out,
                          hipStream_t s);  // diagnostics
hipError_t spec_pixels(const uint4 *ctr, uint32_t P, uint32_t S, const uint32_t *order, uint32_t *d_out,
                       hipStream_t s);  // diagnostics
// after the kSpecFirst pass: assumptions for samples 1.. and the per-pixel ordering keys
// checkpoint rounds: advance each pixel's frontier over finished, valid samples and
// queue a finished sample at the frontier whose assumption was wrong for an exact re-run
// (appended to cont as a restart, at most cap entries in all); then make parked samples at the
// frontier exact (patch unread entries, or restart)
hipError_t launch_iow03_frontier(const Frame &f, const SpecRecs &R, float4 *cont, unsigned *count, uint32_t cap,
                                 hipStream_t s);
hipError_t launch_iow03_fixf(const Frame &f, const SpecRecs &R, float4 *cont, const unsigned *count, int max_lanes,
                             hipStream_t s);
// heavy-first enumeration: per sample index cost from the probe pixels' records and the parked
// lanes' progress -> R.sorder; per pixel cost of its heavy samples -> key (sort -> R.order)
hipError_t launch_iow03_sample_order(const Frame &f, const SpecRecs &R, const float4 *cont, const unsigned *count,
                                     int max_lanes, unsigned long long *fcost, uint32_t *sorder, hipStream_t s);
hipError_t launch_iow03_pixel_key(const Frame &f, const SpecRecs &R, const float4 *cont, const unsigned *count,
                                  int max_lanes, unsigned *key, hipStream_t s);
// rt_math.hpp's shortened sequences against the compiler's for all 2^32 x (k_check_fastmath):
// mismatch count, lowest bad x
hipError_t launch_check_fastmath(int which, unsigned long long *bad, unsigned *first, hipStream_t s);
hipError_t launch_iow03_altspawn(const Frame &f, const SpecRecs &R, float4 *cont, unsigned *count, uint32_t cap,
                                 hipStream_t s);
hipError_t launch_iow03_prep(const Frame &f, const SpecRecs &R, unsigned *key, float prior, uint32_t prior_from,
                             hipStream_t s);
// replay each pixel's samples: re-queue wrong assumptions; final: write clean pixels, hand
// the rest (with their resume state in `state`) to the sequential kernel via R.fb_list
hipError_t launch_iow03_resolve(const Frame &f, const SpecRecs &R, bool final_pass, float4 *state, hipStream_t s);

// sample-parallel INW over samples [s0, s0+ns) of every pixel (records indexed (s-s0)*P + pu),
// then End() over that chunk: carry the sum in `state` or write the pixels
// INW with the on-chip End() folds (k_inw_probe + k_inw_pm / k_inw_sm); ring:
// blocks * (kBlock / 64) * max(ring_pm, ring_sm) float4 (powers of two >= 64); counter: 2 queue
// counters 64 B apart; mode: 2 uints; force: 0 = probe decides, 1 = pixel-major, 2 = sample-major
// blocks_ln > 0: the fold kernels run as blocks_ln 768-lane blocks with the top of the wide BVH
// staged in LDS (ring: max(blocks * 4, blocks_ln * 12) waves)
hipError_t launch_inw_fold(const Frame &f, const InwScene &sc, float4 *ring, uint32_t ring_pm, uint32_t ring_sm,
                           unsigned *counter, uint32_t *mode, uint32_t force, int blocks, int blocks_ln,
                           uint32_t *cost, hipStream_t s);
// the pixel beams of a pixel-major frame (sc.beam*; exits when the probe picks sample-major)
hipError_t launch_inw_beam(const Frame &f, const InwScene &sc, const uint32_t *mode, uint32_t force, hipStream_t s);
// resident blocks per CU of the render kernel for `kind` (3 = IOW-03 wide, 4 = IOW-03 narrow,
// 11/14 = INW layout 1/4)
int resident_blocks_per_cu(int kind);  // 5 = sample-parallel IOW-03, 6/7 = sample-parallel INW 1/4,
                                       // 8 = asynchronous-window IOW-03
// IOW-03 kernel variant for this frame: narrow (byte bounce counts, 12-deep BVH stack, 4 waves
// per SIMD with spills) when rt_options.iow_narrow and u_NumOfBounce <= 255; wide otherwise
bool iow_narrow(const Frame &f);
bool iow_lds(const IowScene &sc);  // k_iow03L / k_iow03sL (BVH in LDS) apply (sc.lds_on and it fits); their blocks_cap counts 256-lane slots
// order[i] = unit ids sorted by cost, most expensive first (hipcub radix sort)
hipError_t sort_units_by_cost(const unsigned *cost, unsigned *keys_tmp, const unsigned *iota, unsigned *order,
                              uint32_t n, void *temp, size_t temp_bytes, hipStream_t s);
size_t sort_temp_bytes(uint32_t n);
// descending key/value radix sort over bits [0, end_bit)
size_t sort_pairs_temp_bytes(size_t n, int end_bit);
hipError_t sort_pairs_desc(const unsigned *keys_in, unsigned *keys_out, const unsigned *vals_in, unsigned *vals_out,
                           size_t n, void *temp, size_t temp_bytes, int end_bit, hipStream_t s);
// keys for ordering the re-execution list longest-first: the ray count of each listed unit's
// previous execution (0 beyond the list's count)
hipError_t spec_list_keys(const SpecRecs &R, unsigned *keys, size_t n, hipStream_t s);

}  // namespace rtk
