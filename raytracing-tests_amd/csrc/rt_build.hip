// rt_build.hip -- the INW wide walk's per-redraw structures built on the device (DESIGN.md §4-5
// "Device build"), from the LBVH the device just built (rt_lbvh.hip; the reference rebuilds it on
// every redraw, In-Next-Week/base.h:96-175, ConstructLBVH_Buff at :135-142):
//   - every object's LBVH leaf box, and its culling box (the leaf box inflated as the host build
//     inflates it, rtamd::inw_wide_build);
//   - the depth-first ranks of the objects in the reference walk's order for both child orders,
//     and the walk's stack high-water mark (each from the object's / node's path to the root);
//   - a binary SAH tree over the culling boxes, built top-down one level per launch with 32
//     centroid bins per axis (a block per node range), collapsed to the 4-wide culling BVH the
//     kernels walk, one level per launch, numbered breadth first (top levels first: the LDS
//     staging takes the first nodes);
//   - the surrounding-RI grid (counts, scan, fill).
// The host path (rtamd::inw_wide_build: a full-sweep SAH) stays for fresh scenes; binned with 32
// bins its SAH cost over the C3 leaf boxes is within 0.3% of the sweep's (16.80 against 16.75).
// Every structure is a culling or bookkeeping structure: the walks' results do not depend on
// its shape, so frames are bit-identical to those of the host-built scene.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cstdio>

#include "rt_host.hpp"
#include "rt_kernels.hpp"

namespace rtk {
namespace {

constexpr int kB = 256;
constexpr int kBins = 32;
constexpr int kLevelBatch = 8;   // levels launched between two reads of the pending-task count
constexpr int kSahFirst = 20;    // the binary SAH levels launched before the first read (C3's tree: ~20)
constexpr int kMaxLevels = 256;  // binary SAH levels launched at most; a deeper tree (a chain-like scene,
                                 // where a split peels one object off per level) returns
                                 // hipErrorNotSupported and the caller builds on the host (rt_capi.hip)

// orderable bits of a float (a < b <=> ford(a) < ford(b)) for atomic min / max
__device__ __forceinline__ uint32_t ford(float f) {
    const uint32_t u = __float_as_uint(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fdeo(uint32_t u) { return __uint_as_float((u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); }

__device__ __forceinline__ uint32_t parent_of(const float4 *nodes, uint32_t i) { return (uint32_t)nodes[2 * i + 1].w; }
__device__ __forceinline__ bool lbvh_leaf(const float4 *nodes, uint32_t i) { return !(nodes[2 * i + 1].z > 0.1f); }

// per LBVH node: leaf -> its object's leaf box, culling box (inflated as rtamd::inw_wide_build),
// centroid, leaf node; the largest |coordinate| of the culling boxes (wbound, as uint bits)
__global__ __launch_bounds__(kB) void k_leaves(const float4 *nodes, uint32_t nn, uint32_t n, float4 *leafbox,
                                               float *box, float *cen, uint32_t *leafnode, uint32_t *ids,
                                               uint32_t *meta) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i >= nn) return;  // no cross-lane work in this kernel
    const float4 n0 = nodes[2 * i], n1 = nodes[2 * i + 1];
    if (n1.z > 0.1f) return;
    const uint32_t g = (uint32_t)(-n1.z);
    if (g >= n) return;  // (the device LBVH never does this)
    leafnode[g] = i;
    ids[g] = g;
    leafbox[2 * g] = n0;
    leafbox[2 * g + 1] = n1;
    const float b[6] = {n0.x, n0.y, n0.z, n0.w, n1.x, n1.y};
    float big = 0.0f;
    for (int k = 0; k < 6; k++) big = fmaxf(big, fabsf(b[k]));
    float wb = 0.0f;
    for (int k = 0; k < 3; k++) {
        const float e = (b[3 + k] - b[k]) * 1e-3f + 1e-3f + big * 1e-5f;
        const float lo = b[k] - e, hi = b[3 + k] + e;
        box[6 * g + k] = lo;
        box[6 * g + 3 + k] = hi;
        cen[3 * g + k] = 0.5f * (lo + hi);
        wb = fmaxf(wb, fmaxf(fabsf(lo), fabsf(hi)));
    }
    atomicMax(meta + 3, __float_as_uint(wb));  // non-negative: uint order = value order
}

// depth-first ranks (01_BVH...glsl:456-460: invert = 0 pops the right child, at the even index,
// first; invert = 1 the left one): the leaves of every earlier-visited sibling on the path
__global__ __launch_bounds__(kB) void k_ranks(const float4 *nodes, uint32_t n, const uint32_t *leafnode,
                                              const uint32_t *lcnt, uint32_t *rank) {
    const uint32_t g = blockIdx.x * kB + threadIdx.x;
    if (g >= n) return;  // no cross-lane work in this kernel
    uint32_t i = leafnode[g], r0 = 0, r1 = 0;
    while (i != 0u) {
        const uint32_t sib = (i & 1u) ? i + 1u : i - 1u;
        const uint32_t c = lbvh_leaf(nodes, sib) ? 1u : lcnt[sib];
        if (i & 1u) r0 += c;  // a left child comes after its right sibling when invert = 0
        else r1 += c;         // a right child after its left sibling when invert = 1
        i = parent_of(nodes, i);
    }
    rank[g] = r0;
    rank[n + g] = r1;
}

// the reference walk's stack high-water mark: popping node X leaves s(X) entries, s(root) = 0,
// a first-visited child has its parent's s + 1, the other one its parent's s; pushing X's children
// makes s(X) + 2 (both child orders; at least 1, the root push)
__global__ __launch_bounds__(kB) void k_high(const float4 *nodes, uint32_t nn, uint32_t *meta) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i >= nn) return;  // no cross-lane work in this kernel
    if (lbvh_leaf(nodes, i)) {
        if (i == 0u) atomicMax(meta + 2, 1u);
        return;
    }
    uint32_t s0 = 0, s1 = 0, j = i;
    while (j != 0u) {
        if (j & 1u) s1++;  // invert = 1 visits the left (odd) child first
        else s0++;         // invert = 0 the right (even) one
        j = parent_of(nodes, j);
    }
    atomicMax(meta + 2, (s0 > s1 ? s0 : s1) + 2u);
}

__device__ __forceinline__ float box_area(float x0, float y0, float z0, float x1, float y1, float z1) {
    const float dx = fmaxf(x1 - x0, 0.0f), dy = fmaxf(y1 - y0, 0.0f), dz = fmaxf(z1 - z0, 0.0f);
    return dx * dy + dy * dz + dz * dx;
}
__device__ __forceinline__ int bin_of(float c, float cmn, float scale) {
    return min(kBins - 1, max(0, (int)((c - cmn) * scale)));
}

// One level of the binned SAH build.  Task = (node, lo, hi, cb) over ids[lo, hi), hi - lo >= 2: the
// node takes the split of least SAH cost over 3 x (kBins - 1) bin boundaries (ties to the lower
// (axis, boundary); a range whose centroids share one bin on every axis splits in the middle),
// stably partitions its ids from ids_in into ids_out (the levels ping-pong between the two
// arrays: every range of a level is written by its parent's task) and makes its children.
// Numbering without counters: a range of m objects has 2m - 1 nodes, so a node's descendants own
// the 2m - 2 ids from cb: its children are the pair cb, cb + 1 (the layout the collapse reads),
// the left child's descendants follow from cb + 2, the right child's after those.  A child of one
// object is written as a leaf (first child = -object, as the LBVH layout) by the lane that places
// the object; the others are appended to the next level's tasks.  Ranges of more than kWaveMax
// objects take a block, the others one wave (no barriers; the top levels hold the few big
// ranges, the deep levels thousands of small ones).  Both paths pick the same split from the same
// bins (costs are min / max folds and exact counts); a block bins an evenly spaced sample of a
// range of more than kSahSample objects.
constexpr uint32_t kWaveMax = 256;
constexpr int kU = 8;  // loads in flight per lane in the block path's loops
constexpr uint32_t kSahSample = 2048;  // objects binned per range (evenly spaced) above this
struct SahBins {
    uint32_t cnt[3][kBins];
    uint32_t bb[3][kBins][6];  // orderable bits: lo min, hi max
};
__device__ __forceinline__ void bins_clear(SahBins &sb, uint32_t t, uint32_t nt) {
    for (uint32_t k = t; k < 3u * kBins; k += nt) {
        sb.cnt[k / kBins][k % kBins] = 0u;
        for (int j = 0; j < 6; j++) sb.bb[k / kBins][k % kBins][j] = j < 3 ? 0xffffffffu : 0u;
    }
}
__device__ __forceinline__ void bins_add(SahBins &sb, const float *bx, const float *c, const float *cmn,
                                         const float *scale, const bool *ax_ok) {
    for (int a = 0; a < 3; a++) {
        if (!ax_ok[a]) continue;
        const int b = bin_of(c[a], cmn[a], scale[a]);
        atomicAdd(&sb.cnt[a][b], 1u);
        for (int k = 0; k < 3; k++) {
            atomicMin(&sb.bb[a][b][k], ford(bx[k]));
            atomicMax(&sb.bb[a][b][3 + k], ford(bx[3 + k]));
        }
    }
}
__device__ __forceinline__ void load_item(const float *box, const float *cen, uint32_t g, float *bx, float *c) {
    for (int k = 0; k < 6; k++) bx[k] = box[6 * g + k];
    for (int k = 0; k < 3; k++) c[k] = cen[3 * g + k];
}
__device__ __forceinline__ void write_leaf(float *bin, uint32_t node, const float *box, uint32_t g) {
    float *o = bin + (size_t)node * 8;
    for (int k = 0; k < 6; k++) o[k] = box[6 * g + k];
    o[6] = -(float)g;
    o[7] = 0.0f;
}
// the object placed at position `dst` of a task split at nl: a child of one object is a leaf
__device__ __forceinline__ void place(uint32_t g, uint32_t dst, const uint4 tk, uint32_t nl, uint32_t *ids_out,
                                      float *bin, const float *box) {
    ids_out[dst] = g;
    const uint32_t lo = tk.y, hi = tk.z;
    if (nl == 1u && dst == lo) write_leaf(bin, tk.w, box, g);
    if (hi - lo - nl == 1u && dst == lo + nl) write_leaf(bin, tk.w + 1u, box, g);
}
// the task's node record and its internal children's tasks (one lane)
__device__ __forceinline__ void sah_emit(const uint4 tk, uint32_t nl, const float *nbox, float *bin, uint4 *tout,
                                         uint32_t *cnt_out) {
    const uint32_t node = tk.x, lo = tk.y, hi = tk.z, cb = tk.w, nr = hi - lo - nl;
    float *o = bin + (size_t)node * 8;
    for (int k = 0; k < 6; k++) o[k] = nbox[k];
    o[6] = (float)cb;
    o[7] = 0.0f;
    const uint32_t k = (nl > 1u ? 1u : 0u) + (nr > 1u ? 1u : 0u);
    if (!k) return;
    uint32_t slot = atomicAdd(cnt_out, k);
    if (nl > 1u) tout[slot++] = make_uint4(cb, lo, lo + nl, cb + 2u);
    if (nr > 1u) tout[slot] = make_uint4(cb + 1u, lo + nl, hi, cb + 2u + 2u * (nl - 1u));
}
__device__ __forceinline__ void bounds_init(float *v) {
    for (int k = 0; k < 3; k++) { v[k] = v[6 + k] = __builtin_huge_valf(); v[3 + k] = v[9 + k] = -__builtin_huge_valf(); }
}
__device__ __forceinline__ void bounds_add(float *v, const float *bx, const float *c) {
    for (int k = 0; k < 3; k++) {
        v[k] = fminf(v[k], bx[k]);
        v[3 + k] = fmaxf(v[3 + k], bx[3 + k]);
        v[6 + k] = fminf(v[6 + k], c[k]);
        v[9 + k] = fmaxf(v[9 + k], c[k]);
    }
}
__device__ __forceinline__ void bounds_wave(float *v) {  // butterfly: every lane holds the result
    for (int k = 0; k < 12; k++) {
        const bool mx = (k % 6) >= 3;
        for (int off = 32; off >= 1; off >>= 1) {
            const float w = __shfl_xor(v[k], off, 64);
            v[k] = mx ? fmaxf(v[k], w) : fminf(v[k], w);
        }
    }
}
__device__ __forceinline__ void bin_frame(const float *v, float *cmn, float *scale, bool *ax_ok) {
    for (int a = 0; a < 3; a++) {
        cmn[a] = v[6 + a];
        const float ext = v[9 + a] - cmn[a];
        ax_ok[a] = ext > 0.0f;
        scale[a] = ax_ok[a] ? (float)kBins / ext : 0.0f;
    }
}
// least-cost boundary over the bins, one wave: lane k < 31 evaluates boundary k of each axis from
// prefix / suffix folds over lanes 0..31 (empty bins fold as the identity); returns (axis *
// (kBins - 1) + boundary, or -1) and the left count in nl
__device__ __forceinline__ int sah_pick(const SahBins &sb, const bool *ax_ok, uint32_t lane, uint32_t m, uint32_t &nl) {
    float bc = __builtin_huge_valf();
    int bi = 0x7fffffff;
    uint32_t pcnt[3] = {0u, 0u, 0u};
    const uint32_t l = lane & 31u;
    for (int a = 0; a < 3; a++) {
        if (!ax_ok[a]) continue;  // uniform
        uint32_t c = sb.cnt[a][l];
        float b[6];
        for (int j = 0; j < 6; j++)
            b[j] = c ? fdeo(sb.bb[a][l][j]) : (j < 3 ? __builtin_huge_valf() : -__builtin_huge_valf());
        uint32_t pc = c, sc = c;
        float p[6], q[6];
        for (int j = 0; j < 6; j++) p[j] = q[j] = b[j];
        for (uint32_t off = 1; off < 32u; off <<= 1) {
            const uint32_t up = __shfl_up(pc, off, 32), dn = __shfl_down(sc, off, 32);
            float pu[6], qd[6];
            for (int j = 0; j < 6; j++) { pu[j] = __shfl_up(p[j], off, 32); qd[j] = __shfl_down(q[j], off, 32); }
            if (l >= off) {
                pc += up;
                for (int j = 0; j < 3; j++) { p[j] = fminf(p[j], pu[j]); p[3 + j] = fmaxf(p[3 + j], pu[3 + j]); }
            }
            if (l + off < 32u) {
                sc += dn;
                for (int j = 0; j < 3; j++) { q[j] = fminf(q[j], qd[j]); q[3 + j] = fmaxf(q[3 + j], qd[3 + j]); }
            }
        }
        // boundary l: left = bins 0..l (prefix at l), right = bins l+1.. (suffix at l+1)
        const uint32_t nr = __shfl_down(sc, 1, 32);
        float r[6];
        for (int j = 0; j < 6; j++) r[j] = __shfl_down(q[j], 1, 32);
        pcnt[a] = pc;
        if (l < (uint32_t)(kBins - 1) && pc && nr) {
            const float cost = box_area(p[0], p[1], p[2], p[3], p[4], p[5]) * (float)pc +
                               box_area(r[0], r[1], r[2], r[3], r[4], r[5]) * (float)nr;
            if (cost < bc) { bc = cost; bi = a * (kBins - 1) + (int)l; }
        }
    }
    for (int off = 32; off >= 1; off >>= 1) {  // least (cost, index)
        const float c2 = __shfl_xor(bc, off, 64);
        const int i2 = __shfl_xor(bi, off, 64);
        if (c2 < bc || (c2 == bc && i2 < bi)) { bc = c2; bi = i2; }
    }
    if (!(bc < __builtin_huge_valf())) { nl = m / 2u; return -1; }
    const int a = bi / (kBins - 1), k = bi % (kBins - 1);
    nl = __shfl(a == 0 ? pcnt[0] : a == 1 ? pcnt[1] : pcnt[2], k, 64);
    return bi;
}
__device__ __forceinline__ bool goes_left(int best, float c, uint32_t pos, uint32_t nl, float cmn, float scale, int k) {
    return best >= 0 ? bin_of(c, cmn, scale) <= k : pos < nl;
}

__global__ __launch_bounds__(kB) void k_sah_level(const uint4 *tin, const uint32_t *cnt_in, uint4 *tout,
                                                  uint32_t *cnt_out, const uint32_t *ids_in, uint32_t *ids_out,
                                                  const float *box, const float *cen, float *bin) {
    __shared__ float s_red[12][kB / 64];
    __shared__ SahBins s_bins;
    __shared__ SahBins s_wbins[kB / 64];
    __shared__ uint32_t s_wl[kB / 64];
    __shared__ float s_box[12];
    __shared__ int s_split[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t ntask = *cnt_in;
    // big ranges: a block each
    for (uint32_t t = blockIdx.x; t < ntask; t += gridDim.x) {  // uniform per block
        const uint4 tk = tin[t];
        const uint32_t lo = tk.y, hi = tk.z, m = hi - lo;
        if (m <= kWaveMax) continue;
        float v[12];
        bounds_init(v);
        for (uint32_t base = lo + tid; base < hi; base += kB * kU) {
            uint32_t g[kU];
            for (int u = 0; u < kU; u++) g[u] = base + u * kB < hi ? ids_in[base + u * kB] : 0xffffffffu;
            for (int u = 0; u < kU; u++)
                if (g[u] != 0xffffffffu) {
                    float bx[6], c[3];
                    load_item(box, cen, g[u], bx, c);
                    bounds_add(v, bx, c);
                }
        }
        bounds_wave(v);
        if (lane < 12u) {
            float x = v[0];
            for (int k = 1; k < 12; k++) x = lane == (uint32_t)k ? v[k] : x;
            s_red[lane][wv] = x;
        }
        bins_clear(s_bins, tid, kB);
        __syncthreads();
        if (tid < 12u) {
            const bool mx = (tid % 6u) >= 3u;
            float r = s_red[tid][0];
            for (uint32_t w = 1; w < kB / 64; w++) r = mx ? fmaxf(r, s_red[tid][w]) : fminf(r, s_red[tid][w]);
            s_box[tid] = r;
        }
        __syncthreads();
        float cmn[3], scale[3];
        bool ax_ok[3];
        bin_frame(s_box, cmn, scale, ax_ok);
        // bins: each thread takes a contiguous run of the range (neighbouring ids are often
        // neighbouring objects, which share bins: spread them over the wave's lanes).  A range of
        // more than kSahSample objects bins kSahSample of them, evenly spaced: the split is chosen
        // from the sample, the partition below counts the true sides (the top levels' LDS atomics
        // otherwise serialise one block on 21 atomics per object)
        {
            const bool smp = m > kSahSample;
            const uint32_t ms = smp ? kSahSample : m;
            const uint32_t per = (ms + kB - 1) / kB, k0 = tid * per, k1 = min(ms, k0 + per);
            for (uint32_t base = k0; base < k1; base += kU) {
                uint32_t g[kU];
                for (int u = 0; u < kU; u++) {
                    const uint32_t k = base + u;
                    const uint32_t q = smp ? lo + (uint32_t)(((uint64_t)k * m) / kSahSample) : lo + k;
                    g[u] = k < k1 ? ids_in[q] : 0xffffffffu;
                }
                for (int u = 0; u < kU; u++)
                    if (g[u] != 0xffffffffu) {
                        float bx[6], c[3];
                        load_item(box, cen, g[u], bx, c);
                        bins_add(s_bins, bx, c, cmn, scale, ax_ok);
                    }
            }
        }
        __syncthreads();
        if (wv == 0) {
            uint32_t nl = 0;
            const int best = sah_pick(s_bins, ax_ok, lane, m, nl);
            if (lane == 0) { s_split[0] = best; s_split[1] = (int)nl; }
        }
        __syncthreads();
        const int best = s_split[0];
        const uint32_t nl_pick = (uint32_t)s_split[1];  // the sample's left count when sampled
        // stable partition by side: a wave per quarter of the range (64-aligned), a count pass,
        // then each wave places its quarter from the counts of the quarters before it
        const int a = best >= 0 ? best / (kBins - 1) : 0, k = best >= 0 ? best % (kBins - 1) : 0;
        const uint32_t seg = ((m + 4u * 64u - 1u) / (4u * 64u)) * 64u;
        const uint32_t s0 = min(hi, lo + wv * seg), s1 = min(hi, s0 + seg);
        const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
        uint32_t nleft = 0;
        for (uint32_t base = s0; base < s1; base += 64u * kU) {
            float c[kU];
            for (int u = 0; u < kU; u++) {
                const uint32_t q = base + 64u * u + lane;
                c[u] = q < s1 && best >= 0 ? cen[3 * ids_in[q] + a] : 0.0f;
            }
            for (int u = 0; u < kU; u++) {
                const uint32_t q = base + 64u * u + lane;
                nleft += (uint32_t)__popcll(__ballot(q < s1 && goes_left(best, c[u], q - lo, nl_pick, cmn[a], scale[a], k)));
            }
        }
        if (lane == 0) s_wl[wv] = nleft;
        __syncthreads();
        uint32_t left = 0, nl = 0;  // nl: the true left count
        for (uint32_t w = 0; w < kB / 64; w++) {
            if (w < wv) left += s_wl[w];
            nl += s_wl[w];
        }
        uint32_t right = (s0 - lo) - left;
        for (uint32_t base = s0; base < s1; base += 64u * kU) {
            uint32_t g[kU];
            float c[kU];
            for (int u = 0; u < kU; u++) {
                const uint32_t q = base + 64u * u + lane;
                g[u] = q < s1 ? ids_in[q] : 0u;
                c[u] = q < s1 && best >= 0 ? cen[3 * g[u] + a] : 0.0f;
            }
            for (int u = 0; u < kU; u++) {
                const uint32_t q = base + 64u * u + lane;
                const bool has = q < s1, isl = has && goes_left(best, c[u], q - lo, nl, cmn[a], scale[a], k);
                const uint64_t ml = __ballot(isl), mh = __ballot(has);
                const uint32_t bl = (uint32_t)__popcll(ml & lt), bh = (uint32_t)__popcll(mh & lt);
                if (has) place(g[u], isl ? lo + left + bl : lo + nl + right + (bh - bl), tk, nl, ids_out, bin, box);
                left += (uint32_t)__popcll(ml);
                right += (uint32_t)(__popcll(mh) - __popcll(ml));
            }
        }
        if (tid == 0) sah_emit(tk, nl, s_box, bin, tout, cnt_out);
        __syncthreads();  // s_wl, s_box and s_split are the next task's
    }
    // small ranges: a wave each
    SahBins &wb = s_wbins[wv];
    const uint32_t nw = gridDim.x * (kB / 64);
    for (uint32_t t = blockIdx.x * (kB / 64) + wv; t < ntask; t += nw) {  // uniform per wave
        const uint4 tk = tin[t];
        const uint32_t lo = tk.y, hi = tk.z, m = hi - lo;
        if (m > kWaveMax) continue;
        uint32_t g[kWaveMax / 64];
        for (uint32_t j = 0; j < kWaveMax / 64; j++) {
            const uint32_t q = lo + lane + 64u * j;
            g[j] = q < hi ? ids_in[q] : 0u;
        }
        float v[12];
        bounds_init(v);
        for (uint32_t j = 0; j < kWaveMax / 64; j++)
            if (lo + lane + 64u * j < hi) {
                float bx[6], c[3];
                load_item(box, cen, g[j], bx, c);
                bounds_add(v, bx, c);
            }
        bounds_wave(v);
        float cmn[3], scale[3];
        bool ax_ok[3];
        bin_frame(v, cmn, scale, ax_ok);
        bins_clear(wb, lane, 64u);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        for (uint32_t j = 0; j < kWaveMax / 64; j++)
            if (lo + lane + 64u * j < hi) {
                float bx[6], c[3];
                load_item(box, cen, g[j], bx, c);
                bins_add(wb, bx, c, cmn, scale, ax_ok);
            }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
        uint32_t nl = 0;
        const int best = sah_pick(wb, ax_ok, lane, m, nl);
        const int a = best >= 0 ? best / (kBins - 1) : 0, k = best >= 0 ? best % (kBins - 1) : 0;
        uint32_t left = 0, right = 0;
        const uint64_t lt = lane ? (~0ull >> (64u - lane)) : 0ull;
        for (uint32_t j = 0; j < kWaveMax / 64 && lo + 64u * j < hi; j++) {  // uniform
            const uint32_t q = lo + lane + 64u * j;
            const bool has = q < hi;
            const bool isl = has && goes_left(best, best >= 0 ? cen[3 * g[j] + a] : 0.0f, q - lo, nl, cmn[a], scale[a], k);
            const uint64_t ml = __ballot(isl), mh = __ballot(has);
            const uint32_t bl = (uint32_t)__popcll(ml & lt), bh = (uint32_t)__popcll(mh & lt);
            if (has) place(g[j], isl ? lo + left + bl : lo + nl + right + (bh - bl), tk, nl, ids_out, bin, box);
            left += (uint32_t)__popcll(ml);
            right += (uint32_t)(__popcll(mh) - __popcll(ml));
        }
        if (lane == 0) {
            float nb[6];
            for (int j = 0; j < 6; j++) nb[j] = v[j];
            sah_emit(tk, nl, nb, bin, tout, cnt_out);
        }
        // the bins are reused by the wave's next task: its reads above are done (wave in order)
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
    }
}

// One level of the 4-wide collapse (rtamd::bvh4_collapse): a wide node gathers its binary node's
// children and opens the largest-area internal one until it holds four; internal children become
// the next level's wide nodes.  Wide node = 10 float4: lx ly lz hx hy hz (SoA over the 4
// children), lx ly lz again, the links (int bits: wide index + 1, or -object; an empty slot is a
// box at 1e30 with link 1e9, culled by every ray).  Numbering breadth first without a node
// counter: level wl + 1's wide nodes follow all earlier levels' (the prefix of the level counts),
// in the order of their task slots; a wave takes its slots with one atomic.  meta[1] sums the
// wide nodes (the root counted by the caller).
__device__ __forceinline__ float bin_area(const float *bin, int i) {
    const float *b = bin + (size_t)i * 8;
    const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    return dx * dy + dy * dz + dz * dx;
}
__global__ __launch_bounds__(kB) void k_collapse_level(const uint2 *tin, uint32_t *wlvl_cnt, int wl, uint2 *tout,
                                                       const float *bin, float4 *wnodes, uint32_t *meta) {
    const uint32_t t = blockIdx.x * kB + threadIdx.x, lane = threadIdx.x & 63u;
    const uint32_t ntask = wlvl_cnt[wl];
    if (blockIdx.x * kB + (threadIdx.x & ~63u) >= ntask) return;  // whole waves only (the scan below)
    // wide nodes before level wl + 1: the level counts 0..wl
    uint32_t before = 0;
    for (int i = (int)lane; i <= wl; i += 64) before += wlvl_cnt[i];
    for (int off = 32; off >= 1; off >>= 1) before += (uint32_t)__shfl_xor((int)before, off, 64);
    const bool act = t < ntask;
    auto is_leaf = [&](int i) { return !(bin[(size_t)i * 8 + 6] > 0.1f); };
    auto first = [&](int i) { return (int)bin[(size_t)i * 8 + 6]; };
    int ch[4] = {-1, -1, -1, -1};
    int nch = 0;
    uint2 tk = make_uint2(0u, 0u);
    if (act) {
        tk = tin[t];
        ch[0] = first((int)tk.x);
        ch[1] = ch[0] + 1;
        nch = 2;
        while (nch < 4) {
            int pick = -1;
            for (int k = 0; k < nch; k++)
                if (!is_leaf(ch[k]) && (pick < 0 || bin_area(bin, ch[k]) > bin_area(bin, ch[pick]))) pick = k;
            if (pick < 0) break;
            const int b = ch[pick];
            for (int k = pick; k < nch - 1; k++) ch[k] = ch[k + 1];
            ch[nch - 1] = first(b);
            ch[nch] = first(b) + 1;
            nch++;
        }
    }
    bool internal[4];
    uint32_t nk = 0;
    for (int k = 0; k < 4; k++) {
        internal[k] = k < nch && !is_leaf(ch[k]);
        nk += internal[k] ? 1u : 0u;
    }
    uint32_t incl = nk;  // inclusive scan of the wave's internal-child counts
    for (uint32_t off = 1; off < 64u; off <<= 1) {
        const uint32_t y = __shfl_up(incl, off, 64);
        if (lane >= off) incl += y;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    uint32_t base = 0;
    if (lane == 63u && total) {
        base = atomicAdd(wlvl_cnt + wl + 1, total);
        atomicAdd(meta + 1, total);
    }
    base = __shfl(base, 63, 64);
    if (!act) return;
    uint32_t slot = base + incl - nk;
    float pl[6][4];
    int lk[4];
    for (int k = 0; k < 4; k++) {
        if (k >= nch) {
            for (int a = 0; a < 6; a++) pl[a][k] = 1e30f;
            lk[k] = 1000000000;
            continue;
        }
        const float *bb = bin + (size_t)ch[k] * 8;
        for (int a = 0; a < 6; a++) pl[a][k] = bb[a];
        if (!internal[k]) lk[k] = (int)bb[6];
        else {
            const uint32_t w = before + slot;
            tout[slot++] = make_uint2((uint32_t)ch[k], w);
            lk[k] = (int)w + 1;
        }
    }
    float4 *o = wnodes + (size_t)tk.y * 10;
    for (int a = 0; a < 6; a++) o[a] = make_float4(pl[a][0], pl[a][1], pl[a][2], pl[a][3]);
    for (int a = 0; a < 3; a++) o[6 + a] = o[a];
    o[9] = make_float4(__int_as_float(lk[0]), __int_as_float(lk[1]), __int_as_float(lk[2]), __int_as_float(lk[3]));
}

// ---- surrounding-RI grid (rtamd::ri_grid_build): bounds, per-cell counts, offsets, ids
__global__ __launch_bounds__(kB) void k_ri_bounds(const float4 *leafbox, uint32_t n, uint32_t *bnd) {
    const uint32_t g = blockIdx.x * kB + threadIdx.x;
    uint32_t v[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    if (g < n) {
        const float4 n0 = leafbox[2 * g], n1 = leafbox[2 * g + 1];
        v[0] = ford(n0.x); v[1] = ford(n0.y); v[2] = ford(n0.z);
        v[3] = ford(n0.w); v[4] = ford(n1.x); v[5] = ford(n1.y);
    }
    for (int off = 32; off >= 1; off >>= 1)  // a wave's bounds, then one atomic per wave and bound
        for (int a = 0; a < 6; a++) {
            const uint32_t w = (uint32_t)__shfl_xor((int)v[a], off, 64);
            v[a] = a < 3 ? min(v[a], w) : max(v[a], w);
        }
    if ((threadIdx.x & 63u) == 0u)
        for (int a = 0; a < 3; a++) {
            atomicMin(bnd + a, v[a]);
            atomicMax(bnd + 3 + a, v[3 + a]);
        }
}
struct RiDims { double lo[3], inv[3]; int dim[3]; };
__device__ __forceinline__ void ri_range(const RiDims &d, float lo_v, float hi_v, int a, int &c0, int &c1) {
    const double m = 1e-3 / d.inv[a];
    c0 = max(0, min(d.dim[a] - 1, (int)floor(((double)lo_v - m - d.lo[a]) * d.inv[a])));
    c1 = max(0, min(d.dim[a] - 1, (int)floor(((double)hi_v + m - d.lo[a]) * d.inv[a])));
}
// pass 0: counts (cnt[c + 1]; flag when a cell lists more than 64); pass 1: ids through fill[c]
__global__ __launch_bounds__(kB) void k_ri_cells(const float4 *leafbox, uint32_t n, RiDims d, int pass, uint32_t *cnt,
                                                 uint32_t *fill, uint32_t *ids, uint32_t *flag) {
    const uint32_t g = blockIdx.x * kB + threadIdx.x;
    if (g >= n) return;  // no cross-lane work in this kernel
    // pass 0 stops once a cell is known to list more than 64 objects (the grid is dropped then, as
    // the host build stops at the first such cell): the count does not grow to O(n x cells) atomics
    if (pass == 0 && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    const float4 n0 = leafbox[2 * g], n1 = leafbox[2 * g + 1];
    const float lo[3] = {n0.x, n0.y, n0.z}, hi[3] = {n0.w, n1.x, n1.y};
    int r0[3], r1[3];
    for (int a = 0; a < 3; a++) ri_range(d, lo[a], hi[a], a, r0[a], r1[a]);
    for (int z = r0[2]; z <= r1[2]; z++) {
        if (pass == 0 && __hip_atomic_load(flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        for (int y = r0[1]; y <= r1[1]; y++)
            for (int x = r0[0]; x <= r1[0]; x++) {
                const size_t c = ((size_t)z * (size_t)d.dim[1] + (size_t)y) * (size_t)d.dim[0] + (size_t)x;
                if (pass == 0) {
                    if (atomicAdd(cnt + c + 1, 1u) >= 64u) atomicOr(flag, 1u);
                } else {
                    ids[atomicAdd(fill + c, 1u)] = g;
                }
            }
    }
}

inline uint32_t nblk(size_t n) { return (uint32_t)((n + kB - 1) / kB); }

// ---- quantised wide nodes (InwScene::qnodes, DESIGN.md §5.2 "Quantised nodes")
// Per node and axis: origin o (a float at or below the lowest child plane minus the margin m) and
// scale s >= 1e-4 (o + 255 s at or above the highest plane plus m); a child's low plane becomes
// the byte q with o + q s <= lo - m, its high plane the byte with o + q s >= hi + m (real
// arithmetic, checked in double on the exact float values).  An empty slot (link 1e9) gets low
// bytes 255 and high bytes 0: an interval reversed by 255 s >= 0.0255, which no rounding of the
// walk's fma closes.  The walk computes t = fma(q, s / d, (o - ray origin) / d); DESIGN.md §2 bounds
// its error below m / |d| while every coordinate and ray origin lies within 1000 of the origin (the
// fused cull's condition, required for these nodes), so the decoded boxes stay conservative.
__device__ __forceinline__ float f32_next_up(float f) {  // finite f: the next float above
    if (f == 0.0f) return __uint_as_float(1u);
    const uint32_t u = __float_as_uint(f);
    return __uint_as_float(f > 0.0f ? u + 1u : u - 1u);
}
__device__ __forceinline__ float f32_next_down(float f) { return -f32_next_up(-f); }
__device__ __forceinline__ float f32_down(double x) {
    float f = (float)x;
    if ((double)f > x) f = f32_next_down(f);
    return f;
}
__device__ __forceinline__ float f32_up(double x) {
    float f = (float)x;
    if ((double)f < x) f = f32_next_up(f);
    return f;
}
__global__ __launch_bounds__(kB) void k_quantize_wnodes(const float4 *wn, uint32_t nw, float4 *qn, float margin) {
    const uint32_t w = blockIdx.x * kB + threadIdx.x;
    if (w >= nw) return;  // no cross-lane work in this kernel
    const float4 *nd = wn + (size_t)w * 10;
    const float4 pl4[6] = {nd[0], nd[1], nd[2], nd[3], nd[4], nd[5]};
    const float4 lk = nd[9];
    auto comp = [](const float4 &v, int k) { return k == 0 ? v.x : k == 1 ? v.y : k == 2 ? v.z : v.w; };
    bool empty[4];
    for (int k = 0; k < 4; k++) empty[k] = __float_as_int(comp(lk, k)) == 1000000000;
    const double m = (double)margin;
    float org[3], scl[3];
    uint32_t qlo[3] = {0u, 0u, 0u}, qhi[3] = {0u, 0u, 0u};
    for (int a = 0; a < 3; a++) {
        double nlo = 0.0, nhi = 0.0;
        bool any = false;
        for (int k = 0; k < 4; k++) {
            if (empty[k]) continue;
            const double lo = comp(pl4[a], k), hi = comp(pl4[3 + a], k);
            nlo = any ? fmin(nlo, lo) : lo;
            nhi = any ? fmax(nhi, hi) : hi;
            any = true;
        }
        const float o = f32_down(nlo - m);
        float s = f32_up(fmax(((nhi + m) - (double)o) / 255.0, 1e-4));
        while ((double)o + 255.0 * (double)s < nhi + m) s = f32_next_up(s);
        org[a] = o;
        scl[a] = s;
        for (int k = 0; k < 4; k++) {
            uint32_t ql = 255u, qh = 0u;
            if (!empty[k]) {
                const double lo = (double)comp(pl4[a], k) - m, hi = (double)comp(pl4[3 + a], k) + m;
                int q = (int)floor((lo - (double)o) / (double)s);
                q = q < 0 ? 0 : (q > 255 ? 255 : q);
                while (q > 0 && (double)o + (double)q * (double)s > lo) q--;
                int r = (int)ceil((hi - (double)o) / (double)s);
                r = r < 0 ? 0 : (r > 255 ? 255 : r);
                while (r < 255 && (double)o + (double)r * (double)s < hi) r++;
                ql = (uint32_t)q;
                qh = (uint32_t)r;
            }
            qlo[a] |= ql << (8 * k);
            qhi[a] |= qh << (8 * k);
        }
    }
    float4 *o4 = qn + (size_t)w * kQNodeF4;
    o4[0] = make_float4(org[0], org[1], org[2], scl[0]);
    o4[1] = make_float4(scl[1], scl[2], __uint_as_float(qlo[0]), __uint_as_float(qlo[1]));
    o4[2] = make_float4(__uint_as_float(qlo[2]), __uint_as_float(qhi[0]), __uint_as_float(qhi[1]), __uint_as_float(qhi[2]));
    o4[3] = lk;
}

}  // namespace

hipError_t inw_quantize_wnodes(const float4 *wnodes, uint32_t nw, float4 *qnodes, float margin, hipStream_t s) {
    if (!nw) return hipSuccess;
    if (!wnodes || !qnodes || !(margin > 0.0f)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_quantize_wnodes, dim3(nblk(nw)), dim3(kB), 0, s, wnodes, nw, qnodes, margin);
    return hipGetLastError();
}

// workspace carve-up (256-B aligned pieces)
struct BuildWs {
    float *box, *cen, *bin;
    uint32_t *leafnode, *ids, *ids2, *meta, *lvl_cnt, *wlvl_cnt;
    uint4 *task[2];
    uint2 *wtask[2];
    uint32_t *ri_bnd, *ri_flag;
};
static size_t carve(void *ws, uint32_t n, BuildWs *w) {
    const size_t nn = 2 * (size_t)n - 1;
    size_t off = 0;
    auto take = [&](size_t bytes) {
        char *p = static_cast<char *>(ws) + off;
        off += (bytes + 255) & ~(size_t)255;
        return static_cast<void *>(p);
    };
    BuildWs t{};
    t.box = static_cast<float *>(take((size_t)n * 6 * 4));
    t.cen = static_cast<float *>(take((size_t)n * 3 * 4));
    t.bin = static_cast<float *>(take(nn * 8 * 4));
    t.leafnode = static_cast<uint32_t *>(take((size_t)n * 4));
    t.ids = static_cast<uint32_t *>(take((size_t)n * 4));
    t.ids2 = static_cast<uint32_t *>(take((size_t)n * 4));
    t.meta = static_cast<uint32_t *>(take(16 * 4));
    t.lvl_cnt = static_cast<uint32_t *>(take((kMaxLevels + 1) * 4));
    t.wlvl_cnt = static_cast<uint32_t *>(take((kMaxLevels + 1) * 4));
    t.task[0] = static_cast<uint4 *>(take((size_t)n * 16));
    t.task[1] = static_cast<uint4 *>(take((size_t)n * 16));
    t.wtask[0] = static_cast<uint2 *>(take((size_t)n * 8));
    t.wtask[1] = static_cast<uint2 *>(take((size_t)n * 8));
    t.ri_bnd = static_cast<uint32_t *>(take(8 * 4));
    t.ri_flag = static_cast<uint32_t *>(take(4));
    if (w) *w = t;
    return off;
}

size_t inw_build_workspace_bytes(uint32_t n) { return n ? carve(reinterpret_cast<void *>(256), n, nullptr) + 256 : 0; }

#define BUILD_HIP(expr)                                                                   \
    do {                                                                                  \
        const hipError_t e_ = (expr);                                                     \
        if (e_ != hipSuccess) return e_;                                                  \
    } while (0)

hipError_t inw_wide_build_device(const float4 *nodes, const uint32_t *lcnt, uint32_t n, void *ws, size_t ws_bytes,
                                 InwWideDev &out, hipStream_t s, int max_levels) {
    const int lvl_cap = max_levels > 0 && max_levels < kMaxLevels ? max_levels : kMaxLevels;
    if (n < 2 || !nodes || !lcnt || !ws || ws_bytes < inw_build_workspace_bytes(n) || !out.wnodes || !out.rank || !out.leafbox)
        return hipErrorInvalidValue;
    BuildWs w;
    carve(ws, n, &w);
    const uint32_t nn = 2 * n - 1;
    BUILD_HIP(hipMemsetAsync(w.meta, 0, 16 * 4, s));
    BUILD_HIP(hipMemsetAsync(w.lvl_cnt, 0, (kMaxLevels + 1) * 4, s));
    BUILD_HIP(hipMemsetAsync(w.wlvl_cnt, 0, (kMaxLevels + 1) * 4, s));
    hipLaunchKernelGGL(k_leaves, dim3(nblk(nn)), dim3(kB), 0, s, nodes, nn, n, out.leafbox, w.box, w.cen, w.leafnode,
                       w.ids, w.meta);
    hipLaunchKernelGGL(k_ranks, dim3(nblk(n)), dim3(kB), 0, s, nodes, n, w.leafnode, lcnt, out.rank);
    hipLaunchKernelGGL(k_high, dim3(nblk(nn)), dim3(kB), 0, s, nodes, nn, w.meta);
    // the RI grid's bounds (the leaf boxes'), read back with the counts below
    const uint32_t binit[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    BUILD_HIP(hipMemcpyAsync(w.ri_bnd, binit, sizeof(binit), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_ri_bounds, dim3(nblk(n)), dim3(kB), 0, s, out.leafbox, n, w.ri_bnd);
    BUILD_HIP(hipGetLastError());
    // binary SAH tree: root task (node 0, all objects, its descendants from node 1)
    const uint32_t one = 1u;
    const uint4 root = make_uint4(0u, 0u, n, 1u);
    BUILD_HIP(hipMemcpyAsync(w.task[0], &root, sizeof(root), hipMemcpyHostToDevice, s));
    BUILD_HIP(hipMemcpyAsync(w.lvl_cnt, &one, 4, hipMemcpyHostToDevice, s));
    int lvl = 0;
    for (int batch = kSahFirst;; batch = kLevelBatch) {
        for (int k = 0; k < batch && lvl < lvl_cap; k++, lvl++)
            hipLaunchKernelGGL(k_sah_level, dim3(1024), dim3(kB), 0, s, w.task[lvl & 1], w.lvl_cnt + lvl,
                               w.task[(lvl + 1) & 1], w.lvl_cnt + lvl + 1, (lvl & 1) ? w.ids2 : w.ids,
                               (lvl & 1) ? w.ids : w.ids2, w.box, w.cen, w.bin);
        BUILD_HIP(hipGetLastError());
        uint32_t pending = 0;
        BUILD_HIP(hipMemcpyAsync(&pending, w.lvl_cnt + lvl, 4, hipMemcpyDeviceToHost, s));
        BUILD_HIP(hipStreamSynchronize(s));
        if (pending == 0) break;
        if (lvl >= lvl_cap) return hipErrorNotSupported;  // deeper than the cap: the caller builds on the host
    }
    // 4-wide collapse; meta[1] = wide node counter (1: the root, from binary node 0)
    const uint2 wroot = make_uint2(0u, 0u);
    BUILD_HIP(hipMemcpyAsync(w.wtask[0], &wroot, sizeof(wroot), hipMemcpyHostToDevice, s));
    BUILD_HIP(hipMemcpyAsync(w.wlvl_cnt, &one, 4, hipMemcpyHostToDevice, s));
    BUILD_HIP(hipMemcpyAsync(w.meta + 1, &one, 4, hipMemcpyHostToDevice, s));
    int wl = 0;
    for (;;) {
        for (int k = 0; k < kLevelBatch && wl < lvl_cap; k++, wl++)
            hipLaunchKernelGGL(k_collapse_level, dim3(nblk(n)), dim3(kB), 0, s, w.wtask[wl & 1], w.wlvl_cnt, wl,
                               w.wtask[(wl + 1) & 1], w.bin, out.wnodes, w.meta);
        BUILD_HIP(hipGetLastError());
        // this batch's level counts, the counters (meta) and the RI bounds in one read
        uint32_t rb[kLevelBatch + 1 + 4 + 6];
        BUILD_HIP(hipMemcpyAsync(rb, w.wlvl_cnt + wl - kLevelBatch, (kLevelBatch + 1) * 4, hipMemcpyDeviceToHost, s));
        BUILD_HIP(hipMemcpyAsync(rb + kLevelBatch + 1, w.meta, 4 * 4, hipMemcpyDeviceToHost, s));
        BUILD_HIP(hipMemcpyAsync(rb + kLevelBatch + 5, w.ri_bnd, 6 * 4, hipMemcpyDeviceToHost, s));
        BUILD_HIP(hipStreamSynchronize(s));
        if (rb[kLevelBatch] == 0) {
            int d = wl - kLevelBatch;
            while (d < wl && rb[d - (wl - kLevelBatch)] != 0) d++;
            out.depth = d;
            const uint32_t *meta = rb + kLevelBatch + 1, *b = rb + kLevelBatch + 5;
            out.n_wnodes = meta[1];
            out.dfs_high = meta[2] ? meta[2] : 1u;
            out.wbound = __builtin_bit_cast(float, meta[3]);
            auto dec = [](uint32_t u) { return __builtin_bit_cast(float, (u & 0x80000000u) ? (u & 0x7fffffffu) : ~u); };
            for (int a = 0; a < 3; a++) { out.ri_lo[a] = dec(b[a]); out.ri_hi[a] = dec(b[3 + a]); }
            break;
        }
        if (wl >= lvl_cap) return hipErrorNotSupported;
    }
    return hipSuccess;
}

// The wide nodes without the repeated low planes (InwScene::cnodes): 7 float4 per node, lx ly lz
// hx hy hz links, for the buffer-load walk (a ray's far plane of axis a sits at a + 3 (1 - s_a))
__global__ __launch_bounds__(kB) void k_compact_wnodes(const float4 *wn, uint32_t nw, float4 *cn) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i >= nw * 7u) return;
    const uint32_t w = i / 7u, k = i - 7u * w;
    cn[i] = wn[(size_t)w * 10 + (k < 6u ? k : 9u)];
}
hipError_t inw_compact_wnodes(const float4 *wnodes, uint32_t nw, float4 *cnodes, hipStream_t s) {
    if (!nw) return hipSuccess;
    hipLaunchKernelGGL(k_compact_wnodes, dim3(nblk(nw * 7u)), dim3(kB), 0, s, wnodes, nw, cnodes);
    return hipGetLastError();
}

size_t ri_scan_temp_bytes(size_t cells) {
    size_t sb = 0;
    (void)hipcub::DeviceScan::InclusiveSum(nullptr, sb, (uint32_t *)nullptr, (uint32_t *)nullptr, (int)cells);
    return sb;
}

static RiDims ri_dims(const double lo[3], const double inv[3], const int dim[3]) {
    RiDims d{};
    for (int a = 0; a < 3; a++) { d.lo[a] = lo[a]; d.inv[a] = inv[a]; d.dim[a] = dim[a]; }
    return d;
}

hipError_t ri_count_device(const float4 *leafbox, uint32_t n, void *ws, const double lo[3], const double inv[3],
                           const int dim[3], uint32_t *cells, void *tmp, size_t tmp_bytes, uint32_t *total,
                           uint32_t *over, hipStream_t s) {
    BuildWs w;
    carve(ws, n, &w);
    const RiDims d = ri_dims(lo, inv, dim);
    const size_t nc = (size_t)dim[0] * dim[1] * dim[2];
    BUILD_HIP(hipMemsetAsync(cells, 0, (nc + 1) * 4, s));
    BUILD_HIP(hipMemsetAsync(w.ri_flag, 0, 4, s));
    hipLaunchKernelGGL(k_ri_cells, dim3(nblk(n)), dim3(kB), 0, s, leafbox, n, d, 0, cells, nullptr, nullptr, w.ri_flag);
    BUILD_HIP(hipGetLastError());
    size_t sb = tmp_bytes;
    BUILD_HIP(hipcub::DeviceScan::InclusiveSum(tmp, sb, cells, cells, (int)(nc + 1), s));
    uint32_t tail[2];
    BUILD_HIP(hipMemcpyAsync(tail, cells + nc, 4, hipMemcpyDeviceToHost, s));
    BUILD_HIP(hipMemcpyAsync(tail + 1, w.ri_flag, 4, hipMemcpyDeviceToHost, s));
    BUILD_HIP(hipStreamSynchronize(s));
    *total = tail[0];
    *over = tail[1];
    return hipSuccess;
}

hipError_t ri_fill_device(const float4 *leafbox, uint32_t n, const double lo[3], const double inv[3], const int dim[3],
                          const uint32_t *cells, uint32_t *fill, uint32_t *ids, hipStream_t s) {
    const RiDims d = ri_dims(lo, inv, dim);
    const size_t nc = (size_t)dim[0] * dim[1] * dim[2];
    BUILD_HIP(hipMemcpyAsync(fill, cells, nc * 4, hipMemcpyDeviceToDevice, s));
    hipLaunchKernelGGL(k_ri_cells, dim3(nblk(n)), dim3(kB), 0, s, leafbox, n, d, 1, nullptr, fill, ids, nullptr);
    return hipGetLastError();
}

}  // namespace rtk
