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
constexpr int kMaxLevels = 256;  // binary SAH levels (a chain over n objects is at most n deep; the
                                 // binned split halves a degenerate range, so depth <= ~2 log2 n)

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

// leaf counts of the LBVH's internal nodes (each object adds one to every ancestor)
__global__ __launch_bounds__(kB) void k_leaf_counts(const float4 *nodes, uint32_t n, const uint32_t *leafnode,
                                                    uint32_t *lcnt) {
    const uint32_t g = blockIdx.x * kB + threadIdx.x;
    if (g >= n) return;  // no cross-lane work in this kernel
    uint32_t i = leafnode[g];
    while (i != 0u) {
        i = parent_of(nodes, i);
        atomicAdd(lcnt + i, 1u);
    }
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

// One level of the binned SAH build.  Task = (node, lo, hi, parent) over ids[lo, hi); a block per
// task.  A range of one object is a leaf (first child = -object, as the LBVH layout); else the
// node takes the split of least SAH cost over 3 x (kBins - 1) bin boundaries (a range whose
// centroids share one bin on every axis splits in the middle), stably partitions its ids, and
// appends its children (allocated as a contiguous pair) to the next level's tasks.
__global__ __launch_bounds__(kB) void k_sah_level(const uint4 *tin, const uint32_t *cnt_in, uint4 *tout,
                                                  uint32_t *cnt_out, uint32_t *ids, uint32_t *ids2, const float *box,
                                                  const float *cen, float *bin, uint32_t *node_ctr) {
    __shared__ float s_red[12][kB / 64];
    __shared__ uint32_t s_cnt[3][kBins];
    __shared__ uint32_t s_bb[3][kBins][6];
    __shared__ float s_cost[3 * (kBins - 1)];
    __shared__ uint32_t s_scan[kB];
    __shared__ float s_box[12];
    __shared__ int s_split[2];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
    const uint32_t ntask = *cnt_in;
    for (uint32_t t = blockIdx.x; t < ntask; t += gridDim.x) {  // uniform per block
        const uint4 tk = tin[t];
        const uint32_t node = tk.x, lo = tk.y, hi = tk.z, par = tk.w, m = hi - lo;
        float *o = bin + (size_t)node * 8;
        if (m == 1u) {
            if (tid == 0) {
                const uint32_t g = ids[lo];
                for (int k = 0; k < 6; k++) o[k] = box[6 * g + k];
                o[6] = -(float)g;
                o[7] = (float)par;
            }
            continue;
        }
        // the node's box and its centroids' bounds
        float v[12];
        for (int k = 0; k < 3; k++) { v[k] = v[6 + k] = __builtin_huge_valf(); v[3 + k] = v[9 + k] = -__builtin_huge_valf(); }
        for (uint32_t q = lo + tid; q < hi; q += kB) {
            const uint32_t g = ids[q];
            for (int k = 0; k < 3; k++) {
                v[k] = fminf(v[k], box[6 * g + k]);
                v[3 + k] = fmaxf(v[3 + k], box[6 * g + 3 + k]);
                v[6 + k] = fminf(v[6 + k], cen[3 * g + k]);
                v[9 + k] = fmaxf(v[9 + k], cen[3 * g + k]);
            }
        }
        for (int k = 0; k < 12; k++) {  // wave reduction, then across the 4 waves
            const bool mx = (k % 6) >= 3;
            for (int off = 32; off >= 1; off >>= 1) {
                const float w = __shfl_xor(v[k], off, 64);
                v[k] = mx ? fmaxf(v[k], w) : fminf(v[k], w);
            }
            if (lane == 0) s_red[k][wv] = v[k];
        }
        if (tid < 3u * kBins) {
            s_cnt[tid / kBins][tid % kBins] = 0u;
            for (int k = 0; k < 6; k++) s_bb[tid / kBins][tid % kBins][k] = k < 3 ? 0xffffffffu : 0u;
        }
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
        for (int a = 0; a < 3; a++) {
            cmn[a] = s_box[6 + a];
            const float ext = s_box[9 + a] - cmn[a];
            ax_ok[a] = ext > 0.0f;
            scale[a] = ax_ok[a] ? (float)kBins / ext : 0.0f;
        }
        // bins: counts and boxes (orderable bits) per axis
        for (uint32_t q = lo + tid; q < hi; q += kB) {
            const uint32_t g = ids[q];
            for (int a = 0; a < 3; a++) {
                if (!ax_ok[a]) continue;
                const int b = bin_of(cen[3 * g + a], cmn[a], scale[a]);
                atomicAdd(&s_cnt[a][b], 1u);
                for (int k = 0; k < 3; k++) {
                    atomicMin(&s_bb[a][b][k], ford(box[6 * g + k]));
                    atomicMax(&s_bb[a][b][3 + k], ford(box[6 * g + 3 + k]));
                }
            }
        }
        __syncthreads();
        // SAH cost of each boundary: area(L) * |L| + area(R) * |R|
        if (tid < 3u * (kBins - 1)) {
            const int a = (int)tid / (kBins - 1), k = (int)tid % (kBins - 1);
            float cost = __builtin_huge_valf();
            if (ax_ok[a]) {
                uint32_t nl = 0, nr = 0;
                float l[6] = {__builtin_huge_valf(), __builtin_huge_valf(), __builtin_huge_valf(),
                              -__builtin_huge_valf(), -__builtin_huge_valf(), -__builtin_huge_valf()};
                float r[6] = {l[0], l[1], l[2], l[3], l[4], l[5]};
                for (int b = 0; b < kBins; b++) {
                    const uint32_t c = s_cnt[a][b];
                    if (!c) continue;
                    float *d = b <= k ? l : r;
                    (b <= k ? nl : nr) += c;
                    for (int j = 0; j < 3; j++) {
                        d[j] = fminf(d[j], fdeo(s_bb[a][b][j]));
                        d[3 + j] = fmaxf(d[3 + j], fdeo(s_bb[a][b][3 + j]));
                    }
                }
                if (nl && nr)
                    cost = box_area(l[0], l[1], l[2], l[3], l[4], l[5]) * (float)nl +
                           box_area(r[0], r[1], r[2], r[3], r[4], r[5]) * (float)nr;
            }
            s_cost[tid] = cost;
        }
        __syncthreads();
        if (tid == 0) {  // least cost, ties to the lower (axis, boundary)
            int best = -1;
            float bc = __builtin_huge_valf();
            for (int c = 0; c < 3 * (kBins - 1); c++)
                if (s_cost[c] < bc) { bc = s_cost[c]; best = c; }
            s_split[0] = best;
            uint32_t nl = m / 2u;
            if (best >= 0) {
                nl = 0;
                for (int b = 0; b <= best % (kBins - 1); b++) nl += s_cnt[best / (kBins - 1)][b];
            }
            s_split[1] = (int)nl;
        }
        __syncthreads();
        const int best = s_split[0];
        const uint32_t nl = (uint32_t)s_split[1];
        if (best >= 0) {  // stable partition of ids[lo, hi) by side, through ids2
            const int a = best / (kBins - 1), k = best % (kBins - 1);
            uint32_t left = 0, right = 0;  // placed so far (uniform)
            for (uint32_t base = lo; base < hi; base += kB) {
                const uint32_t q = base + tid;
                uint32_t g = 0;
                bool isl = false;
                if (q < hi) {
                    g = ids[q];
                    isl = bin_of(cen[3 * g + a], cmn[a], scale[a]) <= k;
                }
                s_scan[tid] = isl ? 1u : 0u;
                __syncthreads();
                for (uint32_t off = 1; off < kB; off <<= 1) {  // inclusive scan
                    const uint32_t x = tid >= off ? s_scan[tid - off] : 0u;
                    __syncthreads();
                    s_scan[tid] += x;
                    __syncthreads();
                }
                const uint32_t incl = s_scan[tid], total = s_scan[kB - 1];
                if (q < hi) {
                    const uint32_t before = incl - (isl ? 1u : 0u);
                    ids2[isl ? lo + left + before : lo + nl + right + (tid - before)] = g;
                }
                const uint32_t chunk = hi - base < (uint32_t)kB ? hi - base : (uint32_t)kB;
                left += total;
                right += chunk - total;
                __syncthreads();
            }
            for (uint32_t q = lo + tid; q < hi; q += kB) ids[q] = ids2[q];
        }
        if (tid == 0) {
            const uint32_t c0 = atomicAdd(node_ctr, 2u);
            for (int k = 0; k < 6; k++) o[k] = s_box[k];
            o[6] = (float)c0;
            o[7] = (float)par;
            const uint32_t slot = atomicAdd(cnt_out, 2u);
            tout[slot] = make_uint4(c0, lo, lo + nl, node);
            tout[slot + 1] = make_uint4(c0 + 1u, lo + nl, hi, node);
        }
        __syncthreads();
    }
}

// One level of the 4-wide collapse (rtamd::bvh4_collapse): a wide node gathers its binary node's
// children and opens the largest-area internal one until it holds four; internal children become
// the next level's wide nodes (indices in level order).  Wide node = 10 float4: lx ly lz hx hy hz
// (SoA over the 4 children), lx ly lz again, the links (int bits: wide index + 1, or -object;
// an empty slot is a box at 1e30 with link 1e9, culled by every ray).
__device__ __forceinline__ float bin_area(const float *bin, int i) {
    const float *b = bin + (size_t)i * 8;
    const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    return dx * dy + dy * dz + dz * dx;
}
__global__ __launch_bounds__(kB) void k_collapse_level(const uint2 *tin, const uint32_t *cnt_in, uint2 *tout,
                                                       uint32_t *cnt_out, const float *bin, float4 *wnodes,
                                                       uint32_t *wide_ctr) {
    const uint32_t t = blockIdx.x * kB + threadIdx.x;
    if (t >= *cnt_in) return;  // no cross-lane work in this kernel
    const uint2 tk = tin[t];
    auto is_leaf = [&](int i) { return !(bin[(size_t)i * 8 + 6] > 0.1f); };
    auto first = [&](int i) { return (int)bin[(size_t)i * 8 + 6]; };
    int ch[4] = {first((int)tk.x), first((int)tk.x) + 1, -1, -1};
    int nch = 2;
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
        if (is_leaf(ch[k])) lk[k] = (int)bb[6];
        else {
            const uint32_t w = atomicAdd(wide_ctr, 1u);
            tout[atomicAdd(cnt_out, 1u)] = make_uint2((uint32_t)ch[k], w);
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
    if (g >= n) return;  // no cross-lane work in this kernel
    const float4 n0 = leafbox[2 * g], n1 = leafbox[2 * g + 1];
    const float lo[3] = {n0.x, n0.y, n0.z}, hi[3] = {n0.w, n1.x, n1.y};
    for (int a = 0; a < 3; a++) {
        atomicMin(bnd + a, ford(lo[a]));
        atomicMax(bnd + 3 + a, ford(hi[a]));
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
    const float4 n0 = leafbox[2 * g], n1 = leafbox[2 * g + 1];
    const float lo[3] = {n0.x, n0.y, n0.z}, hi[3] = {n0.w, n1.x, n1.y};
    int r0[3], r1[3];
    for (int a = 0; a < 3; a++) ri_range(d, lo[a], hi[a], a, r0[a], r1[a]);
    for (int z = r0[2]; z <= r1[2]; z++)
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

inline uint32_t nblk(size_t n) { return (uint32_t)((n + kB - 1) / kB); }

}  // namespace

// workspace carve-up (256-B aligned pieces)
struct BuildWs {
    float *box, *cen, *bin;
    uint32_t *leafnode, *lcnt, *ids, *ids2, *meta, *lvl_cnt, *wlvl_cnt;
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
    t.lcnt = static_cast<uint32_t *>(take(nn * 4));
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

hipError_t inw_wide_build_device(const float4 *nodes, uint32_t n, void *ws, size_t ws_bytes, InwWideDev &out,
                                 hipStream_t s) {
    if (n < 2 || !nodes || !ws || ws_bytes < inw_build_workspace_bytes(n) || !out.wnodes || !out.rank || !out.leafbox)
        return hipErrorInvalidValue;
    BuildWs w;
    carve(ws, n, &w);
    const uint32_t nn = 2 * n - 1;
    BUILD_HIP(hipMemsetAsync(w.meta, 0, 16 * 4, s));
    BUILD_HIP(hipMemsetAsync(w.lcnt, 0, (size_t)nn * 4, s));
    BUILD_HIP(hipMemsetAsync(w.lvl_cnt, 0, (kMaxLevels + 1) * 4, s));
    BUILD_HIP(hipMemsetAsync(w.wlvl_cnt, 0, (kMaxLevels + 1) * 4, s));
    hipLaunchKernelGGL(k_leaves, dim3(nblk(nn)), dim3(kB), 0, s, nodes, nn, n, out.leafbox, w.box, w.cen, w.leafnode,
                       w.ids, w.meta);
    hipLaunchKernelGGL(k_leaf_counts, dim3(nblk(n)), dim3(kB), 0, s, nodes, n, w.leafnode, w.lcnt);
    hipLaunchKernelGGL(k_ranks, dim3(nblk(n)), dim3(kB), 0, s, nodes, n, w.leafnode, w.lcnt, out.rank);
    hipLaunchKernelGGL(k_high, dim3(nblk(nn)), dim3(kB), 0, s, nodes, nn, w.meta);
    // the RI grid's bounds (the leaf boxes'), read back with the counts below
    const uint32_t binit[6] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u};
    BUILD_HIP(hipMemcpyAsync(w.ri_bnd, binit, sizeof(binit), hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_ri_bounds, dim3(nblk(n)), dim3(kB), 0, s, out.leafbox, n, w.ri_bnd);
    BUILD_HIP(hipGetLastError());
    // binary SAH tree: root task (node 0, all objects); meta[0] = node counter (1: the root)
    const uint32_t one = 1u;
    const uint4 root = make_uint4(0u, 0u, n, 0u);
    BUILD_HIP(hipMemcpyAsync(w.task[0], &root, sizeof(root), hipMemcpyHostToDevice, s));
    BUILD_HIP(hipMemcpyAsync(w.lvl_cnt, &one, 4, hipMemcpyHostToDevice, s));
    BUILD_HIP(hipMemcpyAsync(w.meta, &one, 4, hipMemcpyHostToDevice, s));
    int lvl = 0;
    for (int batch = kSahFirst;; batch = kLevelBatch) {
        for (int k = 0; k < batch && lvl < kMaxLevels; k++, lvl++)
            hipLaunchKernelGGL(k_sah_level, dim3(1024), dim3(kB), 0, s, w.task[lvl & 1], w.lvl_cnt + lvl,
                               w.task[(lvl + 1) & 1], w.lvl_cnt + lvl + 1, w.ids, w.ids2, w.box, w.cen, w.bin,
                               w.meta);
        BUILD_HIP(hipGetLastError());
        uint32_t pending = 0;
        BUILD_HIP(hipMemcpyAsync(&pending, w.lvl_cnt + lvl, 4, hipMemcpyDeviceToHost, s));
        BUILD_HIP(hipStreamSynchronize(s));
        if (pending == 0) break;
        if (lvl >= kMaxLevels) return hipErrorNotSupported;  // deeper than any binned split makes
    }
    // 4-wide collapse; meta[1] = wide node counter (1: the root, from binary node 0)
    const uint2 wroot = make_uint2(0u, 0u);
    BUILD_HIP(hipMemcpyAsync(w.wtask[0], &wroot, sizeof(wroot), hipMemcpyHostToDevice, s));
    BUILD_HIP(hipMemcpyAsync(w.wlvl_cnt, &one, 4, hipMemcpyHostToDevice, s));
    BUILD_HIP(hipMemcpyAsync(w.meta + 1, &one, 4, hipMemcpyHostToDevice, s));
    int wl = 0;
    for (;;) {
        for (int k = 0; k < kLevelBatch && wl < kMaxLevels; k++, wl++)
            hipLaunchKernelGGL(k_collapse_level, dim3(nblk(n)), dim3(kB), 0, s, w.wtask[wl & 1], w.wlvl_cnt + wl,
                               w.wtask[(wl + 1) & 1], w.wlvl_cnt + wl + 1, w.bin, out.wnodes, w.meta + 1);
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
        if (wl >= kMaxLevels) return hipErrorNotSupported;
    }
    return hipSuccess;
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
