// rt_lbvh.hip -- LBVH build on the GPU, node-for-node identical to the host
// builder rtamd::lbvh_build and hence to LBVH::ConstructLBVH_Buff (lbvh.h:57-269).
//
// The reference merges adjacent leaf clusters in order of their "highest differing bit", ties
// in index order (lbvh.h:162-210).  Merging adjacent elements in increasing (bit, index) order
// builds the Cartesian tree of the internal-node weights (bit_i, i), so each node's parent is
// the lighter of its nearest heavier neighbours on either side.  Over Morton-sorted codes
// those neighbours are run boundaries of a code prefix and fall out of binary searches:
//   left:  nearest j < i with bit_j > bit_i  = (first leaf k with code_k >> bit_i == code_i >> bit_i) - 1
//   right: nearest j > i with bit_j >= bit_i = last leaf m with code_m >> (bit_i - 1) == code_{i+1} >> (bit_i - 1)
// Boxes propagate bottom-up (second arriving child), then breadth-first indices come from a
// sort on (depth, first leaf) -- the order of the host's FIFO walk (lbvh.h:215-269).
#include <hipcub/hipcub.hpp>

#include "rt_kernels.hpp"

namespace rtk {
namespace {

constexpr int kB = 256;

// MIN / MAX of utility.h:10-11 (x > y ? y : x): on ties the first argument wins, which fixes
// the sign of a zero exactly as the host does
__device__ __forceinline__ float rmin(float x, float y) { return x > y ? y : x; }
__device__ __forceinline__ float rmax(float x, float y) { return x > y ? x : y; }

__device__ __forceinline__ uint32_t expand_bits(uint32_t v) {
    v = (v * 0x00010001u) & 0xFF0000FFu;
    v = (v * 0x00000101u) & 0x0F00F00Fu;
    v = (v * 0x00000011u) & 0xC30C30C3u;
    v = (v * 0x00000005u) & 0x49249249u;
    return v;
}
__device__ __forceinline__ uint32_t quant(float f) {
    return (uint32_t)fminf(fmaxf(f * 1024.0f, 0.0f), 1023.0f);
}

// Scene box.  The host folds smin = MIN(smin, a_i), smax = MAX(smax, a_i) in index order: on
// equal values MIN keeps the earlier element and MAX takes the later one (it decides the sign
// of a zero), so the reduction carries (value, index) and breaks ties the same way.
__device__ __forceinline__ bool better(int a, float x, uint32_t j, float v, uint32_t i) {
    return a < 3 ? (x < v || (x == v && j < i)) : (x > v || (x == v && j > i));
}

__global__ void k_scene_box(const float *aabb, uint32_t n, float *part /* blocks x 6 x 2 */) {
    __shared__ float sv[6][kB];
    __shared__ uint32_t si[6][kB];
    float v[6];
    uint32_t id[6];
    for (int a = 0; a < 6; a++) { v[a] = a < 3 ? __builtin_huge_valf() : -__builtin_huge_valf(); id[a] = 0xffffffffu; }
    for (uint32_t k = blockIdx.x * kB + threadIdx.x; k < n; k += gridDim.x * kB)
        for (int a = 0; a < 6; a++) {
            const float x = aabb[(size_t)k * 6 + a];
            if (id[a] == 0xffffffffu || better(a, x, k, v[a], id[a])) { v[a] = x; id[a] = k; }
        }
    for (int a = 0; a < 6; a++) { sv[a][threadIdx.x] = v[a]; si[a][threadIdx.x] = id[a]; }
    __syncthreads();
    for (int w = kB / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w)
            for (int a = 0; a < 6; a++) {
                const float x = sv[a][threadIdx.x + w];
                const uint32_t j = si[a][threadIdx.x + w];
                const float y = sv[a][threadIdx.x];
                const uint32_t i = si[a][threadIdx.x];
                bool take;
                if (j == 0xffffffffu) take = false;
                else if (i == 0xffffffffu) take = true;
                else take = better(a, x, j, y, i);
                if (take) { sv[a][threadIdx.x] = x; si[a][threadIdx.x] = j; }
            }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int a = 0; a < 6; a++) {
            part[(size_t)blockIdx.x * 12 + a] = sv[a][0];
            part[(size_t)blockIdx.x * 12 + 6 + a] = __uint_as_float(si[a][0]);
        }
}

// fold of the block partials (one wave): the (value, index) order of `better` is a total order,
// so the lane-parallel fold picks the element the host's index-order fold picks
__global__ void k_scene_box_final(const float *part, int blocks, float *box) {
    if (blockIdx.x != 0) return;
    const int lane = (int)threadIdx.x;  // blocks <= 64 (lbvh_build_device)
    for (int a = 0; a < 6; a++) {
        float v = 0.0f;
        uint32_t id = 0xffffffffu;
        if (lane < blocks) {
            v = part[(size_t)lane * 12 + a];
            id = __float_as_uint(part[(size_t)lane * 12 + 6 + a]);
        }
        for (int off = 32; off >= 1; off >>= 1) {
            const float x = __shfl_xor(v, off, 64);
            const uint32_t j = (uint32_t)__shfl_xor((int)id, off, 64);
            const bool take = j != 0xffffffffu && (id == 0xffffffffu || better(a, x, j, v, id));
            if (take) { v = x; id = j; }
        }
        if (lane == 0) box[a] = v;
    }
}

// Morton code and sort key (code, diag^2) per object; values = object ids
__global__ void k_keys(const float *aabb, uint32_t n, const float *box, unsigned long long *key, uint32_t *ids) {
    const uint32_t k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const float *b = aabb + (size_t)k * 6;
    float px = (b[0] + b[3]) * 0.5f, py = (b[1] + b[4]) * 0.5f, pz = (b[2] + b[5]) * 0.5f;
    px = px - box[0]; py = py - box[1]; pz = pz - box[2];
    px = px / (box[3] - box[0]);
    py = py / (box[4] - box[1]);
    pz = pz / (box[5] - box[2]);
    const float dx = b[3] - b[0], dy = b[4] - b[1], dz = b[5] - b[2];
    const float d2 = dx * dx + dy * dy + dz * dz;
    const uint32_t code = expand_bits(quant(px)) * 4 + expand_bits(quant(py)) * 2 + expand_bits(quant(pz));
    key[k] = ((unsigned long long)code << 32) | __float_as_uint(d2);  // diag^2 >= 0: bit order = value order
    ids[k] = k;
}

__device__ __forceinline__ uint32_t code_of(const unsigned long long *key, uint32_t i) { return (uint32_t)(key[i] >> 32); }
__device__ __forceinline__ int hbit(uint32_t x) { return x ? 32 - __clz(x) : 0; }  // highest set bit + 1

// parent / child links of the Cartesian tree.  Nodes: leaves 0..n-1 (sorted order), internal
// n..2n-2 (internal i between leaves i and i+1).
__global__ void k_links(const unsigned long long *key, uint32_t n, int *parent, int *left, int *right) {
    const uint32_t i = blockIdx.x * kB + threadIdx.x;
    if (i + 1 >= n) return;  // n-1 internal nodes
    auto bit = [&](uint32_t j) { return hbit(code_of(key, j) ^ code_of(key, j + 1)); };
    const int bi = bit(i);
    // left: first leaf k <= i whose code agrees with leaf i above bit bi
    const uint32_t pre = code_of(key, i) >> bi;  // bi <= 30 < 32
    uint32_t lo = 0, hi = i;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((code_of(key, mid) >> bi) < pre) lo = mid + 1;
        else hi = mid;
    }
    const int pg = (int)lo - 1;  // -1: none
    // right: last leaf m >= i+1 agreeing with leaf i+1 above bit bi-1 (bi == 0: m = i+1)
    int ng;
    if (bi == 0) ng = (i + 1 < n - 1) ? (int)(i + 1) : -1;
    else {
        const int sh = bi - 1;
        const uint32_t pr = code_of(key, i + 1) >> sh;
        uint32_t l2 = i + 1, h2 = n - 1;  // last index with prefix == pr
        while (l2 < h2) {
            const uint32_t mid = (l2 + h2 + 1) >> 1;
            if ((code_of(key, mid) >> sh) > pr) h2 = mid - 1;
            else l2 = mid;
        }
        ng = (l2 < n - 1) ? (int)l2 : -1;
    }
    // parent = the lighter of the two heavier neighbours (weights (bit, index))
    int p;
    if (pg < 0) p = ng;
    else if (ng < 0) p = pg;
    else {
        const int bp = bit((uint32_t)pg), bn = bit((uint32_t)ng);
        p = (bp < bn || (bp == bn && pg < ng)) ? pg : ng;
    }
    const int me = (int)(n + i);
    if (p < 0) parent[me] = -1;
    else {
        parent[me] = (int)n + p;
        if (p > (int)i) left[n + p] = me;
        else right[n + p] = me;
    }
    // leaf i+1 hangs off the lighter of internal i and i+1; leaf 0 off internal 0
    {
        const uint32_t leaf = i + 1;
        int q = (int)i;
        if (leaf < n - 1) {
            const int b2 = bit(leaf);
            if (b2 < bi || (b2 == bi && (int)leaf < (int)i)) q = (int)leaf;
        }
        parent[leaf] = (int)n + q;
        if (q == (int)i) right[n + q] = (int)leaf;
        else left[n + q] = (int)leaf;
    }
    if (i == 0) { parent[0] = (int)n; left[n] = 0; }
}

// bottom-up boxes: the second child to arrive computes the parent
__global__ void k_boxes(const float *aabb, const uint32_t *ids, uint32_t n, const int *parent, const int *left,
                        const int *right, float *bmin, float *bmax, unsigned *arrive) {
    const uint32_t k = blockIdx.x * kB + threadIdx.x;
    if (k >= n) return;
    const float *b = aabb + (size_t)ids[k] * 6;
    for (int a = 0; a < 3; a++) { bmin[(size_t)k * 3 + a] = b[a]; bmax[(size_t)k * 3 + a] = b[3 + a]; }
    __threadfence();
    int node = parent[k];
    while (node >= 0) {
        if (atomicAdd(arrive + node, 1u) == 0) return;  // first arrival: the sibling continues
        __threadfence();
        const int L = left[node], R = right[node];
        for (int a = 0; a < 3; a++) {
            const float lmn = __hip_atomic_load(bmin + (size_t)L * 3 + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float rmn = __hip_atomic_load(bmin + (size_t)R * 3 + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float lmx = __hip_atomic_load(bmax + (size_t)L * 3 + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const float rmx = __hip_atomic_load(bmax + (size_t)R * 3 + a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bmin + (size_t)node * 3 + a, rmin(lmn, rmn), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(bmax + (size_t)node * 3 + a, rmax(lmx, rmx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __threadfence();
        node = parent[node];
    }
}

// depth and first leaf of every node -> breadth-first key (depth, first leaf); the node's leaf
// count (its leaves are the sorted range first..last)
__global__ void k_bfs_keys(uint32_t n, const int *parent, const int *left, const int *right, unsigned long long *key,
                           uint32_t *vals, uint32_t *cnt) {
    const uint32_t v = blockIdx.x * kB + threadIdx.x;
    if (v >= 2 * n - 1) return;
    uint32_t depth = 0;
    for (int p = parent[v]; p >= 0; p = parent[p]) depth++;
    int first = (int)v, last = (int)v;
    while (first >= (int)n) first = left[first];
    while (last >= (int)n) last = right[last];
    key[v] = ((unsigned long long)depth << 32) | (uint32_t)first;
    vals[v] = v;
    cnt[v] = (uint32_t)(last - first + 1);
}

__global__ void k_rank(const uint32_t *order, uint32_t total, uint32_t *rank) {
    const uint32_t r = blockIdx.x * kB + threadIdx.x;
    if (r < total) rank[order[r]] = r;
}

// ConstructLBVH_Buff layout: {bb_min[3], bb_max[3], leftData, rightData} in BFS order
__global__ void k_write(uint32_t n, const uint32_t *order, const uint32_t *rank, const int *parent, const int *left,
                        const uint32_t *ids, const float *bmin, const float *bmax, const uint32_t *cnt, float *out,
                        uint32_t *lcnt) {
    const uint32_t r = blockIdx.x * kB + threadIdx.x;
    if (r >= 2 * n - 1) return;
    const uint32_t v = order[r];
    float *o = out + (size_t)r * 8;
    for (int a = 0; a < 3; a++) { o[a] = bmin[(size_t)v * 3 + a]; o[3 + a] = bmax[(size_t)v * 3 + a]; }
    o[6] = v >= n ? (float)rank[left[v]] : -(float)ids[v];
    o[7] = parent[v] >= 0 ? (float)rank[parent[v]] : 0.0f;
    if (lcnt) lcnt[r] = cnt[v];
}

}  // namespace

namespace {
struct LbvhWs {
    float *part, *box;
    unsigned long long *k0, *k1;
    uint32_t *v0, *v1, *rank, *cnt;
    int *parent, *left, *right;
    unsigned *arrive;
    float *bmin, *bmax;
    void *sort_tmp;
    size_t sort_bytes, bytes;
};
LbvhWs lbvh_layout(uint32_t n, void *ws) {
    const size_t total = 2 * (size_t)n - 1;
    LbvhWs w{};
    char *base = static_cast<char *>(ws), *p = base;
    auto take = [&](size_t b) { char *q = p; p += (b + 255) & ~size_t(255); return (void *)q; };
    w.part = (float *)take(64 * 12 * 4);
    w.box = (float *)take(64);
    w.k0 = (unsigned long long *)take(total * 8 + 8);
    w.k1 = (unsigned long long *)take(total * 8 + 8);
    w.v0 = (uint32_t *)take(total * 4 + 4);
    w.v1 = (uint32_t *)take(total * 4 + 4);
    w.parent = (int *)take(total * 4 + 4);
    w.left = (int *)take(total * 4 + 4);
    w.right = (int *)take(total * 4 + 4);
    w.arrive = (unsigned *)take(total * 4 + 4);
    w.bmin = (float *)take(total * 12 + 12);
    w.bmax = (float *)take(total * 12 + 12);
    w.rank = (uint32_t *)take(total * 4 + 4);
    w.cnt = (uint32_t *)take(total * 4 + 4);
    w.sort_bytes = 0;
    (void)hipcub::DeviceRadixSort::SortPairs(nullptr, w.sort_bytes, w.k0, w.k1, w.v0, w.v1, (int)total);
    w.sort_tmp = take(w.sort_bytes);
    w.bytes = size_t(p - base);
    return w;
}
const uint32_t kOne = 1u;
__global__ void k_single(const float *aabb, float *out) {  // n == 1: the root is the leaf
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    for (int a = 0; a < 6; a++) out[a] = aabb[a];
    out[6] = -0.0f;  // -float(ObjectID 0)
    out[7] = 0.0f;
}
}  // namespace

size_t lbvh_workspace_bytes(uint32_t n) { return n ? lbvh_layout(n, nullptr).bytes : 0; }

hipError_t lbvh_build_device(const float *aabb, uint32_t n, float *out, void *ws, size_t ws_bytes, hipStream_t s,
                             uint32_t *lcnt) {
    if (n == 0) return hipErrorInvalidValue;
    if (n == 1) {
        hipLaunchKernelGGL(k_single, dim3(1), dim3(64), 0, s, aabb, out);
        if (lcnt) return hipMemcpyAsync(lcnt, &kOne, 4, hipMemcpyHostToDevice, s);
        return hipGetLastError();
    }
    const LbvhWs w = lbvh_layout(n, ws);
    if (ws_bytes < w.bytes) return hipErrorInvalidValue;
    const size_t total = 2 * (size_t)n - 1;
    float *part = w.part, *box = w.box, *bmin = w.bmin, *bmax = w.bmax;
    unsigned long long *k0 = w.k0, *k1 = w.k1;
    uint32_t *v0 = w.v0, *v1 = w.v1, *rank = w.rank;
    int *parent = w.parent, *left = w.left, *right = w.right;
    unsigned *arrive = w.arrive;
    void *sort_tmp = w.sort_tmp;
    size_t sort_bytes = w.sort_bytes;
    hipError_t e = hipSuccess;
    const unsigned gb = (unsigned)std::min<uint32_t>(64, (n + kB - 1) / kB);
    const unsigned gn = (n + kB - 1) / kB, gt = (unsigned)((total + kB - 1) / kB);
    hipLaunchKernelGGL(k_scene_box, dim3(gb), dim3(kB), 0, s, aabb, n, part);
    hipLaunchKernelGGL(k_scene_box_final, dim3(1), dim3(64), 0, s, part, (int)gb, box);
    hipLaunchKernelGGL(k_keys, dim3(gn), dim3(kB), 0, s, aabb, n, box, k0, v0);
    // (code, diag^2) ascending, ties by object id (the radix sort is stable over ids 0..n-1)
    if ((e = hipcub::DeviceRadixSort::SortPairs(sort_tmp, sort_bytes, k0, k1, v0, v1, (int)n, 0, 62, s)) != hipSuccess)
        return e;
    if ((e = hipMemsetAsync(parent, 0xff, total * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(left, 0xff, total * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(right, 0xff, total * 4, s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(arrive, 0, total * 4, s)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_links, dim3((n - 1 + kB - 1) / kB), dim3(kB), 0, s, k1, n, parent, left, right);
    hipLaunchKernelGGL(k_boxes, dim3(gn), dim3(kB), 0, s, aabb, v1, n, parent, left, right, bmin, bmax, arrive);
    hipLaunchKernelGGL(k_bfs_keys, dim3(gt), dim3(kB), 0, s, n, parent, left, right, k0, v0, w.cnt);
    if ((e = hipcub::DeviceRadixSort::SortPairs(sort_tmp, sort_bytes, k0, k1, v0, rank, (int)total, 0, 64, s)) !=
        hipSuccess)
        return e;
    // rank[] now holds the BFS order (node ids); invert into v0 = rank of each node
    hipLaunchKernelGGL(k_rank, dim3(gt), dim3(kB), 0, s, rank, (uint32_t)total, v0);
    hipLaunchKernelGGL(k_write, dim3(gt), dim3(kB), 0, s, n, rank, v0, parent, left, v1, bmin, bmax, w.cnt, out, lcnt);
    return hipGetLastError();
}

}  // namespace rtk
