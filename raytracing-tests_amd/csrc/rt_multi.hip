// rt_multi.hip -- the multi-GPU partition behind the C ABI (BASELINE configs[3]):
// one host thread drives several devices of this process (SURVEY 8b "one host thread drives
// all devices"), the frame's tiles are dealt across them, every device renders its share with
// rt_render_tiles_async on a stream of its own, and the packed tiles travel to device 0 in one
// RCCL exchange (grouped ncclSend / ncclRecv over xGMI), where one kernel unpacks them into the
// W x H image.  This generalises the reference's per-tile dispatch loop
// (In-One-Weekend/03_Shadows_and_Materials/materials.cpp:98-152) to devices and replaces the
// single-device dispatch of RT_Base<>::OnUpdateBase (In-Next-Week/base.h:148-173) for a C++ host.
// bench.py's one-process-per-GPU torchrun path (the driver's scaling run) deals the same tiles
// (rt_tile_deal == bench.deal_order) and gathers them with torch.distributed on RCCL.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <new>
#include <vector>

#include "../../include/rt_hip.h"
#include "rt_host.hpp"

namespace {

// ------------------------------------------------------------------ unpack + counter sum
// recv: the gathered packed tiles, device after device (device r's tiles at its slot offset,
// in its deal order); tiles: their (tx, ty) in the same order.  One thread per pixel of the
// gathered tiles; pixels outside the image (the ragged right / top tiles) are skipped.
__global__ __launch_bounds__(256) void k_unpack_tiles(const float4 *recv, const float *recv_depth, const int2 *tiles,
                                                      uint32_t n_px, int T, int W, int H, float4 *rgba, float *depth) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= n_px) return;  // no cross-lane work in this kernel
    const uint32_t area = uint32_t(T) * uint32_t(T);
    const int2 t = tiles[i / area];
    const uint32_t r = i % area;
    const int x = t.x * T + int(r % uint32_t(T)), y = t.y * T + int(r / uint32_t(T));
    if (x >= W || y >= H) return;
    const size_t o = size_t(y) * size_t(W) + size_t(x);
    rgba[o] = recv[i];
    if (depth) depth[o] = recv_depth[i];
}

// d_counters[k] += sum over devices of their 6 counters (one 64-lane block)
__global__ __launch_bounds__(64) void k_sum_counters(const unsigned long long *all, int n_dev,
                                                     unsigned long long *out) {
    const int k = int(threadIdx.x);
    if (k >= 6) return;  // no cross-lane work in this kernel
    unsigned long long s = 0;
    for (int r = 0; r < n_dev; r++) s += all[r * 6 + k];
    out[k] += s;
}

struct Buf {  // a device allocation on a given device (freed there)
    void *p = nullptr;
    size_t bytes = 0;
    int dev = 0;
    Buf() = default;
    Buf(const Buf &) = delete;
    Buf &operator=(const Buf &) = delete;
    ~Buf() {
        if (p) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(dev);
            (void)hipFree(p);
            (void)hipSetDevice(cur);
        }
    }
    // (re)allocate on the current device, `d`, when smaller than b
    hipError_t ensure(size_t b, int d) {
        if (p && bytes >= b) return hipSuccess;
        if (p) { (void)hipFree(p); p = nullptr; }
        dev = d;
        bytes = b;
        return hipMalloc(&p, b ? b : 16);
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

#define MULTI_HIP(expr)                                                                             \
    do {                                                                                           \
        hipError_t e_ = (expr);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            std::fprintf(stderr, "[rt_hip] %s failed: %s\n", #expr, hipGetErrorString(e_));         \
            return RT_E_HIP;                                                                       \
        }                                                                                          \
    } while (0)
#define MULTI_NCCL(expr)                                                                            \
    do {                                                                                           \
        ncclResult_t r_ = (expr);                                                                  \
        if (r_ != ncclSuccess) {                                                                   \
            std::fprintf(stderr, "[rt_hip] %s failed: %s\n", #expr, ncclGetErrorString(r_));       \
            return RT_E_HIP;                                                                       \
        }                                                                                          \
    } while (0)

// restores the caller's current device on scope exit
struct DeviceGuard {
    int cur = 0;
    DeviceGuard() { (void)hipGetDevice(&cur); }
    ~DeviceGuard() { (void)hipSetDevice(cur); }
};

}  // namespace

struct rt_group {
    int n = 0;
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;
    std::vector<hipStream_t> st;  // st[0] unused: device 0 works on the caller's stream
    struct Share {                // one device's share of the frame
        Buf tiles, packed, depth, counters;
        int n_tiles = 0;
    };
    std::vector<std::unique_ptr<Share>> share;
    Buf recv, recv_depth, recv_tiles, recv_ctr;  // on device 0
    // the deal the buffers hold (re-uploaded when the frame or tile size changes)
    int W = 0, H = 0, T = 0;
    std::vector<uint32_t> off;  // device r's first tile in the gathered order
    ~rt_group() {
        share.clear();
        for (ncclComm_t c : comm)
            if (c) (void)ncclCommDestroy(c);
        for (size_t r = 0; r < st.size(); r++)
            if (st[r]) {
                (void)hipSetDevice(dev[r]);
                (void)hipStreamDestroy(st[r]);
            }
    }
};

namespace {

// the deal of a W x H frame in T x T tiles over g's devices, uploaded to every device's tile list
// and to device 0's gathered order.  The buffers are reused when large enough, so an earlier frame
// still running on the group's streams (device 0: the caller's stream s0) is waited for first: the
// API is asynchronous, and a null-stream copy does not wait for non-blocking streams
int set_deal(rt_group *g, int W, int H, int T, hipStream_t s0) {
    if (g->W == W && g->H == H && g->T == T) return RT_OK;
    for (int r = 0; r < g->n; r++) {
        MULTI_HIP(hipSetDevice(g->dev[size_t(r)]));
        MULTI_HIP(hipStreamSynchronize(r == 0 ? s0 : g->st[size_t(r)]));
    }
    const std::vector<std::pair<int, int>> order = rtamd::tile_deal(W, H, T, g->n);
    std::vector<std::vector<int>> lists(size_t(g->n));
    for (size_t k = 0; k < order.size(); k++) {
        auto &l = lists[k % size_t(g->n)];
        l.push_back(order[k].first);
        l.push_back(order[k].second);
    }
    std::vector<int> all;
    g->off.assign(size_t(g->n) + 1, 0);
    const size_t area = size_t(T) * size_t(T);
    for (int r = 0; r < g->n; r++) {
        auto &S = *g->share[size_t(r)];
        S.n_tiles = int(lists[size_t(r)].size() / 2);
        g->off[size_t(r) + 1] = g->off[size_t(r)] + uint32_t(S.n_tiles);
        all.insert(all.end(), lists[size_t(r)].begin(), lists[size_t(r)].end());
        MULTI_HIP(hipSetDevice(g->dev[size_t(r)]));
        const size_t nt = size_t(std::max(S.n_tiles, 1));
        MULTI_HIP(S.tiles.ensure(nt * 2 * sizeof(int), g->dev[size_t(r)]));
        MULTI_HIP(S.packed.ensure(nt * area * 4 * sizeof(float), g->dev[size_t(r)]));
        MULTI_HIP(S.depth.ensure(nt * area * sizeof(float), g->dev[size_t(r)]));
        MULTI_HIP(S.counters.ensure(6 * sizeof(unsigned long long), g->dev[size_t(r)]));
        if (S.n_tiles)
            MULTI_HIP(hipMemcpy(S.tiles.p, lists[size_t(r)].data(), size_t(S.n_tiles) * 2 * sizeof(int),
                                hipMemcpyHostToDevice));
    }
    MULTI_HIP(hipSetDevice(g->dev[0]));
    const size_t total = order.size();
    MULTI_HIP(g->recv.ensure(total * area * 4 * sizeof(float), g->dev[0]));
    MULTI_HIP(g->recv_depth.ensure(total * area * sizeof(float), g->dev[0]));
    MULTI_HIP(g->recv_tiles.ensure(total * 2 * sizeof(int), g->dev[0]));
    MULTI_HIP(g->recv_ctr.ensure(size_t(g->n) * 6 * sizeof(unsigned long long), g->dev[0]));
    MULTI_HIP(hipMemcpy(g->recv_tiles.p, all.data(), all.size() * sizeof(int), hipMemcpyHostToDevice));
    g->W = W; g->H = H; g->T = T;
    return RT_OK;
}

}  // namespace

extern "C" {

int rt_tile_deal(int width, int height, int tile_size, int n_dev, int *order_out, int cap) {
    if (width <= 0 || height <= 0 || tile_size <= 0 || n_dev <= 0 || cap < 0 || (cap > 0 && !order_out))
        return RT_E_ARG;
    try {
        const std::vector<std::pair<int, int>> order = rtamd::tile_deal(width, height, tile_size, n_dev);
        for (size_t k = 0; k < order.size() && k < size_t(cap); k++) {
            order_out[2 * k] = order[k].first;
            order_out[2 * k + 1] = order[k].second;
        }
        return int(order.size());
    } catch (...) {
        return RT_E_ARG;
    }
}

rt_group *rt_group_create(const int *devices, int n_dev) {
    if (!devices || n_dev <= 0 || n_dev > 64) return nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) return nullptr;
    for (int r = 0; r < n_dev; r++) {
        if (devices[r] < 0 || devices[r] >= count) return nullptr;
        for (int q = 0; q < r; q++)
            if (devices[q] == devices[r]) return nullptr;  // one rank per device (RCCL refuses duplicates)
        if (rt_device_info(devices[r], nullptr, 0, nullptr) != RT_OK) return nullptr;  // a gfx950 device
    }
    DeviceGuard guard;
    std::unique_ptr<rt_group> g(new (std::nothrow) rt_group());
    if (!g) return nullptr;
    try {
        g->n = n_dev;
        g->dev.assign(devices, devices + n_dev);
        g->comm.assign(size_t(n_dev), nullptr);
        g->st.assign(size_t(n_dev), nullptr);
        for (int r = 0; r < n_dev; r++) g->share.push_back(std::make_unique<rt_group::Share>());
    } catch (...) {
        return nullptr;
    }
    if (ncclCommInitAll(g->comm.data(), n_dev, g->dev.data()) != ncclSuccess) {
        g->comm.assign(size_t(n_dev), nullptr);
        return nullptr;
    }
    for (int r = 1; r < n_dev; r++) {
        if (hipSetDevice(devices[r]) != hipSuccess) return nullptr;
        if (hipStreamCreateWithFlags(&g->st[size_t(r)], hipStreamNonBlocking) != hipSuccess) return nullptr;
    }
    return g.release();
}

void rt_group_free(rt_group *g) {
    if (!g) return;
    DeviceGuard guard;
    for (int d : g->dev) {
        (void)hipSetDevice(d);
        (void)hipDeviceSynchronize();
    }
    delete g;
}

int rt_render_multi_async(rt_group *g, rt_dev_scene *const *scenes, const rt_camera *cam, const rt_params *p,
                          int tile_size, float *d_rgba, float *d_depth, uint64_t *d_counters, void *stream) {
    if (!g || !scenes || !cam || !p || !d_rgba || p->width <= 0 || p->height <= 0 || tile_size <= 0 ||
        tile_size % 16 != 0)
        return RT_E_ARG;
    // every scene must live on its group device (its buffers are that device's; a scene of another
    // device would launch there with this device's stream)
    for (int r = 0; r < g->n; r++)
        if (!scenes[r] || rtamd::scene_device(scenes[r]) != g->dev[size_t(r)]) return RT_E_ARG;
    DeviceGuard guard;
    const hipStream_t s0 = static_cast<hipStream_t>(stream);
    if (int rc = set_deal(g, p->width, p->height, tile_size, s0); rc != RT_OK) {
        g->W = 0;  // rebuild the deal next time
        return rc;
    }
    auto stream_of = [&](int r) { return r == 0 ? s0 : g->st[size_t(r)]; };
    const size_t area = size_t(tile_size) * size_t(tile_size);
    rt_params q = *p;
    q.tile_x0 = q.tile_y0 = q.tile_w = q.tile_h = 0;  // the whole frame
    // every device renders its share on its own stream
    for (int r = 0; r < g->n; r++) {
        auto &S = *g->share[size_t(r)];
        MULTI_HIP(hipSetDevice(g->dev[size_t(r)]));
        MULTI_HIP(hipMemsetAsync(S.counters.p, 0, 6 * sizeof(unsigned long long), stream_of(r)));
        if (S.n_tiles == 0) continue;
        const int rc = rt_render_tiles_async(scenes[r], cam, &q, S.tiles.as<int>(), S.n_tiles, tile_size,
                                             S.packed.as<float>(), d_depth ? S.depth.as<float>() : nullptr,
                                             S.counters.as<uint64_t>(), stream_of(r));
        if (rc != RT_OK) return rc;
    }
    // the one exchange step: every device's packed tiles, depth and counters to device 0
    // (device 0 sends to itself too, so one code path serves every group size).  An error inside
    // the group still ends it, so later RCCL calls of this thread are not left inside an open group
    MULTI_NCCL(ncclGroupStart());
    ncclResult_t nr = ncclSuccess;
    auto call = [&](ncclResult_t r_) { if (nr == ncclSuccess) nr = r_; };
    for (int r = 0; r < g->n && nr == ncclSuccess; r++) {
        auto &S = *g->share[size_t(r)];
        if (S.n_tiles) {
            call(ncclSend(S.packed.p, size_t(S.n_tiles) * area * 4, ncclFloat32, 0, g->comm[size_t(r)], stream_of(r)));
            if (d_depth)
                call(ncclSend(S.depth.p, size_t(S.n_tiles) * area, ncclFloat32, 0, g->comm[size_t(r)], stream_of(r)));
        }
        call(ncclSend(S.counters.p, 6, ncclUint64, 0, g->comm[size_t(r)], stream_of(r)));
    }
    for (int r = 0; r < g->n && nr == ncclSuccess; r++) {
        auto &S = *g->share[size_t(r)];
        const size_t o = g->off[size_t(r)];
        if (S.n_tiles) {
            call(ncclRecv(g->recv.as<float>() + o * area * 4, size_t(S.n_tiles) * area * 4, ncclFloat32, r, g->comm[0],
                          s0));
            if (d_depth)
                call(ncclRecv(g->recv_depth.as<float>() + o * area, size_t(S.n_tiles) * area, ncclFloat32, r,
                              g->comm[0], s0));
        }
        call(ncclRecv(g->recv_ctr.as<unsigned long long>() + size_t(r) * 6, 6, ncclUint64, r, g->comm[0], s0));
    }
    const ncclResult_t ne = ncclGroupEnd();
    MULTI_NCCL(nr);
    MULTI_NCCL(ne);
    // device 0 assembles the frame
    MULTI_HIP(hipSetDevice(g->dev[0]));
    const uint32_t n_px = uint32_t(size_t(g->off[size_t(g->n)]) * area);
    if (n_px)
        hipLaunchKernelGGL(k_unpack_tiles, dim3((n_px + 255u) / 256u), dim3(256), 0, s0, g->recv.as<float4>(),
                           g->recv_depth.as<float>(), g->recv_tiles.as<int2>(), n_px, tile_size, p->width, p->height,
                           reinterpret_cast<float4 *>(d_rgba), d_depth);
    if (d_counters)
        hipLaunchKernelGGL(k_sum_counters, dim3(1), dim3(64), 0, s0, g->recv_ctr.as<unsigned long long>(), g->n,
                           reinterpret_cast<unsigned long long *>(d_counters));
    MULTI_HIP(hipGetLastError());
    return RT_OK;
}

int rt_render_inw_multi(const float *geom, uint32_t n, int layout, const float *nodes, const float *lights,
                        uint32_t n_lights, const rt_camera *cam, const rt_params *p, const int *devices, int n_dev,
                        int tile_size, float *rgba, float *depth, rt_stats *st) {
    if (!geom || !nodes || n == 0 || !cam || !p || p->width <= 0 || p->height <= 0 || p->spp < 1 || !rgba ||
        !devices || n_dev <= 0 || (layout != 1 && layout != 4))
        return RT_E_ARG;
    DeviceGuard guard;
    struct SceneDel { void operator()(rt_dev_scene *s) const { rt_dev_scene_free(s); } };
    struct GroupDel { void operator()(rt_group *g) const { rt_group_free(g); } };
    std::vector<std::unique_ptr<rt_dev_scene, SceneDel>> own;
    std::vector<rt_dev_scene *> scenes;
    for (int r = 0; r < n_dev; r++) {  // the scene replicated on every device (< 2 MB at C3)
        rt_dev_scene *s = rt_dev_scene_inw(geom, n, layout, nodes, lights, n_lights, p->spp, devices[r]);
        if (!s) return RT_E_NODEVICE;
        own.emplace_back(s);
        scenes.push_back(s);
    }
    std::unique_ptr<rt_group, GroupDel> g(rt_group_create(devices, n_dev));
    if (!g) return RT_E_NODEVICE;
    MULTI_HIP(hipSetDevice(devices[0]));
    const size_t npx = size_t(p->width) * size_t(p->height);
    Buf d_rgba, d_depth, d_ctr;
    MULTI_HIP(d_rgba.ensure(npx * 16, devices[0]));
    MULTI_HIP(hipMemcpy(d_rgba.p, rgba, npx * 16, hipMemcpyHostToDevice));
    if (depth) {
        MULTI_HIP(d_depth.ensure(npx * 4, devices[0]));
        MULTI_HIP(hipMemcpy(d_depth.p, depth, npx * 4, hipMemcpyHostToDevice));
    }
    MULTI_HIP(d_ctr.ensure(6 * sizeof(unsigned long long), devices[0]));
    MULTI_HIP(hipMemset(d_ctr.p, 0, 6 * sizeof(unsigned long long)));
    hipEvent_t e0 = nullptr, e1 = nullptr;
    MULTI_HIP(hipEventCreate(&e0));
    MULTI_HIP(hipEventCreate(&e1));
    MULTI_HIP(hipEventRecord(e0, nullptr));
    int rc = rt_render_multi_async(g.get(), scenes.data(), cam, p, tile_size, d_rgba.as<float>(),
                                   depth ? d_depth.as<float>() : nullptr, d_ctr.as<uint64_t>(), nullptr);
    (void)hipSetDevice(devices[0]);
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc != RT_OK) return rc;
    MULTI_HIP(hipDeviceSynchronize());
    MULTI_HIP(hipMemcpy(rgba, d_rgba.p, npx * 16, hipMemcpyDeviceToHost));
    if (depth) MULTI_HIP(hipMemcpy(depth, d_depth.p, npx * 4, hipMemcpyDeviceToHost));
    if (st) {
        unsigned long long c[6];
        MULTI_HIP(hipMemcpy(c, d_ctr.p, sizeof(c), hipMemcpyDeviceToHost));
        st->segments = c[0]; st->node_visits = c[1]; st->prim_tests = c[2];
        st->shadow_queries = c[3]; st->stack_drops = c[4]; st->nan_drops = c[5];
        st->ms = ms;
    }
    return RT_OK;
}

}  // extern "C"
