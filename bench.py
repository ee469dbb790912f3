#!/usr/bin/env python3
"""bench.py -- Mrays/s of the MI355X render path on BASELINE.json's 1/2/4/8-GPU configuration.

Workload (default, --config c3): BASELINE.json configs[2] at N=1 and configs[3] at N>1, the
In-Next-Week 01 LBVH scene: 10k random moving spheres (seed 1234), 1920x1080,
500 spp, 50 bounces (In-Next-Week/base.h:148-173, 01_BoundingVolumeHierarchy/computeShaderSrc.glsl).
One step = one full frame: every pixel, every sample, every bounce of the reference's INW-01 loop.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|ns]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Secondary lines: --config c2 (configs[1]: In-One-Weekend 03 final scene, 1200x800, 100 spp) and
--config ns (the north star's IOW-03 final scene at 1920x1080, 500 spp).

Multi-GPU (configs[3]): the frame is cut into tiles dealt to the ranks (one process per GPU):
16x16 tiles across ranks, in a hashed order (deal_order), 64x64 on one GPU (RT_BENCH_TILE
overrides both).  Each rank renders its tiles into a packed buffer and the tiles are gathered
to rank 0 with one RCCL gather over xGMI, where the image is assembled.  Total work is fixed,
so the scaling mode is "strong".

Metric: Mrays/s = W*H*spp*mean_bounces / t = (rays cast, counted by the kernels) / t, summed
over ranks, t = max over ranks of the timed region (barrier + synchronize on both sides).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import rt_amd as R  # noqa: E402

TILE = 64        # tile edge on one GPU
TILE_MULTI = 16  # tile edge of a multi-rank partition: finer tiles deal the heavy pixels out more evenly


def tile_for(world: int) -> int:
    """Tile edge (a multiple of 8) for a partition over `world` ranks; RT_BENCH_TILE overrides."""
    env = os.environ.get("RT_BENCH_TILE", "")
    return int(env) if env else (TILE if world == 1 else TILE_MULTI)
FP32_PEAK_TFLOPS = 157.3   # MI355X FP32 vector peak (= f32 MFMA rate), MI355X_MICROARCH.md
HBM_PEAK_GBPS = 8000.0     # MI355X HBM3E peak, MI355X_MICROARCH.md
CUS = 256                  # MI355X compute units
CLOCK_HZ = 2.4e9           # MI355X peak engine clock
METRIC = "Mrays/s (W\u00d7H\u00d7spp\u00d7mean_bounces/t) + achieved HBM GB/s, 1/2/4/8 MI355X"  # BASELINE.json
# --config -> (preset, seed, n_hint, overrides, workload at N=1, workload at N>1, data)
CONFIGS = {
    "c3": ("INW01_RANDOM", 1234, 10_000, {},
           "In-Next-Week 01 LBVH: 10k random moving spheres, 1920x1080, 500 spp, 50 bounces, 1 MI355X "
           "(BASELINE configs[2])",
           "In-Next-Week 01 LBVH: 10k random moving spheres, 1920x1080, 500 spp, 50 bounces, tile-partitioned "
           "across {n} MI355X with an RCCL gather over xGMI (BASELINE configs[3])",
           "synthetic (seeded C3 generator, SURVEY 8d seed 1234; LBVH built by rt_lbvh_build)"),
    "c2": ("IOW03_FINAL", 20250131, 0, {},
           "In-One-Weekend 03_Adding_Materials final scene (~500 random spheres + ground cuboid), 1200x800, "
           "100 spp, 50 bounces (BASELINE configs[1])",
           "In-One-Weekend 03_Adding_Materials final scene, 1200x800, 100 spp, 50 bounces, tile-partitioned "
           "across {n} MI355X with an RCCL gather",
           "synthetic (seeded final-scene generator, SURVEY 8d seed 20250131)"),
    "c5": ("INW04_CORNELL", 7, 0, {},
           "In-Next-Week 04_Lighting Cornell-box emissive scene, 4096x4096, 2000 spp, 50 bounces, 1 MI355X "
           "(BASELINE configs[4])",
           "In-Next-Week 04_Lighting Cornell-box emissive scene, 4096x4096, 2000 spp, 50 bounces, tile-partitioned "
           "across {n} MI355X with an RCCL gather",
           "synthetic (Cornell-style box generator, SURVEY 8d seed 7)"),
    "ns": ("IOW03_FINAL", 20250131, 0, {"width": 1920, "height": 1080, "spp": 500},
           "In-One-Weekend 03 final scene, 1920x1080, 500 spp, 50 bounces (BASELINE north_star workload)",
           "In-One-Weekend 03 final scene, 1920x1080, 500 spp, 50 bounces, tile-partitioned across {n} MI355X "
           "with an RCCL gather (BASELINE north_star workload)",
           "synthetic (seeded final-scene generator, SURVEY 8d seed 20250131)"),
}


def algorithmic_flops(st: dict) -> float:
    """SURVEY.md 8d contract: F_alg = 40*node_visits + 70*prim_tests + 60*segments."""
    return 40.0 * st["node_visits"] + 70.0 * st["prim_tests"] + 60.0 * st["segments"]


def algorithmic_bytes(st: dict, pixels: int, inw: bool = False) -> float:
    """SURVEY.md 8d contract: B_alg = 32*node_visits + 96*prim_tests (IOW records) + 16*W*H;
    INW: 112-B records, 28 B per shadow query's light record and 20 B per pixel (colour + depth)."""
    if inw:  # + the 28-B light record each shadow query reads (INW-04)
        return 32.0 * st["node_visits"] + 112.0 * st["prim_tests"] + 28.0 * st["shadow_queries"] + 20.0 * pixels
    return 32.0 * st["node_visits"] + 96.0 * st["prim_tests"] + 16.0 * pixels


def deal_order(nx: int, ny: int, world: int):
    """The order tiles are dealt in: row-major on one GPU; across ranks, row-major tiles permuted
    by a multiplicative hash of their index.  A plain round-robin over rows gives rank r the
    tile columns r, r+N, ... whenever the row length is a multiple of N (1920 px / 16 = 120
    tiles), so a heavy vertical region (a glass sphere) lands on a few ranks."""
    tiles = [(tx, ty) for ty in range(ny) for tx in range(nx)]
    if world == 1:
        return tiles
    perm = sorted(range(len(tiles)), key=lambda i: ((i * 2654435761) & 0xFFFFFFFF, i))
    return [tiles[i] for i in perm]


def tiles_for_rank(W: int, H: int, world: int, rank: int, tile: int = TILE):
    """(deal order of all tiles, this rank's tiles = order[rank::world], tiles per rank)."""
    nx, ny = math.ceil(W / tile), math.ceil(H / tile)
    order = deal_order(nx, ny, world)
    return order, order[rank::world], math.ceil(len(order) / world)


def lpt_deal(costs, nx: int, ny: int, world: int):
    """Tile lists per rank by longest-processing-time-first: tiles in decreasing measured cost
    (ties: row-major index), each to the rank with the least cost so far (ties: lowest rank).
    costs[ty * nx + tx] = rays the tile took in an earlier frame of the same view."""
    import heapq
    order = sorted(range(nx * ny), key=lambda i: (-float(costs[i]), i))
    heap = [(0.0, r) for r in range(world)]
    lists = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        lists[r].append((i % nx, i // nx))
        heapq.heappush(heap, (load + float(costs[i]), r))
    return lists


def refine_deal(lists, costs, times, nx: int, tol: float = 0.003):
    """Rebalance a deal by measured rank times (the view is static, so a frame's times predict the
    next one's).  Each rank's time per unit of tile cost k_r = time_r / load_r folds in what rays
    alone miss (the long dependent chains of IOW-03 samples, the tail of a rank's last pixels);
    the equal-time target T solves sum_r T / k_r = sum_r load_r.  Ranks above their share T / k_r
    hand their cheapest tiles to the rank furthest below its share until within `tol`, so the
    heavy tiles -- where the long chains are -- stay where they were measured.  Deterministic:
    every rank computes the same lists from the same reduced costs and gathered times.
    costs[ty * nx + tx] = rays per tile; times[r] = rank r's frame time."""
    lists = [[tuple(t) for t in lst] for lst in lists]
    cost = lambda t: float(costs[t[1] * nx + t[0]])  # noqa: E731
    load = [sum(cost(t) for t in lst) for lst in lists]
    if min(load) <= 0.0 or min(times) <= 0.0:
        return lists
    k = [float(tm) / ld for tm, ld in zip(times, load)]
    target = sum(load) / sum(1.0 / kr for kr in k)
    want = [target / kr for kr in k]
    for r in sorted(range(len(lists)), key=lambda r: (want[r] - load[r], r)):
        movable = sorted(lists[r], key=lambda t: (cost(t), t[1], t[0]))  # cheapest first
        for t in movable:
            if load[r] - want[r] <= tol * want[r]:
                break
            s = min(range(len(lists)), key=lambda q: ((load[q] - want[q]) / want[q], q))
            c = cost(t)
            if load[s] + c > want[s] * (1.0 + tol) or c > load[r] - want[r]:
                continue
            lists[r].remove(t)
            lists[s].append(t)
            load[r] -= c
            load[s] += c
    return lists


def assemble_lists(src, lists, nx: int, ny: int):
    """src: [world, per_rank, T, T, C] packed tiles as gathered on rank 0 (C = 4 colour channels,
    1 for depth), where tile t of rank r is lists[r][t].  Returns the [ny*T, nx*T, C] frame (crop
    to W x H)."""
    T, Cn = src.shape[2], src.shape[4]
    sel = [(r, t) for r, lst in enumerate(lists) for t in range(len(lst))]
    rr = torch.tensor([a for a, _ in sel], dtype=torch.long, device=src.device)
    tt = torch.tensor([b for _, b in sel], dtype=torch.long, device=src.device)
    idx = torch.tensor([ty * nx + tx for lst in lists for tx, ty in lst], dtype=torch.long, device=src.device)
    grid = torch.empty((nx * ny, T, T, Cn), dtype=src.dtype, device=src.device)
    grid[idx] = src[rr, tt]
    return grid.view(ny, nx, T, T, Cn).permute(0, 2, 1, 3, 4).reshape(ny * T, nx * T, Cn)


def message_views(msg, per_rank: int, T: int, with_depth: bool):
    """A rank's one gather message: its packed colour tiles [per_rank, T, T, 4] followed by their
    r32f depth tiles [per_rank, T, T] (INW writes both images per dispatch, 01_BVH...glsl:667-668;
    In-Next-Week/base.h:148-173), as views of one flat buffer."""
    n = per_rank * T * T
    col = msg[:4 * n].view(per_rank, T, T, 4)
    dep = msg[4 * n:5 * n].view(per_rank, T, T) if with_depth else None
    return col, dep


def assemble_message(gathered, lists, nx: int, ny: int, per_rank: int, T: int, with_depth: bool):
    """Rank 0: the gathered messages (one per rank) -> the [ny*T, nx*T, 4] colour frame and the
    [ny*T, nx*T] depth frame (None without depth)."""
    views = [message_views(g, per_rank, T, with_depth) for g in gathered]
    img = assemble_lists(torch.stack([v[0] for v in views], 0), lists, nx, ny)
    dimg = None
    if with_depth:
        dimg = assemble_lists(torch.stack([v[1] for v in views], 0).unsqueeze(-1), lists, nx, ny)[..., 0]
    return img, dimg


def assemble_frame(src, order, nx: int, ny: int):
    """src: [world, per_rank, T, T, 4] packed tiles as gathered on rank 0, where tile t of rank r
    is order[r + world*t].  Returns the [ny*T, nx*T, 4] frame (crop to W x H)."""
    world = src.shape[0]
    return assemble_lists(src, [order[r::world] for r in range(world)], nx, ny)


def host_cores() -> int:
    """The GPU box's host cores as `nproc` reports them (it honours the CPU affinity mask and
    OMP_NUM_THREADS, i.e. this job's share of the host); os.cpu_count() as a fallback."""
    import subprocess
    try:
        return max(1, int(subprocess.run(["nproc"], capture_output=True, text=True, check=True).stdout))
    except Exception:  # noqa: BLE001
        return os.cpu_count() or 1


def cpu_baseline(sc, threads: int, spp: int, bw: int = 64, rows_per_core: int = 1) -> dict:
    """The CPU oracle (the C restatement of the reference shader, OpenMP schedule(dynamic, 1) over
    pixel rows) on all `threads` host cores, on a bounded sample of the same frame: the central
    bw x (rows_per_core * threads) pixel block (every core has rows to take), at `spp` samples
    (Mrays/s is a rate) and the full bounce count."""
    from oracle import oracle as O
    O.set_threads(threads)
    p = R.RtParams()
    C.memmove(C.addressof(p), C.addressof(sc.params), C.sizeof(p))
    bh = max(threads, 8) * rows_per_core
    p.spp = min(spp, sc.params.spp)
    p.tile_x0, p.tile_y0 = sc.params.width // 2 - bw // 2, sc.params.height // 2 - bh // 2
    p.tile_w, p.tile_h = bw, bh
    t0 = time.perf_counter()
    rgba, depth, st = O.render(sc, p)
    dt = time.perf_counter() - t0
    rect = (p.tile_x0, p.tile_y0, bw, bh)
    return {"value": st["segments"] / dt / 1e6, "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"central {bw}x{bh} pixel block of the same frame at {p.spp} spp / "
                      f"{sc.params.max_bounces} bounces, one OpenMP thread per core = nproc "
                      f"({st['segments']} rays, {dt:.1f} s, oracle/librt_oracle.so)"}, (rect, rgba, depth, p.spp)


def block_parity(rect, ref_rgba, ref_depth, img, dep) -> dict:
    """The GPU frame's pixels in `rect` against the oracle's render of that block (bit
    comparison, NaN == NaN): max |delta| per channel, the fraction of bit-identical values, pixels."""
    x0, y0, w, h = rect
    a = np.ascontiguousarray(img[y0:y0 + h, x0:x0 + w], np.float32)
    b = np.ascontiguousarray(ref_rgba[y0:y0 + h, x0:x0 + w], np.float32)
    pairs = [(a, b)]
    if dep is not None and ref_depth is not None:
        pairs.append((np.ascontiguousarray(dep[y0:y0 + h, x0:x0 + w], np.float32),
                      np.ascontiguousarray(ref_depth[y0:y0 + h, x0:x0 + w], np.float32)))
    same, total, mx, nan_mis = 0, 0, 0.0, 0
    for u, v in pairs:
        nu, nv = np.isnan(u), np.isnan(v)
        both = ~(nu | nv)
        d = np.abs(u[both].astype(np.float64) - v[both].astype(np.float64))
        mx = max(mx, float(d.max()) if d.size else 0.0)
        same += int(((u.view(np.uint32) == v.view(np.uint32)) | (nu & nv)).sum())
        total += u.size
        nan_mis += int((nu != nv).sum())
    return {"max_abs": mx, "exact_frac": same / max(total, 1), "nan_mismatch": nan_mis, "pixels": w * h,
            "rect": list(rect), "depth": len(pairs) > 1, "tol": 1e-3,
            "oracle": "oracle/librt_oracle.so render of the same block at the same spp (the cpu_baseline run)"}


def apply_opts(opts):
    """--opt FIELD=VALUE: set rt_options fields (rejecting names the struct lacks)."""
    if not opts:
        return
    o = R.get_options()
    fields = dict(R.RtOptions._fields_)
    for kv in opts:
        k, sep, v = kv.partition("=")
        if not sep or k not in fields or k == "size":  # a ctypes Structure would accept any name
            raise SystemExit(f"--opt {kv!r}: not FIELD=VALUE with an rt_options field "
                             f"({', '.join(f for f in fields if f != 'size')})")
        setattr(o, k, float(v) if k == "spec_max_gb" else int(v))
    R.set_options(o)


def main_group(args):
    """--group: the C ABI's multi-GPU path (rt_multi.hip) timed from one process -- the host a C++
    OnUpdateBase replacement would be.  The scene is replicated on devices
    0..gpus-1, rt_render_multi_async deals the frame's 16x16 tiles across them (rt_tile_deal), every
    device renders its share on its own stream and one grouped RCCL send/recv brings the colour,
    depth and counter tiles to device 0, which assembles the W x H images.  Timed like main():
    warm-up frames, then K frames between device synchronisations of every group device."""
    n = args.gpus
    if n < 1 or n > torch.cuda.device_count():
        raise SystemExit(f"--group --gpus {n}: {torch.cuda.device_count()} devices visible")
    lib = R.load()
    apply_opts(args.opt)
    cfg = "c3" if args.config == "c4" else args.config
    preset, seed, n_hint, base_over, wl1, wln, data = CONFIGS[cfg]
    over = {k: v for k, v in (("spp", args.spp), ("width", args.width), ("height", args.height)) if v}
    sc = R.make_scene(getattr(R, "PRESET_" + preset), seed, n_hint, **{**base_over, **over})
    if sc.stage == R.RT_STAGE_IOW03:
        raise SystemExit("--group: INW configs (c3 / c4 / c5)")
    W, H, spp = sc.params.width, sc.params.height, sc.params.spp
    lt = sc.lights if sc.lights is not None and len(sc.lights) else None
    scenes = []
    for d in range(n):
        s_ = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, sc.layout, R.fptr(sc.nodes), R.fptr(lt), sc.n_lights, spp, d)
        if not s_:
            raise RuntimeError(f"rt_dev_scene_inw on device {d} failed")
        scenes.append(s_)
    grp = lib.rt_group_create((C.c_int * n)(*range(n)), n)
    if not grp:
        raise RuntimeError("rt_group_create failed")
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    img = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
    dep = torch.zeros((H, W), dtype=torch.float32, device=dev)
    ctr = torch.zeros(6, dtype=torch.int64, device=dev)
    sl = (C.c_void_p * n)(*scenes)
    stream = torch.cuda.current_stream(dev).cuda_stream

    def frame():
        rc = lib.rt_render_multi_async(grp, sl, C.byref(sc.camera), C.byref(sc.params), TILE_MULTI, img.data_ptr(),
                                       dep.data_ptr(), ctr.data_ptr(), stream)
        if rc != 0:
            raise RuntimeError(f"rt_render_multi_async -> {rc}")

    def sync_all():
        for d in range(n):
            torch.cuda.synchronize(d)

    for _ in range(args.warmup):
        frame()
    sync_all()
    ctr.zero_()
    sync_all()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        frame()
    sync_all()
    elapsed = time.perf_counter() - t0
    c = [int(v) for v in ctr.cpu().tolist()]
    st = dict(zip(("segments", "node_visits", "prim_tests", "shadow_queries", "stack_drops", "nan_drops"), c))
    per_step = {k: v // args.steps for k, v in st.items()}
    path = R.debug_path(scenes[0])
    out = {
        "metric": METRIC, "value": round(st["segments"] / elapsed / 1e6, 3), "unit": "Mrays/s", "n_gpus": n,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": data,
        "config": {"workload": (wl1 if n == 1 else wln.format(n=n)) + " (--group: one process, C-ABI device group)",
                   "width": W, "height": H, "spp": spp, "max_bounces": sc.params.max_bounces, "objects": sc.n,
                   "tile": TILE_MULTI, "parallelism": f"group{n}+rccl_send_recv"},
        "mean_bounces": round(st["segments"] / (W * H * spp * args.steps), 3),
        "rays_per_step": per_step["segments"], "counters_per_step": per_step, "path": path,
        "options": {k: v for k, v in R.get_options().as_dict().items()
                    if v != R.default_options().as_dict()[k]} or "defaults",
        "timed_region": "rt_render_multi_async of one full frame per step: every device's share, the grouped "
                        "RCCL send/recv of colour + depth + counters to device 0, its unpack kernel",
    }
    print(json.dumps(out), flush=True)
    if args.save_image:
        np.save(args.save_image, img.cpu().numpy())
        np.save(os.path.splitext(args.save_image)[0] + ".depth.npy", dep.cpu().numpy())
    lib.rt_group_free(grp)
    for s_ in scenes:
        lib.rt_dev_scene_free(s_)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--spp", type=int, default=0, help="override spp (default: the config's 100)")
    ap.add_argument("--width", type=int, default=0)
    ap.add_argument("--height", type=int, default=0)
    ap.add_argument("--cpu-spp", type=int, default=0,
                    help="CPU baseline samples per pixel (default: the config's spp)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="host cores for the CPU baseline (default: nproc)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--balance", action="store_true",
                    help="multi-rank: deal the timed frames' tiles by LPT over the warm-up frame's tile costs "
                         "(measured neutral on the 8-way frames: their time is set by long samples, not by rays)")
    ap.add_argument("--balance-time", action="store_true",
                    help="multi-rank: after the warm-up frames (hashed deal), move each rank's cheapest tiles "
                         "from ranks above the equal-time share to ranks below it, by the warm-up frame's "
                         "measured rank times and per-tile rays (bench.refine_deal)")
    ap.add_argument("--occupancy", action="store_true", help="report per-phase lane occupancy (diagnostic)")
    ap.add_argument("--save-image", default="", help="rank 0 saves the assembled frame (.npy) for checking")
    ap.add_argument("--rebuild", action="store_true",
                    help="secondary line: every step also does the reference's per-redraw scene work "
                         "(RT_Base::OnUpdateBase, In-Next-Week/base.h:96-175): rt_pack_inw of the scene "
                         "descriptions, then rt_dev_scene_inw_update with the LBVH built on the device, then the frame")
    ap.add_argument("--opt", action="append", default=[], metavar="FIELD=VALUE",
                    help="set an rt_options field for this run (A/B of the exact strategies; recorded in the line)")
    ap.add_argument("--group", action="store_true",
                    help="one process drives --gpus devices through the C ABI's device group "
                         "(rt_group_create + rt_render_multi_async: tiles dealt across the devices, one "
                         "grouped RCCL send/recv of colour, depth and counters to device 0); INW configs")
    ap.add_argument("--config", default="c3", choices=("c3", "c4", "c2", "c5", "ns"),
                    help="c3 (= c4): BASELINE configs[2] / configs[3], the headline; c2: configs[1]; "
                         "c5: configs[4]; ns: the north star's IOW-03 workload")
    args = ap.parse_args()
    if args.group:
        return main_group(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # RT_BENCH_BACKEND=gloo: multi-rank rehearsal on a box with fewer GPUs than ranks (ranks
    # share devices, collectives go through host memory); the measured path is nccl (RCCL)
    backend = os.environ.get("RT_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    host_coll = world > 1 and backend != "nccl"

    lib = R.load()
    apply_opts(args.opt)
    over = {}
    if args.spp:
        over["spp"] = args.spp
    if args.width:
        over["width"] = args.width
    if args.height:
        over["height"] = args.height
    cfg = "c3" if args.config == "c4" else args.config
    preset, seed, n_hint, base_over, wl1, wln, data = CONFIGS[cfg]
    sc = R.make_scene(getattr(R, "PRESET_" + preset), seed, n_hint, **{**base_over, **over})
    inw = sc.stage != R.RT_STAGE_IOW03
    W, H, spp = sc.params.width, sc.params.height, sc.params.spp
    T = tile_for(world)
    nparts, part = world, rank  # partition size and this process's part
    shard = os.environ.get("RT_BENCH_SHARD", "")  # diagnostic "r/N": one process renders rank r's tiles of N
    if shard and world == 1:
        part, nparts = (int(v) for v in shard.split("/"))
        T = tile_for(nparts)
    nx, ny = math.ceil(W / T), math.ceil(H / T)
    allt = deal_order(nx, ny, nparts)
    lists = [allt[r::nparts] for r in range(nparts)]  # the hashed deal (first frame)
    deal_file = os.environ.get("RT_BENCH_DEAL", "")  # diagnostic: a deal computed elsewhere (tools/gpu/shares_refined.sh)
    if deal_file:
        with open(deal_file) as fh:
            lists = [[tuple(t) for t in lst] for lst in json.load(fh)]
        if len(lists) != nparts:
            raise SystemExit(f"RT_BENCH_DEAL holds {len(lists)} lists for {nparts} parts")

    if inw:
        lt = sc.lights if sc.lights is not None and len(sc.lights) else None
        scene = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, sc.layout, R.fptr(sc.nodes), R.fptr(lt), sc.n_lights, spp,
                                     local)
    else:
        scene = lib.rt_dev_scene_iow03(R.fptr(sc.types), R.fptr(sc.records), sc.n, spp, local)
    if not scene:
        raise RuntimeError("rt_dev_scene_iow03 failed (no gfx950 device?)")
    counters = torch.zeros(6, dtype=torch.int64, device=dev)
    dbg = torch.zeros(16, dtype=torch.int64, device=dev)
    buf = {}

    def use_tiles(my_tiles, per_rank):
        """(Re)allocate this rank's tile list and packed buffers (outside the timed region): one flat
        message of the packed colour tiles and (INW) their r32f depth tiles, gathered in one call."""
        buf["mine"] = my_tiles
        buf["per_rank"] = per_rank
        buf["d_tiles"] = torch.tensor(my_tiles, dtype=torch.int32, device=dev).reshape(-1, 2).contiguous()
        buf["msg"] = torch.zeros(per_rank * T * T * (5 if inw else 4), dtype=torch.float32, device=dev)
        buf["packed"], buf["depth"] = message_views(buf["msg"], per_rank, T, inw)
        buf["px_rays"] = torch.zeros(max(1, len(my_tiles)) * T * T, dtype=torch.int32, device=dev)
        buf["gathered"] = [torch.empty_like(buf["msg"]) for _ in range(world)] if (world > 1 and rank == 0) else None

    per_rank = max(len(v) for v in lists)
    use_tiles(lists[part], per_rank)
    if args.rebuild and not inw:
        raise SystemExit("--rebuild: INW configs only (c3 / c4)")
    rb_ms = np.zeros(6)  # per timed step: pack, records, LBVH, walk structures, their upload, (unused)
    rb_on = [False]
    lib.rt_debug_time_kernels(1)
    if args.occupancy:
        lib.rt_debug_counters(dbg.data_ptr())
    image = torch.empty((ny * T, nx * T, 4), dtype=torch.float32, device=dev) if rank == 0 else None
    dimage = torch.empty((ny * T, nx * T), dtype=torch.float32, device=dev) if rank == 0 and inw else None
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def rebuild():
        """RT_Base<>::OnUpdateBase's per-redraw scene work on the device scene: FillBuffer and the
        swept boxes (rt_pack_inw), the records, the LBVH on the device (ConstructLBVH_Buff,
        base.h:135-142), the wide walk and RI grid on the device (rt_options.inw_device_build;
        0: on the host from the read-back LBVH, then uploaded)."""
        t0 = time.perf_counter()
        pk = R.pack(sc.desc, sc.n, sc.stage, build_lbvh=False)
        t1 = time.perf_counter()
        lt = pk["lights"] if len(pk["lights"]) else None
        tm = (C.c_double * 4)()
        rc = lib.rt_dev_scene_inw_update(scene, R.fptr(pk["geom"]), sc.n, None, R.fptr(pk["aabbs"]), R.fptr(lt),
                                         pk["n_lights"], tm)
        if rc != 0:
            raise RuntimeError(f"rt_dev_scene_inw_update -> {rc}")
        if rb_on[0]:
            rb_ms[:5] += [(t1 - t0) * 1e3, tm[0], tm[1], tm[2], tm[3]]

    def step(i=None, evp=None):
        """One frame; `i`: timed step i (events ev[i]); `evp`: an event pair around the render alone
        (the --balance-time warm-up frame: the gather below would make every rank wait for the slowest)."""
        mine, d_tiles, packed, depth = buf["mine"], buf["d_tiles"], buf["packed"], buf["depth"]
        gathered = buf["gathered"]
        stream = torch.cuda.current_stream()
        if args.rebuild:
            rebuild()
        if evp is None and i is not None:
            evp = ev[i]
        if evp is not None:
            evp[0].record(stream)
        if mine:
            rc = lib.rt_render_tiles_async(scene, C.byref(sc.camera), C.byref(sc.params), d_tiles.data_ptr(),
                                           len(mine), T, packed.data_ptr(),
                                           depth.data_ptr() if depth is not None else None, counters.data_ptr(),
                                           stream.cuda_stream)
            if rc != 0:
                raise RuntimeError(f"rt_render_tiles_async -> {rc}")
        if evp is not None:
            evp[1].record(stream)
        msg = buf["msg"]
        if world > 1 and not host_coll:  # the one exchange step: RCCL gather of colour + depth tiles to rank 0
            dist.gather(msg, gathered, dst=0)
        elif world > 1:
            hg = [torch.empty_like(msg, device="cpu") for _ in range(world)] if rank == 0 else None
            dist.gather(msg.cpu(), hg, dst=0)
            if rank == 0:
                for g_, h_ in zip(gathered, hg):
                    g_.copy_(h_)
        if rank == 0 and not shard:  # assemble the frame: tile t of rank r is lists[r][t]
            img, dimg = assemble_message(gathered if world > 1 else [msg], lists, nx, ny, buf["per_rank"], T, inw)
            image.copy_(img)
            if dimage is not None:
                dimage.copy_(dimg)

    def barrier():
        if world > 1:
            if host_coll:
                dist.barrier()
            else:
                dist.barrier(device_ids=[local])
        torch.cuda.synchronize()

    def tile_costs():
        """Rays per tile over the whole frame from the last rendered frame's per-pixel counts."""
        mine = buf["mine"]
        g = torch.zeros(nx * ny, dtype=torch.float64, device=dev)
        if mine:
            per = buf["px_rays"][:len(mine) * T * T].view(len(mine), T * T).sum(1).double()
            idx = torch.tensor([ty * nx + tx for tx, ty in mine], dtype=torch.long, device=dev)
            g[idx] = per
        if world > 1:
            if host_coll:
                g = g.cpu()
            dist.all_reduce(g)
        return g.cpu().numpy()

    # Load balance (multi-rank partitions, --balance; off by default): the warm-up
    # frames record rays per pixel; the timed frames deal tiles by LPT over those per-tile costs
    # (the view is static, so a frame's costs predict the next one's).  A shard-diagnostic
    # process renders every tile in its warm-up to get them (cached in RT_BENCH_COSTS).
    balance = nparts > 1 and args.balance and args.warmup > 0
    tbal = nparts > 1 and args.balance_time and args.warmup > 0 and not shard
    if tbal:
        lib.rt_debug_pixel_rays(buf["px_rays"].data_ptr())
    costs = None
    cache = os.environ.get("RT_BENCH_COSTS", "")
    if balance and shard and cache and os.path.exists(cache):
        costs = np.load(cache)
    if balance and costs is None and shard:
        use_tiles(allt, len(allt))
    if balance and costs is None:
        lib.rt_debug_pixel_rays(buf["px_rays"].data_ptr())
    wt = 0.0
    wev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    for w in range(args.warmup):
        if (balance and costs is None or tbal) and w == args.warmup - 1:
            buf["px_rays"].zero_()
        # --balance-time: this rank's own render time of the last warm-up frame (HIP events on the
        # render stream, before the gather, which would make every rank wait for the slowest)
        step(evp=wev if tbal and w == args.warmup - 1 else None)
    barrier()
    if tbal:
        wt = wev[0].elapsed_time(wev[1]) * 1e-3
    if tbal:  # refine the hashed deal by the last warm-up frame's rank times
        tcosts = tile_costs()
        lib.rt_debug_pixel_rays(None)
        tt = torch.tensor([wt], dtype=torch.float64, device="cpu" if host_coll else dev)
        gl = [torch.zeros_like(tt) for _ in range(world)]
        dist.all_gather(gl, tt)
        lists = refine_deal(lists, tcosts, [float(x.item()) for x in gl], nx)
        per_rank = max(len(v) for v in lists)
        use_tiles(lists[part], per_rank)
        step()  # one frame on the final partition (first use of its buffers)
        barrier()
    if balance:
        if costs is None:
            costs = tile_costs()
            if shard and cache:
                np.save(cache, costs)
        lib.rt_debug_pixel_rays(None)
        lists = lpt_deal(costs, nx, ny, nparts)
        per_rank = max(len(v) for v in lists)
        use_tiles(lists[part], per_rank)
        step()  # one frame on the final partition (first use of its buffers)
        barrier()
    if args.occupancy:
        lib.rt_debug_pixel_rays(buf["px_rays"].data_ptr())
    counters.zero_()
    rb_on[0] = True
    barrier()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = sum(a.elapsed_time(b) for a, b in ev) / args.steps
    rb_on[0] = False
    blocking_ms = None
    if args.rebuild and world == 1:  # the blocking entry point INTEGRATION.md binds (rt_render_inw): host in / out
        tb = time.perf_counter()
        R.render(sc)
        blocking_ms = (time.perf_counter() - tb) * 1e3

    t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
    ctr = counters.clone()
    if world > 1:
        if host_coll:
            t, ctr = t.cpu(), ctr.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(ctr, op=dist.ReduceOp.SUM)
    elapsed, kernel_ms = float(t[0]), float(t[1])
    c = [int(v) for v in ctr.cpu().tolist()]
    st = dict(zip(("segments", "node_visits", "prim_tests", "shadow_queries", "stack_drops", "nan_drops"), c))
    per_step = {k: v / args.steps for k, v in st.items()}

    path = R.debug_path(scene)  # the kernel and the exact shortcuts the last frame ran (rt_debug_path)
    if inw:  # the last frame's closest-hit queries handed to the reference's LBVH walks (rt_path_info.ref_walks)
        q = per_step["segments"] + per_step["shadow_queries"]
        rw_all = path["ref_walks"]
        if world > 1:
            t_ = torch.tensor([rw_all], dtype=torch.float64, device="cpu" if host_coll else dev)
            dist.all_reduce(t_)
            rw_all = int(t_.item())
        path["ref_walk_frac"] = round(rw_all / q, 6) if q else None
    launches = max(1, path["launches"])  # main-kernel launches per frame (planned)
    kname = path["kernel"]
    # the main kernel's own launches in the last timed frame, each bracketed by HIP events on its
    # stream inside the library (rt_debug_time_kernels): what rocprofv3's per-kernel stats see
    kt_ms, kt_n = C.c_double(0.0), C.c_int(0)
    if lib.rt_debug_kernel_time(scene, C.byref(kt_ms), C.byref(kt_n)) == 0 and kt_n.value > 0:
        launches, main_ms = kt_n.value, kt_ms.value
    else:
        main_ms = kernel_ms
    if world > 1:
        mt = torch.tensor([main_ms], dtype=torch.float64, device=dev)
        if host_coll:
            mt = mt.cpu()
        dist.all_reduce(mt, op=dist.ReduceOp.MAX)
        main_ms = float(mt[0])
    if rank == 0:
        value = st["segments"] / elapsed / 1e6
        flops = algorithmic_flops(per_step)
        # per launch of the main kernel: the frame's algorithmic flops (all of its rays; the
        # sequential leftover pass traces ~2% of them) over the main kernel's launches
        achieved = flops / (main_ms * 1e-3) / 1e12
        balg = algorithmic_bytes(per_step, W * H / world, inw) / launches
        avg_s = main_ms / launches * 1e-3
        traffic, valu, lane_issue, prof_src = None, None, None, None
        prof = os.path.join(ROOT, "profiles", f"pmc_{cfg}.json")  # PMC passes of this config's command
        if os.path.exists(prof) and world == 1:
            try:
                pm = json.load(open(prof))
                if (pm.get("config") == [W, H, spp] and pm.get("kernel") == kname
                        and pm.get("launches_per_frame") == launches):
                    prof_src = "profiles/" + os.path.basename(prof)
                    traffic = pm.get("hbm_bytes_per_launch")
                    # VALU issue: a wave64 VALU instruction holds its SIMD's issue for 2 cycles
                    # (MI355X_MICROARCH.md); capacity = CUs x 4 SIMDs x clock x main-kernel time
                    insts = pm["counters"]["SQ_INSTS_VALU"] / pm["frames"]
                    busy = 2.0 * insts / (CUS * 4 * CLOCK_HZ * (main_ms * 1e-3))
                    util = pm["valu_lane_utilisation"]
                    lane_issue = busy * util
                    valu = {"busy_frac": round(busy, 4), "lane_util": round(util, 4),
                            "lane_issue_frac": round(lane_issue, 4), "insts_per_frame": insts,
                            "clock_hz": CLOCK_HZ,
                            "source": prof_src + " (SQ_INSTS_VALU, SQ_THREAD_CYCLES_VALU / SQ_ACTIVE_INST_VALU)"}
            except Exception:  # noqa: BLE001
                traffic, valu, lane_issue, prof_src = None, None, None, None
        # the same roofline over the reference's own walk: F_alg with the node visits and object
        # tests of the reference's LBVH walk of this frame (inw_wide_walk=0, the oracle's counts;
        # profiles/refwalk_<cfg>.json), a fixed amount of work per frame whatever walk runs
        ref_walk = None
        rw = os.path.join(ROOT, "profiles", f"refwalk_{cfg}.json")
        if inw and world == 1 and os.path.exists(rw):
            try:
                rj = json.load(open(rw))
                rc = rj["counters_per_step"]
                if ([rj["config"]["width"], rj["config"]["height"], rj["config"]["spp"]] == [W, H, spp]
                        and rc["segments"] == int(per_step["segments"])):
                    fr = algorithmic_flops(rc) / launches
                    ref_walk = {"flops_per_launch": fr, "equivalent_TFLOPs": round(fr / avg_s / 1e12, 3),
                                "equivalent_frac": round(fr / avg_s / 1e12 / FP32_PEAK_TFLOPS, 4),
                                "node_visits": rc["node_visits"], "prim_tests": rc["prim_tests"],
                                "note": "NOT achieved: the reference LBVH walk's flops for this frame over this "
                                        "kernel's time -- work the kernel did not do (its own walk is 'frac')",
                                "source": "profiles/" + os.path.basename(rw)}
            except Exception:  # noqa: BLE001
                ref_walk = None
        cpu, parity = None, None
        if world == 1 and not args.no_cpu_baseline:
            cores = args.cpu_threads or host_cores()
            # ~10-20 s of host work on the GPU box (C3: 3.2 Mrays/s on 16 cores for the central block)
            if cfg == "c3":
                cpu, ref = cpu_baseline(sc, cores, args.cpu_spp or sc.params.spp, bw=256, rows_per_core=4)
            elif cfg == "c5":  # 2000 spp, ~6 rays per sample with the shadow queries
                cpu, ref = cpu_baseline(sc, cores, args.cpu_spp or sc.params.spp, bw=32, rows_per_core=2)
            else:  # IOW-03: ~280 rays per sample; ns has 5x the samples per pixel of c2
                cpu, ref = cpu_baseline(sc, cores, args.cpu_spp or sc.params.spp, bw=16 if cfg == "ns" else 64)
            rect, ref_rgba, ref_depth, ref_spp = ref
            if ref_spp == spp and not shard:  # the oracle rendered the same block at the frame's spp
                dimg = dimage.cpu().numpy() if dimage is not None else None  # the last timed frame's depth
                parity = block_parity(rect, ref_rgba, ref_depth, image.cpu().numpy(), dimg)
        out = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": data,
            "config": {"workload": wl1 if world == 1 else wln.format(n=world), "width": W, "height": H,
                       "spp": spp, "max_bounces": sc.params.max_bounces, "objects": sc.n, "tile": T,
                       "parallelism": f"tiles_rr{world}" + ("+rccl_gather" if world > 1 else ""),
                       "deal": ("lpt_rays" if balance else "time_refined" if tbal else "hashed") if world > 1 else None},
            "roofline": {"bound": "valu", "achieved": round(achieved, 3), "peak": FP32_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                         "traffic": traffic, "lane_issue_frac": round(lane_issue, 4) if lane_issue else None,
                         "kernel": kname, "launches_per_frame": launches,
                         "avg_launch_ms": round(main_ms / launches, 3),
                         "main_kernel_ms_per_frame": round(main_ms, 3),
                         "render_ms_per_frame": round(kernel_ms, 3),
                         "flops_per_launch": flops / launches,
                         "source": prof_src,
                         "ref_walk": ref_walk,
                         "note": "fp32 VALU kernel (no MFMA on this path); peak = FP32 vector peak; "
                                 "achieved = SURVEY 8d F_alg per launch / average launch time (HIP events "
                                 "on the launch stream); F_alg counts this build's own node visits and object "
                                 "tests (4-wide culling walk, pixel beams), so it shrinks as the walk improves; "
                                 "ref_walk.equivalent_frac = the reference LBVH walk's flops of this frame over "
                                 "this kernel's time (not achieved work); "
                                 "lane_issue_frac = VALU busy x lane utilisation (PMC); traffic = PMC HBM "
                                 "bytes per launch"},
            "valu": valu,
            "hbm": {"measured_GBps": round(traffic / avg_s / 1e9, 2) if traffic else None,
                    "measured_frac": round(traffic / avg_s / 1e9 / HBM_PEAK_GBPS, 5) if traffic else None,
                    "peak_GBps": HBM_PEAK_GBPS, "bytes_per_launch": traffic,
                    "note": "PMC: 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md HBM section)"},
            "onchip": {"alg_GBps": round(balg / avg_s / 1e9, 1), "alg_bytes_per_launch": balg,
                       "note": "SURVEY 8d algorithmic bytes (node, object and framebuffer reads at their "
                               "nominal size) per launch / average launch time; served from LDS, L1 and L2, "
                               "so not an HBM rate"},
            "mean_bounces": round(st["segments"] / (W * H * spp * args.steps), 3),
            "rays_per_step": int(per_step["segments"]),
            "counters_per_step": {k: int(v) for k, v in per_step.items()},
            "cpu_baseline": cpu,
            "parity": parity,
            "path": path,
            "options": {k: v for k, v in R.get_options().as_dict().items()
                        if v != R.default_options().as_dict()[k]} or "defaults",
            "timed_region": ("per step: rt_pack_inw + rt_dev_scene_inw_update (records, device LBVH, the wide "
                             "walk's BVH + ranks + RI grid built on the "
                             + ("device" if R.get_options().inw_device_build else "host, uploads")
                             + ") + rt_render_tiles_async of one full frame (the reference's whole redraw, "
                             "RT_Base::OnUpdateBase); only the first frame's device allocations are outside it")
                            if args.rebuild else
                            ("rt_render_tiles_async of one full frame per step (+ the RCCL gather and rank 0's "
                             "frame assembly at N > 1) on a device scene built before timing: the host "
                             "acceleration structures, the scene upload and the device allocations of the first "
                             "frame are outside it (bench.py --rebuild times them per step)"),
        }
        if args.rebuild:
            out["rebuild_ms_per_step"] = dict(zip(("pack", "records", "lbvh_device", "walk_structures", "upload"),
                                                  [round(v / args.steps, 3) for v in rb_ms[:5]]))
            out["rebuild_ms_per_step"]["render_events"] = round(kernel_ms, 3)
            out["rebuild_ms_per_step"]["walk_structures_on"] = ("device" if R.get_options().inw_device_build
                                                                else "host")
            out["blocking_rt_render_inw_ms"] = round(blocking_ms, 1) if blocking_ms is not None else None
            out["config"]["workload"] += " + per-step scene rebuild (--rebuild)"
        if args.occupancy:
            d = [int(v) for v in dbg.cpu().tolist()]
            out["lane_occupancy"] = {name: round(d[2 * i + 1] / max(d[2 * i], 1) / 64, 4)
                                     for i, name in enumerate(("outer", "bvh_walk", "leaf_tests", "segments"))}
            out["wave_iterations"] = {name: d[2 * i] for i, name in enumerate(("outer", "bvh_walk", "leaf_tests", "segments"))}
            # wave cycles per phase (shader clock, summed over waves; kDbgCyc* slots)
            out["wave_cycles"] = dict(zip(("camera", "launch_ray", "bvh_walk", "leaf_tests", "segment", "coop_query",
                                           "coop_shade", "coop_pop"), d[8:16]))
            px_rays = buf["px_rays"]
            pr = px_rays[px_rays > 0].double()
            q = torch.quantile(pr.float().cpu(), torch.tensor([0.5, 0.9, 0.99, 0.999])).tolist()
            out["pixel_rays"] = {"mean": round(float(pr.mean()), 1), "p50": q[0], "p90": q[1], "p99": q[2],
                                 "p999": q[3], "max": int(pr.max())}
            rounds = (C.c_uint32 * 16)()
            nr = lib.rt_debug_rounds(scene, rounds, 16)
            out["parked_per_round"] = [int(rounds[i]) for i in range(max(nr, 0))]
            h = (C.c_uint64 * 66)()
            if lib.rt_debug_spec_hist(scene, h) == 0 and h[1]:
                out["sample_rays"] = {"max": h[0], "samples": h[1],
                                      "log2_hist": {b: [h[2 + b], h[34 + b]] for b in range(32) if h[2 + b]}}
            h = (C.c_uint64 * 66)()
            if lib.rt_debug_spec_list_hist(scene, h) == 0 and h[1]:  # the re-execution list after the pass
                out["relist_rays"] = {"max": h[0], "samples": h[1],
                                      "log2_hist": {b: [h[2 + b], h[34 + b]] for b in range(32) if h[2 + b]}}
            cyc = dict(zip(("camera", "closest_hit", "bvh_walk", "leaf_tests", "segment", "coop_query", "coop_shade",
                            "coop_pop"), d[8:16]))
            out["wave_cycles_share"] = {k: round(v / max(1, cyc["camera"] + cyc["segment"]), 4) for k, v in cyc.items()}
        print(json.dumps(out), flush=True)
        if args.save_image:
            np.save(args.save_image, image[:H, :W].cpu().numpy())
            if dimage is not None:  # the r32f depth image beside it (<path>.depth.npy)
                np.save(os.path.splitext(args.save_image)[0] + ".depth.npy", dimage[:H, :W].cpu().numpy())
    lib.rt_dev_scene_free(scene)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
