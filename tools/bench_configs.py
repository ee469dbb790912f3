#!/usr/bin/env python3
"""Secondary measurements for BASELINE.json's other configs (DESIGN.md "Other configs").

bench.py measures configs[1] (the headline).  This script measures the remaining configs on one
GPU as Mrays/s (segments counted by the kernels / device time), each at full resolution.

Every render row runs on a persistent device scene (rt_dev_scene_* + rt_render_image_async),
as bench.py does: the first render allocates the scene's record and continuation buffers and is
reported apart (first_call_ms); the timed renders that follow allocate nothing, and their
device time is bracketed by HIP events on the launch stream.  Each row also records the main
kernel, its launches and the sample chunks the render was split into (rt_debug_launches,
rt_debug_chunks), so two runs of a row can be told apart.

  python tools/bench_configs.py [--quick | --full] [--reps N]

  (default)  C1 full; C3, C5 and the IOW-03 scene at C3 resolution at reduced spp; LBVH builds
  --quick    the same rows at smaller spp
  --full     C3 (500 spp), C5 (2000 spp) and the IOW-03 final scene at 1920x1080 / 500 spp, the
             north star's single-GPU target, at BASELINE's full sample counts
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rt_amd as R  # noqa: E402


def dev_scene(lib, sc, device=0):
    if sc.stage == 3:
        return lib.rt_dev_scene_iow03(R.fptr(sc.types), R.fptr(sc.records), sc.n, sc.params.spp, device)
    lights = sc.lights if sc.lights is not None and len(sc.lights) else None
    return lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, sc.layout, R.fptr(sc.nodes), R.fptr(lights), sc.n_lights,
                                sc.params.spp, device)


def run(name, preset, seed, n_hint, spp=None, reps=1, **over):
    """Warm-up render (allocates), then `reps` timed renders of the same frame on the persistent scene."""
    if spp is not None:
        over["spp"] = spp
    sc = R.make_scene(preset, seed, n_hint, **over)
    p = sc.params
    lib = R.load()
    dev = torch.device("cuda", 0)
    scene = dev_scene(lib, sc)
    if not scene:
        raise RuntimeError("rt_dev_scene_* failed")
    W, H = p.width, p.height
    rgba = torch.zeros((H, W, 4), dtype=torch.float32, device=dev)
    depth = torch.zeros((H, W), dtype=torch.float32, device=dev) if sc.stage != 3 else None
    ctr = torch.zeros(6, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()

    def render():
        rc = lib.rt_render_image_async(scene, C.byref(sc.camera), C.byref(p), rgba.data_ptr(),
                                       depth.data_ptr() if depth is not None else None, ctr.data_ptr(),
                                       stream.cuda_stream)
        if rc != 0:
            raise RuntimeError(f"rt_render_image_async -> {rc}")

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    render()
    torch.cuda.synchronize()
    first_ms = (time.perf_counter() - t0) * 1e3
    ctr.zero_()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        render()
        b.record(stream)
    torch.cuda.synchronize()
    times = [a.elapsed_time(b) for a, b in ev]
    c = [int(v) for v in ctr.cpu().tolist()]
    seg = c[0] // reps
    kname = C.create_string_buffer(64)
    launches = lib.rt_debug_launches(scene, kname, 64)
    chunks = lib.rt_debug_chunks(scene)
    lib.rt_dev_scene_free(scene)
    ms = float(np.median(times))
    return {"config": name, "width": W, "height": H, "spp": p.spp, "max_bounces": p.max_bounces, "objects": sc.n,
            "segments": seg, "shadow_queries": c[3] // reps, "device_ms": round(ms, 2),
            "device_ms_all": [round(t, 2) for t in times], "first_call_ms": round(first_ms, 2),
            "Mrays_per_s": round(seg / (ms * 1e-3) / 1e6, 1), "kernel": kname.value.decode(),
            "launches": launches, "chunks": chunks, "timing": "persistent scene, HIP events, allocation excluded"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--full", action="store_true", help="C3, C5 and IOW-03 at 1920x1080 at BASELINE's full spp")
    ap.add_argument("--reps", type=int, default=1, help="timed renders per row (after the warm-up)")
    ap.add_argument("--inw-only", action="store_true", help="with --full: C3 and C5 only")
    ap.add_argument("--row", choices=("c3", "c5", "ns", "c2"), help="one row only, at --spp (and --reps)")
    ap.add_argument("--spp", type=int, default=0)
    a = ap.parse_args()
    if a.row:
        preset = {"c3": (R.PRESET_INW01_RANDOM, 1234, 10_000), "c5": (R.PRESET_INW04_CORNELL, 7, 0),
                  "ns": (R.PRESET_IOW03_FINAL, 20250131, 0), "c2": (R.PRESET_IOW03_FINAL, 20250131, 0)}[a.row]
        kw = dict(width=1920, height=1080) if a.row == "ns" else {}
        if a.spp:
            kw["spp"] = a.spp
        elif a.row == "ns":
            kw["spp"] = 500
        row = run(a.row, *preset, reps=a.reps, **kw)
        row["env"] = {k: v for k, v in os.environ.items() if k.startswith("RT_")}
        print(json.dumps(row), flush=True)
        return
    if a.full:
        rows = [(("C3 INW-01 LBVH 10k moving spheres (full)", R.PRESET_INW01_RANDOM, 1234, 10_000), dict(spp=500)),
                (("C5 INW-04 Cornell (full)", R.PRESET_INW04_CORNELL, 7, 0), dict(spp=2000))]
        if not a.inw_only:
            rows.append((("IOW-03 final scene, 1920x1080, 500 spp (north-star target)", R.PRESET_IOW03_FINAL,
                          20250131, 0), dict(spp=500, width=1920, height=1080)))
        for args, kw in rows:
            print(json.dumps(run(*args, reps=a.reps, **kw)), flush=True)
        return
    q = a.quick
    out = []
    d = R.iow01_defaults()
    out.append({"config": "C1 IOW-01 400x225 1spp"})
    try:
        rgba, st = R.render_iow01(*d)
        t0 = time.perf_counter()
        rgba, st = R.render_iow01(*d)
        out[-1].update(device_ms=round(st["ms"], 3), wall_ms=round((time.perf_counter() - t0) * 1e3, 3))
    except Exception as e:  # noqa: BLE001
        out[-1]["error"] = str(e)
    for o in out:
        print(json.dumps(o), flush=True)
    out = [run("C3 INW-01 LBVH 10k moving spheres", R.PRESET_INW01_RANDOM, 1234, 10_000, spp=16 if q else 64,
               reps=a.reps),
           run("C5 INW-04 Cornell", R.PRESET_INW04_CORNELL, 7, 0, spp=4 if q else 16, reps=a.reps),
           run("IOW-03 final scene at C3 resolution (north-star target)", R.PRESET_IOW03_FINAL, 20250131, 0,
               spp=8 if q else 32, width=1920, height=1080, reps=a.reps)]
    for n in (10_000, 100_000):
        rng = np.random.default_rng(n)
        c = rng.uniform(-50, 50, (n, 3)).astype(np.float32)
        r = rng.uniform(0.1, 0.4, (n, 1)).astype(np.float32)
        boxes = np.concatenate([c - r, c + r], 1).astype(np.float32)
        R.lbvh_build_gpu(boxes)
        _, ms = R.lbvh_build_gpu(boxes)
        t0 = time.perf_counter()
        R.lbvh_build(boxes)
        host_ms = (time.perf_counter() - t0) * 1e3
        out.append({"config": f"LBVH build N={n}", "gpu_ms": round(ms, 3), "host_ms_1thread": round(host_ms, 3)})
    for o in out:
        print(json.dumps(o), flush=True)


if __name__ == "__main__":
    main()
