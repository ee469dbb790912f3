#!/usr/bin/env python3
"""Secondary measurements for BASELINE.json's other configs (DESIGN.md "Other configs").

bench.py measures configs[1] (the headline).  This script measures the remaining configs on one
GPU as Mrays/s (segments counted by the kernels / device time), each at full resolution; spp is
reduced where the full count would take minutes (Mrays/s is a rate; the reduced spp is in the
output).  It also times the LBVH build on the GPU against the host builder.

  python tools/bench_configs.py [--quick]
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
import rt_amd as R  # noqa: E402


def run(name, preset, seed, n_hint, spp=None, **over):
    if spp is not None:
        over["spp"] = spp
    sc = R.make_scene(preset, seed, n_hint, **over)
    p = sc.params
    R.render(sc, p)  # warm-up (allocations, code objects)
    t0 = time.perf_counter()
    _, _, st = R.render(sc, p)
    wall = time.perf_counter() - t0
    return {"config": name, "width": p.width, "height": p.height, "spp": p.spp, "max_bounces": p.max_bounces,
            "objects": sc.n, "segments": st["segments"], "shadow_queries": st["shadow_queries"],
            "device_ms": round(st["ms"], 2), "wall_ms": round(wall * 1e3, 2),
            "Mrays_per_s": round(st["segments"] / (st["ms"] * 1e-3) / 1e6, 1)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quick", action="store_true")
    ap.add_argument("--full", action="store_true", help="C3 and C5 at BASELINE's full spp only")
    a = ap.parse_args()
    if a.full:
        for o in (run("C3 INW-01 LBVH 10k moving spheres (full)", R.PRESET_INW01_RANDOM, 1234, 10_000, spp=500),
                  run("C5 INW-04 Cornell (full)", R.PRESET_INW04_CORNELL, 7, 0, spp=2000)):
            print(json.dumps(o), flush=True)
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
    out.append(run("C3 INW-01 LBVH 10k moving spheres", R.PRESET_INW01_RANDOM, 1234, 10_000, spp=16 if q else 64))
    out.append(run("C5 INW-04 Cornell", R.PRESET_INW04_CORNELL, 7, 0, spp=4 if q else 16))
    out.append(run("IOW-03 final scene at C3 resolution (north-star target)", R.PRESET_IOW03_FINAL, 20250131, 0,
                   spp=8 if q else 32, width=1920, height=1080))
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
