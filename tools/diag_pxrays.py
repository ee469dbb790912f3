"""Diagnose rt_debug_pixel_rays attribution (VERDICT r04 "What's weak" 1).

Renders C3 at a reduced spp with the per-pixel ray map, with the claim order on and off, and
compares the maps with each other and, on a few tiles, with the oracle's per-pixel ray counts
(1x1 rectangles at the same spp).  Prints one JSON line.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd"), os.path.join(ROOT, "tests")]
import rt_amd as R  # noqa: E402
from oracle import oracle as O  # noqa: E402  (the checker)


def pixel_rays(sc, p):
    import torch
    lib = R.load()
    W, H = p.width, p.height
    px = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    lib.rt_debug_pixel_rays(px.data_ptr())
    try:
        _, _, st = R.render(sc, p)
    finally:
        lib.rt_debug_pixel_rays(None)
    m = px.cpu().numpy().view(np.uint32).reshape(H, W).astype(np.int64)
    return m, st


def main():
    spp = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 10_000, width=1920, height=1080, spp=500, max_bounces=50)
    p = R.RtParams.from_buffer_copy(sc.params)
    p.spp = spp
    out = {"spp": spp}
    m1, st1 = pixel_rays(sc, p)
    with R.options(inw_claim_order=0):
        m0, st0 = pixel_rays(sc, p)
    with R.options(inw_order=2):
        m2, st2 = pixel_rays(sc, p)
    out["sum_claim"] = int(m1.sum()); out["seg_claim"] = st1["segments"]
    out["sum_noclaim"] = int(m0.sum()); out["seg_noclaim"] = st0["segments"]
    out["sum_sm"] = int(m2.sum()); out["seg_sm"] = st2["segments"]
    out["maps_equal_claim_vs_noclaim"] = bool((m1 == m0).all())
    out["maps_equal_claim_vs_sm"] = bool((m1 == m2).all())
    out["pixels_differ_claim_vs_sm"] = int((m1 != m2).sum())
    out["pixels_hit_claim"] = int((m1 > spp).sum())
    out["pixels_hit_sm"] = int((m2 > spp).sum())
    ts = 16
    H, W = m1.shape
    t = m1[: H - H % ts, : W - W % ts].reshape(H // ts, ts, W // ts, ts).sum(axis=(1, 3))
    out["tile_min"] = int(t.min())
    out["busy_tiles"] = int((t > t.min()).sum())
    out["tiles"] = int(t.size)
    # oracle per-pixel counts on a few busy tiles
    rng = np.random.default_rng(4)
    busy = np.argwhere(t > t.min())
    pick = busy[rng.choice(len(busy), size=min(3, len(busy)), replace=False)]
    O.set_threads(os.cpu_count() or 1)
    checks = []
    for ty, tx in pick:
        x0, y0 = int(tx) * ts, int(ty) * ts
        om = np.zeros((ts, ts), np.int64)
        for yy in range(ts):
            for xx in range(ts):
                q = R.RtParams.from_buffer_copy(p)
                q.tile_x0, q.tile_y0, q.tile_w, q.tile_h = x0 + xx, y0 + yy, 1, 1
                _, _, ost = O.render(sc, q)
                om[yy, xx] = ost["segments"]
        g1 = m1[y0:y0 + ts, x0:x0 + ts]
        g2 = m2[y0:y0 + ts, x0:x0 + ts]
        checks.append({"tile": [x0, y0], "gpu_pm": int(g1.sum()), "gpu_sm": int(g2.sum()), "oracle": int(om.sum()),
                       "pm_eq_oracle": bool((g1 == om).all()), "sm_eq_oracle": bool((g2 == om).all())})
    out["checks"] = checks
    print(json.dumps(out))


if __name__ == "__main__":
    main()
