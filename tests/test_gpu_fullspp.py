"""Oracle parity of BASELINE.json's configs at their FULL sizes and sample counts.

The other parity tests run the oracle on reduced frames (tests/cases.py, <= 37 spp).  The
sunflower lens and ring tables depend on spp, and the reference's headline loop runs at its real
sample count (01_BVH...glsl:383, 625-653 with local_size_x = spp; 04...glsl:476-773;
03...glsl:362-430), so here every full frame is rendered on the GPU exactly as the bench renders
it, and a fixed set of its pixels is compared bit for bit -- colour and depth -- with oracle
renders of the same rectangles at the same spp:
- C3 (configs[2]: 10k moving spheres, 1920x1080, 500 spp, 50 bounces): the central 256x64 block
  (the bench's CPU-baseline block), seven 16x16 tiles drawn from those where some sample hits an
  object, and the costliest 16x16 tile;
- C5 (configs[4]: INW-04 Cornell box, 4096x4096, 2000 spp): the central 16x16 tile and the
  costliest one, shadow queries included;
- C2 (configs[1]: IOW-03 final scene, 1200x800, 100 spp): the central 64x16 block.
Per rectangle the ray-level counters (segments, shadow queries, stack drops, NaN directions) of
the oracle must equal those of a GPU render of that rectangle alone (the reference's per-tile
dispatch rectangle, materials.cpp:126-143), whose pixels must also equal the full frame's.
The costliest tile is found from the per-pixel ray counts (rt_debug_pixel_rays) of a render of
the same view at reduced spp (one atomic per ray segment would slow the full-spp frame down).
"""
import os
import subprocess

import numpy as np
import pytest

import rt_amd as R
from cases import TOL, compare
from oracle import oracle as O

pytestmark = pytest.mark.gpu
RAY_COUNTERS = ("segments", "shadow_queries", "stack_drops", "nan_drops")


def _threads() -> int:
    try:
        return max(1, int(subprocess.run(["nproc"], capture_output=True, text=True, check=True).stdout))
    except Exception:  # noqa: BLE001
        return os.cpu_count() or 1


def _rect_params(sc, x0, y0, w, h):
    p = R.RtParams.from_buffer_copy(sc.params)
    p.tile_x0, p.tile_y0, p.tile_w, p.tile_h = x0, y0, w, h
    return p


def _tile_rays(sc, spp: int, ts: int = 16):
    """Rays per ts x ts tile ([ty, tx]) in a render of the same view at `spp` samples (per-pixel
    ray counts of the INW fold kernels, rt_debug_pixel_rays)."""
    import torch

    lib = R.load()
    W, H = sc.params.width, sc.params.height
    p = R.RtParams.from_buffer_copy(sc.params)
    p.spp = spp
    px = torch.zeros(W * H, dtype=torch.int32, device="cuda")
    lib.rt_debug_pixel_rays(px.data_ptr())
    try:
        _, _, st = R.render(sc, p)
    finally:
        lib.rt_debug_pixel_rays(None)
    rays = px.cpu().numpy().view(np.uint32).reshape(H, W).astype(np.int64)
    assert int(rays.sum()) == st["segments"]
    return rays[: H - H % ts, : W - W % ts].reshape(H // ts, ts, W // ts, ts).sum(axis=(1, 3))


def _pick_tiles(t, k, seed, ts=16):
    """The costliest tile and k tiles drawn at random from those whose rays go beyond the primary
    ones (some sample hits an object), as (x0, y0, ts, ts)."""
    ty, tx = np.unravel_index(int(np.argmax(t)), t.shape)
    busy = np.argwhere(t > t.min())
    rng = np.random.default_rng(seed)
    pick = busy[rng.choice(len(busy), size=min(k, len(busy)), replace=False)]
    rects = [(int(x) * ts, int(y) * ts, ts, ts) for y, x in pick]
    heavy = (int(tx) * ts, int(ty) * ts, ts, ts)
    return rects + ([heavy] if heavy not in rects else [])


def _check_rects(name, sc, img, dep, rects):
    O.set_threads(_threads())
    for (x0, y0, w, h) in rects:
        p = _rect_params(sc, x0, y0, w, h)
        o, od, ost = O.render(sc, p)
        sl = (slice(y0, y0 + h), slice(x0, x0 + w))
        c = compare(img[sl], o[sl])
        print(f"{name} rect {(x0, y0, w, h)}: {c}  oracle {ost['segments']} rays, {ost['ms']:.0f} ms")
        assert c["nan_mismatch"] == 0 and c["max_abs"] <= TOL, c
        assert c["exact_frac"] == 1.0, c
        if dep is not None:
            cd = compare(dep[sl], od[sl])
            assert cd["exact_frac"] == 1.0, cd
        # the same rectangle rendered alone: the reference's per-tile dispatch
        g, gd, gst = R.render(sc, p)
        assert compare(g[sl], img[sl])["exact_frac"] == 1.0
        if dep is not None:
            assert compare(gd[sl], dep[sl])["exact_frac"] == 1.0
        for k in RAY_COUNTERS:
            assert gst[k] == ost[k], (k, gst[k], ost[k])


def test_c3_full_frame_matches_oracle_at_500spp(gpu):
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 10_000, width=1920, height=1080, spp=500, max_bounces=50)
    img, dep, st = R.render(sc)
    W, H = 1920, 1080
    rects = [(W // 2 - 128, H // 2 - 32, 256, 64)] + _pick_tiles(_tile_rays(sc, 32), 7, 4)
    print("C3 tiles (the last is the costliest at 32 spp):", rects)
    _check_rects("c3", sc, img, dep, rects)


def test_c5_full_frame_matches_oracle_at_2000spp(gpu):
    sc = R.make_scene(R.PRESET_INW04_CORNELL, 7, 0, width=4096, height=4096, spp=2000, max_bounces=50)
    img, dep, st = R.render(sc)
    assert st["shadow_queries"] > 0
    t = _tile_rays(sc, 16)
    ty, tx = np.unravel_index(int(np.argmax(t)), t.shape)
    rects = [(2048 - 8, 2048 - 8, 16, 16)] + ([(int(tx) * 16, int(ty) * 16, 16, 16)] if (tx, ty) != (127, 127) else [])
    print("C5 tiles (the last is the costliest at 16 spp):", rects)
    _check_rects("c5", sc, img, dep, rects)


def test_c2_full_frame_matches_oracle_at_100spp(gpu):
    sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=1200, height=800, spp=100, max_bounces=50)
    img, _, _ = R.render(sc)
    _check_rects("c2", sc, img, None, [(600 - 32, 400 - 8, 64, 16)])
