"""Oracle parity of BASELINE.json's configs at their FULL sizes and sample counts.

The other parity tests run the oracle on reduced frames (tests/cases.py, <= 37 spp).  The
sunflower lens and ring tables depend on spp, and the reference's headline loop runs at its real
sample count (01_BVH...glsl:383, 625-653 with local_size_x = spp; 04...glsl:476-773;
03...glsl:362-430), so here every full frame is rendered on the GPU exactly as the bench renders
it, and a fixed set of its pixels is compared bit for bit -- colour and depth -- with oracle
renders of the same rectangles at the same spp:
- C3 (configs[2]: 10k moving spheres, 1920x1080, 500 spp, 50 bounces): the central 256x64 block
  (the bench's CPU-baseline block), eight 16x16 tiles drawn from those whose samples hit objects
  (at least twice the rays of an all-sky tile in a reduced-spp render), and the costliest tile;
- C5 (configs[4]: INW-04 Cornell box, 4096x4096, 2000 spp): the central 16x16 tile, a tile on
  the upper part of the glass ellipsoid, one tile drawn at random and the costliest one, shadow queries
  included;
- C2 (configs[1]: IOW-03 final scene, 1200x800, 100 spp): the central 64x16 block, the 16x16
  tile on the big glass sphere's centre and one 16x16 tile drawn at random.
Every rectangle must cast more rays than one per pixel-sample in the oracle (some sample hits an
object), so no check is spent on sky.  The glass tiles sit on the projection of a point of the
object through the pinhole camera (the lens offsets move a ray by far less than the object's
radius in pixels).
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


def _pick_tiles(t, k, seed, ts=16, factor=2.0):
    """The costliest tile and k tiles drawn at random from those that cast at least `factor` times
    the rays of the cheapest (all-sky) tile, as (x0, y0, ts, ts)."""
    ty, tx = np.unravel_index(int(np.argmax(t)), t.shape)
    busy = np.argwhere(t >= factor * t.min())
    rng = np.random.default_rng(seed)
    pick = busy[rng.choice(len(busy), size=min(k, len(busy)), replace=False)]
    rects = [(int(x) * ts, int(y) * ts, ts, ts) for y, x in pick]
    heavy = (int(tx) * ts, int(ty) * ts, ts, ts)
    return rects + ([heavy] if heavy not in rects else [])


def _project(sc, X, ts=16):
    """The ts x ts tile centred on the pinhole projection of world point X: both camera models put
    pixel (x, y) on the direction D*sd + (D x up)*(x/W - 1/2)*aspect + ((D x up) x D)*(y/H - 1/2)
    (03...glsl:370-377, 01_BVH...glsl:366-386), with sd = 1 / (2 tan(fov/2))."""
    W, H = sc.params.width, sc.params.height
    D = np.array(sc.camera.dir, np.float64)
    P = np.array(sc.camera.pos, np.float64)
    cr = np.cross(D, [0.0, 1.0, 0.0])
    cu = np.cross(cr, D)
    sd = 1.0 / (2.0 * np.tan(sc.camera.fov_y_rad * 0.5))
    v = np.asarray(X, np.float64) - P
    a = v @ D / (D @ D)
    sx, sy = (v @ cr / (cr @ cr)) / a * sd, (v @ cu / (cu @ cu)) / a * sd
    x, y = W * (sx / (W / H) + 0.5), H * (sy + 0.5)
    x0 = int(min(max(round(x) - ts // 2, 0), W - ts))
    y0 = int(min(max(round(y) - ts // 2, 0), H - ts))
    return (x0, y0, ts, ts)


def _glass_point(sc, up=0.0):
    """A point of the largest refractive object of the scene (its rt_geom_desc): the centre raised by
    `up` times its y scale."""
    best = max((i for i in range(sc.n) if sc.desc[i].refractivity > 0.5), key=lambda i: sc.desc[i].scale[0])
    d = sc.desc[best]
    return [d.position[0], d.position[1] + up * d.scale[1], d.position[2]]


def _check_rects(name, sc, img, dep, rects):
    O.set_threads(_threads())
    spp = sc.params.spp
    for (x0, y0, w, h) in rects:
        p = _rect_params(sc, x0, y0, w, h)
        o, od, ost = O.render(sc, p)
        sl = (slice(y0, y0 + h), slice(x0, x0 + w))
        c = compare(img[sl], o[sl])
        print(f"{name} rect {(x0, y0, w, h)}: {c}  oracle {ost['segments']} rays "
              f"({ost['segments'] / (w * h * spp):.2f} per pixel-sample), {ost['ms']:.0f} ms")
        # not sky: some sample of the rectangle hits an object
        assert ost["segments"] > w * h * spp, (name, (x0, y0, w, h), ost["segments"])
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
    rects = [(W // 2 - 128, H // 2 - 32, 256, 64)] + _pick_tiles(_tile_rays(sc, 32), 8, 4)
    assert len(rects) >= 9
    print("C3 tiles (the last is the costliest at 32 spp):", rects)
    _check_rects("c3", sc, img, dep, rects)


def test_c5_full_frame_matches_oracle_at_2000spp(gpu):
    sc = R.make_scene(R.PRESET_INW04_CORNELL, 7, 0, width=4096, height=4096, spp=2000, max_bounces=50)
    img, dep, st = R.render(sc)
    assert st["shadow_queries"] > 0
    # the ellipsoid's upper part: its centre's shadow rays pass through the ellipsoid itself, so
    # is_lit = 0 ends those samples at once (04...glsl:604-660); near the top they reach the light
    # and refract through the glass (about 9 rays per pixel-sample)
    rects = [(2048 - 8, 2048 - 8, 16, 16), _project(sc, _glass_point(sc, 0.75))]
    rects += [r for r in _pick_tiles(_tile_rays(sc, 16), 1, 7, factor=1.5) if r not in rects]
    print("C5 tiles (central, glass ellipsoid, random, costliest at 16 spp):", rects)
    assert len(rects) >= 3
    _check_rects("c5", sc, img, dep, rects)


def test_c2_full_frame_matches_oracle_at_100spp(gpu):
    sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=1200, height=800, spp=100, max_bounces=50)
    img, _, _ = R.render(sc)
    rng = np.random.default_rng(5)
    rnd = (int(rng.integers(0, 1200 // 16)) * 16, int(rng.integers(0, 400 // 16)) * 16, 16, 16)  # lower half: ground
    rects = [(600 - 32, 400 - 8, 64, 16), _project(sc, _glass_point(sc)), rnd]
    print("C2 blocks (central, glass sphere, random):", rects)
    _check_rects("c2", sc, img, None, rects)
