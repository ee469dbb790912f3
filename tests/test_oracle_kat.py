"""Known-answer tests that pin the CPU oracle independently of its own output.

The reference has no golden vectors, so these are analytic: closed-form ray /
sphere distances of the IOW-01 default stage, the GLSL sky gradient, the structure of the
sample schedules, and single-object scenes whose pixel values follow from the shader algebra.
"""
import math

import numpy as np

import rt_amd as R
from oracle import oracle as O


def test_iow01_center_pixel_closed_form():
    # Sphere.h defaults: cam (0,1,10) looking -z (yaw -90), focus 1; sphere (0,3,-1) r=3.
    cam, sph, p = R.iow01_defaults(400, 225)
    img, _ = O.render_iow01(cam, sph, p)
    # pixel (200,112.5) is the optical axis; (200,112) is 0.5 px below it
    x, y = 200, 112
    sy = (y * 2.0 - 225) / (2.0 * 225)
    d = np.array([0.0, sy, -1.0])
    d /= np.linalg.norm(d)
    o = np.array([0.0, 1.0, 10.0])
    c = np.array([0.0, 3.0, -1.0])
    rs = o - c
    hb = d @ rs
    t = -hb - math.sqrt(hb * hb - (rs @ rs - 9.0))
    n = (o + t * d - c) / 3.0
    assert np.allclose(img[y, x, :3], n, atol=2e-5), (img[y, x], n)
    assert img[y, x, 3] == 1.0


def test_iow01_floor_and_sky():
    cam, sph, p = R.iow01_defaults(400, 225)
    img, _ = O.render_iow01(cam, sph, p)
    assert np.allclose(img[0, 0, :3], [0.8, 0.1, 0.7])      # bottom-left looks down onto y=-2
    # top-left corner misses everything: sky gradient (1-t)*(1,1,1) + t*(0.3,0.4,1)
    x, y = 0, 224
    sx = (x * 2.0 - 400) / 800.0 * (400 / 225)
    sy = (y * 2.0 - 225) / 450.0
    d = np.array([sx, sy, -1.0])
    d /= np.linalg.norm(d)
    t = (d[1] + 1) * 0.5
    sky = (1 - t) * np.ones(3) + t * np.array([0.3, 0.4, 1.0])
    assert np.allclose(img[y, x, :3], sky, atol=1e-6)


def test_ring_schedule_is_a_stratified_permutation():
    for grid in (1, 2, 3, 10):
        spp = grid * grid
        _, _, ring = O.sample_tables(spp)
        cells = {tuple(r) for r in ring}
        assert len(cells) == spp                          # every sample its own sub-pixel
        assert all(max(i, j) >= 1 for i, j in cells)      # rings start at focus 1
        assert tuple(ring[0]) == (1, 1)
        assert tuple(ring[-1]) == (grid, grid)


def test_sunflower_and_fibonacci_tables():
    for spp in (2, 36, 500):
        sf, fib, _ = O.sample_tables(spp)
        r = np.hypot(sf[:, 0], sf[:, 1])
        assert r[0] == 0.0
        b = round(2 * math.sqrt(spp))
        outer = (np.arange(spp) > spp - b) & (np.arange(spp) > 0)
        assert np.allclose(r[outer], 1.0, atol=1e-6)  # outer boundary ring
        assert np.all(r <= 1.0 + 1e-6)
        assert np.allclose(np.linalg.norm(fib, axis=1), 1.0, atol=1e-6)   # unit Fibonacci sphere
        assert np.isclose(fib[0, 1], 1.0) and np.isclose(fib[-1, 1], 0.0, atol=1e-6)


def _one_object(stage, typ, color, **mat):
    d = (R.RtGeomDesc * 1)()
    g = d[0]
    g.type = typ
    g.scale[:] = (1.0, 1.0, 1.0)
    g.color[:] = color
    g.refractive_index = 1.5
    for k, v in mat.items():
        setattr(g, k, v)
    return d


def test_iow03_absorbing_cuboid_pixel_equals_color():
    # refractivity = reflectivity = 0: spawned rays carry contribution 0, so a pixel whose
    # samples all hit the cuboid sums contribution^2 * Color = Color (03...glsl:253,304).
    d = _one_object(R.RT_STAGE_IOW03, R.RT_IOW_CUBOID, (0.25, 0.5, 0.75), refractivity=0.0, reflectivity=0.0)
    pk = R.pack(d, 1, R.RT_STAGE_IOW03)
    cd = R.RtCamDesc()
    cd.position[:] = (0.0, 0.0, 5.0)
    cd.pitch_deg, cd.yaw_deg, cd.fov_y_deg, cd.aperture, cd.focus_dist = 0.0, -90.0, 30.0, 0.0, 5.0
    cam = R.camera_from_desc(cd, R.RT_STAGE_IOW03)
    p = R.RtParams(32, 32, 4, 5, 0, 0, 0, 0, 0, -1)
    sc = R.Scene(stage=R.RT_STAGE_IOW03, desc=d, n=1, camera=cam, params=p, types=pk["types"], records=pk["records"])
    img, _, st = O.render(sc)
    assert np.allclose(img[16, 16, :3], [0.25, 0.5, 0.75], atol=1e-6)
    assert st["prim_tests"] == st["segments"]  # one object: one test per ray


def test_inw01_absorbing_sphere_pixel_is_sqrt_color():
    # INW stores sqrt(colour) per sample (01_BVH...glsl:670); with nothing reflected or
    # refracted the centre pixel is sqrt(Color).
    d = _one_object(R.RT_STAGE_INW01, R.RT_INW_ELLIPSOID, (0.36, 0.49, 0.64), refractivity=0.0, reflectivity=0.0)
    pk = R.pack(d, 1, R.RT_STAGE_INW01)
    cd = R.RtCamDesc()
    cd.position[:] = (0.0, 0.0, 5.0)
    cd.pitch_deg, cd.yaw_deg, cd.fov_y_deg, cd.aperture, cd.focus_dist = 0.0, -90.0, 30.0, 0.0, 5.0
    cam = R.camera_from_desc(cd, R.RT_STAGE_INW01)
    p = R.RtParams(32, 32, 3, 5, 0, 0, 0, 0, 0, -1)
    sc = R.Scene(stage=R.RT_STAGE_INW01, desc=d, n=1, camera=cam, params=p, geom=pk["geom"], aabbs=pk["aabbs"],
                 nodes=R.lbvh_build(pk["aabbs"]))
    img, depth, st = O.render(sc)
    assert np.allclose(img[16, 16, :3], np.sqrt([0.36, 0.49, 0.64]), atol=1e-6)
    assert depth[16, 16] == 0.0        # final_depth is only written on a miss
    assert depth[0, 0] == 32000.0      # corner ray misses: MAX_T_DEPTH
