"""Parity cases shared by the CPU (oracle vs golden) and GPU (HIP vs oracle) tests.

Each case is a reference stage + scene + reduced render parameters, sized so the CPU oracle
finishes in about a second on a few cores.  The full BASELINE configs are covered on the GPU
through size-independent properties (tests/test_gpu_properties.py).
"""
from __future__ import annotations

import numpy as np

import rt_amd as R


def _scene(preset, seed=0, n_hint=0, **over):
    return R.make_scene(preset, seed, n_hint, **over)


def _no_lights(sc):
    """INW-04 with zero light sources: exercises the `contribution *= 0/1` quirk (04...glsl:660)."""
    arr = sc.desc
    for i in range(sc.n):
        arr[i].emissive = 0
    for k, v in R.pack(arr, sc.n, sc.stage).items():
        setattr(sc, k, v)
    return sc


def _touching_cuboids(n=25, **over):
    """INW-01 with unit cubes at unit spacing on the grid stage's layout: neighbouring cubes share
    faces, and every face lies on its LBVH leaf box, where rounding can put an object's hit an ulp
    before its box's entry t (the wide walk's leaf-entry guard, rt_kernels.hip inw_traverse_wide)."""
    sc = R.make_scene(R.PRESET_INW01_GRID, 0, n, **over)
    arr = sc.desc
    for i in range(sc.n):
        d = arr[i]
        d.type = R.RT_INW_CUBOID
        for k in range(3):
            d.scale[k] = 1.0
        d.position[2] = float(i % 2)  # a second row of faces along z
        d.last_position[0], d.last_position[1], d.last_position[2] = d.position[0], d.position[1], d.position[2]
        d.refractivity, d.reflectivity = (0.3, 0.6) if i % 3 else (0.0, 0.8)
        d.scat_reflect = 0.0
        d.scat_refract = 0.0
    for k, v in R.pack(arr, sc.n, sc.stage).items():
        setattr(sc, k, v)
    return sc


def _scene_cam(preset, seed, n_hint, cam_over, **over):
    """make_scene with camera-description overrides (aperture, focus_dist, position, ...)."""
    stage = R.PRESET_STAGE[preset]
    arr, n, cd, par = R.preset_desc(preset, seed, n_hint)
    for k, v in over.items():
        setattr(par, k, v)
    for k, v in cam_over.items():
        if k == "position":
            for i in range(3):
                cd.position[i] = v[i]
        else:
            setattr(cd, k, v)
    sc = R.Scene(stage=stage, desc=arr, n=n, camera=R.camera_from_desc(cd, stage), params=par)
    for k, v in R.pack(arr, n, stage).items():
        setattr(sc, k, v)
    return sc


def _dense_glass(n=160, **over):
    """INW-01 with n refractive spheres of radius 1.5 packed into a 6-unit cube: points lie inside
    many objects at once (more than the 8 the RI grid / wide RI walk sum before handing the query to
    the reference walk, and cells listing more objects than the grid keeps), and the pixel beam
    lists overflow their 32 entries."""
    sc = _scene_cam(R.PRESET_INW01_RANDOM, 99, n, {"position": (-7.0, 2.5, -7.0), "focus_dist": 8.0}, **over)
    arr = sc.desc
    rng = np.random.default_rng(7)
    for i in range(sc.n):
        d = arr[i]
        p = rng.uniform(-3.0, 3.0, 3)
        for k in range(3):
            d.position[k] = float(p[k])
            d.last_position[k] = float(p[k]) - 0.1
            d.scale[k] = 1.5
        d.refractivity, d.reflectivity, d.refractive_index = 0.65, 0.15, 1.3 + 0.05 * (i % 8)
    for k, v in R.pack(arr, sc.n, sc.stage).items():
        setattr(sc, k, v)
    return sc


CASES = {
    # name: callable -> Scene (IOW-01 handled separately)
    "iow03_ref3": lambda: _scene(R.PRESET_IOW03_REF3, spp=4),
    "iow03_ref3_normals": lambda: _scene(R.PRESET_IOW03_REF3, spp=9, show_normal=1),
    "iow03_ref3_spp1": lambda: _scene(R.PRESET_IOW03_REF3, spp=1),
    "iow03_ref3_tile": lambda: _scene(R.PRESET_IOW03_REF3, spp=4, tile_x0=100, tile_y0=100, tile_w=100, tile_h=100),
    "iow03_final": lambda: _scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=32, height=20, spp=2),
    "iow03_final_b8": lambda: _scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=96, height=64, spp=3, max_bounces=8),
    "inw01_grid": lambda: _scene(R.PRESET_INW01_GRID, 0, 9, spp=16),
    "inw01_random": lambda: _scene(R.PRESET_INW01_RANDOM, 1234, 10000, width=96, height=54, spp=8),
    "inw01_random_spp37": lambda: _scene(R.PRESET_INW01_RANDOM, 1234, 3000, width=64, height=36, spp=37),
    "inw04_refset": lambda: _scene(R.PRESET_INW04_REFSET, spp=16),
    "inw04_nolights": lambda: _no_lights(_scene(R.PRESET_INW04_REFSET, spp=8)),
    "inw04_cornell": lambda: _scene(R.PRESET_INW04_CORNELL, 7, 0, width=64, height=64, spp=8),
    # edge cases: ragged frames (no tile or wave multiple), a single pixel, one bounce, and
    # LBVHs whose root is a leaf (one object) or has two leaves
    "iow03_final_odd": lambda: _scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=67, height=5, spp=2),
    "iow03_final_1px": lambda: _scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=1, height=1, spp=3),
    "iow03_ref3_b1": lambda: _scene(R.PRESET_IOW03_REF3, spp=2, max_bounces=1),
    "inw01_random_one": lambda: _scene(R.PRESET_INW01_RANDOM, 5, 1, width=17, height=3, spp=4),
    "inw01_random_two": lambda: _scene(R.PRESET_INW01_RANDOM, 5, 2, width=33, height=7, spp=4),
    "inw01_touching_cuboids": lambda: _touching_cuboids(25, width=64, height=64, spp=4, max_bounces=12),
    "inw04_cornell_odd": lambda: _scene(R.PRESET_INW04_CORNELL, 7, 0, width=13, height=11, spp=3, max_bounces=3),
    # pixel beams (k_inw_beam): a wide lens makes the lists overflow (their cut decides), a focus
    # distance near the lens turns them off; a dense glass cluster for the RI grid's fallbacks
    "inw01_random_aperture": lambda: _scene_cam(R.PRESET_INW01_RANDOM, 1234, 3000, {"aperture": 4.0},
                                                width=64, height=36, spp=12),
    "inw01_random_focus1": lambda: _scene_cam(R.PRESET_INW01_RANDOM, 1234, 3000, {"focus_dist": 1.05},
                                              width=48, height=27, spp=8),
    "inw01_dense_glass": lambda: _dense_glass(160, width=48, height=48, spp=6, max_bounces=10),
}

GOLDEN_CASES = ["iow01_c1", "iow03_ref3", "iow03_ref3_normals", "iow03_final", "inw01_grid",
                "inw01_random", "inw04_refset", "inw04_cornell"]


def iow01_c1():
    """Config C1 exactly: IOW-01 400x225, 1 spp, primary rays only, stage defaults."""
    return R.iow01_defaults(400, 225)


def compare(a: np.ndarray, b: np.ndarray) -> dict:
    """Per-channel comparison that treats NaN == NaN (the reference can produce NaN)."""
    a = np.asarray(a, np.float32)
    b = np.asarray(b, np.float32)
    na, nb = np.isnan(a), np.isnan(b)
    both = ~(na | nb)
    d = np.abs(a[both].astype(np.float64) - b[both].astype(np.float64))
    bits_equal = (a.view(np.uint32) == b.view(np.uint32)) | (na & nb)
    return {
        "nan_mismatch": int((na != nb).sum()),
        "max_abs": float(d.max()) if d.size else 0.0,
        "n_over_1e-3": int((d > 1e-3).sum()),
        "exact_frac": float(bits_equal.mean()),
    }


TOL = 1e-3  # north_star: per-channel |delta| <= 1e-3
