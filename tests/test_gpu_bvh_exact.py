"""Full-frame exactness of the IOW-03 kernel's execution strategies against each other.

- RT_IOW_LINEAR=1: the reference's linear object loop instead of the culling BVH;
- RT_IOW_NARROW=1: the byte-bounce stack layout (12-deep BVH stack) instead of the 9-float one;
- RT_ROUNDS=0/6:   no tail compaction (no parking / resume launches) / six compaction rounds
  per pass (default 1 on the sample-parallel path);
- RT_SOLO=0/10^5:  the re-run pass's longest samples share waves / take a wave each up to the
  resident wave count (default 4096, clamped to the 3072 resident waves on MI355X; DESIGN.md
  "Solo head");
- RT_IOW_SPEC=0:   the sequential per-pixel kernel instead of sample-parallel speculation;
- RT_SPEC_ITERS=0/3/10: other numbers of resolve passes (default 1), more pixels finished by the sequential kernel (which
  takes the still-exact records; RT_SPEC_VALIDATE=0 re-runs every sample from the first bad one);
- RT_SPEC_PRIOR_FROM: from which sample on the scene's RI prior is guessed for entries sample 0
  left unwritten (default 2; 10^6 = never, with the former 10 re-run passes);
- RT_SPEC_TAIL_ROUNDS=0/3: no budgeted tail rounds (the round-1 default) / three, with
  RT_SPEC_TAIL_BUDGET segments per unit and round (default 60 rounds of 3072);
- RT_SPEC_SCAN=0/4: no anchored scan past the frontier (default 128 samples; DESIGN.md
  "Anchored scan") / a short one;
- RT_SPEC_CHAIN=0: exact restarts stop after their own sample (default: they go on down the
  pixel's chain of mispredicted samples);
- RT_SPEC_ALT=0 / RT_SPEC_ALT_SEG small: no alternative runs / alternatives for almost every
  sample that read a stale entry (default 16384 segments), so adoption runs often;
- RT_SPEC_ROUNDS=k: the speculative pass as k checkpoint rounds (default 24; 0 = one launch)
  with pixel frontiers and immediate exact re-runs of mispredicted samples;
- RT_IOW_LDS=0: the BVH read from global memory instead of staged in LDS (768-lane blocks);
- RT_COOP=0/64: no wave-cooperative closest hits / every closest hit wave-cooperative (default:
  waves with at most 4 tracing lanes);
- a scene with 12 distinct refractive indices (more than the 8 alternative-run values the
  speculation tracks, DESIGN.md "Alternative runs"), default against the sequential kernel;
- INW: RT_INW_ORDER=1/2 (the pixel- / sample-major on-chip fold instead of the probe's pick, with
  small fold windows RT_INW_RING_PM / RT_INW_RING_SM), RT_INW_ORDER=-1 (the per-pixel sequential
  kernel k_inw), RT_INW_LDS=0 (no LDS-staged BVH top) and RT_INW_FAST=0 (the reference's LBVH walk
  instead of the wide walk; images and ray counts equal).
Each must give a bit-identical image of the final scene with identical ray counts.  The
renders run in subprocesses because the switches are read by the library at scene build /
launch time."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = r"""
import sys, json, numpy as np
sys.path[:0] = [{root!r}, {root!r} + '/raytracing-tests_amd']
import rt_amd as R
sc = R.make_scene({preset}, {seed}, {n_hint}, width={w}, height={h}, spp={spp})
if {many_ri}:  # 12 distinct refractive indices over a third of the objects
    for i in range(sc.n):
        if i % 3 == 0 and sc.desc[i].type == R.RT_IOW_ELLIPSOID:
            sc.desc[i].refractivity = 0.9
            sc.desc[i].refractive_index = 1.1 + 0.07 * (i % 12)
    for k, v in R.pack(sc.desc, sc.n, sc.stage).items():
        setattr(sc, k, v)
img, depth, st = R.render(sc)
if depth is not None:
    img = np.concatenate([img, depth[..., None]], axis=2)
np.save({out!r}, img)
print(json.dumps(st))
"""


IOW = (2, 20250131, 0)     # PRESET_IOW03_FINAL
INW1 = (4, 1234, 3000)     # PRESET_INW01_RANDOM, 3000 objects
INW4 = (6, 7, 0)           # PRESET_INW04_CORNELL
IOW_RI = (2, 20250131, 0, True)  # the final scene with 12 distinct refractive indices


def _render(tmp_path, over, w, h, spp, scene=IOW):
    out = str(tmp_path / f"img_{len(os.listdir(tmp_path))}.npy")
    env = dict(os.environ)
    for k in ("RT_IOW_LINEAR", "RT_IOW_NARROW", "RT_ROUNDS", "RT_CHUNKS", "RT_IOW_SPEC", "RT_SPEC_ITERS",
              "RT_INW_ORDER", "RT_INW_RING_PM", "RT_INW_RING_SM", "RT_INW_LDS",
              "RT_SPEC_VALIDATE", "RT_SPEC_PRIOR_FROM", "RT_COOP", "RT_IOW_LDS",
              "RT_SPEC_ROUNDS", "RT_SOLO", "RT_SPEC_HEAVY",
              "RT_SPEC_TAIL_ROUNDS", "RT_SPEC_TAIL_BUDGET", "RT_SPEC_SCAN",
              "RT_SPEC_CHAIN", "RT_INW_FAST", "RT_SPEC_ALT", "RT_SPEC_ALT_SEG", "RT_SPEC_ALT_EVERY"):
        env.pop(k, None)
    env.update(over)
    code = SCRIPT.format(root=ROOT, w=w, h=h, spp=spp, out=out, preset=scene[0], seed=scene[1], n_hint=scene[2],
                         many_ri=len(scene) > 3 and scene[3])
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stderr[-2000:]
    return np.load(out), json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("over,w,h,spp", [
    ({"RT_IOW_LINEAR": "1"}, 600, 400, 2),
    ({"RT_IOW_LINEAR": "1"}, 1200, 800, 1),
    ({"RT_IOW_NARROW": "1"}, 600, 400, 8),
    ({"RT_ROUNDS": "0"}, 600, 400, 8),
    ({"RT_CHUNKS": "lpt", "RT_IOW_SPEC": "0"}, 300, 200, 24),
    ({"RT_IOW_SPEC": "0"}, 600, 400, 8),
    ({"RT_SPEC_ITERS": "0"}, 300, 200, 16),
    ({"RT_SPEC_ITERS": "1"}, 300, 200, 16),
    ({"RT_SPEC_ITERS": "0", "RT_SPEC_VALIDATE": "0"}, 300, 200, 16),
    ({"RT_SPEC_ITERS": "10", "RT_SPEC_PRIOR_FROM": "1000000"}, 300, 200, 16),
    ({"RT_SPEC_ITERS": "3", "RT_SPEC_PRIOR_FROM": "1"}, 600, 400, 12),
    ({"RT_COOP": "0"}, 600, 400, 8),
    ({"RT_IOW_LDS": "0"}, 600, 400, 8),
    ({"RT_SPEC_ROUNDS": "0"}, 600, 400, 12),
    ({"RT_SPEC_ROUNDS": "8"}, 600, 400, 12),
    ({"RT_SPEC_ROUNDS": "24", "RT_SPEC_PRIOR_FROM": "1"}, 300, 200, 16),
    ({"RT_SPEC_ROUNDS": "5"}, 300, 200, 9),
    ({"RT_IOW_LDS": "0", "RT_IOW_SPEC": "0"}, 300, 200, 8),
    ({"RT_COOP": "64"}, 300, 200, 4),
    ({"RT_COOP": "64", "RT_IOW_SPEC": "0"}, 300, 200, 4),
    ({"RT_COOP": "64", "RT_IOW_LINEAR": "1"}, 200, 100, 2),
    ({"RT_SPEC_ITERS": "2"}, 300, 200, 16),
    ({"RT_ROUNDS": "6"}, 600, 400, 12),
    ({"RT_SOLO": "0"}, 600, 400, 12),
    ({"RT_SOLO": "100000", "RT_SPEC_ITERS": "2"}, 300, 200, 16),
    ({"RT_SPEC_HEAVY": "0"}, 300, 200, 16),
    ({"RT_SPEC_TAIL_ROUNDS": "0"}, 600, 400, 12),
    ({"RT_SPEC_SCAN": "0"}, 600, 400, 12),
    ({"RT_SPEC_CHAIN": "0"}, 600, 400, 12),
    ({"RT_SPEC_ALT": "0"}, 600, 400, 12),
    ({"RT_SPEC_ALT_SEG": "8", "RT_SPEC_ALT_EVERY": "1", "RT_SPEC_TAIL_BUDGET": "64"}, 300, 200, 24),
    ({"RT_SPEC_ALT_SEG": "1", "RT_SPEC_ALT_EVERY": "2", "RT_SPEC_TAIL_BUDGET": "16", "RT_SPEC_ROUNDS": "4",
      "RT_SPEC_PRIOR_FROM": "1"}, 200, 100, 40),
    ({"RT_SPEC_CHAIN": "0", "RT_SPEC_SCAN": "0"}, 300, 200, 24),
    ({"RT_SPEC_SCAN": "4", "RT_SPEC_TAIL_BUDGET": "32"}, 300, 200, 24),
    ({"RT_SPEC_SCAN": "1000", "RT_SPEC_TAIL_BUDGET": "16", "RT_SPEC_ROUNDS": "6"}, 200, 100, 40),
    ({"RT_SPEC_TAIL_ROUNDS": "3", "RT_SPEC_TAIL_BUDGET": "64"}, 300, 200, 16),
    ({"RT_SPEC_TAIL_ROUNDS": "40", "RT_SPEC_TAIL_BUDGET": "16", "RT_SPEC_ROUNDS": "3"}, 300, 200, 16),
])
def test_strategies_bit_identical(tmp_path, gpu, over, w, h, spp):
    _same_frames(tmp_path, over, w, h, spp, IOW)


@pytest.mark.parametrize("over,w,h,spp", [
    ({"RT_IOW_SPEC": "0"}, 300, 200, 24),
    ({"RT_SPEC_ALT_SEG": "8", "RT_SPEC_ALT_EVERY": "1", "RT_SPEC_TAIL_BUDGET": "64"}, 300, 200, 24),
])
def test_many_refractive_indices_bit_identical(tmp_path, gpu, over, w, h, spp):
    """More distinct RIs than the alternative runs track: speculation must stay exact."""
    _same_frames(tmp_path, over, w, h, spp, IOW_RI)


def _same_frames(tmp_path, over, w, h, spp, scene):
    a, sa = _render(tmp_path, {}, w, h, spp, scene)
    b, sb = _render(tmp_path, over, w, h, spp, scene)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    bad = np.argwhere(~same.all(axis=2))
    print("mismatching pixels:", len(bad), bad[:10].tolist())
    print("default", sa, over, sb)
    assert len(bad) == 0
    for k in ("segments", "stack_drops", "nan_drops"):
        assert sa[k] == sb[k], k


@pytest.mark.parametrize("over,scene,w,h,spp", [
    ({"RT_INW_ORDER": "-1"}, INW1, 192, 108, 24),     # the per-pixel sequential kernel k_inw
    ({"RT_INW_ORDER": "1"}, INW1, 200, 100, 37),       # pixel-major fold, spp not a multiple of the wave
    ({"RT_INW_ORDER": "2"}, INW1, 200, 100, 37),       # sample-major fold
    ({"RT_INW_ORDER": "1"}, INW1, 160, 96, 1),         # more than 64 pixels per fold window
    ({"RT_INW_ORDER": "2"}, INW1, 160, 96, 1),
    ({"RT_INW_ORDER": "1"}, INW1, 97, 43, 3),          # ragged 8x8 units (padding samples)
    ({"RT_INW_ORDER": "2"}, INW1, 97, 43, 3),
    ({"RT_INW_ORDER": "1", "RT_INW_RING_PM": "64"}, INW1, 128, 72, 300),  # a window smaller than a pixel
    ({"RT_INW_ORDER": "2", "RT_INW_RING_SM": "64"}, INW1, 128, 72, 20),   # a window of one sample row
    ({"RT_INW_ORDER": "-1"}, INW4, 128, 128, 16),
    ({"RT_INW_ORDER": "1"}, INW4, 128, 128, 16),
    ({"RT_INW_ORDER": "-1", "RT_INW_FAST": "0"}, INW4, 96, 96, 8),
    ({"RT_INW_ORDER": "-1"}, INW4, 96, 96, 12),
    ({"RT_INW_FAST": "0"}, INW1, 480, 270, 16),          # the reference's LBVH walk
    ({"RT_INW_FAST": "0"}, INW4, 256, 256, 12),
    ({"RT_INW_FAST": "0", "RT_INW_ORDER": "-1"}, INW1, 192, 108, 24),
    ({"RT_INW_LDS": "0"}, INW1, 192, 108, 24),          # every wide node from global memory
    ({"RT_INW_LDS": "0", "RT_INW_ORDER": "2"}, INW4, 128, 128, 16),
])
def test_inw_strategies_bit_identical(tmp_path, gpu, over, scene, w, h, spp):
    a, sa = _render(tmp_path, {}, w, h, spp, scene)
    b, sb = _render(tmp_path, over, w, h, spp, scene)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), np.argwhere(~same.all(axis=2))[:10].tolist()
    # the wide walk's node and primitive counts depend on which rays share a wave (postponed
    # leaves are tested together), so only the ray-level counters must agree
    for k in ("segments", "shadow_queries", "stack_drops", "nan_drops"):
        assert sa[k] == sb[k], k
