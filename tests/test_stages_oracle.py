"""CPU checks of the oracle's IOW-00 / IOW-02 / MULTIFOCUS restatements:
known answers derived by hand from the shaders, the committed golden fixtures, and the IOW-02
packer of librt_hip.so (host code, no GPU) against the oracle's IOW-03 packer."""
import os

import numpy as np
import pytest

import rt_amd as R
import stages as S
from cases import compare
from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def test_iow00_gradient_formula():
    """base.cpp:13-15: r = x / (W - 1.0), g = y / (H - 1.0), b = 0.25 (a/b = a * RN(1/b))."""
    for w, h in ((100, 100), (7, 5), (1920, 3)):
        img = O.render_iow00(S.iow00_params(w, h))
        x = np.arange(w, dtype=np.float32)[None, :] * (np.float32(1) / np.float32(w - 1))
        y = np.arange(h, dtype=np.float32)[:, None] * (np.float32(1) / np.float32(h - 1))
        assert np.array_equal(img[..., 0], np.broadcast_to(x, (h, w)))
        assert np.array_equal(img[..., 1], np.broadcast_to(y, (h, w)))
        assert (img[..., 2] == np.float32(0.25)).all() and (img[..., 3] == 1).all()


def _bg(dy):
    t = (np.float32(dy) + np.float32(1)) * np.float32(0.5)
    return np.array([(1 - t) + t * np.float32(0.3), (1 - t) + t * np.float32(0.4), 1.0], np.float32)


def test_iow02_default_scene_known_answers():
    """One red unit cube at the origin seen from (0,1,10) along -z (groups.h defaults).  Pixel
    (50, 40): sy = -0.1, the ray meets the front face (z = 0.5) at y ~ 0.05 -> red.  Column 50
    above the cube shows the sky gradient of the ray's own y direction."""
    c = S.iow02_default()
    img, st = O.render_iow02(c["types"], c["records"], c["camera"], c["params"], 0, 1)
    assert np.array_equal(img[40, 50], np.array([1, 0, 0, 1], np.float32))
    assert st["segments"] == 100 * 100 and st["prim_tests"] == 100 * 100
    # a sky pixel: colour is the background of the normalised ray (02.glsl:172-175)
    D = np.array(c["camera"].dir, np.float32)
    assert abs(D[2] + 1) < 1e-6
    # pixel (50, 90): sx = 0, sy = 0.4, plus the ring schedule's first sub-pixel (1, 1) of a
    # 1x1 grid: + (aspect / W, 1 / H) = (0.01, 0.01)  (02.glsl:146-166)
    assert np.allclose(img[90, 50, :3], _bg(0.41 / np.sqrt(0.01 ** 2 + 0.41 ** 2 + 1)), atol=1e-6)
    # culling both sides hides every object (02.glsl:55-61, 81-89)
    img2, _ = O.render_iow02(c["types"], c["records"], c["camera"], c["params"], 1, 1)
    assert np.array_equal(img2[..., 0], img2[..., 0]) and not np.any(
        (img2[..., 0] == 1) & (img2[..., 1] == 0) & (img2[..., 2] == 0))
    # show-normal: the front face's local normal (0, 0, 1)
    c["params"].show_normal = 1
    img3, _ = O.render_iow02(c["types"], c["records"], c["camera"], c["params"], 0, 1)
    assert np.array_equal(img3[40, 50, :3], np.array([0, 0, 1], np.float32))


def test_iow02_bounce_weights():
    """A pixel whose first hit is the cube and whose mirror bounce escapes: red + 0.4 * sky."""
    c = S.iow02_default()
    c["params"].max_bounces = 2
    img, _ = O.render_iow02(c["types"], c["records"], c["camera"], c["params"], 0, 1)
    px = img[40, 50, :3]
    assert px[0] > 1.0 and 0.0 < px[1] < 0.4 and 0.0 < px[2] <= 0.4 + 1e-6


def test_pack_iow02_is_iow03_prefix():
    """Groups::Geometry::FillBuffer packs what the IOW-03 FillBuffer packs first (groups.h:45-64,
    materials.h:48-76): position, inverse rotation, scale, colour."""
    arr, n, _, _ = R.preset_desc(R.PRESET_IOW03_FINAL, 20250131, 0)
    t2, r2 = R.pack_iow02(arr, n)
    o = O.pack(arr, n, 3)
    assert np.array_equal(t2, o["types"]) and np.array_equal(r2, o["records"][:, :18])


@pytest.mark.parametrize("name", S.GOLDEN_STAGE_CASES)
def test_stage_oracle_matches_golden(name):
    gold = np.load(os.path.join(GOLDEN, name + ".npz"))
    img, depth, st = S.render_oracle(name)
    assert compare(img, gold["rgba"])["exact_frac"] == 1.0
    if depth is not None and "depth" in gold:
        assert compare(depth, gold["depth"])["exact_frac"] == 1.0
    for k in gold.files:
        if k.startswith("stat_"):
            assert st[k[5:]] == int(gold[k]), k


def test_multifocus_differs_from_single_focus_and_keeps_finite_hits():
    """MULTIFOCUS rebuilds the primary ray (BVH.glsl:388-400), so even one focus distance renders
    differently from the single-focus camera; pixels whose sample 0 hits before the first lens
    limit (focus / 2) stay finite (the lens record is dropped after the hit, :544-549)."""
    sc, focus = S.MF_CASES["inw01_mf1"]()
    a, da, sa = O.render_inw_mf(sc, focus)
    b, db, sb = O.render(sc)
    finite = np.isfinite(a[..., 0])
    assert 0 < finite.sum() < finite.size
    assert not np.array_equal(a[finite], b[finite])
    assert np.isfinite(b).all()
    assert sa["segments"] > 0 and sa["node_visits"] > 0
