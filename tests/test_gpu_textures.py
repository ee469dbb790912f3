"""GPU texture path against the CPU oracle, through the C ABI:
- textured INW-04 renders (rt_render_inw_tex, both the sample-parallel and the per-pixel
  kernel): cube-projected nearest-texel colour (04...glsl:416-464), bit-identical;
- noise textures (rt_noise_texture, MakeTexture utility.h:69-192), byte-identical, the three
  noise kinds, the stage's own 600x100 size and others the reference's batches tile;
- Mercator <-> cubic re-projection (rt_texture_remap, utility.cpp:266-463), byte-identical,
  both directions, RGB and RGBA, including the dice.png size (1003x176).
"""
import os

import numpy as np
import pytest

import rt_amd as R
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _same(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint8 if a.dtype == np.uint8 else np.uint32),
                                                 b.view(np.uint8 if b.dtype == np.uint8 else np.uint32))


NOISE = [
    (600, 100, 0, 0.01, 2.0, 0.5, 5),
    (600, 100, 1, 0.01, 2.5, 0.5, 5),
    (600, 100, 2, 0.01, 2.5, 0.5, 5),
    (1003, 176, 2, 0.05, 2.0, 0.6, 7),
    (7, 5, 1, 0.7, 2.0, 0.5, 3),
    (4096, 1024, 1, 0.004, 2.1, 0.5, 8),
]


@pytest.mark.parametrize("w,h,kind,freq,lac,gain,octaves", NOISE)
def test_noise_texture_matches_oracle(gpu, w, h, kind, freq, lac, gain, octaves):
    g, ms = R.noise_texture(w, h, kind, freq=freq, lac=lac, gain=gain, octaves=octaves)
    o = O.noise_texture(w, h, kind, freq=freq, lac=lac, gain=gain, octaves=octaves)
    print(f"noise {w}x{h} kind {kind}: {ms:.3f} ms")
    assert _same(g, o), np.argwhere(g != o)[:10].tolist()


def test_noise_texture_gradients_match_oracle(gpu):
    grads = [[], [(0.2, 0.4, 0.9)], [(1, 0, 0), (0, 1, 0), (0, 0, 1), (1, 1, 1)], [(-0.5, 2.0, 0.5), (1, 1, 1)]]
    for grad in grads:
        g, _ = R.noise_texture(600, 100, 1, gradient=grad, freq=0.02, lac=2.5)
        o = O.noise_texture(600, 100, 1, gradient=grad, freq=0.02, lac=2.5)
        assert _same(g, o), grad


def test_noise_texture_rejects_what_the_reference_cannot_do(gpu):
    with pytest.raises(RuntimeError):
        R.noise_texture(8, 8)
    with pytest.raises(RuntimeError):
        R.noise_texture(600, 100, 1, octaves=0)


@pytest.mark.parametrize("w,h,c", [(600, 100, 3), (1003, 176, 4), (2048, 1024, 3), (7, 3, 4)])
@pytest.mark.parametrize("load_as,map_to", [(0, 1), (1, 0), (1, 1)])
def test_remap_matches_oracle(gpu, w, h, c, load_as, map_to):
    rng = np.random.default_rng(w * 7 + c)
    img = rng.integers(0, 256, (h, w, c)).astype(np.uint8)
    g, ms = R.texture_remap(img, load_as, map_to)
    o = O.texture_remap(img, load_as, map_to)
    print(f"remap {w}x{h}x{c} {load_as}->{map_to}: {ms:.3f} ms")
    assert _same(g, o), np.argwhere((g != o).any(axis=2))[:10].tolist()


def _textured_scene(preset, seed, w, h, spp, tex_ids):
    sc = R.make_scene(preset, seed, 0, width=w, height=h, spp=spp)
    for i, t in enumerate(tex_ids):
        sc.geom[i % sc.n, 27] = float(t)
    rng = np.random.default_rng(seed)
    sc.textures = [O.noise_texture(600, 100, 2, freq=0.02, lac=2.5, octaves=5),
                   rng.integers(0, 256, (176, 1003, 4)).astype(np.uint8),
                   O.noise_texture(600, 100, 0, gradient=[(1, 0.2, 0.1), (0.1, 0.3, 1)], freq=0.05)]
    return sc


TEXTURED = [
    ("refset", R.PRESET_INW04_REFSET, 0, 96, 64, 4, [1, 2, 3, 0, 2]),
    ("cornell", R.PRESET_INW04_CORNELL, 7, 128, 128, 6, [1, 2, 3, 1, 2, 3, 9, 0, 1]),
]


@pytest.mark.parametrize("name,preset,seed,w,h,spp,ids", TEXTURED, ids=[t[0] for t in TEXTURED])
@pytest.mark.parametrize("order,wide", [("0", "1"), ("1", "1"), ("2", "1"), ("-1", "1"), ("0", "0")])
def test_textured_render_matches_oracle(gpu, name, preset, seed, w, h, spp, ids, order, wide):
    """order: rt_options.inw_order (0 the probe's pick, 1 / 2 the pixel- / sample-major fold, -1 the
    per-pixel kernel k_inw); wide: rt_options.inw_wide_walk."""
    sc = _textured_scene(preset, seed, w, h, spp, ids)
    with R.options(inw_order=int(order), inw_wide_walk=int(wide)):
        g, gd, gst = R.render(sc)
    o, od, ost = O.render(sc)
    assert _same(g, o), np.argwhere(~(g.view(np.uint32) == o.view(np.uint32)).all(axis=2))[:10].tolist()
    assert _same(gd, od)
    ks = ("segments", "shadow_queries", "stack_drops", "nan_drops")  # the wide walk counts its own nodes
    for k in ks + (("node_visits", "prim_tests") if wide == "0" else ()):
        assert gst[k] == ost[k], k
    sc.textures = None
    sc.geom[:, 27] = 0.0
    u, _, _ = R.render(sc)
    assert not np.array_equal(u, g)  # the textures did change the image


def test_textured_records_without_textures_fail_loudly(gpu):
    sc = _textured_scene(R.PRESET_INW04_REFSET, 0, 32, 32, 1, [1])
    sc.textures = None
    with pytest.raises(RuntimeError):
        R.render(sc)
