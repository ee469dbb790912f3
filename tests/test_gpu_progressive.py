"""Progressive rendering and the display pass on the GPU:
- rt_render_spiral_async, a few spiral tiles per update (Adding_Materials::OnUpdate with
  m_NumberOfTilesAtATime > 1, materials.cpp:98-152), assembles the same image, bit for bit, as
  one full-frame render, for IOW-03 and INW;
- rt_display_rgba8_async (the quad blit, BVH.cpp:6-43) equals GL's unorm8 store of the colour
  or depth image restated in numpy.
"""
import ctypes as C

import numpy as np
import pytest

import rt_amd as R

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


def _scene(sc):
    lib = R.load()
    if sc.stage == R.RT_STAGE_IOW03:
        return lib.rt_dev_scene_iow03(R.fptr(sc.types), R.fptr(sc.records), sc.n, sc.params.spp, -1)
    lights = sc.lights if sc.lights is not None and len(sc.lights) else None
    return lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, sc.layout, R.fptr(sc.nodes), R.fptr(lights), sc.n_lights,
                                sc.params.spp, -1)


@pytest.mark.parametrize("preset,seed,n_hint,w,h,spp,tile,per_update", [
    (R.PRESET_IOW03_FINAL, 20250131, 0, 300, 200, 6, 64, 3),
    (R.PRESET_IOW03_REF3, 0, 0, 300, 300, 4, 100, 1),
    (R.PRESET_INW01_RANDOM, 1234, 2000, 240, 135, 8, 32, 5),
])
def test_spiral_progressive_equals_full_frame(gpu, preset, seed, n_hint, w, h, spp, tile, per_update):
    sc = R.make_scene(preset, seed, n_hint, width=w, height=h, spp=spp)
    full, full_depth, _ = R.render(sc)
    lib = R.load()
    dev = torch.device("cuda")
    img = torch.zeros((h, w, 4), dtype=torch.float32, device=dev)
    dep = torch.zeros((h, w), dtype=torch.float32, device=dev)
    ctr = torch.zeros(6, dtype=torch.int64, device=dev)
    s = _scene(sc)
    assert s
    stream = torch.cuda.current_stream().cuda_stream
    n = len(R.tile_spiral(w, h, tile, tile))
    updates = 0
    try:
        cur = 0
        while cur < n:
            nxt = lib.rt_render_spiral_async(s, C.byref(sc.camera), C.byref(sc.params), tile, tile, cur, per_update,
                                             img.data_ptr(), dep.data_ptr(), ctr.data_ptr(), stream)
            assert nxt > cur, nxt
            cur = nxt
            updates += 1
        torch.cuda.synchronize()
    finally:
        lib.rt_dev_scene_free(s)
    assert updates == (n + per_update - 1) // per_update
    g = img.cpu().numpy()
    assert np.array_equal(g.view(np.uint32), full.view(np.uint32))
    if full_depth is not None:
        assert np.array_equal(dep.cpu().numpy().view(np.uint32), full_depth.view(np.uint32))


def _unorm8(x):
    x = np.asarray(x, np.float32)
    # NaN -> 0 before the cast (casting NaN to uint8 is undefined and warns)
    out = np.floor(np.nan_to_num(np.clip(x, 0, 1), nan=0.0) * np.float32(255) + np.float32(0.5)).astype(np.uint8)
    out[~(x > 0)] = 0
    out[x >= 1] = 255
    return out


@pytest.mark.parametrize("use_depth", [0, 1])
def test_display_pass_matches_unorm8_store(gpu, use_depth):
    rng = np.random.default_rng(5)
    h, w = 77, 131
    rgba = rng.uniform(-0.5, 1.5, (h, w, 4)).astype(np.float32)
    rgba[0, :8, 0] = [np.nan, np.inf, -np.inf, 0.0, -0.0, 1.0, 0.5 / 255, 254.5 / 255]
    depth = rng.uniform(-1, 2, (h, w)).astype(np.float32)
    dev = torch.device("cuda")
    d_rgba = torch.from_numpy(rgba).to(dev)
    d_depth = torch.from_numpy(depth).to(dev)
    out = torch.zeros((h, w, 4), dtype=torch.uint8, device=dev)
    rc = R.load().rt_display_rgba8_async(d_rgba.data_ptr(), d_depth.data_ptr(), w, h, use_depth, out.data_ptr(),
                                         torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    if use_depth:
        ref = np.stack([depth, depth, depth, np.ones_like(depth)], axis=2)
    else:
        ref = rgba
    assert np.array_equal(out.cpu().numpy(), _unorm8(ref))
