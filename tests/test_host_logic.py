"""Host half of the path (product C++ in librt_hip.so) against the oracle's independent
restatement: record packers, light SSBO, camera uniforms, LBVH node buffers, sample tables.
All byte-exact; none of this needs a GPU."""
import math

import numpy as np
import pytest

import rt_amd as R
from oracle import oracle as O

PRESETS = [(R.PRESET_IOW03_REF3, 0, 0), (R.PRESET_IOW03_FINAL, 20250131, 0), (R.PRESET_INW01_GRID, 0, 9),
           (R.PRESET_INW01_GRID, 0, 50), (R.PRESET_INW01_RANDOM, 1234, 10000), (R.PRESET_INW04_REFSET, 0, 0),
           (R.PRESET_INW04_CORNELL, 7, 0)]


@pytest.mark.parametrize("preset,seed,n", PRESETS)
def test_packers_match_oracle(preset, seed, n):
    arr, cnt, _, _ = R.preset_desc(preset, seed, n)
    stage = R.PRESET_STAGE[preset]
    a = R.pack(arr, cnt, stage, build_lbvh=False)
    b = O.pack(arr, cnt, stage)
    for k, v in b.items():
        if k == "n_lights":
            assert a[k] == v
        else:
            assert a[k].tobytes() == v.tobytes(), k


@pytest.mark.parametrize("preset,seed,n", [p for p in PRESETS if R.PRESET_STAGE[p[0]] != R.RT_STAGE_IOW03])
def test_lbvh_matches_oracle(preset, seed, n):
    arr, cnt, _, _ = R.preset_desc(preset, seed, n)
    aabbs = R.pack(arr, cnt, R.PRESET_STAGE[preset], build_lbvh=False)["aabbs"]
    assert R.lbvh_build(aabbs).tobytes() == O.lbvh_build(aabbs).tobytes()


def _check_lbvh_structure(nodes, aabbs):
    n = aabbs.shape[0]
    assert nodes.shape == (2 * n - 1, 8)
    seen = []
    stack = [0]
    while stack:
        i = stack.pop()
        left = nodes[i, 6]
        if left <= 0.1:
            obj = int(-left)
            seen.append(obj)
            assert np.array_equal(nodes[i, :6], aabbs[obj])
        else:
            l = int(left)
            for ch in (l, l + 1):  # children contiguous, rightData = parent
                assert int(nodes[ch, 7]) == i
                assert np.all(nodes[i, :3] <= nodes[ch, :3]) and np.all(nodes[i, 3:6] >= nodes[ch, 3:6])
                stack.append(ch)
    assert sorted(seen) == list(range(n))


@pytest.mark.parametrize("n", [1, 2, 3, 7, 64, 1000])
def test_lbvh_structure_random(n):
    rng = np.random.default_rng(n)
    c = rng.uniform(-10, 10, (n, 3)).astype(np.float32)
    r = rng.uniform(0.1, 1, (n, 1)).astype(np.float32)
    aabbs = np.concatenate([c - r, c + r], axis=1).astype(np.float32)
    nodes = R.lbvh_build(aabbs)
    assert nodes.tobytes() == O.lbvh_build(aabbs).tobytes()
    _check_lbvh_structure(nodes, aabbs)
    if n == 1:
        assert nodes[0, 6] == 0.0 and math.copysign(1.0, nodes[0, 6]) < 0  # -float(ObjectID 0)


def test_lbvh_duplicates_and_ties():
    # identical boxes: equal Morton codes AND equal diagonals -> contract tie-break by ObjectID
    aabbs = np.tile(np.array([[0, 0, 0, 1, 1, 1]], np.float32), (9, 1))
    aabbs[5] = [0, 0, 0, 2, 2, 2]
    nodes = R.lbvh_build(aabbs)
    assert nodes.tobytes() == O.lbvh_build(aabbs).tobytes()
    _check_lbvh_structure(nodes, aabbs)


@pytest.mark.parametrize("spp", [1, 2, 3, 36, 100, 500, 1024, 2000])
def test_sample_tables_match_oracle(spp):
    for a, b in zip(R.sample_tables(spp), O.sample_tables(spp)):
        assert a.tobytes() == b.tobytes()


def test_camera_uniforms():
    cd = R.RtCamDesc()
    cd.position[:] = (1, 2, 3)
    cd.pitch_deg, cd.yaw_deg, cd.fov_y_deg, cd.aperture, cd.focus_dist = -30.0, 45.0, 60.0, 0.5, 10.0
    iow = R.camera_from_desc(cd, R.RT_STAGE_IOW03)
    inw = R.camera_from_desc(cd, R.RT_STAGE_INW01)
    p, y = math.radians(-30), math.radians(45)
    ref = [math.cos(y) * math.cos(p), math.sin(p), math.sin(y) * math.cos(p)]
    assert np.allclose(list(inw.dir), ref, atol=1e-6)
    assert abs(np.linalg.norm(list(iow.dir)) - 1) < 1e-6
    assert abs(iow.fov_y_rad - math.radians(60)) < 1e-6
    with pytest.raises(RuntimeError):
        R.camera_from_desc(cd, 99)


def test_presets_deterministic_and_seeded():
    a = R.pack(*R.preset_desc(R.PRESET_INW01_RANDOM, 1, 500)[:2], R.RT_STAGE_INW01, build_lbvh=False)["geom"]
    b = R.pack(*R.preset_desc(R.PRESET_INW01_RANDOM, 1, 500)[:2], R.RT_STAGE_INW01, build_lbvh=False)["geom"]
    c = R.pack(*R.preset_desc(R.PRESET_INW01_RANDOM, 2, 500)[:2], R.RT_STAGE_INW01, build_lbvh=False)["geom"]
    assert a.tobytes() == b.tobytes() and a.tobytes() != c.tobytes()


def test_final_scene_shape():
    arr, n, cd, par = R.preset_desc(R.PRESET_IOW03_FINAL, 20250131)
    assert 450 <= n <= 500  # "~500 random spheres": 22x22 grid minus the clearance + 3 big + ground
    assert (par.width, par.height, par.spp, par.max_bounces) == (1200, 800, 100, 50)
    types = {arr[i].type for i in range(n)}
    assert types == {R.RT_IOW_CUBOID, R.RT_IOW_ELLIPSOID}


def test_inw04_light_ssbo():
    arr, n, _, _ = R.preset_desc(R.PRESET_INW04_REFSET)
    pk = R.pack(arr, n, R.RT_STAGE_INW04, build_lbvh=False)
    assert pk["n_lights"] == 2
    idx = pk["lights"][:, 6].view(np.uint32)
    assert list(idx) == [0, 1]
    assert np.array_equal(pk["lights"][:, :6], pk["aabbs"][[0, 1]])
    g = pk["geom"]
    assert np.all(g[[0, 1], 24:27] == 1.0) and np.all(g[[0, 1], 20:22] == 0.0)  # emissive packing


@pytest.mark.parametrize("preset,seed,n_hint", [(R.PRESET_INW01_RANDOM, 1234, 10_000), (R.PRESET_INW01_RANDOM, 5, 2),
                                                (R.PRESET_INW04_CORNELL, 7, 0), (R.PRESET_INW01_GRID, 0, 9)])
def test_inw_host_structures(preset, seed, n_hint):
    """The INW device scene's host-built structures (rt_inw_host_build, what rt_dev_scene_inw
    uploads): the wide walk applies to every well-formed LBVH of 2+ objects, its stack high-water
    mark fits the shader's 40-float stack, and the RI grid covers C3's objects."""
    sc = R.make_scene(preset, seed, n_hint, width=8, height=8, spp=1)
    info = R.inw_host_build(sc.nodes, sc.n)
    print(sc.n, info)
    assert info["wide_nodes"] >= 1 and 1 <= info["dfs_high"] <= 40 and info["wide_depth"] >= 1
    assert info["wide_nodes"] <= sc.n  # 4-wide: fewer nodes than objects
    if sc.n >= 1000:
        assert info["ri_grid"] == 1 and info["ri_cells"] >= sc.n and info["ri_ids"] >= sc.n
    # a malformed LBVH (a leaf id out of range) turns the wide walk off instead of failing
    bad = sc.nodes.copy()
    bad[np.argmax(bad[:, 6] <= 0.1), 6] = -float(sc.n + 5)
    assert R.inw_host_build(bad, sc.n)["wide_nodes"] == 0


def test_iow_host_structures():
    """The IOW-03 culling BVH (rt_iow_host_build): built for the final scene, absent (linear
    loop) for a single object."""
    sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=8, height=8, spp=1)
    info = R.iow_host_build(sc.types, sc.records, sc.n)
    assert 1 <= info["wide_nodes"] < sc.n
    assert R.iow_host_build(sc.types[:1], sc.records[:1], 1)["wide_nodes"] == 0


def test_tile_deal_matches_bench():
    """rt_tile_deal (the C ABI's multi-GPU deal, rt_multi.hip) is bench.py's deal_order: every
    tile once, row-major on one device, the multiplicative-hash permutation across devices; device
    r's share is entries r, r + n, ... (bench.tiles_for_rank)."""
    import bench
    for (W, H, T) in ((1920, 1080, 16), (1920, 1080, 64), (100, 60, 16), (4096, 4096, 32), (17, 9, 16)):
        nx, ny = -(-W // T), -(-H // T)
        for n in (1, 2, 3, 8):
            got = R.tile_deal(W, H, T, n)
            assert got == bench.deal_order(nx, ny, n), (W, H, T, n)
            assert sorted(got) == sorted((tx, ty) for ty in range(ny) for tx in range(nx))
            for r in range(n):
                assert got[r::n] == bench.tiles_for_rank(W, H, n, r, T)[1]
    assert R.load().rt_tile_deal(0, 10, 16, 1, None, 0) < 0
    assert R.load().rt_tile_deal(10, 10, 16, 0, None, 0) < 0
