"""GPU parity: the HIP kernels (through the C ABI) against the CPU oracle on the same scene
bytes, and against the committed golden fixtures.

Bar (north_star): per-channel |delta| <= 1e-3 with identical NaN positions.  Under the
numerics contract the kernels are expected to be bit-identical to the oracle; the exact-match
fraction is printed and the integer counters (segments, node visits, primitive tests, shadow
queries, stack drops) must agree exactly -- that checks the traversal, not just the image.
"""
import os

import numpy as np
import pytest

import rt_amd as R
from cases import CASES, GOLDEN_CASES, TOL, compare, iow01_c1
from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
COUNTERS = ("segments", "node_visits", "prim_tests", "shadow_queries", "stack_drops", "nan_drops")

pytestmark = pytest.mark.gpu


def _check(name, g, o):
    c = compare(g, o)
    print(f"{name}: {c}")
    assert c["nan_mismatch"] == 0, c
    assert c["max_abs"] <= TOL, c
    return c


def test_iow01_c1_matches_oracle(gpu):
    cam, sph, p = iow01_c1()
    g, gst = R.render_iow01(cam, sph, p)
    o, ost = O.render_iow01(cam, sph, p)
    c = _check("iow01_c1", g, o)
    assert c["exact_frac"] == 1.0
    assert gst["segments"] == ost["segments"] == 400 * 225


@pytest.mark.parametrize("wide,order", [("1", "0"), ("0", "0"), ("1", "1"), ("1", "2")])
@pytest.mark.parametrize("name", sorted(CASES))
def test_render_matches_oracle(gpu, name, wide, order):
    """wide: rt_options.inw_wide_walk (the INW wide walk, 1, or the reference's LBVH walk, 0);
    order: rt_options.inw_order (0: the probe picks the INW fold kernel, 1: pixel-major, 2:
    sample-major)."""
    sc = CASES[name]()
    if sc.stage == R.RT_STAGE_IOW03 and (wide == "0" or order != "0"):
        pytest.skip("inw_wide_walk / inw_order only switch the INW kernels")
    with R.options(inw_wide_walk=int(wide), inw_order=int(order)):
        g, gd, gst = R.render(sc)
    o, od, ost = O.render(sc)
    c = _check(name, g, o)
    if gd is not None:
        _check(name + ":depth", gd, od)
    print(name, "gpu", {k: gst[k] for k in COUNTERS}, "ms %.2f" % gst["ms"])
    print(name, "cpu", {k: ost[k] for k in COUNTERS}, "ms %.2f" % ost["ms"])
    # IOW-03 walks a culling BVH instead of the reference's linear object loop, and INW's wide
    # walk (inw_wide_walk, default on) a 4-wide culling BVH instead of the reference's LBVH walk, so
    # their node / primitive counts are their own; every ray-level counter must still match
    # exactly.  With inw_wide_walk=0 the INW kernels walk the LBVH as the reference does, and the
    # node and primitive counts match too.
    own = sc.stage == R.RT_STAGE_IOW03 or wide == "1"
    exact = ("segments", "shadow_queries", "stack_drops", "nan_drops") if own else COUNTERS
    for k in exact:
        assert gst[k] == ost[k], (k, gst[k], ost[k])
    assert c["exact_frac"] == 1.0, c


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_render_matches_golden(gpu, name):
    gold = np.load(os.path.join(GOLDEN, name + ".npz"))
    if name == "iow01_c1":
        cam, sph, p = iow01_c1()
        g, _ = R.render_iow01(cam, sph, p)
    else:
        g, gd, _ = R.render(CASES[name]())
        if "depth" in gold:
            _check(name + ":depth", gd, gold["depth"])
    _check(name, g, gold["rgba"])


def test_tile_list_matches_full_image(gpu):
    """rt_render_tiles_async (the multi-GPU path's tile scheduler) == a full-frame render."""
    import ctypes as C

    import torch

    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 2000, width=80, height=48, spp=4)
    full, full_depth, _ = R.render(sc)
    lib = R.load()
    ts = 16
    tiles = [(tx, ty) for ty in range((48 + ts - 1) // ts) for tx in range((80 + ts - 1) // ts)]
    tiles = tiles[::-1]  # arbitrary order
    dev = torch.device("cuda")
    d_tiles = torch.tensor(tiles, dtype=torch.int32, device=dev).contiguous()
    out = torch.zeros((len(tiles), ts, ts, 4), dtype=torch.float32, device=dev)
    dep = torch.zeros((len(tiles), ts, ts), dtype=torch.float32, device=dev)
    ctr = torch.zeros(6, dtype=torch.int64, device=dev)
    s = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, 1, R.fptr(sc.nodes), None, 0, sc.params.spp, -1)
    assert s
    try:
        rc = lib.rt_render_tiles_async(s, C.byref(sc.camera), C.byref(sc.params), d_tiles.data_ptr(), len(tiles), ts,
                                       out.data_ptr(), dep.data_ptr(), ctr.data_ptr(),
                                       torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
    finally:
        lib.rt_dev_scene_free(s)
    img = np.zeros((48, 80, 4), np.float32)
    dimg = np.zeros((48, 80), np.float32)
    o = out.cpu().numpy()
    d = dep.cpu().numpy()
    for i, (tx, ty) in enumerate(tiles):
        h = min(ts, 48 - ty * ts)
        w = min(ts, 80 - tx * ts)
        img[ty * ts:ty * ts + h, tx * ts:tx * ts + w] = o[i, :h, :w]
        dimg[ty * ts:ty * ts + h, tx * ts:tx * ts + w] = d[i, :h, :w]
    assert compare(img, full)["exact_frac"] == 1.0
    assert compare(dimg, full_depth)["exact_frac"] == 1.0


def test_unsupported_texture_index_fails_loudly(gpu):
    sc = R.make_scene(R.PRESET_INW04_REFSET, spp=1)
    sc.geom[2, 27] = 1.0  # TextureIndex > 0 with no texture bound (rt_render_inw_tex binds them)
    with pytest.raises(RuntimeError):
        R.render(sc)


def test_repeated_frames_on_one_device_scene(gpu):
    """A device scene renders frame after frame with its fold rings kept (their tags carry a
    frame epoch; they are cleared only when it wraps every 63 frames): 70 frames, alternating two
    cameras (so a stale ring entry of the other view would change the image), the fold windows
    (global rings, k_inw_pm's LDS ring) and the fold order between them; every frame is
    bit-identical to the oracle's render of its camera, colour and depth, with the same ray counts."""
    import copy
    import ctypes as C

    import torch

    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 3000, width=64, height=40, spp=37)
    sc2 = copy.copy(sc)
    sc2.camera = R.RtCamera.from_buffer_copy(sc.camera)
    sc2.camera.pos[0] += 3.0
    sc2.camera.pos[1] -= 1.5
    lib = R.load()
    dev = torch.device("cuda")
    s = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, 1, R.fptr(sc.nodes), None, 0, sc.params.spp, -1)
    assert s
    frames = []
    try:
        for i in range(70):
            o = R.default_options()
            # pixel-major ring: global (64, 1024 entries) or in LDS (0); sample-major windows
            o.inw_ring_pm, o.inw_ring_sm = ((64, 128), (0, 256), (1024, 256), (0, 64))[i % 4]
            o.inw_order = (0, 1, 2)[i % 3]
            assert lib.rt_dev_scene_set_options(s, C.byref(o)) == 0
            cam = (sc.camera, sc2.camera)[i % 2]
            img = torch.zeros((40, 64, 4), dtype=torch.float32, device=dev)
            dep = torch.zeros((40, 64), dtype=torch.float32, device=dev)
            ctr = torch.zeros(6, dtype=torch.int64, device=dev)
            rc = lib.rt_render_image_async(s, C.byref(cam), C.byref(sc.params), img.data_ptr(), dep.data_ptr(),
                                           ctr.data_ptr(), torch.cuda.current_stream().cuda_stream)
            assert rc == 0
            torch.cuda.synchronize()
            frames.append((img.cpu().numpy(), dep.cpu().numpy(), int(ctr[0].item())))
    finally:
        lib.rt_dev_scene_free(s)
    refs = [O.render(x) for x in (sc, sc2)]
    assert int((refs[0][0] != refs[1][0]).any(axis=-1).sum()) > 200  # the two views differ (the sky is shared)
    for i, (a, d, n) in enumerate(frames):
        o, od, ost = refs[i % 2]
        assert compare(a, o)["exact_frac"] == 1.0, i
        assert compare(d, od)["exact_frac"] == 1.0, i
        assert n == ost["segments"], i


def test_scene_update_deep_tree_falls_back_to_host_build(gpu):
    """the device build of the walk structures stops at its level cap (a chain-like
    scene can split one object off per SAH level); the update then builds them on the host from
    the device LBVH instead of failing and leaving the scene unrenderable.  The cap is lowered
    (rt_debug_build_level_cap) so an ordinary scene is 'too deep': the update succeeds, reports the
    host fallback (info[7] = 2), and its frame equals a fresh scene's and the oracle's."""
    import ctypes as C

    import torch

    b = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 3000, width=64, height=36, spp=8)
    lib = R.load()
    dev = torch.device("cuda")

    def frame(s):
        img = torch.zeros((36, 64, 4), dtype=torch.float32, device=dev)
        dep = torch.zeros((36, 64), dtype=torch.float32, device=dev)
        ctr = torch.zeros(6, dtype=torch.int64, device=dev)
        assert lib.rt_render_image_async(s, C.byref(b.camera), C.byref(b.params), img.data_ptr(), dep.data_ptr(),
                                         ctr.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        return img.cpu().numpy(), dep.cpu().numpy(), int(ctr[0].item())

    s = lib.rt_dev_scene_inw(R.fptr(b.geom), b.n, 1, R.fptr(b.nodes), None, 0, b.params.spp, -1)
    f = lib.rt_dev_scene_inw(R.fptr(b.geom), b.n, 1, R.fptr(b.nodes), None, 0, b.params.spp, -1)
    assert s and f
    try:
        for cap, site in ((4, 2), (0, 1)):  # a cap below the tree's depth, then the default
            assert lib.rt_debug_build_level_cap(cap) == 0
            tm = (C.c_double * 4)()
            assert lib.rt_dev_scene_inw_update(s, R.fptr(b.geom), b.n, None, R.fptr(b.aabbs), None, 0, tm) == 0
            info = (C.c_uint32 * 8)()
            assert lib.rt_debug_wide_info(s, info, None) == 0
            assert info[7] == site and info[0] > 0, list(info)
            g, gd, gs = frame(s)
            h, hd, hs = frame(f)
            assert compare(g, h)["exact_frac"] == 1.0 and compare(gd, hd)["exact_frac"] == 1.0 and gs == hs
    finally:
        lib.rt_debug_build_level_cap(0)
        lib.rt_dev_scene_free(s)
        lib.rt_dev_scene_free(f)
    o, od, ost = O.render(b)
    assert compare(g, o)["exact_frac"] == 1.0 and gs == ost["segments"]


@pytest.mark.parametrize("device_lbvh,n_new", [(False, 3000), (True, 3000), (True, 3600), (False, 2200)])
def test_scene_update_matches_fresh_scene(gpu, device_lbvh, n_new):
    """rt_dev_scene_inw_update (the per-redraw work of RT_Base::OnUpdateBase, In-Next-Week/base.h:
    96-175) on an existing device scene: moved objects (n_new of them: the same count, more or
    fewer), the LBVH given or built on the device, then a frame -- bit-identical to a scene built
    from scratch for the moved objects, and to the oracle."""
    import ctypes as C

    import torch

    a = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 3000, width=64, height=36, spp=12)
    b = R.make_scene(R.PRESET_INW01_RANDOM, 1234, n_new, width=64, height=36, spp=12)
    for i in range(b.n):  # every object moves
        for k in range(3):
            b.desc[i].position[k] += 0.25 * ((i + k) % 3 - 1)
    for k, v in R.pack(b.desc, b.n, b.stage).items():
        setattr(b, k, v)
    lib = R.load()
    dev = torch.device("cuda")

    def frame(s):
        img = torch.zeros((36, 64, 4), dtype=torch.float32, device=dev)
        dep = torch.zeros((36, 64), dtype=torch.float32, device=dev)
        ctr = torch.zeros(6, dtype=torch.int64, device=dev)
        assert lib.rt_render_image_async(s, C.byref(b.camera), C.byref(b.params), img.data_ptr(), dep.data_ptr(),
                                         ctr.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        return img.cpu().numpy(), dep.cpu().numpy(), int(ctr[0].item())

    s = lib.rt_dev_scene_inw(R.fptr(a.geom), a.n, 1, R.fptr(a.nodes), None, 0, a.params.spp, -1)
    f = lib.rt_dev_scene_inw(R.fptr(b.geom), b.n, 1, R.fptr(b.nodes), None, 0, b.params.spp, -1)
    assert s and f
    try:
        frame(s)  # a frame of the old geometry first
        tm = (C.c_double * 4)()
        rc = lib.rt_dev_scene_inw_update(s, R.fptr(b.geom), b.n, None if device_lbvh else R.fptr(b.nodes),
                                         R.fptr(b.aabbs), None, 0, tm)
        assert rc == 0
        print("update ms", list(tm))
        g, gd, gs = frame(s)
        h, hd, hs = frame(f)
        # the walk structures: with the device LBVH they are built on the device (rt_build.hip,
        # binned SAH), else on the host as for the fresh scene; the depth-first ranks and the stack
        # high-water mark are functions of the LBVH alone, so they must equal the fresh scene's
        info_s, info_f = (C.c_uint32 * 8)(), (C.c_uint32 * 8)()
        rank_s, rank_f = (C.c_uint32 * (2 * b.n))(), (C.c_uint32 * (2 * b.n))()
        assert lib.rt_debug_wide_info(s, info_s, rank_s) == 0 and lib.rt_debug_wide_info(f, info_f, rank_f) == 0
        print("wide info update", list(info_s), "fresh", list(info_f))
        assert info_s[0] > 0 and info_s[3] == 1 and info_s[5] == 1 and info_s[6] == b.n
        assert info_s[1] == info_f[1]
        assert list(rank_s) == list(rank_f)
        if not device_lbvh:
            assert list(info_s) == list(info_f)
    finally:
        lib.rt_dev_scene_free(s)
        lib.rt_dev_scene_free(f)
    o, od, ost = O.render(b)
    for x, y in ((g, h), (gd, hd), (g, o), (gd, od)):
        assert compare(x, y)["exact_frac"] == 1.0
    assert gs == hs == ost["segments"]


def test_debug_path_reports_the_fold_ring(gpu):
    """rt_debug_path names the kernel and where its fold ring lived: k_inw_pm's ring in LDS by
    default (256 entries per wave, 5 staged nodes), a global ring with inw_ring_pm > 0 (236 staged
    nodes); the sample-major kernel keeps its global ring."""
    import ctypes as C

    import torch

    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 3000, width=64, height=40, spp=8)
    lib = R.load()
    dev = torch.device("cuda")
    s = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, 1, R.fptr(sc.nodes), None, 0, sc.params.spp, -1)
    assert s
    paths = {}
    try:
        for name, over in (("lds", {"inw_order": 1, "inw_qnodes": 0}), ("gq", {"inw_order": 1, "inw_qnodes": 1}),
                           ("global", {"inw_order": 1, "inw_ring_pm": 1024}), ("sm", {"inw_order": 2})):
            o = R.default_options()
            for k, v in over.items():
                setattr(o, k, v)
            assert lib.rt_dev_scene_set_options(s, C.byref(o)) == 0
            img = torch.zeros((40, 64, 4), dtype=torch.float32, device=dev)
            ctr = torch.zeros(6, dtype=torch.int64, device=dev)
            rc = lib.rt_render_image_async(s, C.byref(sc.camera), C.byref(sc.params), img.data_ptr(), None,
                                           ctr.data_ptr(), torch.cuda.current_stream().cuda_stream)
            assert rc == 0
            torch.cuda.synchronize()
            paths[name] = R.debug_path(s)
    finally:
        lib.rt_dev_scene_free(s)
    print(paths)
    p = paths["lds"]
    assert p["kernel"].startswith("k_inw_pm") and p["ring_lds"] == 1 and p["ring_entries"] == 256
    assert p["lds_nodes"] == 0  # the FStack LDS-ring instances read every node from L1 / L2
    assert p["time_bins"] == 2  # moving spheres: the walks pick one of 2 time-bin trees
    assert p["beam_bins"] == 2  # ... and the primary rays one of 2 beam lists per pixel
    assert p["sphere_records"] == 1  # equal-scale unrotated ellipsoids: the 2-float4 object records
    assert paths["gq"]["time_bins"] == 0 and paths["global"]["time_bins"] == 0 and paths["sm"]["time_bins"] == 0
    assert p["qnodes"] == 0 and p["global_stack"] == 0 and p["walk_stack"] == 37
    p = paths["gq"]  # GQ: quantised nodes, the top ones staged in LDS, the 40-float stacks in global memory
    assert p["kernel"].startswith("k_inw_pm") and p["ring_lds"] == 1 and p["ring_entries"] == 256
    assert p["qnodes"] == 1 and p["global_stack"] == 1 and p["walk_stack"] == 16 and p["lds_nodes"] > 5
    p = paths["global"]
    assert p["kernel"].startswith("k_inw_pm") and p["ring_lds"] == 0 and p["ring_entries"] == 1024
    assert p["lds_nodes"] > 5
    p = paths["sm"]
    assert p["kernel"].startswith("k_inw_sm") and p["ring_lds"] == 0 and p["lds_nodes"] > 5
    assert p["sphere_records"] == 1
    # INW-04's room (4 wide nodes): the sample-major ring goes to LDS as well (inw_ring_sm = 0),
    # beside every node the staging would take anyway; a power of two keeps the global ring
    sc = R.make_scene(R.PRESET_INW04_CORNELL, 7, 0, width=64, height=64, spp=8)
    s = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, sc.layout, R.fptr(sc.nodes),
                             R.fptr(sc.lights if sc.n_lights else None), sc.n_lights, sc.params.spp, -1)
    assert s
    try:
        for name, over in (("sm4", {"inw_order": 2}), ("sm4g", {"inw_order": 2, "inw_ring_sm": 256})):
            o = R.default_options()
            for k, v in over.items():
                setattr(o, k, v)
            assert lib.rt_dev_scene_set_options(s, C.byref(o)) == 0
            img = torch.zeros((64, 64, 4), dtype=torch.float32, device=dev)
            ctr = torch.zeros(6, dtype=torch.int64, device=dev)
            rc = lib.rt_render_image_async(s, C.byref(sc.camera), C.byref(sc.params), img.data_ptr(), None,
                                           ctr.data_ptr(), torch.cuda.current_stream().cuda_stream)
            assert rc == 0
            torch.cuda.synchronize()
            paths[name] = R.debug_path(s)
    finally:
        lib.rt_dev_scene_free(s)
    print(paths["sm4"], paths["sm4g"])
    p = paths["sm4"]
    assert p["kernel"].startswith("k_inw_sm") and p["ring_lds"] == 1 and p["ring_entries"] == 256
    assert p["lds_nodes"] == 4
    p = paths["sm4g"]
    assert p["kernel"].startswith("k_inw_sm") and p["ring_lds"] == 0 and p["lds_nodes"] == 4


def test_iow03_tile_after_full_frame_uses_its_own_records(gpu):
    """Sample-parallel IOW-03 records are tagged per frame: a fresh scene (rt_render_iow03 builds
    one per call) whose record buffers reuse a freed scene's memory must not take that scene's
    finished records for its own.  Render the full frame, then one tile alone, twice: the tile's
    pixels and ray counts equal the oracle's each time (before the process-wide tags, the tile
    returned the full frame's colours at its own record indices)."""
    sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=120, height=80, spp=9)
    R.render(sc)
    p = R.RtParams.from_buffer_copy(sc.params)
    p.tile_x0, p.tile_y0, p.tile_w, p.tile_h = 40, 16, 16, 16
    o, _, ost = O.render(sc, p)
    sl = (slice(16, 32), slice(40, 56))
    for _ in range(2):
        g, _, gst = R.render(sc, p)
        assert compare(g[sl], o[sl])["exact_frac"] == 1.0
        assert gst["segments"] == ost["segments"], (gst["segments"], ost["segments"])
