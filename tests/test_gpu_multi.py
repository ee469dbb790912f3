"""The multi-GPU partition behind the C ABI (BASELINE configs[3]): rt_group_create
(one RCCL communicator per device, ncclCommInitAll), rt_render_multi_async (every device renders
its tile share, grouped ncclSend / ncclRecv to device 0, unpack there) and the blocking
rt_render_inw_multi a C++ host calls in place of RT_Base<>::OnUpdateBase's dispatch
(In-Next-Week/base.h:148-173).  The box has one GPU, so the group holds one device: its tiles
still travel through RCCL (device 0 sends to itself), and the frame must be bit-identical to the
single-device render, with the same ray counts.  The deal itself is checked on the CPU
(tests/test_host_logic.py::test_tile_deal_matches_bench)."""
import ctypes as C

import numpy as np
import pytest

import rt_amd as R
from cases import compare

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("preset,n,w,h,spp,tile", [
    (R.PRESET_INW01_RANDOM, 2000, 100, 60, 12, 16),   # ragged: 100 x 60 is not a multiple of 16
    (R.PRESET_INW01_RANDOM, 3000, 96, 64, 7, 64),     # one ragged 64 x 64 tile row
    (R.PRESET_INW04_CORNELL, 0, 64, 48, 9, 32),       # INW-04: lights, shadow queries
])
def test_blocking_multi_matches_single_device(gpu, preset, n, w, h, spp, tile):
    sc = R.make_scene(preset, 7 if preset == R.PRESET_INW04_CORNELL else 1234, n, width=w, height=h, spp=spp)
    g, gd, gst = R.render(sc)
    m, md, mst = R.render_inw_multi(sc, [0], tile=tile)
    assert compare(m, g)["exact_frac"] == 1.0
    assert compare(md, gd)["exact_frac"] == 1.0
    # the wide walk's node and object counts depend on which rays share a wave (postponed leaves
    # are tested together; tiles regroup the pixels), so the ray-level counters must agree
    for k in ("segments", "shadow_queries", "stack_drops", "nan_drops"):
        assert mst[k] == gst[k], (k, mst[k], gst[k])


def test_group_async_frames_match_image_render(gpu):
    """A persistent group renders frame after frame (two cameras alternating) into device-0
    buffers: each frame equals rt_render_image_async of the same camera, counters included."""
    import copy

    import torch

    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 2500, width=80, height=48, spp=10)
    sc2 = copy.copy(sc)
    sc2.camera = R.RtCamera.from_buffer_copy(sc.camera)
    sc2.camera.pos[2] += 4.0
    lib = R.load()
    dev = torch.device("cuda")
    s = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, 1, R.fptr(sc.nodes), None, 0, sc.params.spp, 0)
    assert s
    devs = (C.c_int * 1)(0)
    grp = lib.rt_group_create(devs, 1)
    assert grp
    scenes = (C.c_void_p * 1)(s)
    stream = torch.cuda.current_stream().cuda_stream
    try:
        for i in range(4):
            cam = (sc.camera, sc2.camera)[i % 2]
            out = []
            for multi in (True, False):
                img = torch.zeros((48, 80, 4), dtype=torch.float32, device=dev)
                dep = torch.zeros((48, 80), dtype=torch.float32, device=dev)
                ctr = torch.zeros(6, dtype=torch.int64, device=dev)
                if multi:
                    rc = lib.rt_render_multi_async(grp, scenes, C.byref(cam), C.byref(sc.params), 16, img.data_ptr(),
                                                   dep.data_ptr(), ctr.data_ptr(), stream)
                else:
                    rc = lib.rt_render_image_async(s, C.byref(cam), C.byref(sc.params), img.data_ptr(),
                                                   dep.data_ptr(), ctr.data_ptr(), stream)
                assert rc == 0
                torch.cuda.synchronize()
                out.append((img.cpu().numpy(), dep.cpu().numpy(), ctr.cpu().numpy()))
            (a, ad, ac), (b, bd, bc) = out
            assert compare(a, b)["exact_frac"] == 1.0, i
            assert compare(ad, bd)["exact_frac"] == 1.0, i
            assert ac[0] == bc[0] and np.array_equal(ac[3:], bc[3:]), (i, ac, bc)  # ray-level counters
    finally:
        lib.rt_group_free(grp)
        lib.rt_dev_scene_free(s)


def test_group_rejects_bad_device_lists(gpu):
    lib = R.load()
    assert not lib.rt_group_create((C.c_int * 2)(0, 0), 2)   # one rank per device
    assert not lib.rt_group_create((C.c_int * 1)(4096), 1)   # no such device
    assert not lib.rt_group_create(None, 1)


def test_bench_group_mode_matches_single_device(gpu, tmp_path):
    """bench.py --group (the C-ABI device group timed from one process, rt_render_multi_async) on a
    reduced C3 frame: its assembled colour and depth images equal a single-device render of the
    same scene bit for bit, and the line reports the frame's ray count."""
    import json
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    img = str(tmp_path / "g.npy")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--group", "--gpus", "1", "--config", "c3",
                        "--width", "96", "--height", "54", "--spp", "6", "--steps", "1", "--warmup", "1",
                        "--save-image", img], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 1 and line["config"]["parallelism"] == "group1+rccl_send_recv"
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 10_000, width=96, height=54, spp=6)
    g, gd, gst = R.render(sc)
    assert compare(np.load(img), g)["exact_frac"] == 1.0
    assert compare(np.load(str(tmp_path / "g.depth.npy")), gd)["exact_frac"] == 1.0
    assert line["rays_per_step"] == gst["segments"]


def test_group_refuses_a_scene_of_another_device(gpu):
    """rt_render_multi_async checks that scenes[r] was built on the group's device r (a scene's
    buffers belong to its device).  With one GPU the mismatch is a scene list whose entry is not
    on device 0 -- here a null entry and, when a second device exists, a scene built there."""
    import torch

    lib = R.load()
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 500, width=32, height=16, spp=2)
    grp = lib.rt_group_create((C.c_int * 1)(0), 1)
    assert grp
    dev = torch.device("cuda", 0)
    img = torch.zeros((16, 32, 4), dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream
    other = None
    try:
        assert lib.rt_render_multi_async(grp, (C.c_void_p * 1)(None), C.byref(sc.camera), C.byref(sc.params), 16,
                                         img.data_ptr(), None, None, stream) == R.RT_E_ARG
        if torch.cuda.device_count() > 1:
            other = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, 1, R.fptr(sc.nodes), None, 0, sc.params.spp, 1)
            assert other
            assert lib.rt_render_multi_async(grp, (C.c_void_p * 1)(other), C.byref(sc.camera), C.byref(sc.params),
                                             16, img.data_ptr(), None, None, stream) == R.RT_E_ARG
        mine = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, 1, R.fptr(sc.nodes), None, 0, sc.params.spp, 0)
        assert mine
        try:
            assert lib.rt_render_multi_async(grp, (C.c_void_p * 1)(mine), C.byref(sc.camera), C.byref(sc.params), 16,
                                             img.data_ptr(), None, None, stream) == 0
            torch.cuda.synchronize()
        finally:
            lib.rt_dev_scene_free(mine)
    finally:
        if other:
            lib.rt_dev_scene_free(other)
        lib.rt_group_free(grp)


def test_group_frame_size_changes_between_async_frames(gpu):
    """a new frame or tile size re-deals the tiles; the re-upload waits for the group's
    earlier frame, so two async frames of different sizes with no host sync between them are both
    bit-identical to single-device renders."""
    import torch

    lib = R.load()
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 2000, width=80, height=48, spp=5)
    s = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, 1, R.fptr(sc.nodes), None, 0, sc.params.spp, 0)
    grp = lib.rt_group_create((C.c_int * 1)(0), 1)
    assert s and grp
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream().cuda_stream
    try:
        outs = []
        for (w, h, tile) in ((80, 48, 16), (64, 40, 32), (80, 48, 16)):
            p = R.RtParams.from_buffer_copy(sc.params)
            p.width, p.height = w, h
            img = torch.zeros((h, w, 4), dtype=torch.float32, device=dev)
            assert lib.rt_render_multi_async(grp, (C.c_void_p * 1)(s), C.byref(sc.camera), C.byref(p), tile,
                                             img.data_ptr(), None, None, stream) == 0
            outs.append((w, h, img))
        torch.cuda.synchronize()
        for w, h, img in outs:
            ref = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 2000, width=w, height=h, spp=5)
            g, _, _ = R.render(ref)
            assert compare(img.cpu().numpy(), g)["exact_frac"] == 1.0, (w, h)
    finally:
        lib.rt_group_free(grp)
        lib.rt_dev_scene_free(s)
