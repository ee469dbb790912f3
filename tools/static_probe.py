#!/usr/bin/env python3
"""Experiment: how much of the C3 frame do the moving spheres' swept boxes cost?

Renders the C3 scene with every sphere's motion scaled by m (last_position = position - m * motion;
m = 1 is the bench scene, m = 0 static) and prints the frame time and the walk's node / object
counts.  m = 1/K approximates culling with per-time-bin boxes (K bins of the shutter interval).
  python3 tools/static_probe.py [spp] [m ...]
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import torch  # noqa: E402

import rt_amd as R  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 500
ms_list = [float(v) for v in sys.argv[2:]] or [1.0, 0.5, 0.25, 0.0]
lib = R.load()
if os.environ.get("STATIC_OPTS"):  # rt_options fields for the scenes, "a=1,b=2"
    o = R.get_options()
    for kv in os.environ["STATIC_OPTS"].split(","):
        k, v = kv.split("=", 1)
        setattr(o, k, int(v))
    R.set_options(o)
dev = torch.device("cuda", 0)
arr, n, cd, par = R.preset_desc(R.PRESET_INW01_RANDOM, 1234, 10_000)
par.spp = spp
cam = R.camera_from_desc(cd, R.RT_STAGE_INW01)
base = [(tuple(arr[i].position), tuple(arr[i].last_position)) for i in range(n)]
st = torch.cuda.current_stream()
rgba = torch.zeros((par.height, par.width, 4), dtype=torch.float32, device=dev)
depth = torch.zeros((par.height, par.width), dtype=torch.float32, device=dev)
ctr = torch.zeros(6, dtype=torch.int64, device=dev)
for m in ms_list:
    for i, (p, lp) in enumerate(base):
        for a in range(3):
            arr[i].last_position[a] = p[a] - m * (p[a] - lp[a])
    pk = R.pack(arr, n, R.RT_STAGE_INW01)
    scene = lib.rt_dev_scene_inw(R.fptr(pk["geom"]), n, 1, R.fptr(pk["nodes"]), None, 0, spp, 0)
    assert scene
    res = []
    for rep in range(3):
        ctr.zero_()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        rc = lib.rt_render_image_async(scene, C.byref(cam), C.byref(par), rgba.data_ptr(), depth.data_ptr(),
                                       ctr.data_ptr(), st.cuda_stream)
        assert rc == 0, rc
        b.record(st)
        torch.cuda.synchronize()
        res.append(a.elapsed_time(b))
    c = [int(v) for v in ctr.cpu().tolist()]
    print(json.dumps({"motion_scale": m, "spp": spp, "ms": [round(v, 2) for v in res], "segments": c[0],
                      "node_visits": c[1], "prim_tests": c[2]}), flush=True)
    lib.rt_dev_scene_free(scene)
