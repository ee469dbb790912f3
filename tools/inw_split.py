#!/usr/bin/env python3
"""Phase split of the INW fold kernel (diagnostic build with -DRT_DIAG_SPLIT):

  make -C raytracing-tests_amd variant VARIANT=split VDEFS=-DRT_DIAG_SPLIT
  RT_HIP_LIB=raytracing-tests_amd/librt_hip_split.so python3 tools/inw_split.py [c3|c5] [spp]

Prints the shader-clock cycles the waves spent per phase (summed over waves): closest-hit walk,
surrounding-RI walk (both inside the segment), fold, claim + issue, and the whole segment step.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import torch  # noqa: E402

import rt_amd as R  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
spp = int(sys.argv[2]) if len(sys.argv) > 2 else 0
over = {"spp": spp} if spp else {}
sc = (R.make_scene(R.PRESET_INW01_RANDOM, 1234, 10_000, **over) if cfg == "c3"
      else R.make_scene(R.PRESET_INW04_CORNELL, 7, 0, **over))
lib = R.load()
dev = torch.device("cuda", 0)
lights = sc.lights if sc.lights is not None and len(sc.lights) else None
scene = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, sc.layout, R.fptr(sc.nodes), R.fptr(lights), sc.n_lights,
                             sc.params.spp, 0)
p = sc.params
rgba = torch.zeros((p.height, p.width, 4), dtype=torch.float32, device=dev)
depth = torch.zeros((p.height, p.width), dtype=torch.float32, device=dev)
ctr = torch.zeros(6, dtype=torch.int64, device=dev)
dbg = torch.zeros(16, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream()


def render():
    rc = lib.rt_render_image_async(scene, C.byref(sc.camera), C.byref(p), rgba.data_ptr(), depth.data_ptr(),
                                   ctr.data_ptr(), st.cuda_stream)
    assert rc == 0, rc


render()
torch.cuda.synchronize()
lib.rt_debug_counters(dbg.data_ptr())
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(st)
render()
b.record(st)
torch.cuda.synchronize()
lib.rt_debug_counters(None)
d = [int(v) for v in dbg.cpu().tolist()]
names = ("closest_hit", "ri_walk", "fold", "claim_issue", "segment_step")
cyc = dict(zip(names, d[8:13]))
tot = cyc["fold"] + cyc["claim_issue"] + cyc["segment_step"]
kname = C.create_string_buffer(64)
lib.rt_debug_launches(scene, kname, 64)
print(json.dumps({"config": cfg, "spp": p.spp, "kernel": kname.value.decode(), "ms": round(a.elapsed_time(b), 2),
                  "wave_cycles": cyc, "share_of_loop": {k: round(v / max(tot, 1), 4) for k, v in cyc.items()}}))
lib.rt_dev_scene_free(scene)
