"""INW lane occupancy per phase of the fold kernel (diagnostic build with -DRT_DIAG_OCC):
    make -C raytracing-tests_amd variant VARIANT=occ VDEFS=-DRT_DIAG_OCC
    RT_HIP_LIB=raytracing-tests_amd/librt_hip_occ.so python tools/inw_occ.py [c3|c5] [spp] [FIELD=VALUE ...]
Prints, per phase, the wave iterations, the lanes doing that phase's work per iteration (of 64)
and the share of wave iterations; slots as rt_kernels.hip kOcc*."""
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
if len(sys.argv) > 3:
    o = R.get_options()
    for kv in sys.argv[3:]:
        k, v = kv.split("=", 1)
        setattr(o, k, int(v))
    R.set_options(o)
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
dbg = torch.zeros(64, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream().cuda_stream
lib.rt_render_image_async(scene, C.byref(sc.camera), C.byref(p), rgba.data_ptr(), depth.data_ptr(), ctr.data_ptr(), st)
torch.cuda.synchronize()
ctr.zero_()
lib.rt_debug_counters(dbg.data_ptr())
lib.rt_render_image_async(scene, C.byref(sc.camera), C.byref(p), rgba.data_ptr(), depth.data_ptr(), ctr.data_ptr(), st)
torch.cuda.synchronize()
lib.rt_debug_counters(None)
d = [int(v) for v in dbg.cpu().tolist()][32:50]
names = ("segment_iterations", "walk_trips", "node_steps", "leaf_batches", "beam_trips", "reference_walks", "ri_queries",
         "node_steps_same_node_as_first", "node_steps_all_one_node")
out = {"config": cfg, "spp": p.spp, "path": R.debug_path(scene), "segments": int(ctr[0].item()),
       "node_visits": int(ctr[1].item()), "prim_tests": int(ctr[2].item())}
tot = sum(d[2 * i] for i in (1, 3, 4))
for i, n in enumerate(names):
    it, lanes = d[2 * i], d[2 * i + 1]
    out[n] = {"wave_iterations": it, "lanes_per_iteration": round(lanes / max(it, 1), 2),
              "lane_occupancy": round(lanes / max(it, 1) / 64, 4)}
out["walk_trip_share_of_walk+leaf+beam"] = round(d[2] / max(tot, 1), 4)
lib.rt_dev_scene_free(scene)
print(json.dumps(out))
