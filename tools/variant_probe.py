"""Probe one build of librt_hip (RT_HIP_LIB selects a variant built with `make variant`):
IOW-03 parity against the oracle on a small frame, the lone-pixel wave-cooperative segment cost
with its phase split (RT_DIAG_SPLIT builds).
    RT_HIP_LIB=raytracing-tests_amd/librt_hip_diag.so python tools/variant_probe.py"""
import ctypes as C, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import numpy as np, torch  # noqa: E402
import rt_amd as R  # noqa: E402
from oracle import oracle as O  # the checker

lib = R.load()
out = {"lib": os.path.basename(R.LIB_PATH)}
sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=40, height=24, spp=6)
g, _, gs = R.render(sc, sc.params)
o, _, os_ = O.render(sc, sc.params)
out["parity_small"] = bool(np.array_equal(g, o)) and gs["segments"] == os_["segments"]
# lone pixel, sequential kernel, cooperative closest hits
o = R.get_options(); o.iow_spec, o.iow_coop_max = 0, 4; R.set_options(o)
sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0)
q = R.RtParams(); C.memmove(C.addressof(q), C.addressof(sc.params), C.sizeof(q))
q.tile_x0, q.tile_y0, q.tile_w, q.tile_h = 553, 404, 1, 1
img0, _, _ = R.render(sc, q)
dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
lib.rt_debug_counters(dbg.data_ptr())
img1, _, st = R.render(sc, q)
lib.rt_debug_counters(None)
names = ["outer", "outer_lanes", "cull", "exact", "reduce", "leaf_lanes", "seg", "seg_lanes", "cyc_loop_top",
         "eval", "shade", "cyc_leaf", "cyc_seg", "cyc_coop_query", "cyc_coop_shade", "cyc_pop"]
n = max(1, st["segments"])
out["lone"] = {"segments": st["segments"], "us_per_segment": st["ms"] * 1e3 / n,
               "cyc_per_segment": {k: round(v / n, 1) for k, v in zip(names, dbg.cpu().numpy().tolist()) if v}}
out["lone_rgba"] = [float(v) for v in img1.reshape(-1)[:3]]
R.set_options(R.default_options())
print(json.dumps(out))
