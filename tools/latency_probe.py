"""Single-pixel latency probe: find the heaviest pixel of a central region, then time it alone
(sequential kernel vs sample-parallel) to measure per-segment latency of a lone lane."""
import ctypes as C, os, sys, time, json
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import numpy as np, torch
import rt_amd as R
lib = R.load()
sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0)
W, H = sc.params.width, sc.params.height
x0, y0, tw, th = W // 2 - 64, H // 2 - 64, 128, 128
units = ((tw + 7) // 8) * ((th + 7) // 8) * 64
pr = torch.zeros(units, dtype=torch.int32, device="cuda")
lib.rt_debug_pixel_rays(pr.data_ptr())
p = R.RtParams(); C.memmove(C.addressof(p), C.addressof(sc.params), C.sizeof(p))
p.tile_x0, p.tile_y0, p.tile_w, p.tile_h = x0, y0, tw, th
with R.options(iow_spec=0):
    R.render(sc, p)
lib.rt_debug_pixel_rays(None)
u = int(torch.argmax(pr).item()); mx = int(pr.max().item())
b, l = u >> 6, u & 63; nbx = (tw + 7) >> 3
px, py = x0 + (b % nbx) * 8 + (l & 7), y0 + (b // nbx) * 8 + (l >> 3)
out = {"pixel": [px, py], "rays": mx}
for coop, mode in (("0", "0"), ("4", "0"), ("0", "1"), ("4", "1")):
    o = R.default_options(); o.iow_spec, o.iow_coop_max = int(mode), int(coop); R.set_options(o)
    q = R.RtParams(); C.memmove(C.addressof(q), C.addressof(sc.params), C.sizeof(q))
    q.tile_x0, q.tile_y0, q.tile_w, q.tile_h = px, py, 1, 1
    R.render(sc, q)
    dbg = torch.zeros(16, dtype=torch.int64, device="cuda")
    lib.rt_debug_counters(dbg.data_ptr())
    t0 = time.perf_counter(); _, _, st = R.render(sc, q); dt = time.perf_counter() - t0
    lib.rt_debug_counters(None)
    d = dbg.cpu().numpy().tolist()
    names = ["outer", "outer_lanes", "trav", "trav_lanes", "leaf", "leaf_lanes", "seg", "seg_lanes",
             "cyc_loop_top", "cyc_ray", "cyc_trav", "cyc_leaf", "cyc_seg", "cyc_coop_query", "cyc_coop_shade", "cyc_pop"]
    out["spec" + mode + "_coop" + coop] = {"ms": st["ms"], "wall_ms": dt * 1e3, "segments": st["segments"],
                          "us_per_segment": st["ms"] * 1e3 / max(1, st["segments"]),
                          "dbg_per_segment": {k: round(v / max(1, st["segments"]), 1) for k, v in zip(names, d)}}
print(json.dumps(out))
