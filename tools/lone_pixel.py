"""One pixel of the bench frame rendered alone (the latency probe's heaviest pixel, 553,404):
a lone wave's cost per ray segment, for PMC passes.  python tools/lone_pixel.py [x y]"""
import ctypes as C, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import rt_amd as R  # noqa: E402
x, y = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (553, 404)
o = R.default_options(); o.iow_spec, o.iow_coop_max = 0, 4; R.set_options(o)  # sequential, cooperative hits
sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0)
q = R.RtParams(); C.memmove(C.addressof(q), C.addressof(sc.params), C.sizeof(q))
q.tile_x0, q.tile_y0, q.tile_w, q.tile_h = x, y, 1, 1
R.render(sc, q)
t0 = time.perf_counter(); _, _, st = R.render(sc, q); dt = time.perf_counter() - t0
print(json.dumps({"pixel": [x, y], "segments": st["segments"], "ms": st["ms"], "wall_ms": dt * 1e3,
                  "us_per_segment": st["ms"] * 1e3 / max(1, st["segments"])}))
