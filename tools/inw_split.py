#!/usr/bin/env python3
"""Phase split of the INW fold kernel (diagnostic build with -DRT_DIAG_SPLIT):

  make -C raytracing-tests_amd variant VARIANT=split VDEFS=-DRT_DIAG_SPLIT
  RT_HIP_LIB=raytracing-tests_amd/librt_hip_split.so python3 tools/inw_split.py [c3|c5] [spp]

  ... tools/inw_split.py c3 500 r/N     (rank r's tiles of an N-way partition, as bench.py deals them)

Prints the shader-clock cycles the waves spent per phase (summed over waves): closest-hit walk,
surrounding-RI walk (both inside the segment), fold, claim + issue, and the whole segment step;
and, for k_inw_pm, the wall-clock timeline of one launch: waves' first / last start, the first
wave to find the pixel queue drained, and the first / last wave exit (the tail).
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
shard = sys.argv[3] if len(sys.argv) > 3 else ""
if len(sys.argv) > 4:  # rt_options fields, FIELD=VALUE
    o = R.get_options()
    for kv in sys.argv[4:]:
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
dbg = torch.zeros(32, dtype=torch.int64, device=dev)  # slots 8-15 phases, 16-20 timeline, 24-25 rounds
st = torch.cuda.current_stream()
if shard:
    from bench import tile_for, tiles_for_rank
    r, n = (int(v) for v in shard.split("/"))
    T = tile_for(n)
    _, mine, per_rank = tiles_for_rank(p.width, p.height, n, r, T)
    if os.environ.get("RT_SPLIT_ROWS"):  # experiment: the share's tiles in row-major order
        mine = sorted(mine, key=lambda t: (t[1], t[0]))
    d_tiles = torch.tensor(mine, dtype=torch.int32, device=dev).reshape(-1, 2).contiguous()
    packed = torch.zeros((per_rank, T, T, 4), dtype=torch.float32, device=dev)
    tdepth = torch.zeros((per_rank, T, T), dtype=torch.float32, device=dev)


def render():
    if shard:
        rc = lib.rt_render_tiles_async(scene, C.byref(sc.camera), C.byref(p), d_tiles.data_ptr(), len(mine), T,
                                       packed.data_ptr(), tdepth.data_ptr(), ctr.data_ptr(), st.cuda_stream)
    else:
        rc = lib.rt_render_image_async(scene, C.byref(sc.camera), C.byref(p), rgba.data_ptr(), depth.data_ptr(),
                                       ctr.data_ptr(), st.cuda_stream)
    assert rc == 0, rc


render()
torch.cuda.synchronize()
big = (1 << 63) - 1
dbg[16], dbg[18], dbg[19] = big, big, big
lib.rt_debug_counters(dbg.data_ptr())
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record(st)
render()
b.record(st)
torch.cuda.synchronize()
lib.rt_debug_counters(None)
d = [int(v) for v in dbg.cpu().tolist()]
names = ("closest_hit", "ri_walk", "fold", "claim_issue", "segment_step", "seg_prologue", "seg_material",
         "seg_tail")
cyc = dict(zip(names, d[8:16]))
tot = cyc["fold"] + cyc["claim_issue"] + cyc["segment_step"]
# k_inw_pm: whole-wave cycles of the primary round (beam lists) and the bounce round (wide walk)
cyc["round0_primary"], cyc["round1_bounce"] = d[24], d[25]
kname = C.create_string_buffer(64)
lib.rt_debug_launches(scene, kname, 64)
t = d[16:21]  # wall clock, 100 MHz
tl = None
if t[0] != big and t[3] != big:
    ms = lambda v: round((v - t[0]) / 1e5, 3)  # noqa: E731
    tl = {"last_wave_start_ms": ms(t[1]), "queue_drained_ms": ms(t[2]) if t[2] != big else None,
          "first_wave_exit_ms": ms(t[3]), "last_wave_exit_ms": ms(t[4]),
          "tail_after_drain_ms": round((t[4] - t[2]) / 1e5, 3) if t[2] != big else None}
print(json.dumps({"config": cfg, "spp": p.spp, "shard": shard or None, "kernel": kname.value.decode(),
                  "ms": round(a.elapsed_time(b), 2), "wave_cycles": cyc,
                  "share_of_loop": {k: round(v / max(tot, 1), 4) for k, v in cyc.items()}, "timeline": tl}))
lib.rt_dev_scene_free(scene)
