"""rt_dev_scene_inw_update timing (the reference's per-redraw scene work, In-Next-Week/base.h:96-175)
on the C3 scene: `steps` updates with the LBVH and the walk structures built on the device, host
wall time per phase (rt_dev_scene_inw_update's timing_ms).  For rocprofv3 kernel traces of the
device build: python tools/prof_update.py [steps] [device_build 0|1]."""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import rt_amd as R  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    dev = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 10_000)
    lib = R.load()
    with R.options(inw_device_build=dev):
        s = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, 1, R.fptr(sc.nodes), None, 0, sc.params.spp, 0)
    assert s
    tm = (C.c_double * 4)()
    tot = [0.0] * 5
    try:
        for i in range(steps + 1):
            pk = R.pack(sc.desc, sc.n, sc.stage, build_lbvh=False)
            t0 = time.perf_counter()
            rc = lib.rt_dev_scene_inw_update(s, R.fptr(pk["geom"]), sc.n, None, R.fptr(pk["aabbs"]), None, 0, tm)
            dt = (time.perf_counter() - t0) * 1e3
            assert rc == 0, rc
            if i:
                for k in range(4):
                    tot[k] += tm[k]
                tot[4] += dt
        info = (C.c_uint32 * 8)()
        lib.rt_debug_wide_info(s, info, None)
    finally:
        lib.rt_dev_scene_free(s)
    print(json.dumps({"device_build": dev, "steps": steps,
                      "ms_per_update": dict(zip(("records", "lbvh", "walk_structures", "upload", "call"),
                                                [round(v / steps, 3) for v in tot])),
                      "wide_info": list(info)}))


if __name__ == "__main__":
    main()
