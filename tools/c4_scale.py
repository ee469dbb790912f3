"""Predicted strong scaling of BASELINE config C4: the C3 scene (INW-01, 10k moving spheres,
LBVH, 1920x1080) tile-partitioned over 1/2/4/8 ranks as bench.py partitions it.  Every rank's
share is rendered on its own on one GPU (device-resident scene, the library's tile entry point);
the N-rank frame time is the maximum over ranks.  INW samples are independent invocations
(01_BVH...glsl:601-675), so unlike IOW-03 this path has no cross-sample chains.

  python tools/c4_scale.py [spp]      (default 32; Mrays/s is a rate, the full 500 spp scales it)
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import torch  # noqa: E402

import rt_amd as R  # noqa: E402
from bench import tile_for, tiles_for_rank  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 32
lib = R.load()
sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 10_000, spp=spp)
W, H = sc.params.width, sc.params.height
scene = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, sc.layout, R.fptr(sc.nodes), None, 0, spp, 0)
assert scene, "rt_dev_scene_inw failed"
dev = torch.device("cuda", 0)
st = torch.cuda.current_stream()


def share(n, r):
    T = tile_for(n)
    _, mine, per_rank = tiles_for_rank(W, H, n, r, T)
    d_tiles = torch.tensor(mine, dtype=torch.int32, device=dev).reshape(-1, 2).contiguous()
    packed = torch.zeros((per_rank, T, T, 4), dtype=torch.float32, device=dev)
    depth = torch.zeros((per_rank, T, T), dtype=torch.float32, device=dev)
    ctr = torch.zeros(6, dtype=torch.int64, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    rc = lib.rt_render_tiles_async(scene, C.byref(sc.camera), C.byref(sc.params), d_tiles.data_ptr(), len(mine), T,
                                   packed.data_ptr(), depth.data_ptr(), ctr.data_ptr(), st.cuda_stream)
    assert rc == 0, rc
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3, int(ctr[0].item())


share(1, 0)  # warm-up: workspace for the largest share, code objects
base = None
for n in (1, 2, 4, 8):
    res = [share(n, r) for r in range(n)]
    t = [round(v[0], 2) for v in res]
    rays = sum(v[1] for v in res)
    base = base or max(t)
    print(json.dumps({"config": "C4 = C3 tile-partitioned", "spp": spp, "n_ranks": n, "tile": tile_for(n),
                      "max_ms": max(t), "per_rank_ms": t, "speedup": round(base / max(t), 3),
                      "Mrays_per_s": round(rays / (max(t) * 1e-3) / 1e6, 1)}), flush=True)
lib.rt_dev_scene_free(scene)
