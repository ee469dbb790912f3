"""Diagnostic: when the long samples of one rank's share start, restart and finish (launch
sequence numbers of the sample-parallel IOW-03 pipeline, RT_DEBUG_TIMES=1).
  python tools/spec_times.py r N [W H spp]"""
import ctypes as C
import json
import os
import sys

import numpy as np

os.environ["RT_DEBUG_TIMES"] = "1"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import torch  # noqa: E402

import rt_amd as R  # noqa: E402
from bench import tile_for, tiles_for_rank  # noqa: E402

r, n = int(sys.argv[1]), int(sys.argv[2])
over = dict(zip(("width", "height", "spp"), (int(v) for v in sys.argv[3:6])))
lib = R.load()
sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0, **over)
W, H = sc.params.width, sc.params.height
T = tile_for(n)
_, mine, per_rank = tiles_for_rank(W, H, n, r, T)
scene = lib.rt_dev_scene_iow03(R.fptr(sc.types), R.fptr(sc.records), sc.n, sc.params.spp, 0)
dev = torch.device("cuda", 0)
d_tiles = torch.tensor(mine, dtype=torch.int32, device=dev).reshape(-1, 2).contiguous()
packed = torch.zeros((per_rank, T, T, 4), dtype=torch.float32, device=dev)
ctr = torch.zeros(6, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream()
lib.rt_debug_time_kernels(1)
rc = lib.rt_render_tiles_async(scene, C.byref(sc.camera), C.byref(sc.params), d_tiles.data_ptr(), len(mine), T,
                               packed.data_ptr(), None, ctr.data_ptr(), st.cuda_stream)
assert rc == 0, rc
torch.cuda.synchronize()
cap = len(mine) * T * T * sc.params.spp + 64 * sc.params.spp
rays = np.zeros(cap, np.uint32)
lst = np.zeros(1 << 22, np.uint32)
dims = np.zeros(4, np.uint32)
assert lib.rt_debug_spec_dump(scene, C.c_void_p(rays.ctypes.data), cap, C.c_void_p(lst.ctypes.data), len(lst),
                              C.c_void_p(dims.ctypes.data)) == 0
P, S, nl, nfb = (int(v) for v in dims)
t0 = np.zeros(cap, np.uint32)
t1 = np.zeros(cap, np.uint32)
assert lib.rt_debug_spec_times(scene, C.c_void_p(t0.ctypes.data), C.c_void_p(t1.ctypes.data), cap) == 0
rays, t0, t1 = rays[:P * S], t0[:P * S], t1[:P * S]
ms = C.c_double(0.0)
nk = C.c_int(0)
lib.rt_debug_kernel_time(scene, C.byref(ms), C.byref(nk))
top = np.argsort(-rays.astype(np.int64))[:30]
out = {"share": f"{r}/{n}", "P": P, "S": S, "launches": nk.value, "relist": nl, "seq_leftover_pixels": nfb,
       "restarted_samples": int(((t0 >> 16) > 1).sum()),
       "last_end_launch": int(t1.max()),
       "top": [{"pu": int(i % P), "s": int(i // P), "rays": int(rays[i]), "start": int(t0[i] & 0xffff),
                "starts": int(t0[i] >> 16), "end": int(t1[i])} for i in top]}
late = np.nonzero(t1 >= t1.max() - 3)[0]
out["finished_last"] = [{"pu": int(i % P), "s": int(i // P), "rays": int(rays[i]), "start": int(t0[i] & 0xffff),
                         "starts": int(t0[i] >> 16), "end": int(t1[i])} for i in late[np.argsort(-rays[late].astype(np.int64))][:15]]
# units in flight per launch (started at or before it, finished at or after it), and how many
# of them are long (> 10k rays)
st_l, en_l = (t0 & 0xffff).astype(np.int64), t1.astype(np.int64)
ok = (t1 > 0) | (st_l > 0)
alive, heavy = [], []
for L in range(int(t1.max()) + 1):
    a = ok & (st_l <= L) & (en_l >= L)
    alive.append(int(a.sum()))
    heavy.append(int((a & (rays > 10000)).sum()))
out["alive_per_launch"] = alive
out["alive_long_per_launch"] = heavy
print(json.dumps(out))
lib.rt_dev_scene_free(scene)
