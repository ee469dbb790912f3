"""Diagnostic: how well does the heaviest-first pixel order (by sample 0's ray count) place the
heaviest samples of the bench frame?  Renders the bench frame once (device scene, full image)
and summarises rt_debug_spec_pixels as JSON."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import torch  # noqa: E402

import rt_amd as R  # noqa: E402

lib = R.load()
sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0)
W, H, spp = sc.params.width, sc.params.height, sc.params.spp
scene = lib.rt_dev_scene_iow03(R.fptr(sc.types), R.fptr(sc.records), sc.n, spp, 0)
img = torch.zeros((H, W, 4), dtype=torch.float32, device="cuda")
ctr = torch.zeros(6, dtype=torch.int64, device="cuda")
rc = lib.rt_render_image_async(scene, C.byref(sc.camera), C.byref(sc.params), img.data_ptr(), None, ctr.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
assert rc == 0, rc
torch.cuda.synchronize()
P = ((W + 7) // 8) * ((H + 7) // 8) * 64
out = np.zeros((P, 4), np.uint32)
n = lib.rt_debug_spec_pixels(scene, out.ctypes.data_as(C.POINTER(C.c_uint32)), P)
assert n > 0, n
out = out[:n]
s0, mx, arg = out[:, 0].astype(np.int64), out[:, 1].astype(np.int64), out[:, 2]
rank_of = np.empty(n, np.int64)
rank_of[out[:, 3]] = np.arange(n)
valid = mx > 0
top = np.argsort(-mx)[:200]
res = {
    "units": int(n), "valid": int(valid.sum()),
    "max_sample_rays": int(mx.max()),
    "top_samples": [{"pixel_unit": int(p), "rays": int(mx[p]), "sample": int(arg[p]), "s0_rays": int(s0[p]),
                     "order_rank": int(rank_of[p])} for p in top[:25]],
    "top200_rank_quantiles": [float(q) for q in np.quantile(rank_of[top] / n, [0.1, 0.5, 0.9, 1.0])],
    "spearman_s0_vs_max": float(np.corrcoef(np.argsort(np.argsort(s0[valid])),
                                            np.argsort(np.argsort(mx[valid])))[0, 1]),
    "top200_sample_index_quantiles": [float(q) for q in np.quantile(arg[top], [0.1, 0.5, 0.9])],
}
for thr in (32768, 65536, 100000):
    sel = mx >= thr
    res[f"pixels_max_ge_{thr}"] = int(sel.sum())
    if sel.any():
        res[f"rank_frac_quantiles_ge_{thr}"] = [float(q) for q in np.quantile(rank_of[sel] / n, [0.5, 0.9, 1.0])]
h = (C.c_uint64 * 66)()
lib.rt_debug_spec_list_hist(scene, h)
res["relist"] = {"samples": int(h[1]), "max_rays": int(h[0]),
                 "log2_hist": {b: [int(h[2 + b]), int(h[34 + b])] for b in range(32) if h[2 + b]}}
if os.environ.get("RT_DEBUG_FIRST_STALE") == "1":
    h2 = (C.c_uint64 * 32)()
    lib.rt_debug_spec_list_stale(scene, h2)
    res["first_stale_16ths"] = {"samples": [int(h2[b]) for b in range(16)], "rays": [int(h2[16 + b]) for b in range(16)]}
print(json.dumps(res))
