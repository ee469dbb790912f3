"""Diagnostic: the heaviest samples of one rank's share of an N-way tile partition and the chains
they form inside their pixels.  python tools/chain_stats.py [r N [W H spp]]   (default 0 1 = whole
bench frame; W H spp: another resolution / sample count of the same scene)

Renders the share once (as bench.py does), then reads rt_debug_spec_dump: the rays of every
(pixel, sample) record (their last execution), the re-execution list after the pass, and the
count of pixels left to the sequential kernel."""
import ctypes as C
import json
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import torch  # noqa: E402

import rt_amd as R  # noqa: E402
from bench import tile_for, tiles_for_rank  # noqa: E402

r, n = (int(sys.argv[1]), int(sys.argv[2])) if len(sys.argv) > 2 else (0, 1)
lib = R.load()
over = dict(zip(("width", "height", "spp"), (int(v) for v in sys.argv[3:6])))
sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0, **over)
W, H = sc.params.width, sc.params.height
TILE = tile_for(n)
_, mine, per_rank = tiles_for_rank(W, H, n, r, TILE)
scene = lib.rt_dev_scene_iow03(R.fptr(sc.types), R.fptr(sc.records), sc.n, sc.params.spp, 0)
dev = torch.device("cuda", 0)
d_tiles = torch.tensor(mine, dtype=torch.int32, device=dev).reshape(-1, 2).contiguous()
packed = torch.zeros((per_rank, TILE, TILE, 4), dtype=torch.float32, device=dev)
ctr = torch.zeros(6, dtype=torch.int64, device=dev)
st = torch.cuda.current_stream()
rc = lib.rt_render_tiles_async(scene, C.byref(sc.camera), C.byref(sc.params), d_tiles.data_ptr(), len(mine), TILE,
                               packed.data_ptr(), None, ctr.data_ptr(), st.cuda_stream)
assert rc == 0, rc
torch.cuda.synchronize()
cap = len(mine) * TILE * TILE * sc.params.spp + 64 * sc.params.spp
rays = np.zeros(cap, np.uint32)
lst = np.zeros(1 << 22, np.uint32)
dims = np.zeros(4, np.uint32)
rc = lib.rt_debug_spec_dump(scene, rays.ctypes.data, cap, lst.ctypes.data, len(lst), dims.ctypes.data)
assert rc == 0, rc
P, S, nl, nfb = (int(v) for v in dims)
rays = rays[:P * S].reshape(S, P)
inlist = np.zeros((S, P), bool)
lu = lst[:min(nl, len(lst))]
inlist[lu // P, lu % P] = True
flat = np.argsort(-rays.astype(np.int64), axis=None)[:40]
top = [{"pu": int(i % P), "s": int(i // P), "rays": int(rays.flat[i]), "relisted": bool(inlist.flat[i])}
       for i in flat]
chains = []
for pu in list(dict.fromkeys(t["pu"] for t in top))[:10]:
    col = rays[:, pu]
    heavy = [(int(s), int(col[s]), bool(inlist[s, pu])) for s in np.nonzero(col > 4096)[0]]
    chains.append({"pu": pu, "total": int(col.sum()), "heavy_samples": heavy})
rl = np.sort(rays[inlist])[::-1]
out = {"share": f"{r}/{n}", "P": P, "S": S, "relist": nl, "seq_leftover_pixels": nfb,
       "relist_top_rays": [int(v) for v in rl[:20]], "relist_rays_total": int(rl.sum()),
       "top_samples": top, "pixel_chains": chains,
       "max_sample_rays": int(rays.max()), "pixel_max_total": int(rays.sum(0).max())}
print(json.dumps(out))
lib.rt_dev_scene_free(scene)
