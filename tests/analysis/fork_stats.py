"""Offline analysis: the cost of evaluating IOW-03 samples for every value of the stale RI entries
they read (fork on read, tools/fork_stats.c) on random pixels of the bench frame (C2).

  python tests/analysis/fork_stats.py [npix] [seed] [extra px,py ...]

Offline study on the CPU oracle (test infrastructure, hence under tests/); not collected by pytest.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd")]
import rt_amd as R  # noqa: E402

SO = "/tmp/libfork_stats.so"
subprocess.run(["gcc", "-O2", "-fopenmp", "-ffp-contract=off", "-fPIC", "-shared", "-o", SO,
                os.path.join(ROOT, "tests", "analysis", "fork_stats.c"), "-lm"], check=True)
lib = C.CDLL(SO)
npix = int(sys.argv[1]) if len(sys.argv) > 1 else 128
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1
extra = [tuple(int(v) for v in a.split(",")) for a in sys.argv[3:]]
sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0)
W, H, S = sc.params.width, sc.params.height, sc.params.spp
rng = np.random.default_rng(seed)
pix = np.stack([rng.integers(0, W, npix), rng.integers(0, H, npix)], 1).astype(np.int32)
if extra:
    pix = np.concatenate([pix, np.array(extra, np.int32)], 0)
rec = np.asarray(sc.records).reshape(-1, 24)
vals = np.unique(np.concatenate([[0.0, 1.0], rec[:, 20]])).astype(np.float32)
if os.environ.get("FORK_VALS"):
    vals = np.array([float(v) for v in os.environ["FORK_VALS"].split(",")], np.float32)
out = np.zeros((len(pix), S, 12), np.uint64)
FP = C.POINTER(C.c_float)
lib.fork_stats(R.fptr(sc.types), R.fptr(sc.records), C.c_uint32(sc.n), C.byref(sc.camera), C.byref(sc.params),
               C.c_void_p(pix.ctypes.data), C.c_int(len(pix)), vals.ctypes.data_as(FP), C.c_int(len(vals)), C.c_void_p(out.ctypes.data))
ex, fw, lv, lg, rd, pre, gl, bad, wr = (out[..., k].astype(np.int64) for k in range(9))
res = {
    "pixels": int(len(pix)), "values": vals.tolist(),
    "exact_segments": int(ex.sum()), "fork_segments": int(fw.sum()),
    "work_ratio": round(float(fw.sum() / max(1, ex.sum())), 4),
    "samples_reading_incoming": round(float((rd > 0).mean()), 4),
    "samples_forked": round(float((lv > 1).mean()), 4),
    "leaves_mean": round(float(lv.mean()), 3), "leaves_max": int(lv.max()),
    "max_exact_sample": int(ex.max()), "max_branch": int(lg.max()),
    "forked_prefix_frac": round(float(pre[lv > 1].sum() / max(1, ex[lv > 1].sum())), 4),
    "forked_heavy_prefix_frac": round(float(pre[(lv > 1) & (ex > 10000)].sum() / max(1, ex[(lv > 1) & (ex > 10000)].sum())), 4),
    "forked_work_frac": round(float(ex[lv > 1].sum() / max(1, ex.sum())), 4),
    "mispredicted_samples": round(float(bad.mean()), 5), "mispredicted_ray_frac": round(float(gl[bad > 0].sum() / max(1, ex.sum())), 5),
    "max_pixel_exact": int(ex.sum(1).max()), "max_pixel_fork": int(fw.sum(1).max()),
}
for i, (px, py) in enumerate(pix[len(pix) - len(extra):] if extra else []):
    j = len(pix) - len(extra) + i
    res[f"px{px},{py}"] = {"exact": int(ex[j].sum()), "fork": int(fw[j].sum()), "max_branch": int(lg[j].max()),
                            "max_sample": int(ex[j].max())}
print(json.dumps(res))
if os.environ.get("FORK_SAVE"):
    np.savez(os.environ["FORK_SAVE"], out=out, pix=pix)
