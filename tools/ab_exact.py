"""A/B bit-exactness of IOW-03 strategy switches on the final scene (diagnostic).
usage: python tools/ab_exact.py W H SPP 'ENV_A' 'ENV_B' ...  (each ENV as k=v,k=v; '-' = defaults)"""
import json, os, subprocess, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODE = r"""
import sys, json, numpy as np
sys.path[:0] = [{root!r}, {root!r} + '/raytracing-tests_amd']
import rt_amd as R
sc = R.make_scene(2, 20250131, 0, width={w}, height={h}, spp={spp})
img, depth, st = R.render(sc)
np.save({out!r}, img)
print(json.dumps(st))
"""
w, h, spp = map(int, sys.argv[1:4])
res = []
for i, spec in enumerate(sys.argv[4:]):
    env = {k: v for k, v in os.environ.items() if not k.startswith("RT_")}
    if spec != "-":
        env.update(dict(kv.split("=") for kv in spec.split(",")))
    out = f"/tmp/ab_{i}.npy"
    r = subprocess.run([sys.executable, "-c", CODE.format(root=ROOT, w=w, h=h, spp=spp, out=out)], env=env,
                       capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        print(spec, "FAILED", r.stderr[-1500:]); sys.exit(1)
    st = json.loads(r.stdout.strip().splitlines()[-1])
    res.append((spec, np.load(out), st))
a = res[0][1]
for spec, b, st in res:
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    bad = np.argwhere(~same.all(axis=2))
    print(json.dumps({"env": spec, "mismatch_px": len(bad), "first": bad[:6].tolist(), **{k: st[k] for k in ("segments", "node_visits", "prim_tests", "stack_drops", "ms")}}))
