"""Summarise a directory of bench.py A/B lines (gpurun_out/<dir>/<variant>_<i>.json) into one JSON
for profiles/: per run the step time, the main kernel's time, the node / object counts and the path
fields that tell the variants apart.
usage: python tools/ab_summary.py DIR OUT.json 'note' [variant=description ...]"""
import glob
import json
import os
import sys

d, out, note = sys.argv[1], sys.argv[2], sys.argv[3]
desc = dict(kv.split("=", 1) for kv in sys.argv[4:])
res = {"note": note, "variants": desc, "runs": {}}
for f in sorted(glob.glob(os.path.join(d, "*.json"))):
    name = os.path.basename(f)[:-5]
    try:
        j = json.load(open(f))
    except Exception:  # noqa: BLE001  (an occupancy line or an empty file)
        continue
    if "ms_per_step" not in j:
        res["runs"][name] = j
        continue
    p, c = j["path"], j["counters_per_step"]
    res["runs"][name] = {"ms_per_step": j["ms_per_step"], "kernel_ms": j["roofline"]["main_kernel_ms_per_frame"],
                         "node_visits": c["node_visits"], "prim_tests": c["prim_tests"], "segments": c["segments"],
                         "kernel": p["kernel"], "lds_nodes": p["lds_nodes"], "qnodes": p.get("qnodes"),
                         "global_stack": p.get("global_stack"), "ref_walk_frac": p.get("ref_walk_frac"),
                         "options": j["options"]}
by = {}
for k, v in res["runs"].items():
    if "ms_per_step" in v:
        by.setdefault(k.rsplit("_", 1)[0], []).append(v["ms_per_step"])
res["mean_ms_per_step"] = {k: round(sum(v) / len(v), 2) for k, v in by.items()}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res["mean_ms_per_step"]))
