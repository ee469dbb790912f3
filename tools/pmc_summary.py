#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes of one bench run for one kernel into profiles/pmc_<tag>.json.

  python tools/pmc_summary.py --dir gpurun_out/prof --kernel k_iow03 --config 1200 800 100 \
      --launches-per-frame 7 --frames 1 --out profiles/pmc_iow03.json

Each pass directory pmcN/ holds rocprofv3's *counter_collection.csv.  Counter values are summed
over every dispatch of the kernel.  HBM bytes follow MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE is doubled (gfx950 tallies 128-B read requests at 64 B).
"""
import argparse
import collections
import csv
import glob
import json
import os


def collect(d, kernel):
    agg = collections.defaultdict(float)
    dispatches = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", "")
            if ("::" + kernel + "(") in name or name.startswith(kernel + "("):
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                dispatches[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
    return dict(agg), {k: len(v) for k, v in dispatches.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dir", required=True)
    ap.add_argument("--kernel", required=True)
    ap.add_argument("--config", type=int, nargs=3, required=True)
    ap.add_argument("--launches-per-frame", type=int, required=True)
    ap.add_argument("--frames", type=int, default=1)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    agg, nd = {}, {}
    for p in sorted(glob.glob(os.path.join(a.dir, "pmc*"))):
        g, n = collect(p, a.kernel)
        agg.update(g)
        nd.update(n)
    res = {"kernel": a.kernel, "config": a.config, "frames": a.frames,
           "launches_per_frame": a.launches_per_frame, "dispatches": nd, "counters": agg}
    if "FETCH_SIZE" in agg and "WRITE_SIZE" in agg:
        rd = 2.0 * agg["FETCH_SIZE"] * 1024.0
        wr = agg["WRITE_SIZE"] * 1024.0
        per_frame = (rd + wr) / a.frames
        res.update({"hbm_read_bytes_per_frame": rd / a.frames, "hbm_write_bytes_per_frame": wr / a.frames,
                    "hbm_bytes_per_frame": per_frame,
                    "hbm_bytes_per_launch": per_frame / a.launches_per_frame,
                    "hbm_note": "FETCH_SIZE x2 (gfx950 wide-read tally) + WRITE_SIZE, KiB->B; "
                                "read widths here are 16 B node/record loads, uncalibrated"})
    if "SQ_THREAD_CYCLES_VALU" in agg and "SQ_ACTIVE_INST_VALU" in agg:
        res["valu_lane_utilisation"] = agg["SQ_THREAD_CYCLES_VALU"] / (64.0 * agg["SQ_ACTIVE_INST_VALU"])
    if "SQ_WAIT_ANY" in agg and "SQ_WAVE_CYCLES" in agg:
        res["wait_fraction"] = agg["SQ_WAIT_ANY"] / agg["SQ_WAVE_CYCLES"]
    if "SQ_WAIT_INST_ANY" in agg and "SQ_WAVE_CYCLES" in agg:
        res["issue_stall_fraction"] = agg["SQ_WAIT_INST_ANY"] / agg["SQ_WAVE_CYCLES"]
    if "SQ_INSTS_VALU" in agg and "SQ_WAVES" in agg:
        res["valu_insts_per_wave"] = agg["SQ_INSTS_VALU"] / agg["SQ_WAVES"]
    if "TA_TA_BUSY_sum" in agg and "GRBM_GUI_ACTIVE" in agg:
        # GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md); one TA per CU (256)
        res["ta_busy_fraction"] = agg["TA_TA_BUSY_sum"] / (256.0 * agg["GRBM_GUI_ACTIVE"] / 8.0)
    if "TCP_TOTAL_CACHE_ACCESSES_sum" in agg and "TCP_TCC_READ_REQ_sum" in agg:
        res["l1_read_miss_per_access"] = agg["TCP_TCC_READ_REQ_sum"] / max(1.0, agg["TCP_TOTAL_CACHE_ACCESSES_sum"])
    if "TCC_HIT_sum" in agg and "TCC_MISS_sum" in agg:
        res["l2_hit_rate"] = agg["TCC_HIT_sum"] / max(1.0, agg["TCC_HIT_sum"] + agg["TCC_MISS_sum"])
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
