"""Diagnose a C2 rectangle rendered alone against the oracle (IOW-03 sample-parallel path).

  python tools/diag_c2_rect.py X0 Y0 W H [spp]
Prints one JSON line per variant: the rect render alone (default options, repeated), with the
sequential kernel (iow_spec=0), and the full frame's pixels, each compared with the oracle.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd"), os.path.join(ROOT, "tests")]
import rt_amd as R  # noqa: E402
from cases import compare  # noqa: E402
from oracle import oracle as O  # noqa: E402  (the checker)


def main():
    x0, y0, w, h = (int(v) for v in sys.argv[1:5])
    spp = int(sys.argv[5]) if len(sys.argv) > 5 else 100
    sc = R.make_scene(R.PRESET_IOW03_FINAL, 20250131, 0, width=1200, height=800, spp=spp, max_bounces=50)
    p = R.RtParams.from_buffer_copy(sc.params)
    p.tile_x0, p.tile_y0, p.tile_w, p.tile_h = x0, y0, w, h
    O.set_threads(os.cpu_count() or 1)
    o, _, ost = O.render(sc, p)
    sl = (slice(y0, y0 + h), slice(x0, x0 + w))
    print(json.dumps({"oracle_segments": ost["segments"], "oracle_nans": ost["nan_drops"]}), flush=True)

    def report(name, img, st=None):
        c = compare(img[sl], o[sl])
        bad = np.argwhere(np.any(img[sl] != o[sl], axis=-1))
        ex = []
        for yy, xx in bad[:4]:
            ex.append({"px": [int(x0 + xx), int(y0 + yy)], "gpu": img[y0 + yy, x0 + xx].tolist(),
                       "oracle": o[y0 + yy, x0 + xx].tolist()})
        print(json.dumps({"variant": name, **c, "bad_px": int(len(bad)), "examples": ex,
                          "segments": st["segments"] if st else None}), flush=True)

    for k in range(3):
        g, _, st = R.render(sc, p)
        report(f"rect_alone_{k}", g, st)
    with R.options(iow_spec=0):
        g, _, st = R.render(sc, p)
        report("rect_alone_seq", g, st)
    with R.options(spec_heavy=0, spec_alt_seg=16384):
        g, _, st = R.render(sc, p)
        report("rect_alone_fullframe_settings", g, st)
    img, _, st = R.render(sc)
    report("full_frame", img)


if __name__ == "__main__":
    main()
