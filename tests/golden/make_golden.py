"""Regenerate tests/golden/*.npz from the CPU oracle (the committed fixtures).

The reference ships no golden images, tests or known-answer vectors, and its
renderer cannot run here (GLSL/OpenGL, Windows-only harness), so these fixtures pin the
ORACLE against regressions; they are not reference outputs.  Run from the repo root:
    python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "raytracing-tests_amd"), os.path.dirname(HERE)]

import cases  # noqa: E402
import stages  # noqa: E402
from oracle import oracle as O  # noqa: E402


def main():
    only = set(sys.argv[1:])  # optional: regenerate just these cases
    for name in cases.GOLDEN_CASES + stages.GOLDEN_STAGE_CASES:
        if only and name not in only:
            continue
        if name in stages.GOLDEN_STAGE_CASES:
            rgba, depth, st = stages.render_oracle(name)
        elif name == "iow01_c1":
            cam, sph, p = cases.iow01_c1()
            rgba, st = O.render_iow01(cam, sph, p)
            depth = None
        else:
            sc = cases.CASES[name]()
            rgba, depth, st = O.render(sc)
        out = {"rgba": rgba}
        if depth is not None:
            out["depth"] = depth
        for k, v in st.items():
            if k != "ms":
                out["stat_" + k] = np.uint64(v)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print(name, rgba.shape, {k: v for k, v in st.items() if k != "ms"})


if __name__ == "__main__":
    main()
