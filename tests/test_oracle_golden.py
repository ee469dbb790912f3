"""The CPU oracle still reproduces the committed golden fixtures bit for bit (regression pin
of the checker itself; tests/golden/make_golden.py regenerates them)."""
import os

import numpy as np
import pytest

from cases import CASES, GOLDEN_CASES, compare, iow01_c1
from oracle import oracle as O

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_matches_golden(name):
    gold = np.load(os.path.join(GOLDEN, name + ".npz"))
    if name == "iow01_c1":
        cam, sph, p = iow01_c1()
        img, st = O.render_iow01(cam, sph, p)
    else:
        img, depth, st = O.render(CASES[name]())
        if "depth" in gold:
            assert compare(depth, gold["depth"])["exact_frac"] == 1.0
    c = compare(img, gold["rgba"])
    assert c["exact_frac"] == 1.0, c
    for k in gold.files:
        if k.startswith("stat_"):
            assert st[k[5:]] == int(gold[k]), k
