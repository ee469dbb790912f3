"""GPU parity of the simple In-One-Weekend stages and of INW-01's MULTIFOCUS branch (SURVEY
8f4): the HIP kernels through the C ABI against the CPU oracle and the golden fixtures.  Same
bar as tests/test_gpu_parity.py: bit-identical images (NaN == NaN) and identical counters."""
import os

import numpy as np
import pytest

import rt_amd as R
import stages as S
from cases import TOL, compare
from oracle import oracle as O

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
COUNTERS = ("segments", "node_visits", "prim_tests", "shadow_queries", "stack_drops", "nan_drops")


def _exact(name, g, o):
    c = compare(g, o)
    print(name, c)
    assert c["nan_mismatch"] == 0 and c["max_abs"] <= TOL, c
    assert c["exact_frac"] == 1.0, c


@pytest.mark.parametrize("wh", [(100, 100), (7, 5), (1920, 1080), (1, 9)])
def test_iow00_matches_oracle(gpu, wh):
    p = S.iow00_params(*wh)
    _exact("iow00", R.render_iow00(p), O.render_iow00(p))


@pytest.mark.parametrize("wide", ["1", "0"])
@pytest.mark.parametrize("name", sorted(S.IOW02_CASES) + sorted(S.MF_CASES))
def test_stage_matches_oracle(gpu, name, wide):
    if name in S.IOW02_CASES and wide == "0":
        pytest.skip("inw_wide_walk only switches the INW walk")
    with R.options(inw_wide_walk=int(wide)):  # the MULTIFOCUS cases run the INW kernels
        g, gd, gst = S.render_gpu(name)
    o, od, ost = S.render_oracle(name)
    _exact(name, g, o)
    if gd is not None:
        _exact(name + ":depth", gd, od)
    print(name, "gpu", {k: gst[k] for k in COUNTERS}, "cpu", {k: ost[k] for k in COUNTERS})
    own = name in S.MF_CASES and wide == "1"  # the wide walk counts its own nodes and primitives
    for k in COUNTERS:
        if not (own and k in ("node_visits", "prim_tests")):
            assert gst[k] == ost[k], (k, gst[k], ost[k])


@pytest.mark.parametrize("name", S.GOLDEN_STAGE_CASES)
def test_stage_matches_golden(gpu, name):
    gold = np.load(os.path.join(GOLDEN, name + ".npz"))
    g, gd, _ = S.render_gpu(name)
    _exact(name, g, gold["rgba"])
    if gd is not None and "depth" in gold:
        _exact(name + ":depth", gd, gold["depth"])


def test_iow02_tile_rect(gpu):
    """u_TileIndex-style rectangles: a tile render writes only its rectangle, identically."""
    c = S.IOW02_CASES["iow02_rotated"]()
    full, _ = R.render_iow02(c["types"], c["records"], c["camera"], c["params"], 0, 1)
    p = c["params"]
    p.tile_x0, p.tile_y0, p.tile_w, p.tile_h = 30, 10, 40, 25
    part, _ = R.render_iow02(c["types"], c["records"], c["camera"], p, 0, 1)
    assert np.array_equal(part[10:35, 30:70], full[10:35, 30:70])
    assert (part[:10] == 0).all() and (part[:, :30] == 0).all()
