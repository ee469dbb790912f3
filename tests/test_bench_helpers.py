"""bench.py's host-side helpers (no GPU): the tile deals of the multi-rank path and the
`parity` field that compares the timed frame's block with the CPU baseline's oracle render."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def test_deal_order_is_a_permutation():
    nx, ny = 120, 68  # 1920 x 1080 in 16 x 16 tiles (the last row ragged)
    one = bench.deal_order(nx, ny, 1)
    assert one == [(tx, ty) for ty in range(ny) for tx in range(nx)]
    for world in (2, 4, 8):
        d = bench.deal_order(nx, ny, world)
        assert sorted(d) == sorted(one)
        # a row-major round robin would hand rank r whole tile columns (120 % 8 == 0): the hash
        # spreads every rank over most columns
        for r in range(world):
            cols = {tx for tx, _ in d[r::world]}
            assert len(cols) > nx // 2


def test_tiles_for_rank_cover_the_frame_once():
    W, H = 1920, 1080
    for world in (1, 3, 8):
        got = []
        for r in range(world):
            order, mine, per = bench.tiles_for_rank(W, H, world, r, 16)
            assert len(mine) <= per
            got += mine
        assert sorted(got) == sorted(order)


def test_lpt_deal_balances_and_assigns_every_tile():
    rng = np.random.default_rng(3)
    nx, ny, world = 30, 17, 8
    costs = rng.pareto(1.5, nx * ny) * 100.0
    lists = bench.lpt_deal(costs, nx, ny, world)
    flat = [t for lst in lists for t in lst]
    assert sorted(flat) == sorted((i % nx, i // nx) for i in range(nx * ny))
    loads = [sum(costs[ty * nx + tx] for tx, ty in lst) for lst in lists]
    # LPT: the spread between ranks is at most the largest single tile
    assert max(loads) - min(loads) <= costs.max() + 1e-9


def test_block_parity_bits_and_nans():
    rect = (2, 1, 4, 3)
    ref = np.random.default_rng(0).random((6, 8, 4), dtype=np.float32)
    img = ref.copy()
    p = bench.block_parity(rect, ref, None, img, None)
    assert p["exact_frac"] == 1.0 and p["max_abs"] == 0.0 and p["pixels"] == 12 and not p["depth"]
    img[1, 2, 0] = np.nextafter(img[1, 2, 0], np.float32(2.0))  # one ulp inside the block
    img[0, 0, 0] += 1.0                                       # outside the block: not compared
    ref_d = np.zeros((6, 8), np.float32)
    ref_d[2, 3] = np.nan
    dep = ref_d.copy()                                        # NaN == NaN
    p = bench.block_parity(rect, ref, ref_d, img, dep)
    assert p["depth"] and p["nan_mismatch"] == 0
    assert p["exact_frac"] == (12 * 4 + 12 - 1) / (12 * 4 + 12)
    assert 0.0 < p["max_abs"] < 1e-6
    dep[2, 3] = 0.0
    assert bench.block_parity(rect, ref, ref_d, img, dep)["nan_mismatch"] == 1


def test_refine_deal_moves_cheap_tiles_off_slow_ranks():
    rng = np.random.default_rng(5)
    nx, ny, world = 24, 12, 4
    costs = rng.uniform(1.0, 2.0, nx * ny)
    costs[5 * nx + 7] = 80.0  # one heavy tile (a long chain) on whichever rank holds it
    order = bench.deal_order(nx, ny, world)
    lists = [order[r::world] for r in range(world)]
    heavy = (7, 5)
    hr = next(r for r in range(world) if heavy in lists[r])
    load = [sum(costs[ty * nx + tx] for tx, ty in lst) for lst in lists]
    times = [ld * (1.3 if r == hr else 1.0) for r, ld in enumerate(load)]  # the heavy rank runs slower per ray
    new = bench.refine_deal(lists, costs, times, nx)
    flat = sorted(t for lst in new for t in lst)
    assert flat == sorted(order)
    assert heavy in new[hr]  # the heavy tile stays where it was measured
    k = [tm / ld for tm, ld in zip(times, load)]
    pred = [k[r] * sum(costs[ty * nx + tx] for tx, ty in new[r]) for r in range(world)]
    assert max(pred) / min(pred) < 1.05 < max(times) / min(times)  # 2.3x apart before
    # deterministic: the same inputs give the same lists on every rank
    assert bench.refine_deal(lists, costs, times, nx) == new
    assert new != lists  # unbalanced shares: the refined deal differs from the hashed one


def test_refine_deal_keeps_a_balanced_deal():
    nx, ny, world = 24, 12, 4
    costs = np.ones(nx * ny)
    order = bench.deal_order(nx, ny, world)
    lists = [order[r::world] for r in range(world)]
    times = [float(len(lst)) for lst in lists]  # every rank at the same time per ray
    assert bench.refine_deal(lists, costs, times, nx) == [list(lst) for lst in lists]


def test_opt_rejects_unknown_fields(monkeypatch):
    """bench.py --opt names an rt_options field or exits (a ctypes Structure accepts any name)."""
    import pytest
    monkeypatch.setattr(sys, "argv", ["bench.py", "--opt", "inw_wide_wlak=0", "--steps", "1"])
    monkeypatch.setenv("WORLD_SIZE", "1")

    class Stop(Exception):
        pass

    def no_device(*a, **k):
        raise Stop()
    monkeypatch.setattr(bench.torch.cuda, "set_device", lambda *a: None)
    monkeypatch.setattr(bench.R, "get_options", lambda: bench.R.RtOptions())
    monkeypatch.setattr(bench.R, "load", lambda *a: None)
    monkeypatch.setattr(bench.R, "set_options", no_device)
    with pytest.raises(SystemExit, match="inw_wide_wlak"):
        bench.main()
