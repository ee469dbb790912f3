"""Progressive tile order on the CPU: rt_tile_spiral against an independent
Python restatement of Adding_Materials::OnUpdate's spiral (materials.cpp:84-152, state widths
materials.h:110-116), and its coverage property: the dispatched rectangles tile the image
exactly once."""
import numpy as np
import pytest

import rt_amd as R


def _py_spiral(W, H, tw, th):
    mx0, mx1 = W // tw, H // th
    i0, i1 = int((np.float32(mx0) - np.float32(0.1)) / np.float32(2)), int((np.float32(mx1) - np.float32(0.1)) / np.float32(2))
    r00, r01, r10, r11 = [i0, i1], [i0, i1 + 1], [i0 + 1, i1 - 1], [i0 + 1, i1 + 1]
    step = [0, 0]
    out = []
    while min(i0, i1) < max(mx0, mx1) + 1:
        if [i0, i1] == r00:
            r00 = [r00[0] - 1, r00[1] - 1]; step = [0, 1]
        if [i0, i1] == r01:
            r01 = [r01[0] - 1, r01[1] + 1]; step = [1, 0]
        if [i0, i1] == r11:
            r11 = [r11[0] + 1, r11[1] + 1]; step = [0, -1]
        if [i0, i1] == r10:
            r10 = [r10[0] + 1, r10[1] - 1]; step = [-1, 0]
        if 0 <= i1 <= mx1 and 0 <= i0 <= mx0:
            out.append([i0, i1, W % tw if i0 >= mx0 else tw, H % th if i1 >= mx1 else th])
        i0, i1 = i0 + step[0], i1 + step[1]
    return out


SIZES = [(300, 300, 100, 100), (1200, 800, 100, 100), (1920, 1080, 100, 100), (4096, 4096, 128, 128),
         (50, 30, 100, 100), (1, 1, 1, 1), (333, 77, 32, 16), (801, 1, 8, 1)]


@pytest.mark.parametrize("W,H,tw,th", SIZES)
def test_spiral_matches_restatement(W, H, tw, th):
    got = R.tile_spiral(W, H, tw, th).tolist()
    assert got == _py_spiral(W, H, tw, th)


@pytest.mark.parametrize("W,H,tw,th", SIZES)
def test_spiral_covers_image_once(W, H, tw, th):
    cov = np.zeros((H, W), np.int32)
    for tx, ty, w, h in R.tile_spiral(W, H, tw, th):
        cov[ty * th:ty * th + h, tx * tw:tx * tw + w] += 1
    assert (cov == 1).all()


def test_spiral_starts_at_centre_tile():
    t = R.tile_spiral(1200, 800, 100, 100)
    assert tuple(t[0, :2]) == (5, 3)  # ((12 - 0.1) / 2, (8 - 0.1) / 2) truncated
    assert len({tuple(r[:2]) for r in t}) == len(t)
