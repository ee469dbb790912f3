"""Host build of the time-bin culling trees and the sphere records, on the CPU
through the C ABI's test hooks: every bin tree holds every object once, its boxes nest, each
object's bin box holds the object at every time ratio of the bin (evaluated in float32 as the
kernels evaluate it), and the sphere records are the hot record's own floats."""
import ctypes as C

import numpy as np
import pytest

import rt_amd as R


def _time_bins(sc, bins):
    lib = R.load()
    info = (C.c_uint32 * 4)()
    nodes = np.ascontiguousarray(sc.nodes, np.float32)
    geom = np.ascontiguousarray(sc.geom, np.float32)
    assert lib.rt_debug_time_bins(R.fptr(nodes), R.fptr(geom), sc.n, bins, None, 0, info) == 0
    n0, nb, stride, total = list(info)
    out = np.zeros(total * 40, np.float32)
    assert lib.rt_debug_time_bins(R.fptr(nodes), R.fptr(geom), sc.n, bins, R.fptr(out), total, info) == 0
    return n0, nb, stride, total, out.reshape(total, 40)


def _links(node):
    return node[36:40].view(np.int32)


def _walk(wn, root, n):
    """Objects reached from `root` (each must appear once), checking that every child's own planes
    lie inside its slot in the parent."""
    seen = np.zeros(n, np.int32)
    stack = [root]
    while stack:
        cur = stack.pop()
        nd = wn[cur - 1]
        for k, l in enumerate(_links(nd)):
            if l == 1000000000:
                continue  # empty slot
            lo = nd[[0 + k, 4 + k, 8 + k]]
            hi = nd[[12 + k, 16 + k, 20 + k]]
            assert (lo <= hi).all()
            if l > 0:
                ch = wn[l - 1]
                for j, cl in enumerate(_links(ch)):
                    if cl == 1000000000:
                        continue
                    assert (ch[[0 + j, 4 + j, 8 + j]] >= lo).all() and (ch[[12 + j, 16 + j, 20 + j]] <= hi).all()
                stack.append(int(l))
            else:
                seen[-l] += 1
    return seen


@pytest.mark.parametrize("bins", [2, 3, 4])
def test_time_bin_trees(bins):
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 600, width=8, height=8, spp=1)
    n0, nb, stride, total, wn = _time_bins(sc, bins)
    assert nb == bins and total == n0 + bins * stride and 1 <= n0 <= sc.n
    # the swept tree and every bin tree hold every object exactly once
    assert (_walk(wn, 1, sc.n) == 1).all()
    for b in range(bins):
        assert (_walk(wn, 1 + n0 + b * stride, sc.n) == 1).all(), b
    # static scenes get no bins
    st = R.make_scene(R.PRESET_INW04_CORNELL, 7, 0, width=8, height=8, spp=1)
    assert _time_bins(st, bins)[1] == 1


@pytest.mark.parametrize("bins", [2, 4, 7])
def test_bin_boxes_hold_the_objects(bins):
    """The object at every time ratio of its bin (the kernels' float32 arithmetic: centre
    p - delta * (1 - r), r = s * (1/spp)) lies inside its bin box, with its radius (equal-scale
    unrotated ellipsoids), and the bin box is no larger than the swept box by more than the margin."""
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 99, 400, width=8, height=8, spp=1)
    g = sc.geom.astype(np.float32)
    pos, scale, delta = g[:, 0:3], g[:, 12:15], g[:, 15:18]
    lib = R.load()
    spp = 500
    inv = np.float32(1.0) / np.float32(spp)
    ratio = np.arange(spp, dtype=np.float32) * inv
    for b in range(bins):
        boxes = np.zeros((sc.n, 6), np.float32)
        assert lib.rt_debug_bin_boxes(R.fptr(g), sc.n, bins, b, R.fptr(boxes)) == 0
        r = ratio[np.minimum((ratio * np.float32(bins)).astype(np.int32), bins - 1) == b]
        assert len(r)
        one_minus = (np.float32(1.0) - r)[:, None, None]
        c = pos[None] - delta[None] * one_minus  # (samples, objects, 3), float32
        assert (c - scale[None] >= boxes[None, :, 0:3]).all() and (c + scale[None] <= boxes[None, :, 3:6]).all()
        swept_lo = np.minimum(pos, pos - delta) - scale
        swept_hi = np.maximum(pos, pos - delta) + scale
        assert (boxes[:, 0:3] >= swept_lo - 0.05).all() and (boxes[:, 3:6] <= swept_hi + 0.05).all()


def test_sphere_records():
    lib = R.load()
    sc = R.make_scene(R.PRESET_INW01_RANDOM, 1234, 300, width=8, height=8, spp=1)
    g = np.ascontiguousarray(sc.geom, np.float32)
    out = np.zeros((sc.n, 12), np.float32)
    assert lib.rt_debug_sphere_records(R.fptr(g), sc.n, 1, R.fptr(out)) == 1
    assert (out[:, 0:3] == g[:, 0:3]).all() and (out[:, 4:7] == g[:, 15:18]).all()
    assert (out[:, 3] == np.float32(1.0) / g[:, 12]).all()  # the hot record's RN(1/scale)
    assert (out[:, 7] == g[:, 20]).all()  # the RI the surrounding-RI walk adds (layout 1)
    assert (out[:, 8:11] == np.float32(1.0) / (g[:, 12:15] * g[:, 12:15])).all() and (out[:, 11] == g[:, 19]).all()
    # a rotated object, unequal scales or a cuboid: no sphere records
    for col, val in ((4, 0.5), (13, 2.0 * g[0, 12]), (18, 2.0)):
        h = g.copy()
        h[0, col] = val
        assert lib.rt_debug_sphere_records(R.fptr(h), sc.n, 1, R.fptr(out)) == 0, col
    cb = R.make_scene(R.PRESET_INW04_CORNELL, 7, 0, width=8, height=8, spp=1)
    g4 = np.ascontiguousarray(cb.geom, np.float32)
    assert lib.rt_debug_sphere_records(R.fptr(g4), cb.n, 4, R.fptr(np.zeros((cb.n, 12), np.float32))) == 0
