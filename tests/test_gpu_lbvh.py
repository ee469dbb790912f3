"""GPU LBVH builder (rt_lbvh_build_gpu / rt_lbvh_build_async): node-for-node
bit-identical to the oracle's restatement of LBVH::ConstructLBVH_Buff (lbvh.h:215-269,
oracle/rt_oracle_host.c via O.lbvh_build), and to the host product builder (rt_lbvh_build).
Edge cases: N = 1 and 2, duplicate
centroids (equal Morton codes: the chain the reference's index-ordered merge builds), a
degenerate scene (every box identical, scene extent 0), signed zeros, and the INW presets'
own boxes, up to N = 200k."""
import numpy as np
import pytest

import rt_amd as R
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _boxes(n, seed, dup=0.0, flat=False):
    rng = np.random.default_rng(seed)
    c = rng.uniform(-50, 50, (n, 3)).astype(np.float32)
    if dup:
        k = max(1, int(n * (1 - dup)))
        c = c[rng.integers(0, k, n)]
    r = rng.uniform(0.1, 0.4, (n, 1)).astype(np.float32)
    if flat:
        r[:] = 0.25
    return np.concatenate([c - r, c + r], axis=1).astype(np.float32)


def _same(a, b):
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


CASES = [
    ("n1", _boxes(1, 1)),
    ("n2", _boxes(2, 2)),
    ("n3", _boxes(3, 3)),
    ("n17", _boxes(17, 4)),
    ("n500", _boxes(500, 5)),
    ("n10k", _boxes(10_000, 6)),
    ("n200k", _boxes(200_000, 7)),
    ("dup50", _boxes(5000, 8, dup=0.5)),
    ("dup99", _boxes(3000, 9, dup=0.99)),
    ("same_box", np.tile(np.array([[1, 2, 3, 2, 3, 4]], np.float32), (257, 1))),
    ("signed_zero", np.array([[-0.0, 0, 0, 1, 1, 1], [0, -0.0, 0, 1, 1, 1], [0.0, 0, -0.0, 2, 2, 2],
                              [-1, -1, -1, -0.0, -0.0, -0.0], [-1, 0, -1, 0.0, 1, 0.0]], np.float32)),
]


@pytest.mark.parametrize("name,boxes", CASES, ids=[c[0] for c in CASES])
def test_gpu_lbvh_equals_oracle(gpu, name, boxes):
    ref = O.lbvh_build(boxes)
    dev, ms = R.lbvh_build_gpu(boxes)
    bad = np.argwhere(~(ref.view(np.uint32) == dev.view(np.uint32)).all(axis=1))
    assert _same(ref, dev), f"{len(bad)} nodes differ from the oracle, first {bad[:5].ravel().tolist()}"
    assert _same(R.lbvh_build(boxes), dev)  # and the host product builder agrees


@pytest.mark.parametrize("preset,seed,n_hint", [(R.PRESET_INW01_RANDOM, 1234, 10_000),
                                                (R.PRESET_INW01_GRID, 0, 0),
                                                (R.PRESET_INW04_CORNELL, 7, 0)])
def test_gpu_lbvh_on_preset_scenes(gpu, preset, seed, n_hint):
    sc = R.make_scene(preset, seed, n_hint)
    dev, _ = R.lbvh_build_gpu(sc.aabbs)
    assert _same(O.lbvh_build(sc.aabbs), dev)
