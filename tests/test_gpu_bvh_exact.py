"""Full-frame exactness of the IOW-03 kernel's execution strategies against each other.

- iow_linear=1: the reference's linear object loop instead of the culling BVH;
- iow_narrow=1: the byte-bounce stack layout (12-deep BVH stack) instead of the 9-float one;
- rounds_spec / rounds_seq=0/6:   no tail compaction (no parking / resume launches) / six compaction rounds
  per pass (default 1 on the sample-parallel path);
- spec_solo=0/10^5:  the re-run pass's longest samples share waves / take a wave each up to the
  resident wave count (default 4096, clamped to the 3072 resident waves on MI355X; DESIGN.md
  "Solo head");
- iow_spec=0:   the sequential per-pixel kernel instead of sample-parallel speculation;
- spec_iters=0/3/10: other numbers of resolve passes (default 1), more pixels finished by the sequential kernel (which
  takes the still-exact records; spec_validate=0 re-runs every sample from the first bad one);
- spec_prior_from: from which sample on the scene's RI prior is guessed for entries sample 0
  left unwritten (default 2; 10^6 = never, with the former 10 re-run passes);
- spec_tail_rounds=0/3: no budgeted tail rounds (the round-1 default) / three, with
  spec_tail_budget segments per unit and round (default 60 rounds of 3072);
- spec_scan=0/4: no anchored scan past the frontier (default 128 samples; DESIGN.md
  "Anchored scan") / a short one;
- spec_chain=0: exact restarts stop after their own sample (default: they go on down the
  pixel's chain of mispredicted samples);
- spec_alt=0 / spec_alt_seg small: no alternative runs / alternatives for almost every
  sample that read a stale entry (default 16384 segments), so adoption runs often;
- spec_rounds=k: the speculative pass as k checkpoint rounds (default 24; 0 = one launch)
  with pixel frontiers and immediate exact re-runs of mispredicted samples;
- iow_lds_bvh=0: the BVH read from global memory instead of staged in LDS (768-lane blocks);
- iow_coop_max=0/64: no wave-cooperative closest hits / every closest hit wave-cooperative (default:
  waves with at most 4 tracing lanes);
- a scene with 12 distinct refractive indices (more than the 8 alternative-run values the
  speculation tracks, DESIGN.md "Alternative runs"), default against the sequential kernel;
- INW: inw_order=1/2 (the pixel- / sample-major on-chip fold instead of the probe's pick, with
  small fold windows inw_ring_pm / inw_ring_sm), inw_order=-1 (the per-pixel sequential
  kernel k_inw), inw_lds_nodes=0 (no LDS-staged BVH top) and inw_wide_walk=0 (the reference's LBVH walk
  instead of the wide walk; images and ray counts equal).
Each must give a bit-identical image of the final scene with identical ray counts.  The
switches are rt_options fields set through the C ABI (R.options) around each render."""
import numpy as np
import pytest

import rt_amd as R

pytestmark = pytest.mark.gpu


def _scene(preset, seed, n_hint, w, h, spp, many_ri=False):
    sc = R.make_scene(preset, seed, n_hint, width=w, height=h, spp=spp)
    if many_ri:  # 12 distinct refractive indices over a third of the objects
        for i in range(sc.n):
            if i % 3 == 0 and sc.desc[i].type == R.RT_IOW_ELLIPSOID:
                sc.desc[i].refractivity = 0.9
                sc.desc[i].refractive_index = 1.1 + 0.07 * (i % 12)
        for k, v in R.pack(sc.desc, sc.n, sc.stage).items():
            setattr(sc, k, v)
    return sc


IOW = (2, 20250131, 0)     # PRESET_IOW03_FINAL
INW1 = (4, 1234, 3000)     # PRESET_INW01_RANDOM, 3000 objects
INW4 = (6, 7, 0)           # PRESET_INW04_CORNELL
IOW_RI = (2, 20250131, 0, True)  # the final scene with 12 distinct refractive indices


def _render(over, w, h, spp, scene=IOW):
    """Render `scene` with the default options changed by `over` (rt_options fields); colour and
    depth stacked as (H, W, 4 or 5)."""
    sc = _scene(scene[0], scene[1], scene[2], w, h, spp, len(scene) > 3 and scene[3])
    with R.options(**{**R.default_options().as_dict(), **over}):
        img, depth, st = R.render(sc)
    if depth is not None:
        img = np.concatenate([img, depth[..., None]], axis=2)
    return img, st


@pytest.mark.parametrize("over,w,h,spp", [
    ({"iow_linear": 1}, 600, 400, 2),
    ({"iow_linear": 1}, 1200, 800, 1),
    ({"iow_narrow": 1}, 600, 400, 8),
    ({"rounds_seq": 0, "rounds_spec": 0}, 600, 400, 8),
    ({"iow_chunks_lpt": 1, "iow_spec": 0}, 300, 200, 24),
    ({"iow_spec": 0}, 600, 400, 8),
    ({"spec_iters": 0}, 300, 200, 16),
    ({"spec_iters": 1}, 300, 200, 16),
    ({"spec_iters": 0, "spec_validate": 0}, 300, 200, 16),
    ({"spec_iters": 10, "spec_prior_from": 1000000}, 300, 200, 16),
    ({"spec_iters": 3, "spec_prior_from": 1}, 600, 400, 12),
    ({"iow_coop_max": 0}, 600, 400, 8),
    ({"iow_lds_bvh": 0}, 600, 400, 8),
    ({"spec_rounds": 0}, 600, 400, 12),
    ({"spec_rounds": 8}, 600, 400, 12),
    ({"spec_rounds": 24, "spec_prior_from": 1}, 300, 200, 16),
    ({"spec_rounds": 5}, 300, 200, 9),
    ({"iow_lds_bvh": 0, "iow_spec": 0}, 300, 200, 8),
    ({"iow_coop_max": 64}, 300, 200, 4),
    ({"iow_coop_max": 64, "iow_spec": 0}, 300, 200, 4),
    ({"iow_coop_max": 64, "iow_linear": 1}, 200, 100, 2),
    ({"spec_iters": 2}, 300, 200, 16),
    ({"rounds_seq": 6, "rounds_spec": 6}, 600, 400, 12),
    ({"spec_solo": 0}, 600, 400, 12),
    ({"spec_solo": 100000, "spec_iters": 2}, 300, 200, 16),
    ({"spec_heavy": 0}, 300, 200, 16),
    ({"spec_tail_rounds": 0}, 600, 400, 12),
    ({"spec_scan": 0}, 600, 400, 12),
    ({"spec_chain": 0}, 600, 400, 12),
    ({"spec_alt": 0}, 600, 400, 12),
    ({"spec_alt_seg": 8, "spec_alt_every": 1, "spec_tail_budget": 64}, 300, 200, 24),
    ({"spec_alt_seg": 1, "spec_alt_every": 2, "spec_tail_budget": 16, "spec_rounds": 4, "spec_prior_from": 1}, 200, 100, 40),
    ({"spec_chain": 0, "spec_scan": 0}, 300, 200, 24),
    ({"spec_scan": 4, "spec_tail_budget": 32}, 300, 200, 24),
    ({"spec_scan": 1000, "spec_tail_budget": 16, "spec_rounds": 6}, 200, 100, 40),
    ({"spec_tail_rounds": 3, "spec_tail_budget": 64}, 300, 200, 16),
    ({"spec_tail_rounds": 40, "spec_tail_budget": 16, "spec_rounds": 3}, 300, 200, 16),
])
def test_strategies_bit_identical(gpu, over, w, h, spp):
    _same_frames(over, w, h, spp, IOW)


@pytest.mark.parametrize("over,w,h,spp", [
    ({"iow_spec": 0}, 300, 200, 24),
    ({"spec_alt_seg": 8, "spec_alt_every": 1, "spec_tail_budget": 64}, 300, 200, 24),
])
def test_many_refractive_indices_bit_identical(gpu, over, w, h, spp):
    """More distinct RIs than the alternative runs track: speculation must stay exact."""
    _same_frames(over, w, h, spp, IOW_RI)


def _same_frames(over, w, h, spp, scene):
    a, sa = _render({}, w, h, spp, scene)
    b, sb = _render(over, w, h, spp, scene)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    bad = np.argwhere(~same.all(axis=2))
    print("mismatching pixels:", len(bad), bad[:10].tolist())
    print("default", sa, over, sb)
    assert len(bad) == 0
    for k in ("segments", "stack_drops", "nan_drops"):
        assert sa[k] == sb[k], k


@pytest.mark.parametrize("over,scene,w,h,spp", [
    ({"inw_order": -1}, INW1, 192, 108, 24),     # the per-pixel sequential kernel k_inw
    ({"inw_order": 1}, INW1, 200, 100, 37),       # pixel-major fold, spp not a multiple of the wave
    ({"inw_order": 2}, INW1, 200, 100, 37),       # sample-major fold
    ({"inw_order": 1}, INW1, 160, 96, 1),         # more than 64 pixels per fold window
    ({"inw_order": 2}, INW1, 160, 96, 1),
    ({"inw_order": 1}, INW1, 97, 43, 3),          # ragged 8x8 units (padding samples)
    ({"inw_order": 2}, INW1, 97, 43, 3),
    ({"inw_order": 1, "inw_ring_pm": 64}, INW1, 128, 72, 300),  # a window smaller than a pixel
    ({"inw_order": 1, "inw_ring_pm": 1024}, INW1, 128, 72, 300),  # the global ring (default: LDS)
    ({"inw_order": 1, "inw_ring_pm": 1024}, INW4, 128, 128, 16),
    ({"inw_order": 2, "inw_ring_sm": 64}, INW1, 128, 72, 20),   # a window of one sample row
    ({"inw_order": 2, "inw_ring_sm": 256}, INW4, 128, 128, 16),  # global ring (default here: LDS)
    ({"inw_order": 2, "inw_ring_sm": 64}, INW4, 97, 43, 300),    # a small global window, ragged units
    ({"inw_order": -1}, INW4, 128, 128, 16),
    ({"inw_order": 1}, INW4, 128, 128, 16),
    ({"inw_order": -1, "inw_wide_walk": 0}, INW4, 96, 96, 8),
    ({"inw_order": -1}, INW4, 96, 96, 12),
    ({"inw_wide_walk": 0}, INW1, 480, 270, 16),          # the reference's LBVH walk
    ({"inw_wide_walk": 0}, INW4, 256, 256, 12),
    ({"inw_wide_walk": 0, "inw_order": -1}, INW1, 192, 108, 24),
    ({"inw_lds_nodes": 0}, INW1, 192, 108, 24),          # every wide node from global memory
    ({"inw_lds_nodes": 0, "inw_order": 2}, INW4, 128, 128, 16),
    # the per-frame shortcuts of the pixel-major kernel, each off (INW4 forced pixel-major)
    ({"inw_beams": 0}, INW1, 192, 108, 24),
    ({"inw_beams": 2}, INW1, 192, 108, 24),              # (id, t) pairs (default: 32-bit entries)
    ({"inw_fused_cull": 0}, INW1, 192, 108, 24),
    ({"inw_ri_grid": 0}, INW1, 192, 108, 24),
    ({"inw_claim_order": 0}, INW1, 192, 108, 24),
    ({"inw_claim_xcd": 0}, INW1, 192, 108, 24),          # one claim queue (default: one per XCD)
    ({"inw_claim_xcd": 0, "inw_claim_order": 0}, INW1, 97, 43, 7),
    # k_inw_pm's GQ instance (the 40-float stacks in global memory, the walk's node stack and the
    # top of the culling BVH in LDS, quantised nodes) against the default FStack instance
    ({"inw_qnodes": 1}, INW1, 192, 108, 24),
    ({"inw_qnodes": 1, "inw_order": 1}, INW1, 97, 43, 7),
    ({"inw_qnodes": 1, "inw_order": 1}, INW1, 160, 96, 300),
    # time-bin culling trees (default 4 for moving objects) against the swept tree alone, other
    # bin counts (uneven sample splits, more bins than some spp), and the kernels that use them
    ({"inw_time_bins": 0}, INW1, 192, 108, 24),
    ({"inw_time_bins": 3}, INW1, 97, 43, 7),
    ({"inw_time_bins": 16, "inw_order": -1}, INW1, 160, 96, 37),
    ({"inw_time_bins": 5, "inw_lds_nodes": 0}, INW1, 128, 72, 300),
    ({"inw_time_bins": 0, "inw_order": 2}, INW1, 200, 100, 37),
    ({"inw_time_bins": 2, "inw_ring_pm": 1024}, INW1, 128, 72, 40),
    ({"inw_beam_bins": 0}, INW1, 192, 108, 24),          # one beam list per pixel, bin trees for the walks
    ({"inw_walk_bins": 0}, INW1, 97, 43, 7),             # beam lists per bin, the swept tree for the walks
    ({"inw_walk_bins": 0, "inw_time_bins": 7}, INW1, 160, 96, 300),
    # the 7-float4 object records against the 2-float4 sphere records (default for sphere scenes)
    ({"inw_sphere_records": 0}, INW1, 192, 108, 24),
    ({"inw_sphere_records": 0, "inw_order": 2}, INW1, 200, 100, 37),
    ({"inw_sphere_records": 0, "inw_order": -1, "inw_beams": 2}, INW1, 97, 43, 7),
    # the buffer-load walk's 10-float4 nodes against the 7-float4 copy (default)
    ({"inw_compact_nodes": 0}, INW1, 192, 108, 24),
    ({"inw_compact_nodes": 0, "inw_lds_nodes": 0, "inw_order": 2}, INW4, 128, 128, 16),
    ({"inw_beams": 0, "inw_order": 1}, INW4, 128, 128, 16),
    ({"inw_fused_cull": 0, "inw_order": 1}, INW4, 128, 128, 16),
    ({"inw_ri_grid": 0, "inw_order": 1}, INW4, 128, 128, 16),
    ({"inw_claim_order": 0, "inw_order": 1}, INW4, 128, 128, 16),
])
def test_inw_strategies_bit_identical(gpu, over, scene, w, h, spp):
    a, sa = _render({}, w, h, spp, scene)
    b, sb = _render(over, w, h, spp, scene)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), np.argwhere(~same.all(axis=2))[:10].tolist()
    # the wide walk's node and primitive counts depend on which rays share a wave (postponed
    # leaves are tested together), so only the ray-level counters must agree
    for k in ("segments", "shadow_queries", "stack_drops", "nan_drops"):
        assert sa[k] == sb[k], k


@pytest.mark.parametrize("over,scene,w,h,spp", [
    ({}, INW1, 160, 90, 12),                       # pixel-major fold (k_inw_pm, LDS ring: no staged nodes)
    ({"inw_order": 2}, INW1, 160, 90, 12),          # sample-major fold (1,180 LBVH nodes in LDS)
    ({"inw_order": -1}, INW1, 160, 90, 12),         # the per-pixel kernel (no LDS staging)
    ({"inw_lds_nodes": 0}, INW1, 160, 90, 12),      # 256-lane instances, every node from global memory
    ({"inw_order": 1}, INW4, 96, 96, 10),           # INW-04: shadow rays, RI walks
    ({"inw_order": 2}, INW4, 96, 96, 10),
])
def test_stackless_walk_equals_stack_walk(gpu, over, scene, w, h, spp):
    """The stackless LBVH walks (rt_options.inw_stackless) against the reference's
    stack walks with the wide walk off: the same image and depth, and -- since they visit the
    same nodes in the same order -- the same node visits and object tests as well as the ray
    counters, all equal to the oracle's."""
    from oracle import oracle as O
    base = {"inw_wide_walk": 0, **over}
    a, sa = _render({**base, "inw_stackless": 0}, w, h, spp, scene)
    b, sb = _render({**base, "inw_stackless": 1}, w, h, spp, scene)
    same = (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))
    assert same.all(), np.argwhere(~same.all(axis=2))[:10].tolist()
    sc = _scene(scene[0], scene[1], scene[2], w, h, spp)
    _, _, so = O.render(sc)
    for k in ("segments", "node_visits", "prim_tests", "shadow_queries", "stack_drops", "nan_drops"):
        assert sa[k] == sb[k] == so[k], (k, sa[k], sb[k], so[k])
    # the path report of a device scene built with those options (inw_wide_walk is a [build] option)
    import ctypes as C

    import torch
    sc = _scene(scene[0], scene[1], scene[2], w, h, spp)
    lib = R.load()
    with R.options(**{**R.default_options().as_dict(), **base, "inw_stackless": 1}):
        s = lib.rt_dev_scene_inw(R.fptr(sc.geom), sc.n, sc.layout, R.fptr(sc.nodes),
                                 R.fptr(sc.lights if sc.n_lights else None), sc.n_lights, spp, -1)
    assert s
    try:
        img = torch.zeros((h, w, 4), dtype=torch.float32, device="cuda")
        ctr = torch.zeros(6, dtype=torch.int64, device="cuda")
        assert lib.rt_render_image_async(s, C.byref(sc.camera), C.byref(sc.params), img.data_ptr(), None,
                                         ctr.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        path = R.debug_path(s)
    finally:
        lib.rt_dev_scene_free(s)
    print(over, path)
    assert path["stackless"] == 1 and path["wide_walk"] == 0
