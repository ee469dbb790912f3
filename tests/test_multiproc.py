"""Multi-GPU partition + exchange, rehearsed on the CPU with gloo (world size 2 and 3).

bench.py deals tiles round-robin to ranks (64x64 on one GPU, 16x16 across ranks in a hashed
order), each rank packs its tiles, one gather brings
them to rank 0, and rank 0 assembles the frame.  Here every rank "renders" a
deterministic per-pixel pattern into its packed tiles (the assembled frame must equal the
pattern everywhere, and the tile lists must cover every tile exactly once), and, with the CPU
oracle as the renderer, the tiles of real INW-01 / IOW-03 frames, whose assembly must equal the
single render bit for bit with the same summed ray count.
"""
import math
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bench


def _pattern(W, H):
    y, x = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    return torch.stack([x, y, x * 1000 + y, torch.ones_like(x)], -1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, W, H, T, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        allt, mine, per_rank = bench.tiles_for_rank(W, H, world, rank, T)
        ref = _pattern(W, H)
        packed = torch.zeros((per_rank, T, T, 4))
        for k, (tx, ty) in enumerate(mine):  # what rt_render_tiles_async writes: 0 outside the image
            y0, x0 = ty * T, tx * T
            blk = ref[y0:y0 + T, x0:x0 + T]
            packed[k, :blk.shape[0], :blk.shape[1]] = blk
        gathered = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
        dist.gather(packed, gathered, dst=0)
        if rank == 0:
            nx, ny = math.ceil(W / T), math.ceil(H / T)
            img = bench.assemble_frame(torch.stack(gathered, 0), allt, nx, ny)[:H, :W]
            q.put(bool(torch.equal(img, ref)))
    finally:
        dist.destroy_process_group()


def _worker_msg(rank, world, port, W, H, T, q):
    """bench.py's one gather message per rank: the colour tiles and their r32f depth tiles in one
    flat buffer (bench.message_views), assembled on rank 0 by bench.assemble_message."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        allt, mine, per_rank = bench.tiles_for_rank(W, H, world, rank, T)
        ref = _pattern(W, H)
        dref = ref[..., 2] * 0.5 + 7.0  # a depth pattern distinct from every colour channel
        msg = torch.zeros(per_rank * T * T * 5)
        col, dep = bench.message_views(msg, per_rank, T, True)
        for k, (tx, ty) in enumerate(mine):
            y0, x0 = ty * T, tx * T
            blk, dblk = ref[y0:y0 + T, x0:x0 + T], dref[y0:y0 + T, x0:x0 + T]
            col[k, :blk.shape[0], :blk.shape[1]] = blk
            dep[k, :dblk.shape[0], :dblk.shape[1]] = dblk
        gathered = [torch.empty_like(msg) for _ in range(world)] if rank == 0 else None
        dist.gather(msg, gathered, dst=0)
        if rank == 0:
            nx, ny = math.ceil(W / T), math.ceil(H / T)
            lists = [allt[r::world] for r in range(world)]
            img, dimg = bench.assemble_message(gathered, lists, nx, ny, per_rank, T, True)
            q.put(bool(torch.equal(img[:H, :W], ref)) and bool(torch.equal(dimg[:H, :W], dref)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,T", [(2, 200, 130, 16), (3, 200, 130, 16), (3, 97, 43, 64)])
def test_gather_message_assembles_colour_and_depth(world, W, H, T):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_msg, args=(r, world, port, W, H, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("world,W,H,T", [(2, 1200, 800, 16), (2, 1200, 800, 64), (3, 200, 130, 16),
                                         (3, 200, 130, 64), (2, 64, 64, 64)])
def test_gather_assembles_frame(world, W, H, T):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, W, H, T, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_tiles_cover_frame_once(world):
    W, H = 1200, 800
    T = bench.tile_for(world)
    assert T == (64 if world == 1 else 16)
    seen = []
    for r in range(world):
        allt, mine, per_rank = bench.tiles_for_rank(W, H, world, r, T)
        assert len(mine) <= per_rank
        seen += mine
    assert sorted(seen) == sorted(allt)
    assert len(set(seen)) == len(allt) == math.ceil(W / T) * math.ceil(H / T)


def test_deal_order_spreads_columns():
    """With 120 tiles per row (1920 px / 16) a row-major round-robin gives each of 8 ranks whole
    tile columns; the hashed deal order gives every rank tiles from every column band."""
    W, H, T, world = 1920, 1080, 16, 8
    for r in range(world):
        _, mine, _ = bench.tiles_for_rank(W, H, world, r, T)
        cols = {tx for tx, _ in mine}
        assert len(cols) > 100, (r, len(cols))


def test_lpt_deal_balances_and_assembles():
    """The LPT deal over measured tile costs covers every tile once, keeps the heaviest rank
    within one tile's cost of the mean, and assemble_lists puts uneven per-rank lists back."""
    W, H, T, world = 200, 130, 16, 3
    nx, ny = math.ceil(W / T), math.ceil(H / T)
    g = torch.Generator().manual_seed(5)
    costs = (torch.rand(nx * ny, generator=g) ** 4 * 1000).tolist()
    lists = bench.lpt_deal(costs, nx, ny, world)
    flat = sorted(t for lst in lists for t in lst)
    assert flat == sorted((tx, ty) for ty in range(ny) for tx in range(nx))
    loads = [sum(costs[ty * nx + tx] for tx, ty in lst) for lst in lists]
    assert max(loads) - sum(loads) / world <= max(costs)
    ref = _pattern(W, H)
    per = max(len(v) for v in lists)
    src = torch.zeros((world, per, T, T, 4))
    for r, lst in enumerate(lists):
        for k, (tx, ty) in enumerate(lst):
            blk = ref[ty * T:ty * T + T, tx * T:tx * T + T]
            src[r, k, :blk.shape[0], :blk.shape[1]] = blk
    assert torch.equal(bench.assemble_lists(src, lists, nx, ny)[:H, :W], ref)


def _render_worker(rank, world, port, T, case, q):
    """One rank of a rendered partition: this rank's tiles of a real frame (rendered by the CPU
    oracle, tile by tile, as the reference dispatches tile rectangles), packed as
    rt_render_tiles_async packs them, gathered to rank 0 and assembled there; the ray counters
    are summed over ranks as bench.py sums them."""
    import sys
    sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__)))]
    import numpy as np

    import rt_amd as R
    from oracle import oracle as O

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        O.set_threads(1)
        preset, seed, n, over = case
        sc = R.make_scene(preset, seed, n, **over)
        W, H = sc.params.width, sc.params.height
        allt, mine, per_rank = bench.tiles_for_rank(W, H, world, rank, T)
        packed = torch.zeros((per_rank, T, T, 4))
        seg = torch.zeros(1, dtype=torch.float64)
        for k, (tx, ty) in enumerate(mine):
            p = R.RtParams.from_buffer_copy(sc.params)
            p.tile_x0, p.tile_y0 = tx * T, ty * T
            p.tile_w, p.tile_h = min(T, W - tx * T), min(T, H - ty * T)
            img, _, st = O.render(sc, p)
            blk = torch.from_numpy(img[p.tile_y0:p.tile_y0 + p.tile_h, p.tile_x0:p.tile_x0 + p.tile_w].copy())
            packed[k, :blk.shape[0], :blk.shape[1]] = blk
            seg += st["segments"]
        gathered = [torch.empty_like(packed) for _ in range(world)] if rank == 0 else None
        dist.gather(packed, gathered, dst=0)
        dist.all_reduce(seg)
        if rank == 0:
            nx, ny = math.ceil(W / T), math.ceil(H / T)
            img = bench.assemble_frame(torch.stack(gathered, 0), allt, nx, ny)[:H, :W].numpy()
            full, _, fst = O.render(sc)
            q.put(bool(np.array_equal(img.view(np.uint32), full.view(np.uint32))) and int(seg.item()) == fst["segments"])
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,T,case", [
    (2, 16, ("INW", 1234, 3000, dict(width=72, height=40, spp=6))),
    (3, 16, ("IOW", 20250131, 0, dict(width=40, height=24, spp=3))),
])
def test_gather_of_rendered_tiles(world, T, case):
    """The multi-GPU exchange on rendered content: ranks render their dealt tiles of a real INW-01 /
    IOW-03 frame, one gather assembles the frame on rank 0, and it equals the single render bit
    for bit with the same ray count (CPU oracle as the renderer, gloo as the transport)."""
    import rt_amd as R
    preset = R.PRESET_INW01_RANDOM if case[0] == "INW" else R.PRESET_IOW03_FINAL
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_render_worker, args=(r, world, port, T, (preset,) + case[1:], q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs)
    assert q.get(timeout=5) is True
