"""A CPU model of k_inw_pm's wave scheduler (raytracing-tests_amd/csrc/rt_kernels.hip, k_inw_pm):
pixel claims at most 64 ordinals ahead of the fold, issue of stream entries g = (pixel ordinal,
sample) to free lanes within the fold window, the LDS ring's finished-entry rule (every issued
entry below the smallest one a busy lane holds is stored), the in-order fold (01_BVH...glsl:
625-653's End() sum order) and the pixel store when its last sample is folded.

Several waves share one claim counter; sample lengths are drawn at random (mostly one segment,
a few very long: stragglers that hold the window). The model checks what the kernel's exactness
rests on: every pixel's samples are folded in sample order, every pixel is stored exactly once
with the right sum while its ordinal slot still holds it, and every wave terminates with its grid
drained.
"""
import random

import pytest

RING = 256  # kPmLdsRing


class Wave:
    def __init__(self, spp, rng, long_frac):
        self.spp, self.rng, self.long_frac = spp, rng, long_frac
        self.gi = self.ji = self.si = 0
        self.gf = self.jf = self.sf = 0
        self.nclaimed = 0
        self.qdone = False
        self.acc = None
        self.pix_slot = [None] * 64
        self.busy = [False] * 64
        self.g = [0] * 64
        self.left = [0] * 64
        self.ring = {}
        self.lane_js = {}

    def length(self):
        return self.rng.randint(20, 60) if self.rng.random() < self.long_frac else self.rng.randint(1, 2)

    def step(self, counter, total, out):
        spp = self.spp
        # fold: entries below the smallest one a busy lane holds are finished
        if self.gf != self.gi:
            held = [self.g[l] - self.gf for l in range(64) if self.busy[l]]
            n = min(min(held) if held else 1 << 30, self.gi - self.gf, 64)
            for k in range(n):
                e = self.gf + k
                val = self.ring.pop(e % RING)
                assert val[0] == e, "ring slot overwritten before its fold"
                j, s, v = val[1], val[2], val[3]
                assert (j, s) == (self.jf, self.sf), "fold out of order"
                self.acc = v if self.sf == 0 else self.acc + v
                self.sf += 1
                if self.sf == spp:
                    unit = self.pix_slot[self.jf & 63]
                    assert unit[0] == self.jf, "ordinal slot holds another pixel"
                    assert unit[1] not in out, "pixel stored twice"
                    out[unit[1]] = self.acc
                    self.sf = 0
                    self.jf += 1
            self.gf += n
        # claims: at most 64 ordinals ahead of the fold
        free = [l for l in range(64) if not self.busy[l]]
        if not self.qdone and free:
            lim = self.jf + 64
            need = min(self.ji + (self.si + len(free) - 1) // spp + 1, lim)
            if need > self.nclaimed:
                want = need - self.nclaimed
                base = counter[0]
                counter[0] += want
                got = want
                if base >= total:
                    got, self.qdone = 0, True
                elif base + want >= total:
                    got, self.qdone = total - base, True
                for r in range(got):
                    j = self.nclaimed + r
                    old = self.pix_slot[j & 63]  # the slot's previous pixel is stored
                    assert old is None or old[0] < self.jf, "slot reclaimed before its pixel was stored"
                    self.pix_slot[j & 63] = (j, base + r)
                self.nclaimed += got
        # issue within the window
        avail = RING - (self.gi - self.gf)
        left = (self.nclaimed - self.ji) * spp - self.si
        take = min(len(free), avail, left)
        for rank in range(take):
            l = free[rank]
            adv = self.si + rank
            q = adv // spp
            j, s = self.ji + q, adv - q * spp
            self.busy[l], self.g[l], self.left[l] = True, self.gi + rank, self.length()
            self.lane_js[l] = (j, s)
        self.gi += take
        a2 = self.si + take
        self.ji += a2 // spp
        self.si = a2 % spp
        if self.qdone and self.ji == self.nclaimed and self.gf == self.gi and not any(self.busy):
            return False
        # one segment per busy lane; a finished sample stores its value
        for l in range(64):
            if self.busy[l]:
                self.left[l] -= 1
                if self.left[l] == 0:
                    j, s = self.lane_js[l]
                    e = self.g[l]
                    assert e % RING not in self.ring, "ring slot still unfolded"
                    self.ring[e % RING] = (e, j, s, value(self.pix_slot[j & 63][1], s))
                    self.busy[l] = False
        return True


def value(unit, s):
    return (unit * 7919 + s * 104729) % 1000003


@pytest.mark.parametrize("spp,units,waves,long_frac,seed", [
    (37, 64 * 8, 3, 0.02, 1),
    (500, 64 * 2, 2, 0.01, 2),     # a pixel's samples span more than the ring window
    (1, 64 * 6, 4, 0.3, 3),        # more than 64 pixels per window
    (3, 64 * 5, 3, 0.5, 4),
    (64, 64 * 3, 5, 0.05, 5),      # more waves than rows per wave
    (7, 64 * 9, 4, 0.2, 7),
])
def test_pixel_major_scheduler_model(spp, units, waves, long_frac, seed):
    rng = random.Random(seed)
    counter = [0]
    out = {}
    ws = [Wave(spp, rng, long_frac) for _ in range(waves)]
    live = list(ws)
    for _ in range(10_000_000):
        if not live:
            break
        w = live[rng.randrange(len(live))]  # waves interleave in any order
        if not w.step(counter, units, out):
            live.remove(w)
    assert not live, "a wave did not terminate"
    assert sorted(out) == list(range(units))
    for u, a in out.items():
        want = 0
        for s in range(spp):
            want = value(u, s) if s == 0 else want + value(u, s)
        assert a == want
