"""Texture producers on the CPU: the oracle's restatements of
Helper::Noise::MakeTexture (utility.h:69-192, utility.cpp:609-769) and of the Mercator <->
cubic re-projection (utility.cpp:266-463), plus the double-precision transcendentals both the
oracle and the GPU kernels use.

Parity is unpinned against the reference itself (its harness needs OpenGL + MSVC; MakeTexture
uploads straight to a GL texture).  The noise oracle is cross-checked here against a second,
pure-Python restatement written from the same source lines; the re-projection against its
own structural properties.
"""
import math

import numpy as np
import pytest

import rt_amd as R
from oracle import oracle as O

F32 = np.float32
PERM = None


def _perm():
    # perm[] of utility.cpp:620-633, taken from the oracle's own noise at one octave would be
    # circular; the table is restated here independently (it is the classic Perlin table)
    global PERM
    if PERM is None:
        PERM = [151, 160, 137, 91, 90, 15, 131, 13, 201, 95, 96, 53, 194, 233, 7, 225, 140, 36, 103, 30, 69, 142,
                8, 99, 37, 240, 21, 10, 23, 190, 6, 148, 247, 120, 234, 75, 0, 26, 197, 62, 94, 252, 219, 203, 117,
                35, 11, 32, 57, 177, 33, 88, 237, 149, 56, 87, 174, 20, 125, 136, 171, 168, 68, 175, 74, 165, 71,
                134, 139, 48, 27, 166, 77, 146, 158, 231, 83, 111, 229, 122, 60, 211, 133, 230, 220, 105, 92, 41,
                55, 46, 245, 40, 244, 102, 143, 54, 65, 25, 63, 161, 1, 216, 80, 73, 209, 76, 132, 187, 208, 89,
                18, 169, 200, 196, 135, 130, 116, 188, 159, 86, 164, 100, 109, 198, 173, 186, 3, 64, 52, 217, 226,
                250, 124, 123, 5, 202, 38, 147, 118, 126, 255, 82, 85, 212, 207, 206, 59, 227, 47, 16, 58, 17, 182,
                189, 28, 42, 223, 183, 170, 213, 119, 248, 152, 2, 44, 154, 163, 70, 221, 153, 101, 155, 167, 43,
                172, 9, 129, 22, 39, 253, 19, 98, 108, 110, 79, 113, 224, 232, 178, 185, 112, 104, 218, 246, 97,
                228, 251, 34, 242, 193, 238, 210, 144, 12, 191, 179, 162, 241, 81, 51, 145, 235, 249, 14, 239, 107,
                49, 192, 214, 31, 181, 199, 106, 157, 184, 84, 204, 176, 115, 121, 50, 45, 127, 4, 150, 254, 138,
                236, 205, 93, 222, 114, 67, 29, 24, 72, 243, 141, 128, 195, 78, 66, 215, 61, 156, 180]
    return PERM


def _py_snoise2(x, y):
    P = _perm()
    x, y = F32(x), F32(y)
    F2, G2 = F32(0.366025403), F32(0.211324865)

    def ffloor(v):
        return int(v) if F32(int(v)) < v else int(v) - 1

    def grad(h, gx, gy):
        h &= 7
        u, v = (gx, F32(2) * gy) if h < 4 else (gy, F32(2) * gx)
        if h & 1:
            u, v = -u, -v
        return F32(u + v)

    def corner(cx, cy, hsh):
        t = F32(0.5 - float(F32(cx * cx)) - float(F32(cy * cy)))
        if t < 0:
            return F32(0)
        t = F32(t * t)
        return F32(F32(t * t) * grad(P[hsh], cx, cy))

    s = F32((x + y) * F2)
    i, j = ffloor(F32(x + s)), ffloor(F32(y + s))
    t = F32(F32(i + j) * G2)
    x0, y0 = F32(x - F32(F32(i) - t)), F32(y - F32(F32(j) - t))
    i1, j1 = (1, 0) if x0 > y0 else (0, 1)
    x1, y1 = F32(F32(x0 - F32(i1)) + G2), F32(F32(y0 - F32(j1)) + G2)
    x2 = F32(float(x0) - 1.0 + 2.0 * float(G2))
    y2 = F32(float(y0) - 1.0 + 2.0 * float(G2))
    ii, jj = i & 255, j & 255
    n0 = corner(x0, y0, (ii + P[jj]) & 255)
    n1 = corner(x1, y1, (ii + i1 + P[(jj + j1) & 255]) & 255)
    n2 = corner(x2, y2, (ii + 1 + P[(jj + 1) & 255]) & 255)
    return F32(F32(n0 + n1) + n2)


def _py_make_texture(W, H, kind, freq, lac, gain, octaves):
    """MakeTexture<glm::vec3>(W, H, kind, {vec3(0), vec3(1)}, ...) restated in Python."""
    noise = np.zeros((H, W), np.float32)
    for Y in range(H):
        for X in range(W):
            if kind == 0:
                v = _py_snoise2(F32(X) * F32(freq), F32(Y) * F32(freq))
            else:
                v, amp, fq = F32(0), F32(1), F32(freq)
                for _ in range(octaves):
                    f = F32(_py_snoise2(F32(X) * fq, F32(Y) * fq) * amp)
                    if kind == 2 and f < 0:
                        f = -f
                    v = F32(v + f)
                    fq, amp = F32(fq * F32(lac)), F32(amp * F32(gain))
            noise[Y, X] = v
    mn, mx = min(F32(1), noise.min()), max(F32(0), noise.max())
    out = np.zeros((H, W, 3), np.uint8)
    for Y in range(H):
        for X in range(W):
            f = F32(F32(noise[Y, X] - mn) / F32(mx - mn))
            f = F32(F32(f - F32(F32(int(F32(f / F32(1))))) * F32(1)) * F32(1))  # MOD(f, 1) * 1, region 0
            out[Y, X] = int(255.999 * float(F32(F32(0) + F32(F32(1) * f)))) & 255
    return out


@pytest.mark.parametrize("kind", [0, 1, 2])
def test_noise_oracle_matches_python_restatement(kind):
    W, H = 6, 3  # 6 is a width the reference's four column batches tile exactly
    got = O.noise_texture(W, H, kind, freq=0.37, lac=2.5, gain=0.5, octaves=4)
    ref = _py_make_texture(W, H, kind, 0.37, 2.5, 0.5, 4)
    assert np.array_equal(got, ref)


def test_noise_oracle_properties():
    t = O.noise_texture(600, 100, 0, freq=0.01)
    assert t.shape == (100, 600, 3)
    assert (t[..., 0] == t[..., 1]).all() and (t[..., 1] == t[..., 2]).all()  # grey gradient {0, 1}
    assert t.min() == 0 and t.max() == 255
    # the reference's MOD(factor, 1/(n-1)) wraps the brightest texel (factor == 1) back to 0
    g = O.noise_texture(600, 100, 1, freq=0.01, lac=2.5, octaves=5)
    assert g.std() > 20


def test_noise_widths_the_batches_do_not_tile_are_rejected():
    with pytest.raises(RuntimeError):
        O.noise_texture(8, 4)  # batch 3 would get a negative width in MakeTexture
    with pytest.raises(RuntimeError):
        O.noise_texture(600, 10, 1, octaves=0)  # constant field: the reference divides by zero


def test_dm_transcendentals_match_libm():
    lib = O.load()
    import ctypes as C
    rng = np.random.default_rng(3)
    worst = 0.0
    for y, x in rng.normal(size=(4000, 2)) * rng.choice([1e-4, 1.0, 1e4], size=(4000, 1)):
        a, b = lib.orc_dm_atan2(y, x), math.atan2(y, x)
        worst = max(worst, abs(a - b) / abs(b))
    assert worst < 4e-15
    for x in np.concatenate([rng.uniform(-1, 1, 4000), [-1.0, -0.5, 0.0, 0.5, 1.0]]):
        a, b = lib.orc_dm_acos(x), math.acos(x)
        assert abs(a - b) <= 4e-15 * max(1.0, b)
    s, c = C.c_double(), C.c_double()
    for x in rng.uniform(-8, 8, 4000):
        lib.orc_dm_sincos(x, C.byref(s), C.byref(c))
        assert abs(s.value - math.sin(x)) < 3e-16 and abs(c.value - math.cos(x)) < 3e-16
    # signed zeros / axes of atan2
    assert lib.orc_dm_atan2(0.0, -1.0) == math.pi and lib.orc_dm_atan2(-0.0, -1.0) == -math.pi
    assert math.copysign(1, lib.orc_dm_atan2(-0.0, 1.0)) == -1.0


@pytest.mark.parametrize("load_as,map_to", [(0, 1), (1, 0)])
def test_remap_oracle_properties(load_as, map_to):
    rng = np.random.default_rng(7)
    flat = np.full((100, 600, 3), 77, np.uint8)
    out = O.texture_remap(flat, load_as, map_to)
    # every texel is a copy of a source texel (unorm8 round trip is exact) or an unwritten 0
    assert set(np.unique(out)) <= {0, 77}
    assert (out == 77).mean() > 0.85
    img = rng.integers(0, 256, (100, 600, 4)).astype(np.uint8)
    assert np.array_equal(O.texture_remap(img, load_as, load_as), img)
    out = O.texture_remap(img, load_as, map_to)
    texels = {tuple(v) for v in img.reshape(-1, 4)}
    written = out.reshape(-1, 4)[(out.reshape(-1, 4) != 0).any(axis=1)]
    assert all(tuple(v) in texels for v in written[::97])


def test_textured_render_oracle_changes_only_textured_objects():
    """TextureIndex k in 1..n_tex multiplies the object's colour by a texel; TextureIndex above
    n_tex leaves the image as the untextured one (04...glsl:416)."""
    sc = R.make_scene(R.PRESET_INW04_REFSET, spp=2, width=48, height=32)
    base, _, _ = O.render(sc)
    white = np.full((100, 600, 3), 255, np.uint8)
    sc.textures = [white]
    sc.geom[:, 27] = 2.0  # above n_tex = 1: no texture
    a, _, _ = O.render(sc)
    assert np.array_equal(a.view(np.uint32), base.view(np.uint32))
    sc.geom[:, 27] = 1.0  # an all-white texture multiplies by 1.0
    b, _, _ = O.render(sc)
    assert np.array_equal(b.view(np.uint32), base.view(np.uint32))
    sc.textures = [O.noise_texture(600, 100, 2, freq=0.02, lac=2.5, octaves=5)]
    c, _, _ = O.render(sc)
    assert not np.array_equal(c, base)
