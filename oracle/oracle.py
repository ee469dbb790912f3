"""ctypes wrapper of the CPU ORACLE (oracle/librt_oracle.so).

TEST INFRASTRUCTURE ONLY: importable by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / the timed CPU baseline.  The product path never uses it.
PARITY UNPINNED against the reference itself -- see rt_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

# RT_ORACLE_LIB: the sanitizer build of the same sources (tools/san/run_san.sh)
LIB_PATH = os.environ.get("RT_ORACLE_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_oracle.so")
_FP = C.POINTER(C.c_float)
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built at {LIB_PATH} (run `make -C oracle`)")
        lib = C.CDLL(LIB_PATH)
        lib.orc_num_threads.restype = C.c_int
        lib.orc_set_threads.argtypes = [C.c_int]
        for fn in ("orc_render_iow01", "orc_render_iow03", "orc_render_inw", "orc_lbvh_build",
                   "orc_pack_iow03", "orc_pack_inw", "orc_sample_tables", "orc_render_inw_tex",
                   "orc_noise_texture", "orc_texture_remap", "orc_render_iow00", "orc_render_iow02",
                   "orc_render_inw_mf"):
            getattr(lib, fn).restype = C.c_int
        lib.orc_noise_texture.argtypes = [C.c_int, C.c_int, C.c_int, _FP, C.c_int, C.c_float, C.c_float,
                                          C.c_float, C.c_int, C.c_void_p]
        lib.orc_texture_remap.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        for fn in ("orc_dm_atan2", "orc_dm_acos"):
            getattr(lib, fn).restype = C.c_double
        lib.orc_dm_atan2.argtypes = [C.c_double, C.c_double]
        lib.orc_dm_acos.argtypes = [C.c_double]
        lib.orc_dm_sincos.argtypes = [C.c_double, C.POINTER(C.c_double), C.POINTER(C.c_double)]
        _lib = lib
    return _lib


def _f(a):
    return None if a is None else a.ctypes.data_as(_FP)


def set_threads(n: int) -> None:
    load().orc_set_threads(int(n))


def num_threads() -> int:
    return load().orc_num_threads()


def _stats_struct():
    class S(C.Structure):
        _fields_ = [("segments", C.c_uint64), ("node_visits", C.c_uint64), ("prim_tests", C.c_uint64),
                    ("shadow_queries", C.c_uint64), ("stack_drops", C.c_uint64), ("nan_drops", C.c_uint64),
                    ("ms", C.c_double)]
    return S()


def _sd(st):
    return {k: getattr(st, k) for k, _ in st._fields_}


def render_iow01(camera, sphere, params):
    lib = load()
    rgba = np.zeros((params.height, params.width, 4), np.float32)
    st = _stats_struct()
    sph = np.asarray(sphere, np.float32)
    rc = lib.orc_render_iow01(C.byref(camera), _f(sph), C.byref(params), _f(rgba), C.byref(st))
    if rc:
        raise RuntimeError(f"orc_render_iow01 -> {rc}")
    return rgba, _sd(st)


def render_iow00(params):
    """IOW-00: the base stage's default compute shader (base.cpp:7-28)."""
    rgba = np.zeros((params.height, params.width, 4), np.float32)
    rc = load().orc_render_iow00(C.byref(params), _f(rgba))
    if rc:
        raise RuntimeError(f"orc_render_iow00 -> {rc}")
    return rgba


def render_iow02(types, records, camera, params, cull_front=0, cull_back=1):
    """IOW-02 groups stage (02_Groups/computeShaderSrc.glsl); records N x 18."""
    types = np.ascontiguousarray(types, np.float32)
    records = np.ascontiguousarray(records, np.float32).reshape(-1, 18)
    rgba = np.zeros((params.height, params.width, 4), np.float32)
    st = _stats_struct()
    rc = load().orc_render_iow02(_f(types), _f(records), C.c_uint32(len(types)), C.byref(camera), C.byref(params),
                                 C.c_int(cull_front), C.c_int(cull_back), _f(rgba), C.byref(st))
    if rc:
        raise RuntimeError(f"orc_render_iow02 -> {rc}")
    return rgba, _sd(st)


def render_inw_mf(scene, focus, params=None):
    """INW-01 with its MULTIFOCUS branch (01_BVH...glsl:388-404, 505-549) and focus distances `focus`."""
    p = params or scene.params
    f = np.ascontiguousarray(focus, np.float32)
    rgba = np.zeros((p.height, p.width, 4), np.float32)
    depth = np.zeros((p.height, p.width), np.float32)
    st = _stats_struct()
    rc = load().orc_render_inw_mf(_f(scene.geom), C.c_uint32(scene.n), _f(scene.nodes), C.byref(scene.camera),
                                  _f(f), C.c_int(len(f)), C.byref(p), _f(rgba), _f(depth), C.byref(st))
    if rc:
        raise RuntimeError(f"orc_render_inw_mf -> {rc}")
    return rgba, depth, _sd(st)


def render(scene, params=None):
    """CPU render of a packed rt_amd.Scene; same return shape as rt_amd.render."""
    lib = load()
    p = params or scene.params
    rgba = np.zeros((p.height, p.width, 4), np.float32)
    st = _stats_struct()
    depth = None
    if scene.stage == 3:
        rc = lib.orc_render_iow03(_f(scene.types), _f(scene.records), C.c_uint32(scene.n), C.byref(scene.camera),
                                  C.byref(p), _f(rgba), C.byref(st))
    else:
        depth = np.zeros((p.height, p.width), np.float32)
        lights = scene.lights if scene.lights is not None and len(scene.lights) else None
        tex = getattr(scene, "textures", None) or []
        keep = [np.ascontiguousarray(t, np.uint8) for t in tex]
        arr = (_OrcTexture * max(1, len(keep)))()
        for i, t in enumerate(keep):
            arr[i] = _OrcTexture(t.ctypes.data, t.shape[1], t.shape[0], t.shape[2])
        rc = lib.orc_render_inw_tex(_f(scene.geom), C.c_uint32(scene.n), C.c_int(scene.layout), _f(scene.nodes),
                                    _f(lights), C.c_uint32(scene.n_lights), arr, C.c_uint32(len(keep)),
                                    C.byref(scene.camera), C.byref(p), _f(rgba), _f(depth), C.byref(st))
    if rc:
        raise RuntimeError(f"oracle render -> {rc}")
    return rgba, depth, _sd(st)


class _OrcTexture(C.Structure):
    _fields_ = [("texels", C.c_void_p), ("width", C.c_int), ("height", C.c_int), ("channels", C.c_int)]


def noise_texture(width=600, height=100, kind=0, gradient=((0, 0, 0), (1, 1, 1)), freq=0.01, lac=2.0, gain=0.5,
                  octaves=5):
    """CPU restatement of Helper::Noise::MakeTexture<glm::vec3> (utility.h:69-192)."""
    g = np.ascontiguousarray(np.asarray(gradient, np.float32).reshape(-1, 3))
    out = np.zeros((height, width, 3), np.uint8)
    rc = load().orc_noise_texture(width, height, kind, _f(g) if len(g) else None, len(g), freq, lac, gain, octaves,
                                  out.ctypes.data)
    if rc:
        raise RuntimeError(f"orc_noise_texture -> {rc}")
    return out


def texture_remap(img, load_as, map_to):
    """CPU restatement of LoadFromDiskToGPU's re-projection (utility.cpp:266-463)."""
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros_like(img)
    rc = load().orc_texture_remap(img.ctypes.data, img.shape[1], img.shape[0], img.shape[2], load_as, map_to,
                                  out.ctypes.data)
    if rc:
        raise RuntimeError(f"orc_texture_remap -> {rc}")
    return out


def lbvh_build(aabbs):
    aabbs = np.ascontiguousarray(aabbs, np.float32)
    n = aabbs.shape[0]
    out = np.zeros((2 * n - 1, 8), np.float32)
    rc = load().orc_lbvh_build(_f(aabbs), C.c_uint32(n), _f(out))
    if rc:
        raise RuntimeError(f"orc_lbvh_build -> {rc}")
    return out


def pack(desc, n, stage):
    lib = load()
    if stage == 3:
        types = np.zeros(n, np.float32)
        rec = np.zeros((n, 24), np.float32)
        rc = lib.orc_pack_iow03(desc, C.c_uint32(n), _f(types), _f(rec))
        if rc:
            raise RuntimeError("orc_pack_iow03")
        return {"types": types, "records": rec}
    layout = 4 if stage == 14 else 1
    geom = np.zeros((n, 28), np.float32)
    aabbs = np.zeros((n, 6), np.float32)
    lights = np.zeros((max(n, 1), 7), np.float32)
    nl = C.c_uint32(0)
    rc = lib.orc_pack_inw(desc, C.c_uint32(n), C.c_int(layout), _f(geom), _f(aabbs), _f(lights), C.byref(nl))
    if rc:
        raise RuntimeError("orc_pack_inw")
    return {"geom": geom, "aabbs": aabbs, "lights": lights[: nl.value].copy(), "n_lights": nl.value}


def sample_tables(spp):
    sf = np.zeros((spp, 2), np.float32)
    fib = np.zeros((spp, 3), np.float32)
    ring = np.zeros((spp, 2), np.int32)
    rc = load().orc_sample_tables(C.c_int(spp), _f(sf), _f(fib), ring.ctypes.data_as(C.POINTER(C.c_int)))
    if rc:
        raise RuntimeError("orc_sample_tables")
    return sf, fib, ring
