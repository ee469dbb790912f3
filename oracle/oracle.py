"""ctypes wrapper of the CPU ORACLE (oracle/librt_oracle.so).

TEST INFRASTRUCTURE ONLY: importable by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, as the checker / the timed CPU baseline.  The product path never uses it.
PARITY UNPINNED against the reference itself -- see rt_oracle.h.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "librt_oracle.so")
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
                   "orc_pack_iow03", "orc_pack_inw", "orc_sample_tables"):
            getattr(lib, fn).restype = C.c_int
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
        rc = lib.orc_render_inw(_f(scene.geom), C.c_uint32(scene.n), C.c_int(scene.layout), _f(scene.nodes),
                                _f(lights), C.c_uint32(scene.n_lights), C.byref(scene.camera), C.byref(p),
                                _f(rgba), _f(depth), C.byref(st))
    if rc:
        raise RuntimeError(f"oracle render -> {rc}")
    return rgba, depth, _sd(st)


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
