"""The C ABI surface of librt_hip.so: it loads on a CPU-only host, exports every function
include/*.h declares, and validates arguments before touching a device."""
import ctypes as C
import os
import re

import numpy as np
import pytest

import rt_amd as R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    names = set()
    for h in ("rt_hip.h", "rt_scene.h"):
        src = open(os.path.join(ROOT, "include", h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:int|void|size_t|rt_dev_scene\s*\*)\s*\*?\s*(rt_\w+)\s*\(", src, re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    lib = R.load()
    declared = _declared()
    assert len(declared) >= 16
    for name in declared:
        assert hasattr(lib, name), name
    assert declared == set(R.SIGNATURES), declared ^ set(R.SIGNATURES)


def test_abi_version():
    assert R.load().rt_abi_version() == 1


def test_argument_validation_without_device():
    lib = R.load()
    st = R.RtStats()
    cam = R.RtCamera()
    p = R.RtParams(0, 0, 1, 1, 0, 0, 0, 0, 0, -1)
    buf = np.zeros(16, np.float32)
    assert lib.rt_render_iow01(None, None, None, None, None) == R.RT_E_ARG
    assert lib.rt_render_iow03(R.fptr(buf), R.fptr(buf), 1, C.byref(cam), C.byref(p), R.fptr(buf), C.byref(st)) == R.RT_E_ARG
    p.width = p.height = 4
    assert lib.rt_render_inw(R.fptr(buf), 1, 3, R.fptr(buf), None, 0, C.byref(cam), C.byref(p), R.fptr(buf), None,
                             C.byref(st)) == R.RT_E_ARG  # bad layout
    assert lib.rt_lbvh_build(None, 0, None) == R.RT_E_ARG
    assert lib.rt_sample_tables(0, None, None, None) == R.RT_E_ARG
    assert lib.rt_scene_preset(999, 0, 0, None, 0, None, None) == R.RT_E_ARG
    assert lib.rt_render_tiles_async(None, None, None, None, 0, 16, None, None, None, None) == R.RT_E_ARG


def test_textured_records_rejected_before_device():
    sc = R.make_scene(R.PRESET_INW04_REFSET, spp=1)
    sc.geom[1, 27] = 2.0
    lib = R.load()
    rgba = np.zeros((100, 100, 4), np.float32)
    rc = lib.rt_render_inw(R.fptr(sc.geom), sc.n, 4, R.fptr(sc.nodes), R.fptr(sc.lights), sc.n_lights,
                           C.byref(sc.camera), C.byref(sc.params), R.fptr(rgba), None, None)
    assert rc == R.RT_E_UNSUPPORTED


def test_no_silent_cpu_fallback():
    """Without a GPU the product path reports an error; it never renders on the CPU."""
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("GPU present")
    cam, sph, p = R.iow01_defaults(8, 8)
    with pytest.raises(RuntimeError):
        R.render_iow01(cam, sph, p)


def test_product_does_not_reference_oracle():
    """The shipped library and the product Python package never name the oracle."""
    with open(R.LIB_PATH, "rb") as f:
        blob = f.read()
    assert b"orc_" not in blob and b"librt_oracle" not in blob
    pkg = os.path.join(ROOT, "raytracing-tests_amd", "rt_amd")
    for fn in os.listdir(pkg):
        if fn.endswith(".py"):
            assert "oracle" not in open(os.path.join(pkg, fn)).read().replace("no CPU fallback", ""), fn
