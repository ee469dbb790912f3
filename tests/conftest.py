"""pytest wiring: the `gpu` marker, import paths, and on-demand builds of the two libraries.

Markers
  gpu  -- needs an MI355X (gfx950) device; the parity tests proper, calling through the C ABI.
Everything unmarked runs on the CPU: oracle vs golden fixtures, host logic (packers, LBVH,
sample tables, tile scheduler), the ABI surface of librt_hip.so, and gloo multi-process tests.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "raytracing-tests_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def _ensure_built():
    if not os.path.exists(os.path.join(ROOT, "oracle", "librt_oracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    if not os.path.exists(os.path.join(PKG, "librt_hip.so")):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True)


_ensure_built()


def gpu_available() -> bool:
    try:
        import rt_amd
        return rt_amd.load().rt_device_info(-1, None, 0, None) == 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    if not gpu_available():
        pytest.fail("no gfx950 device visible to librt_hip.so (gpu tests need an MI355X)")
    return True
