"""rt_amd -- Python mirror of the MI355X render path's C ABI (librt_hip.so).

The package directory is ``raytracing-tests_amd/`` (not importable by name because of the
hyphen); callers add it to ``sys.path`` and ``import rt_amd``.  See ``rt_amd.capi``.
"""
from .capi import *  # noqa: F401,F403
