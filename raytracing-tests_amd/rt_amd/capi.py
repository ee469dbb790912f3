"""ctypes binding of librt_hip.so (include/rt_hip.h + include/rt_scene.h).

This is the Python side of the drop-in boundary: a thin mirror of the C ABI with numpy
arrays in and out.  It loads the in-tree HIP library and fails loudly if it is missing --
there is no CPU fallback anywhere in the product path.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# RT_HIP_LIB: an alternative build of the same library (diagnostic variants, tools/ only)
LIB_PATH = os.environ.get("RT_HIP_LIB") or os.path.join(os.path.dirname(_HERE), "librt_hip.so")

RT_OK, RT_E_ARG, RT_E_HIP, RT_E_NODEVICE, RT_E_UNSUPPORTED = 0, -1, -2, -3, -4

RT_STAGE_IOW01, RT_STAGE_IOW03, RT_STAGE_INW01, RT_STAGE_INW04 = 1, 3, 11, 14
RT_STAGE_IOW02 = 2
RT_IOW_CUBOID, RT_IOW_ELLIPSOID = 1, 2
RT_INW_ELLIPSOID, RT_INW_CUBOID = 1, 2

ABI_VERSION = 5  # RT_ABI_VERSION, include/rt_hip.h

PRESET_IOW03_REF3 = 1
PRESET_IOW03_FINAL = 2
PRESET_INW01_GRID = 3
PRESET_INW01_RANDOM = 4
PRESET_INW04_REFSET = 5
PRESET_INW04_CORNELL = 6


class RtCamera(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("dir", C.c_float * 3), ("fov_y_rad", C.c_float),
                ("aperture", C.c_float), ("focus_dist", C.c_float)]


class RtParams(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("spp", C.c_int), ("max_bounces", C.c_int),
                ("tile_x0", C.c_int), ("tile_y0", C.c_int), ("tile_w", C.c_int), ("tile_h", C.c_int),
                ("show_normal", C.c_int), ("device", C.c_int)]


class RtStats(C.Structure):
    _fields_ = [("segments", C.c_uint64), ("node_visits", C.c_uint64), ("prim_tests", C.c_uint64),
                ("shadow_queries", C.c_uint64), ("stack_drops", C.c_uint64), ("nan_drops", C.c_uint64),
                ("ms", C.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_}


class RtGeomDesc(C.Structure):
    _fields_ = [("type", C.c_int), ("position", C.c_float * 3), ("last_position", C.c_float * 3),
                ("rotation_deg", C.c_float * 3), ("scale", C.c_float * 3), ("color", C.c_float * 3),
                ("refractivity", C.c_float), ("reflectivity", C.c_float), ("refractive_index", C.c_float),
                ("scat_refract", C.c_float), ("scat_reflect", C.c_float), ("emissive", C.c_int),
                ("texture_index", C.c_int)]


class RtCamDesc(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("pitch_deg", C.c_float), ("yaw_deg", C.c_float),
                ("fov_y_deg", C.c_float), ("aperture", C.c_float), ("focus_dist", C.c_float)]


class RtTexture(C.Structure):
    _fields_ = [("texels", C.c_void_p), ("width", C.c_int), ("height", C.c_int), ("channels", C.c_int)]


class RtOptions(C.Structure):
    """rt_options (include/rt_hip.h): the exact strategy switches of the render path."""
    _fields_ = [("size", C.c_uint32)] + [(n, C.c_int) for n in (
        "inw_wide_walk", "inw_order", "inw_beams", "inw_ri_grid", "inw_lds_nodes", "inw_fused_cull",
        "inw_claim_order", "inw_ring_pm", "inw_ring_sm", "inw_stackless", "inw_device_build", "inw_claim_xcd",
        "inw_qnodes", "inw_time_bins", "inw_walk_bins", "inw_beam_bins", "inw_sphere_records", "inw_compact_nodes",
        "iow_spec", "iow_linear", "iow_narrow", "iow_lds_bvh", "iow_leaf_batch", "iow_coop_max", "iow_chunks_lpt",
        "rounds_seq", "rounds_spec", "park_min",
        "spec_iters", "spec_probe", "spec_heavy", "spec_rounds", "spec_tail_rounds", "spec_tail_budget", "spec_scan",
        "spec_chain", "spec_alt", "spec_alt_cap", "spec_alt_seg", "spec_alt_every", "spec_spread", "spec_prior_from",
        "spec_sort", "spec_solo", "spec_validate")] + [("spec_max_gb", C.c_double)]

    def as_dict(self) -> dict:
        return {k: getattr(self, k) for k, _ in self._fields_ if k != "size"}


class RtPathInfo(C.Structure):
    """rt_path_info (include/rt_hip.h): what a scene's last render ran."""
    _fields_ = [("kernel", C.c_char * 64), ("launches", C.c_int), ("order", C.c_int), ("order_forced", C.c_int),
                ("wide_walk", C.c_int), ("beams", C.c_int), ("ri_grid", C.c_int), ("fused_cull", C.c_int),
                ("lds_nodes", C.c_int), ("claim_order", C.c_int), ("ring_entries", C.c_int), ("iow_bvh", C.c_int),
                ("ring_lds", C.c_int), ("stackless", C.c_int), ("lbvh_lds_nodes", C.c_int),
                ("qnodes", C.c_int), ("global_stack", C.c_int), ("walk_stack", C.c_int), ("ref_walks", C.c_uint64),
                ("time_bins", C.c_int), ("beam_bins", C.c_int), ("sphere_records", C.c_int)]

    ORDERS = {0: None, 1: "pixel-major", 2: "sample-major", 3: "per-pixel", 4: "sample-parallel", 5: "sequential"}

    def as_dict(self) -> dict:
        d = {k: getattr(self, k) for k, _ in self._fields_}
        d["kernel"] = self.kernel.decode()
        d["order"] = self.ORDERS.get(self.order, self.order)
        return d


_FP = C.POINTER(C.c_float)
_IP = C.POINTER(C.c_int)
_U32P = C.POINTER(C.c_uint32)
_U64P = C.POINTER(C.c_uint64)

# name -> (restype, argtypes); every symbol include/*.h declares
SIGNATURES = {
    "rt_abi_version": (C.c_int, []),
    "rt_device_info": (C.c_int, [C.c_int, C.c_char_p, C.c_int, _IP]),
    "rt_render_iow01": (C.c_int, [C.POINTER(RtCamera), _FP, C.POINTER(RtParams), _FP, C.POINTER(RtStats)]),
    "rt_render_iow03": (C.c_int, [_FP, _FP, C.c_uint32, C.POINTER(RtCamera), C.POINTER(RtParams), _FP,
                                  C.POINTER(RtStats)]),
    "rt_render_iow00": (C.c_int, [C.POINTER(RtParams), _FP]),
    "rt_pack_iow02": (C.c_int, [C.c_void_p, C.c_uint32, _FP, _FP]),
    "rt_render_iow02": (C.c_int, [_FP, _FP, C.c_uint32, C.POINTER(RtCamera), C.POINTER(RtParams), C.c_int, C.c_int,
                                  _FP, C.POINTER(RtStats)]),
    "rt_render_inw_mf": (C.c_int, [_FP, C.c_uint32, _FP, C.POINTER(RtCamera), _FP, C.c_int, C.POINTER(RtParams), _FP,
                                   _FP, C.POINTER(RtStats)]),
    "rt_render_inw": (C.c_int, [_FP, C.c_uint32, C.c_int, _FP, _FP, C.c_uint32, C.POINTER(RtCamera),
                                C.POINTER(RtParams), _FP, _FP, C.POINTER(RtStats)]),
    "rt_render_inw_tex": (C.c_int, [_FP, C.c_uint32, C.c_int, _FP, _FP, C.c_uint32, C.POINTER(RtTexture), C.c_int,
                                    C.POINTER(RtCamera), C.POINTER(RtParams), _FP, _FP, C.POINTER(RtStats)]),
    "rt_noise_texture": (C.c_int, [C.c_int, C.c_int, C.c_int, _FP, C.c_int, C.c_float, C.c_float, C.c_float,
                                   C.c_int, C.c_void_p, C.c_int, C.POINTER(C.c_double)]),
    "rt_noise_workspace_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "rt_noise_texture_async": (C.c_int, [C.c_int, C.c_int, C.c_int, _FP, C.c_int, C.c_float, C.c_float, C.c_float,
                                         C.c_int, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "rt_texture_remap": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_int,
                                   C.POINTER(C.c_double)]),
    "rt_remap_workspace_bytes": (C.c_size_t, [C.c_int, C.c_int]),
    "rt_texture_remap_async": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                         C.c_void_p, C.c_size_t, C.c_void_p]),
    "rt_lbvh_build": (C.c_int, [_FP, C.c_uint32, _FP]),
    "rt_lbvh_workspace_bytes": (C.c_size_t, [C.c_uint32]),
    "rt_lbvh_build_async": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p]),
    "rt_lbvh_build_gpu": (C.c_int, [_FP, C.c_uint32, _FP, C.c_int, C.POINTER(C.c_double)]),
    "rt_dev_scene_iow03": (C.c_void_p, [_FP, _FP, C.c_uint32, C.c_int, C.c_int]),
    "rt_dev_scene_inw": (C.c_void_p, [_FP, C.c_uint32, C.c_int, _FP, _FP, C.c_uint32, C.c_int, C.c_int]),
    "rt_dev_scene_inw_tex": (C.c_void_p, [_FP, C.c_uint32, C.c_int, _FP, _FP, C.c_uint32, C.POINTER(RtTexture),
                                          C.c_int, C.c_int, C.c_int]),
    "rt_dev_scene_free": (None, [C.c_void_p]),
    "rt_render_tiles_async": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.POINTER(RtParams), C.c_void_p,
                                        C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_render_image_async": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.POINTER(RtParams), C.c_void_p,
                                        C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_scene_preset": (C.c_int, [C.c_int, C.c_uint32, C.c_int, C.POINTER(RtGeomDesc), C.c_int,
                                  C.POINTER(RtCamDesc), C.POINTER(RtParams)]),
    "rt_camera_from_desc": (C.c_int, [C.POINTER(RtCamDesc), C.c_int, C.POINTER(RtCamera)]),
    "rt_pack_iow03": (C.c_int, [C.POINTER(RtGeomDesc), C.c_uint32, _FP, _FP]),
    "rt_pack_inw": (C.c_int, [C.POINTER(RtGeomDesc), C.c_uint32, C.c_int, _FP, _FP, _FP, _U32P]),
    "rt_sample_tables": (C.c_int, [C.c_int, _FP, _FP, _IP]),
    "rt_tile_spiral": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, _IP, C.c_int]),
    "rt_render_spiral_async": (C.c_int, [C.c_void_p, C.POINTER(RtCamera), C.POINTER(RtParams), C.c_int, C.c_int,
                                         C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_display_rgba8_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                         C.c_void_p]),
    "rt_debug_counters": (C.c_int, [C.c_void_p]),
    "rt_debug_pixel_rays": (C.c_int, [C.c_void_p]),
    "rt_debug_rounds": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int]),
    "rt_debug_spec_hist": (C.c_int, [C.c_void_p, C.c_void_p]),
    "rt_debug_launches": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int]),
    "rt_debug_chunks": (C.c_int, [C.c_void_p]),
    "rt_debug_spec_times": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t]),
    "rt_debug_time_kernels": (C.c_int, [C.c_int]),
    "rt_debug_check_fastmath": (C.c_int, [C.c_int, _U64P, _U32P]),
    "rt_debug_kernel_time": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.POINTER(C.c_int)]),
    "rt_debug_spec_pixels": (C.c_int, [C.c_void_p, _U32P, C.c_uint32]),
    "rt_debug_spec_list_hist": (C.c_int, [C.c_void_p, _U64P]),
    "rt_debug_spec_list_stale": (C.c_int, [C.c_void_p, _U64P]),
    "rt_debug_spec_dump": (C.c_int, [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_uint32, C.c_void_p]),
    "rt_inw_host_build": (C.c_int, [_FP, C.c_uint32, _U32P, C.POINTER(C.c_double)]),
    "rt_iow_host_build": (C.c_int, [_FP, _FP, C.c_uint32, _U32P, C.POINTER(C.c_double)]),
    "rt_options_default": (None, [C.POINTER(RtOptions)]),
    "rt_options_set": (C.c_int, [C.POINTER(RtOptions)]),
    "rt_options_get": (C.c_int, [C.POINTER(RtOptions)]),
    "rt_dev_scene_set_options": (C.c_int, [C.c_void_p, C.POINTER(RtOptions)]),
    "rt_dev_scene_inw_update": (C.c_int, [C.c_void_p, _FP, C.c_uint32, _FP, _FP, _FP, C.c_uint32,
                                          C.POINTER(C.c_double)]),
    "rt_debug_path": (C.c_int, [C.c_void_p, C.POINTER(RtPathInfo)]),
    "rt_debug_wide_info": (C.c_int, [C.c_void_p, _U32P, _U32P]),
    "rt_tile_deal": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, _IP, C.c_int]),
    "rt_group_create": (C.c_void_p, [_IP, C.c_int]),
    "rt_debug_build_level_cap": (C.c_int, [C.c_int]),
    "rt_debug_time_bins": (C.c_int, [_FP, _FP, C.c_uint32, C.c_uint32, _FP, C.c_uint32, _U32P]),
    "rt_debug_bin_boxes": (C.c_int, [_FP, C.c_uint32, C.c_uint32, C.c_uint32, _FP]),
    "rt_debug_sphere_records": (C.c_int, [_FP, C.c_uint32, C.c_int, _FP]),
    "rt_group_free": (None, [C.c_void_p]),
    "rt_render_multi_async": (C.c_int, [C.c_void_p, C.c_void_p, C.POINTER(RtCamera), C.POINTER(RtParams), C.c_int,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "rt_render_inw_multi": (C.c_int, [_FP, C.c_uint32, C.c_int, _FP, _FP, C.c_uint32, C.POINTER(RtCamera),
                                      C.POINTER(RtParams), _IP, C.c_int, C.c_int, _FP, _FP, C.POINTER(RtStats)]),
}

_lib = None


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load librt_hip.so.  Raises (never falls back) if the HIP library is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RuntimeError(f"librt_hip.so not built at {path}: run __graft_entry__.build() "
                           "(there is no CPU fallback for the render path)")
    # torch bundles its own libamdhip64 (SONAME libamdhip64.so.7).  Loading torch first makes
    # the dynamic linker resolve our NEEDED libamdhip64.so.7 to that same runtime, so device
    # pointers, streams and RCCL from torch and our kernels share one HIP runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def fptr(a: np.ndarray | None):
    if a is None:
        return None
    assert a.dtype == np.float32 and a.flags.c_contiguous
    return a.ctypes.data_as(_FP)


def check(rc: int, what: str) -> None:
    if rc != RT_OK:
        raise RuntimeError(f"{what} failed with status {rc}")


# ---------------------------------------------------------------------------- options
def default_options() -> RtOptions:
    o = RtOptions()
    load().rt_options_default(C.byref(o))
    return o


def get_options() -> RtOptions:
    o = RtOptions()
    check(load().rt_options_get(C.byref(o)), "rt_options_get")
    return o


def set_options(o: RtOptions) -> None:
    check(load().rt_options_set(C.byref(o)), "rt_options_set")


class options:
    """Context manager: the library-wide rt_options with some fields changed, e.g.
    `with R.options(inw_order=2, inw_ring_sm=64): R.render(sc)`; restores the previous ones."""

    def __init__(self, **fields):
        self.fields = fields

    def __enter__(self) -> RtOptions:
        self.prev = get_options()
        o = RtOptions.from_buffer_copy(self.prev)
        for k, v in self.fields.items():
            if k not in dict(RtOptions._fields_):
                raise KeyError(f"unknown rt_options field {k!r}")
            setattr(o, k, v)
        set_options(o)
        return o

    def __exit__(self, *exc) -> None:
        set_options(self.prev)


def debug_path(scene_handle) -> dict:
    """rt_debug_path of a device scene: the kernel and exact shortcuts of its last render."""
    p = RtPathInfo()
    check(load().rt_debug_path(scene_handle, C.byref(p)), "rt_debug_path")
    return p.as_dict()


# ----------------------------------------------------------------------------- scenes
@dataclass
class Scene:
    """A packed scene in the reference's record layouts (what the GL textures held)."""
    stage: int
    desc: object            # ctypes array of RtGeomDesc
    n: int
    camera: RtCamera
    params: RtParams
    types: np.ndarray | None = None    # IOW-03
    records: np.ndarray | None = None  # IOW-03 (N,24)
    geom: np.ndarray | None = None     # INW (N,28)
    aabbs: np.ndarray | None = None    # INW (N,6)
    nodes: np.ndarray | None = None    # INW (2N-1,8)
    lights: np.ndarray | None = None   # INW-04 (L,7)
    n_lights: int = 0
    textures: list | None = None       # INW-04 u_MaterialTextures: (H, W, 3|4) uint8 images

    @property
    def layout(self) -> int:
        return 4 if self.stage == RT_STAGE_INW04 else 1


PRESET_STAGE = {PRESET_IOW03_REF3: RT_STAGE_IOW03, PRESET_IOW03_FINAL: RT_STAGE_IOW03,
                 PRESET_INW01_GRID: RT_STAGE_INW01, PRESET_INW01_RANDOM: RT_STAGE_INW01,
                 PRESET_INW04_REFSET: RT_STAGE_INW04, PRESET_INW04_CORNELL: RT_STAGE_INW04}


def preset_desc(preset: int, seed: int = 0, n_hint: int = 0):
    lib = load()
    n = lib.rt_scene_preset(preset, seed, n_hint, None, 0, None, None)
    if n < 0:
        raise RuntimeError(f"unknown preset {preset}")
    arr = (RtGeomDesc * max(n, 1))()
    cam, par = RtCamDesc(), RtParams()
    check(lib.rt_scene_preset(preset, seed, n_hint, arr, n, C.byref(cam), C.byref(par)) - n, "rt_scene_preset")
    return arr, n, cam, par


def camera_from_desc(cd: RtCamDesc, stage: int) -> RtCamera:
    cam = RtCamera()
    check(load().rt_camera_from_desc(C.byref(cd), stage, C.byref(cam)), "rt_camera_from_desc")
    return cam


def pack(desc, n: int, stage: int, build_lbvh: bool = True) -> dict:
    lib = load()
    out: dict = {}
    if stage == RT_STAGE_IOW03:
        types = np.zeros(n, np.float32)
        rec = np.zeros((n, 24), np.float32)
        check(lib.rt_pack_iow03(desc, n, fptr(types), fptr(rec)), "rt_pack_iow03")
        out.update(types=types, records=rec)
    else:
        layout = 4 if stage == RT_STAGE_INW04 else 1
        geom = np.zeros((n, 28), np.float32)
        aabbs = np.zeros((n, 6), np.float32)
        lights = np.zeros((max(n, 1), 7), np.float32)
        nl = C.c_uint32(0)
        check(lib.rt_pack_inw(desc, n, layout, fptr(geom), fptr(aabbs), fptr(lights), C.byref(nl)), "rt_pack_inw")
        out.update(geom=geom, aabbs=aabbs, lights=lights[: nl.value].copy(), n_lights=nl.value)
        if build_lbvh:
            out["nodes"] = lbvh_build(aabbs)
    return out


def make_scene(preset: int, seed: int = 0, n_hint: int = 0, **param_overrides) -> Scene:
    stage = PRESET_STAGE[preset]
    arr, n, cd, par = preset_desc(preset, seed, n_hint)
    for k, v in param_overrides.items():
        setattr(par, k, v)
    cam = camera_from_desc(cd, stage)
    sc = Scene(stage=stage, desc=arr, n=n, camera=cam, params=par)
    for k, v in pack(arr, n, stage).items():
        setattr(sc, k, v)
    return sc


def texture_array(textures):
    """rt_texture[] for a list of (H, W, 3|4) uint8 images (row 0 first); returns (array, keep-alive)."""
    keep = [np.ascontiguousarray(t, np.uint8) for t in textures]
    arr = (RtTexture * max(1, len(keep)))()
    for i, t in enumerate(keep):
        assert t.ndim == 3 and t.shape[2] in (3, 4), t.shape
        arr[i] = RtTexture(t.ctypes.data, t.shape[1], t.shape[0], t.shape[2])
    return arr, keep


NOISE_SIMPLEX, NOISE_FBM, NOISE_TURBULENCE = 0, 1, 2
MAP_MERCATOR, MAP_CUBIC = 0, 1


def noise_texture(width=600, height=100, kind=NOISE_SIMPLEX, gradient=((0, 0, 0), (1, 1, 1)), freq=0.01,
                  lac=2.0, gain=0.5, octaves=5, device: int = -1):
    """GPU Helper::Noise::MakeTexture<glm::vec3> (rt_noise_texture): (height, width, 3) uint8, ms."""
    g = np.ascontiguousarray(np.asarray(gradient, np.float32).reshape(-1, 3))
    out = np.zeros((height, width, 3), np.uint8)
    ms = C.c_double(0.0)
    check(load().rt_noise_texture(width, height, kind, fptr(g) if len(g) else None, len(g), freq, lac, gain,
                                  octaves, out.ctypes.data, device, C.byref(ms)), "rt_noise_texture")
    return out, ms.value


def texture_remap(img, load_as, map_to, device: int = -1):
    """GPU re-projection of LoadFromDiskToGPU(loc, loadAs, mapTo) (rt_texture_remap): image, ms."""
    img = np.ascontiguousarray(img, np.uint8)
    out = np.zeros_like(img)
    ms = C.c_double(0.0)
    check(load().rt_texture_remap(img.ctypes.data, img.shape[1], img.shape[0], img.shape[2], load_as, map_to,
                                  out.ctypes.data, device, C.byref(ms)), "rt_texture_remap")
    return out, ms.value


def tile_spiral(width: int, height: int, tile_w: int = 100, tile_h: int = 100) -> np.ndarray:
    """Progressive tile order of Adding_Materials::OnUpdate (rt_tile_spiral): (n, 4) int32 rows
    (tx, ty, dispatch_w, dispatch_h)."""
    lib = load()
    n = lib.rt_tile_spiral(width, height, tile_w, tile_h, None, 0)
    check(min(n, 0), "rt_tile_spiral")
    out = np.zeros((max(n, 1), 4), np.int32)
    lib.rt_tile_spiral(width, height, tile_w, tile_h, out.ctypes.data_as(_IP), n)
    return out[:n]


def tile_deal(width: int, height: int, tile: int, n_dev: int) -> list:
    """rt_tile_deal: the multi-GPU deal order of the frame's tiles, [(tx, ty), ...]; entry k goes to
    device k % n_dev."""
    lib = load()
    n = lib.rt_tile_deal(width, height, tile, n_dev, None, 0)
    check(min(n, 0), "rt_tile_deal")
    out = np.zeros((max(n, 1), 2), np.int32)
    lib.rt_tile_deal(width, height, tile, n_dev, out.ctypes.data_as(_IP), n)
    return [tuple(int(v) for v in row) for row in out[:n]]


def render_inw_multi(sc: "Scene", devices, params: RtParams | None = None, tile: int = 16):
    """rt_render_inw_multi: the INW frame tile-partitioned over `devices` with the RCCL gather to
    devices[0]; returns (rgba, depth, stats) like render()."""
    p = params or sc.params
    devs = (C.c_int * len(devices))(*devices)
    rgba = np.zeros((p.height, p.width, 4), np.float32)
    depth = np.zeros((p.height, p.width), np.float32)
    st = RtStats()
    lights = sc.lights if sc.lights is not None and len(sc.lights) else None
    check(load().rt_render_inw_multi(fptr(sc.geom), sc.n, sc.layout, fptr(sc.nodes), fptr(lights), sc.n_lights,
                                     C.byref(sc.camera), C.byref(p), devs, len(devices), tile, fptr(rgba), fptr(depth),
                                     C.byref(st)), "rt_render_inw_multi")
    return rgba, depth, st.as_dict()


def lbvh_build_gpu(aabbs, device: int = -1):
    """GPU LBVH (rt_lbvh_build_gpu): same (2N-1) x 8 node buffer as lbvh_build; returns (nodes, ms)."""
    aabbs = np.ascontiguousarray(aabbs, np.float32)
    n = aabbs.shape[0]
    nodes = np.zeros((2 * n - 1, 8), np.float32)
    ms = C.c_double(0.0)
    check(load().rt_lbvh_build_gpu(fptr(aabbs), n, fptr(nodes), device, C.byref(ms)), "rt_lbvh_build_gpu")
    return nodes, ms.value


def inw_host_build(nodes: np.ndarray, n: int) -> dict:
    """rt_inw_host_build: the INW device scene's host-built structures (sizes) and host time."""
    info = (C.c_uint32 * 8)()
    ms = C.c_double(0.0)
    check(load().rt_inw_host_build(fptr(np.ascontiguousarray(nodes, np.float32)), n, info, C.byref(ms)),
          "rt_inw_host_build")
    keys = ("wide_nodes", "dfs_high", "wide_depth", "ri_grid", "ri_cells", "ri_ids")
    return {**dict(zip(keys, list(info)[:6])), "ms": ms.value}


def iow_host_build(types: np.ndarray, records: np.ndarray, n: int) -> dict:
    """rt_iow_host_build: the IOW-03 culling BVH's size (0: linear loop) and host time."""
    info = (C.c_uint32 * 4)()
    ms = C.c_double(0.0)
    check(load().rt_iow_host_build(fptr(types), fptr(records), n, info, C.byref(ms)), "rt_iow_host_build")
    return {"wide_nodes": info[0], "ms": ms.value}


def lbvh_build(aabbs: np.ndarray) -> np.ndarray:
    aabbs = np.ascontiguousarray(aabbs, np.float32)
    n = aabbs.shape[0]
    nodes = np.zeros((2 * n - 1, 8), np.float32)
    check(load().rt_lbvh_build(fptr(aabbs), n, fptr(nodes)), "rt_lbvh_build")
    return nodes


def sample_tables(spp: int):
    sf = np.zeros((spp, 2), np.float32)
    fib = np.zeros((spp, 3), np.float32)
    ring = np.zeros((spp, 2), np.int32)
    check(load().rt_sample_tables(spp, fptr(sf), fptr(fib), ring.ctypes.data_as(_IP)), "rt_sample_tables")
    return sf, fib, ring


# ---------------------------------------------------------------------------- render
def render(sc: Scene, params: RtParams | None = None, sphere=None):
    """Blocking GPU render of a packed scene; returns (rgba (H,W,4), depth or None, stats dict)."""
    lib = load()
    p = params or sc.params
    rgba = np.zeros((p.height, p.width, 4), np.float32)
    st = RtStats()
    depth = None
    if sc.stage == RT_STAGE_IOW01:
        sph = np.asarray(sphere, np.float32)
        rc = lib.rt_render_iow01(C.byref(sc.camera), fptr(sph), C.byref(p), fptr(rgba), C.byref(st))
    elif sc.stage == RT_STAGE_IOW03:
        rc = lib.rt_render_iow03(fptr(sc.types), fptr(sc.records), sc.n, C.byref(sc.camera), C.byref(p),
                                 fptr(rgba), C.byref(st))
    else:
        depth = np.zeros((p.height, p.width), np.float32)
        lights = sc.lights if sc.lights is not None and len(sc.lights) else None
        tex = getattr(sc, "textures", None) or []
        if tex:
            arr, keep = texture_array(tex)
            rc = lib.rt_render_inw_tex(fptr(sc.geom), sc.n, sc.layout, fptr(sc.nodes), fptr(lights), sc.n_lights,
                                       arr, len(tex), C.byref(sc.camera), C.byref(p), fptr(rgba), fptr(depth),
                                       C.byref(st))
        else:
            rc = lib.rt_render_inw(fptr(sc.geom), sc.n, sc.layout, fptr(sc.nodes), fptr(lights), sc.n_lights,
                                   C.byref(sc.camera), C.byref(p), fptr(rgba), fptr(depth), C.byref(st))
    check(rc, "render")
    return rgba, depth, st.as_dict()


def render_iow01(camera: RtCamera, sphere, params: RtParams):
    sc = Scene(stage=RT_STAGE_IOW01, desc=None, n=0, camera=camera, params=params)
    rgba, _, st = render(sc, params, sphere=sphere)
    return rgba, st


def render_iow00(params: RtParams) -> np.ndarray:
    """IOW-00 (In-One-Weekend/base.cpp:7-28): the UV gradient of the base stage."""
    rgba = np.zeros((params.height, params.width, 4), np.float32)
    check(load().rt_render_iow00(C.byref(params), fptr(rgba)), "rt_render_iow00")
    return rgba


def pack_iow02(desc, n: int) -> tuple[np.ndarray, np.ndarray]:
    """Groups::Geometry::FillBuffer (groups.h:45-64): types[N], records[N, 18]."""
    types = np.zeros(n, np.float32)
    rec = np.zeros((n, 18), np.float32)
    check(load().rt_pack_iow02(desc, n, fptr(types), fptr(rec)), "rt_pack_iow02")
    return types, rec


def render_iow02(types, records, camera: RtCamera, params: RtParams, cull_front: int = 0, cull_back: int = 1):
    """IOW-02 groups stage (02_Groups/computeShaderSrc.glsl); defaults cull the back side
    (groups.h:91-92)."""
    types = np.ascontiguousarray(types, np.float32)
    records = np.ascontiguousarray(records, np.float32).reshape(-1, 18)
    rgba = np.zeros((params.height, params.width, 4), np.float32)
    st = RtStats()
    check(load().rt_render_iow02(fptr(types), fptr(records), len(types), C.byref(camera), C.byref(params),
                                 int(cull_front), int(cull_back), fptr(rgba), C.byref(st)), "rt_render_iow02")
    return rgba, st.as_dict()


def render_inw_mf(sc: "Scene", focus, params: RtParams | None = None):
    """INW-01 with the shader's MULTIFOCUS branch (01_BVH...glsl:388-404, 505-549), focus distances
    `focus` (1..9)."""
    p = params or sc.params
    f = np.ascontiguousarray(focus, np.float32)
    rgba = np.zeros((p.height, p.width, 4), np.float32)
    depth = np.zeros((p.height, p.width), np.float32)
    st = RtStats()
    check(load().rt_render_inw_mf(fptr(sc.geom), sc.n, fptr(sc.nodes), C.byref(sc.camera), fptr(f), len(f),
                                  C.byref(p), fptr(rgba), fptr(depth), C.byref(st)), "rt_render_inw_mf")
    return rgba, depth, st.as_dict()


def iow01_defaults(width: int = 400, height: int = 225) -> tuple[RtCamera, np.ndarray, RtParams]:
    """IOW-01 stage defaults (Sphere.h:26,34-37): camera (0,1,10), pitch 0 / yaw -90, focus 1,
    sphere (0,3,-1) r 3, ShowNormal = true."""
    cd = RtCamDesc()
    cd.position[:] = (0.0, 1.0, 10.0)
    cd.pitch_deg, cd.yaw_deg, cd.fov_y_deg, cd.aperture, cd.focus_dist = 0.0, -90.0, 0.0, 0.0, 1.0
    cam = camera_from_desc(cd, RT_STAGE_IOW01)
    p = RtParams()
    p.width, p.height, p.spp, p.max_bounces, p.show_normal, p.device = width, height, 1, 1, 1, -1
    return cam, np.array([0.0, 3.0, -1.0, 3.0], np.float32), p
