"""ctypes binding of the C ABI in include/ipt.h (lib/libipt_amd.so).

This is the only way the package reaches native code; there is no Python or
CPU fallback for any compute entry point.  If the library is missing the
import fails loudly (build it with ``python -c "import __graft_entry__ as g;
g.build()"`` or ``make -C inverse_path_tracer_amd/csrc``).
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# IPT_AMD_LIB selects another build of the same library (A/B profiling of
# kernel variants); the default is the in-tree build.
LIB_PATH = os.environ.get("IPT_AMD_LIB") or os.path.join(_HERE, "lib", "libipt_amd.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "ipt.h")
TRI_EXPORT_STRIDE = 57
ACC_WIDTH = 8
# include/ipt.h ipt_abi_version(): the Params layout and signatures below are this version's
ABI_VERSION = 5
# acceleration modes (include/ipt.h IPT_ACCEL_*)
ACCEL_AUTO, ACCEL_BRUTE, ACCEL_BVH = 0, 1, 2


class NativeError(RuntimeError):
    """A C-ABI call failed; the message is ipt_last_error()."""


class Params(C.Structure):
    """ipt_params_t (include/ipt.h)."""

    _fields_ = [
        ("width", C.c_int32),
        ("height", C.c_int32),
        ("spp", C.c_int32),
        ("max_bounces", C.c_int32),
        ("seed", C.c_uint64),
        ("row_begin", C.c_int32),
        ("row_end", C.c_int32),
        ("row_step", C.c_int32),
    ]

    @property
    def rows(self) -> int:
        """Image rows the launch traces (row_begin, row_begin + row_step, ... < row_end)."""
        n = self.row_end - self.row_begin
        return max(0, -(-n // max(1, self.row_step)))


def make_params(width, height, spp, max_bounces=None, seed=0, row_begin=0, row_end=None, row_step=1) -> Params:
    return Params(int(width), int(height), int(spp), -1 if max_bounces is None else int(max_bounces),
                  int(seed) & 0xFFFFFFFFFFFFFFFF, int(row_begin), int(height if row_end is None else row_end),
                  int(row_step))


_lib = None

vp = C.c_void_p
fp = C.POINTER(C.c_float)
dp = C.POINTER(C.c_double)
u8p = C.POINTER(C.c_uint8)
pp = C.POINTER(Params)

# name -> (restype, argtypes); every symbol include/ipt.h declares.
SIGNATURES = {
    # reference symbols (scene.h:177,195; path_trace.cu:227; inv_path_trace.cu:195,210,216)
    "loadScene": (C.c_int, [C.POINTER(fp), C.POINTER(fp), C.POINTER(fp), C.POINTER(C.c_char_p),
                            C.POINTER(C.c_char_p), C.c_int, C.POINTER(vp)]),
    "freeScene": (None, [vp]),
    "createImage": (None, [vp, C.c_char_p]),
    "createGraph": (None, [vp, C.c_char_p, fp]),
    "getMaterials": (None, [vp, fp]),
    "setMaterials": (None, [vp, fp]),
    # explicit API
    "ipt_last_error": (C.c_char_p, []),
    "ipt_clear_error": (None, []),
    "ipt_abi_version": (C.c_int, []),
    "ipt_device_count": (C.c_int, []),
    "ipt_selftest_math": (C.c_int, [C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]),
    "ipt_debug_fail_launches": (None, [C.c_int]),
    "ipt_debug_adju_ring": (None, [C.c_int, C.c_int]),
    "ipt_legacy_config": (None, [C.c_int, C.c_int, C.c_int, C.c_int, C.c_int64]),
    "ipt_load_scene": (C.c_int, [C.c_int, fp, fp, fp, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p), C.POINTER(vp)]),
    "ipt_load_scene_host": (C.c_int, [C.c_int, fp, fp, fp, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p),
                                      C.POINTER(vp)]),
    "ipt_scene_num_triangles": (C.c_int, [vp]),
    "ipt_scene_num_emissives": (C.c_int, [vp]),
    "ipt_scene_export_triangles": (C.c_int, [vp, fp]),
    "ipt_scene_camera": (C.c_int, [vp, fp]),
    "ipt_scene_get_materials": (C.c_int, [vp, fp]),
    "ipt_scene_set_materials": (C.c_int, [vp, fp]),
    "ipt_render_samples_host": (C.c_int, [vp, pp, fp]),
    "ipt_render_host": (C.c_int, [vp, pp, fp, u8p]),
    "ipt_adjoint_host": (C.c_int, [vp, pp, fp, dp]),
    "ipt_graph_host": (C.c_int, [vp, pp, u8p, dp, fp]),
    "ipt_compress": (C.c_int, [C.c_int, dp, fp]),
    "ipt_render_dev": (C.c_int, [vp, pp, vp, vp, vp, vp]),
    "ipt_render_samples_dev": (C.c_int, [vp, pp, vp, vp, vp]),
    "ipt_pixel_mean_dev": (C.c_int, [vp, C.c_int64, C.c_int, vp, vp, vp]),
    "ipt_render_samples_sm_dev": (C.c_int, [vp, pp, vp, vp, vp]),
    "ipt_pixel_mean_sm_dev": (C.c_int, [vp, C.c_int64, C.c_int, vp, vp, vp]),
    "ipt_adjoint_dev": (C.c_int, [vp, pp, vp, vp, vp, vp]),
    "ipt_graph_dev": (C.c_int, [vp, pp, vp, vp, vp]),
    "ipt_render_batch_dev": (C.c_int, [vp, pp, C.c_int, C.c_uint64, vp, vp, vp]),
    "ipt_adjoint_batch_dev": (C.c_int, [vp, pp, C.c_int, C.c_uint64, vp, vp, vp, vp]),
    "ipt_scene_set_accel": (C.c_int, [vp, C.c_int]),
    "ipt_scene_bvh_info": (C.c_int, [vp, C.POINTER(C.c_int32)]),
    "ipt_scene_export_bvh": (C.c_int, [vp, fp, fp, C.POINTER(C.c_int32)]),
    "ipt_scene_export_wide": (C.c_int, [vp, fp]),
    "ipt_closest_hit_host": (C.c_int, [vp, C.c_int64, fp, fp, C.POINTER(C.c_int32), fp, C.POINTER(C.c_int32)]),
    "ipt_closest_hit_dev": (C.c_int, [vp, C.c_int64, vp, vp, vp, vp, vp, vp]),
    "ipt_scene_shadow_masks": (C.c_int, [vp, C.POINTER(C.c_uint32)]),
    "ipt_shadow_hit_host": (C.c_int, [vp, C.c_int64, fp, fp, C.POINTER(C.c_int32), C.POINTER(C.c_int32), fp,
                                      C.POINTER(C.c_int32)]),
    "ipt_png_write": (C.c_int, [C.c_char_p, C.c_int, C.c_int, u8p]),
    "ipt_png_read": (C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), u8p, C.c_int64]),
}


def lib():
    """Load lib/libipt_amd.so once (raises NativeError if absent)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                "native library %s is missing: build it with `make -C inverse_path_tracer_amd/csrc` "
                "(there is no CPU fallback)" % LIB_PATH)
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        v = L.ipt_abi_version()
        if v != ABI_VERSION:  # a stale build would read ipt_params_t / arguments with another layout
            raise NativeError("%s has ABI %d, this binding needs %d: rebuild it" % (LIB_PATH, v, ABI_VERSION))
        _lib = L
    return _lib


def last_error() -> str:
    return (lib().ipt_last_error() or b"").decode(errors="replace")


def check(rc, what="native call"):
    if rc is not None and rc < 0:
        raise NativeError("%s failed: %s" % (what, last_error()))
    return rc


def device_count() -> int:
    return lib().ipt_device_count()
