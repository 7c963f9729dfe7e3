"""ctypes binding of the CPU oracle (oracle/build/libipt_oracle.so).

TEST INFRASTRUCTURE: only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg import this module.  The product never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "libipt_oracle.so")
# -O3 x86-64-v3 build with FMA contraction: timed CPU baseline only, never a checker
FAST_LIB_PATH = os.path.join(ROOT, "oracle", "build", "libipt_oracle_fast.so")
TRI_STRIDE = 57

_lib = None
_libs = {}


def build():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)


def lib(fast=False):
    """The parity build (default) or the fast build of the oracle."""
    global _lib
    if fast:
        if "fast" not in _libs:
            if not os.path.exists(FAST_LIB_PATH):
                build()
            _libs["fast"] = _bind(C.CDLL(FAST_LIB_PATH))
        return _libs["fast"]
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        _lib = _bind(C.CDLL(LIB_PATH))
    return _lib


def _bind(L):
    """ctypes signatures of the oracle's C API."""
    vp, fp, dp, i64 = C.c_void_p, C.POINTER(C.c_float), C.POINTER(C.c_double), C.c_int64
    L.oro_load_scene.restype = vp
    L.oro_load_scene.argtypes = [C.c_int, fp, fp, fp, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p)]
    L.oro_free_scene.argtypes = [vp]
    L.oro_last_error.restype = C.c_char_p
    L.oro_num_triangles.argtypes = [vp]
    L.oro_num_emissives.argtypes = [vp]
    L.oro_export_triangles.argtypes = [vp, fp]
    L.oro_get_materials.argtypes = [vp, fp]
    L.oro_set_materials.argtypes = [vp, fp]
    L.oro_camera_matrix.argtypes = [vp, fp]
    L.oro_render_samples.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, i64, i64, fp, C.POINTER(i64)]
    L.oro_pixel_mean.argtypes = [fp, i64, C.c_int, fp, C.POINTER(C.c_uint8)]
    L.oro_graph.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int, C.POINTER(C.c_uint8), dp, fp]
    L.oro_graph_casts.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int,
                                  C.POINTER(C.c_int64)]
    L.oro_compress.argtypes = [C.c_int, dp, fp]
    L.oro_adjoint.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint64, C.c_int, C.c_int, fp, dp]
    L.oro_uniform_at.restype = C.c_float
    L.oro_uniform_at.argtypes = [C.c_uint64, C.c_int]
    L.oro_sincos.argtypes = [C.c_float, fp, fp]
    L.oro_log.restype = C.c_double
    L.oro_log.argtypes = [C.c_double]
    L.oro_exp.restype = C.c_double
    L.oro_exp.argtypes = [C.c_double]
    L.oro_powf.restype = C.c_float
    L.oro_powf.argtypes = [C.c_float, C.c_float]
    L.oro_set_threads.argtypes = [C.c_int]
    ip = C.POINTER(C.c_int)
    L.oro_closest_hit.argtypes = [vp, i64, fp, fp, fp, ip]
    L.oro_hit_each.argtypes = [vp, fp, fp, fp]
    return L


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _dp(a):
    return a.ctypes.data_as(C.POINTER(C.c_double))


class OracleScene:
    """Scene loaded by the oracle from (pos, ori, scl, obj, mtl) object records."""

    def __init__(self, objects, fast=False):
        self.L = L = lib(fast)
        n = len(objects)
        self._poss = np.array([o[0] for o in objects], np.float32).reshape(n, 3)
        self._oris = np.array([o[1] for o in objects], np.float32).reshape(n, 3)
        self._scls = np.array([o[2] for o in objects], np.float32).reshape(n, 3)
        objs = (C.c_char_p * n)(*[o[3].encode() for o in objects])
        mtls = (C.c_char_p * n)(*[o[4].encode() for o in objects])
        self.ptr = L.oro_load_scene(n, _fp(self._poss), _fp(self._oris), _fp(self._scls), objs, mtls)
        if not self.ptr:
            raise RuntimeError("oracle load failed: %s" % L.oro_last_error().decode())
        self.nT = L.oro_num_triangles(self.ptr)
        self.nE = L.oro_num_emissives(self.ptr)

    def __del__(self):
        try:
            if getattr(self, "ptr", None) and getattr(self, "L", None) is not None:
                self.L.oro_free_scene(self.ptr)
                self.ptr = None
        except Exception:
            pass

    def triangles(self):
        out = np.zeros((self.nT, TRI_STRIDE), np.float32)
        self.L.oro_export_triangles(self.ptr, _fp(out))
        return out

    def camera(self):
        out = np.zeros(16, np.float32)
        self.L.oro_camera_matrix(self.ptr, _fp(out))
        return out.reshape(4, 4)

    def get_materials(self):
        out = np.zeros((self.nT, 3), np.float32)
        self.L.oro_get_materials(self.ptr, _fp(out))
        return out

    def set_materials(self, kd):
        kd = np.ascontiguousarray(kd, np.float32).reshape(self.nT, 3)
        self.L.oro_set_materials(self.ptr, _fp(kd))

    def render_samples(self, W, H, spp, max_bounces, seed, s_begin=0, s_end=None):
        if s_end is None:
            s_end = W * H * spp
        out = np.zeros((s_end - s_begin, 3), np.float32)
        casts = C.c_int64(0)
        rc = self.L.oro_render_samples(self.ptr, W, H, spp, -1 if max_bounces is None else max_bounces,
                                      seed, s_begin, s_end, _fp(out), C.byref(casts))
        if rc:
            raise RuntimeError(self.L.oro_last_error().decode())
        return out, casts.value

    def render(self, W, H, spp, max_bounces, seed):
        s, casts = self.render_samples(W, H, spp, max_bounces, seed)
        hdr, u8 = pixel_mean(s, W * H, spp)
        return hdr.reshape(H, W, 3), u8.reshape(H, W, 3), casts

    def graph(self, W, H, spp, max_bounces, seed, target, row_begin=0, row_end=None):
        row_end = H if row_end is None else row_end
        target = np.ascontiguousarray(target, np.uint8).reshape(H, W, 3)
        acc = np.zeros(((self.nT + 1) * self.nT, 8), np.float64)
        data = np.zeros((self.nT + 1) * self.nT * 7, np.float32)
        rc = self.L.oro_graph(self.ptr, W, H, spp, -1 if max_bounces is None else max_bounces, seed,
                             row_begin, row_end, target.ctypes.data_as(C.POINTER(C.c_uint8)), _dp(acc), _fp(data))
        if rc:
            raise RuntimeError(self.L.oro_last_error().decode())
        return acc, data

    def graph_casts(self, W, H, spp, max_bounces, seed, row_begin=0, row_end=None):
        """Path + shadow casts of createGraph's integrator over rows [row_begin, row_end)."""
        row_end = H if row_end is None else row_end
        n = C.c_int64(0)
        rc = self.L.oro_graph_casts(self.ptr, W, H, spp, -1 if max_bounces is None else max_bounces, seed,
                                    row_begin, row_end, C.byref(n))
        if rc:
            raise RuntimeError(self.L.oro_last_error().decode())
        return n.value

    def adjoint(self, W, H, spp, max_bounces, seed, adj, row_begin=0, row_end=None):
        row_end = H if row_end is None else row_end
        adj = np.ascontiguousarray(adj, np.float32).reshape(H, W, 3)
        grad = np.zeros((self.nT, 3), np.float64)
        rc = self.L.oro_adjoint(self.ptr, W, H, spp, -1 if max_bounces is None else max_bounces, seed, row_begin,
                                row_end, _fp(adj), _dp(grad))
        if rc:
            raise RuntimeError(self.L.oro_last_error().decode())
        return grad


    def closest_hit(self, origins, dirs):
        o = np.ascontiguousarray(np.asarray(origins, np.float32).reshape(-1, 3))
        d = np.ascontiguousarray(np.asarray(dirs, np.float32).reshape(-1, 3))
        n = o.shape[0]
        t = np.zeros(n, np.float32)
        idx = np.zeros(n, np.int32)
        self.L.oro_closest_hit(self.ptr, n, _fp(o), _fp(d), _fp(t), idx.ctypes.data_as(C.POINTER(C.c_int)))
        return t, idx

    def hit_each(self, origin, direction):
        o = np.ascontiguousarray(np.asarray(origin, np.float32).reshape(3))
        d = np.ascontiguousarray(np.asarray(direction, np.float32).reshape(3))
        t = np.zeros(self.L.oro_num_triangles(self.ptr), np.float32)
        self.L.oro_hit_each(self.ptr, _fp(o), _fp(d), _fp(t))
        return t


def pixel_mean(samples, npix, spp):
    samples = np.ascontiguousarray(samples, np.float32)
    hdr = np.zeros((npix, 3), np.float32)
    u8 = np.zeros((npix, 3), np.uint8)
    lib().oro_pixel_mean(_fp(samples), npix, spp, _fp(hdr), u8.ctypes.data_as(C.POINTER(C.c_uint8)))
    return hdr, u8


def compress(nT, acc):
    acc = np.ascontiguousarray(acc, np.float64)
    data = np.zeros((nT + 1) * nT * 7, np.float32)
    lib().oro_compress(nT, _dp(acc), _fp(data))
    return data
