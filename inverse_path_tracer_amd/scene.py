"""Scene: the reference's scene-file format and a handle on the native scene.

Scene text format (ipt_cuda.py:17-59, 91-107): blocks introduced by a line
``OBJECT``, each with optional ``POS x y z``, ``ORI x y z`` (axis*angle),
``SCL x y z`` and mandatory ``OBJ path`` and ``MTL path-or-*Kd r g b*``.
Paths are resolved like the reference (relative to the current directory);
``Scene.from_file`` also accepts a ``root`` to resolve them against.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _native as N


@dataclass
class ObjectSpec:
    """One OBJECT block (the fields of ipt_cuda.ObjParams, ipt_cuda.py:61-78)."""

    obj_file: str
    mtl_file: str
    pos: Sequence[float] = (0.0, 0.0, 0.0)
    ori: Sequence[float] = (0.0, 0.0, 0.0)
    scl: Sequence[float] = (1.0, 1.0, 1.0)


def parse_object_block(text: str) -> ObjectSpec:
    """from_string (ipt_cuda.py:39-59): later keys win, defaults 0/0/1."""
    pos = ori = scl = obj = mtl = None
    for line in text.split("\n"):
        items = line.strip().split(" ")
        token, values = items[0], items[1:]
        if token == "POS":
            pos = [float(x) for x in values]
        elif token == "ORI":
            ori = [float(x) for x in values]
        elif token == "SCL":
            scl = [float(x) for x in values]
        elif token == "OBJ":
            obj = values[0]
        elif token == "MTL":
            mtl = " ".join(values)
    if obj is None or mtl is None:
        raise ValueError("OBJECT block without OBJ/MTL: %r" % text)
    return ObjectSpec(obj, mtl, pos if pos is not None else [0.0] * 3, ori if ori is not None else [0.0] * 3,
                      scl if scl is not None else [1.0] * 3)


def format_object_block(obj_file: str, mtl_file: str, pos=None, ori=None, scl=None) -> str:
    """Inverse of parse_object_block in the reference's spelling (ipt_cuda.py:17-37
    to_string): optional POS/ORI/SCL lines with each value printed by str(),
    then OBJ and MTL."""
    keys = (("POS", pos), ("ORI", ori), ("SCL", scl))
    head = "".join("%s %s\n" % (k, " ".join(str(x) for x in v[:3])) for k, v in keys if v is not None)
    return head + "OBJ %s\nMTL %s\n" % (obj_file, mtl_file)


def inline_kd(kd: Sequence[float]) -> str:
    """The inline material string ``*Kd r g b*`` (ipt_cuda.py:14-15)."""
    return "*Kd %s*" % " ".join(str(x) for x in kd)


def parse_scene_text(text: str) -> List[ObjectSpec]:
    """load_params (ipt_cuda.py:91-107)."""
    objects, cur = [], ""
    for line in text.splitlines(True):
        line = line.strip()
        if line == "OBJECT":
            if len(cur) > 0:
                objects.append(parse_object_block(cur))
            cur = ""
        else:
            cur += line + "\n"
    objects.append(parse_object_block(cur))
    return objects


def _resolve(path: str, roots: Sequence[str]) -> str:
    if path.startswith("*") or os.path.isabs(path):
        return path
    for r in roots:
        cand = os.path.normpath(os.path.join(r, path))
        if os.path.exists(cand):
            return cand
    return path


class Scene:
    """A scene loaded on the current HIP device (loadScene, scene.h:177-193)."""

    def __init__(self, objects: Sequence[ObjectSpec], device: bool = True):
        L = N.lib()
        n = len(objects)
        self.objects = list(objects)
        pos = np.array([o.pos for o in objects], np.float32).reshape(n, 3)
        ori = np.array([o.ori for o in objects], np.float32).reshape(n, 3)
        scl = np.array([o.scl for o in objects], np.float32).reshape(n, 3)
        objs = (C.c_char_p * n)(*[o.obj_file.encode() for o in objects])
        mtls = (C.c_char_p * n)(*[o.mtl_file.encode() for o in objects])
        h = C.c_void_p(0)
        load = L.ipt_load_scene if device else L.ipt_load_scene_host
        nT = load(n, pos.ctypes.data_as(N.fp), ori.ctypes.data_as(N.fp), scl.ctypes.data_as(N.fp),
                              objs, mtls, C.byref(h))
        if nT < 0:
            raise N.NativeError("loadScene failed: %s" % N.last_error())
        self.handle = h
        self.nT = nT
        self.nE = L.ipt_scene_num_emissives(h)

    @classmethod
    def from_file(cls, path: str, root: Optional[str] = None, device: bool = True) -> "Scene":
        with open(path) as f:
            objects = parse_scene_text(f.read())
        roots = [root] if root else []
        roots += [os.getcwd(), os.path.dirname(os.path.dirname(os.path.abspath(path))),
                  os.path.dirname(os.path.abspath(path))]
        for o in objects:
            o.obj_file = _resolve(o.obj_file, roots)
            o.mtl_file = _resolve(o.mtl_file, roots)
        return cls(objects, device=device)

    def close(self):
        if getattr(self, "handle", None) and self.handle.value:
            N.lib().freeScene(self.handle)
            self.handle = C.c_void_p(0)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------- materials
    @property
    def materials(self) -> np.ndarray:
        """Per-triangle diffuse Kd, (nT, 3) float32 (getMaterials)."""
        out = np.zeros((self.nT, 3), np.float32)
        N.check(N.lib().ipt_scene_get_materials(self.handle, out.ctypes.data_as(N.fp)), "getMaterials")
        return out

    @materials.setter
    def materials(self, kd):
        kd = np.ascontiguousarray(np.asarray(kd, np.float32).reshape(self.nT, 3))
        N.check(N.lib().ipt_scene_set_materials(self.handle, kd.ctypes.data_as(N.fp)), "setMaterials")

    def triangles(self) -> np.ndarray:
        out = np.zeros((self.nT, N.TRI_EXPORT_STRIDE), np.float32)
        N.check(N.lib().ipt_scene_export_triangles(self.handle, out.ctypes.data_as(N.fp)), "export")
        return out

    def camera(self) -> np.ndarray:
        out = np.zeros(16, np.float32)
        N.check(N.lib().ipt_scene_camera(self.handle, out.ctypes.data_as(N.fp)), "camera")
        return out.reshape(4, 4)

    # ---------------------------------------------------------- acceleration
    def set_accel(self, mode: int):
        """IPT_ACCEL_AUTO / _BRUTE / _BVH (N.ACCEL_*): which closest-hit loop
        the kernels run.  Results are identical; only speed differs."""
        N.check(N.lib().ipt_scene_set_accel(self.handle, int(mode)), "set_accel")

    def bvh_info(self) -> dict:
        info = (C.c_int32 * 8)()
        has = N.lib().ipt_scene_bvh_info(self.handle, info)
        N.check(has, "bvh_info")
        return {"has_bvh": bool(has), "nodes": info[0], "pairs": info[1], "depth": info[2], "big_pairs": info[4],
                "wide_nodes": info[5], "wide_depth": info[6], "wide_tris": info[7],
                "accel": {N.ACCEL_BRUTE: "brute", N.ACCEL_BVH: "bvh"}.get(info[3], "?"),
                "status": "ok" if has else N.last_error()}

    def export_bvh(self):
        """(nodes[n,16] float32, pairs[m,40] float32, big_idx[2k] int32) --
        BvhNode / BvhPair records (scene_layout.h; child links and indices are
        int32 bits) and the large triangles tested before the traversal."""
        i = self.bvh_info()
        nodes = np.zeros((i["nodes"], 16), np.float32)
        pairs = np.zeros((i["pairs"], 40), np.float32)
        big = np.zeros(2 * i["big_pairs"], np.int32)
        N.check(N.lib().ipt_scene_export_bvh(self.handle, nodes.ctypes.data_as(N.fp), pairs.ctypes.data_as(N.fp),
                                             big.ctypes.data_as(C.POINTER(C.c_int32))), "export_bvh")
        return nodes, pairs, big

    def export_wide(self):
        """wide[n,8,8] float32: the cooperative traversal's 8-wide nodes
        (WideNode, scene_layout.h; child refs are int32 bits)."""
        n = self.bvh_info()["wide_nodes"]
        wide = np.zeros((n, 8, 8), np.float32)
        N.check(N.lib().ipt_scene_export_wide(self.handle, wide.ctypes.data_as(N.fp)), "export_wide")
        return wide

    def closest_hit(self, origins, dirs, targets=None):
        """The kernels' cast on caller rays: (t float32[n], idx int32[n])."""
        o = np.ascontiguousarray(np.asarray(origins, np.float32).reshape(-1, 3))
        d = np.ascontiguousarray(np.asarray(dirs, np.float32).reshape(-1, 3))
        n = o.shape[0]
        t = np.zeros(n, np.float32)
        idx = np.zeros(n, np.int32)
        tg = None
        if targets is not None:
            tg = np.ascontiguousarray(np.asarray(targets, np.int32).reshape(n))
        ip = C.POINTER(C.c_int32)
        N.check(N.lib().ipt_closest_hit_host(self.handle, n, o.ctypes.data_as(N.fp), d.ctypes.data_as(N.fp),
                                             tg.ctypes.data_as(ip) if tg is not None else None,
                                             t.ctypes.data_as(N.fp), idx.ctypes.data_as(ip)), "closest_hit")
        return t, idx

    def shadow_masks(self):
        """uint32[nT, max(nE, 1)]: the shadow rays' potential-occluder pair masks."""
        m = np.zeros((self.nT, max(1, self.nE)), np.uint32)
        N.check(N.lib().ipt_scene_shadow_masks(self.handle, m.ctypes.data_as(C.POINTER(C.c_uint32))), "shadow_masks")
        return m

    def shadow_hit(self, origins, dirs, targets, sources):
        """Shadow rays as the megakernel casts them from a vertex on triangle
        sources[i] (< 0: unknown) towards emitter triangle targets[i]."""
        o = np.ascontiguousarray(np.asarray(origins, np.float32).reshape(-1, 3))
        d = np.ascontiguousarray(np.asarray(dirs, np.float32).reshape(-1, 3))
        n = o.shape[0]
        t = np.zeros(n, np.float32)
        idx = np.zeros(n, np.int32)
        tg = np.ascontiguousarray(np.asarray(targets, np.int32).reshape(n))
        sr = np.ascontiguousarray(np.asarray(sources, np.int32).reshape(n))
        ip = C.POINTER(C.c_int32)
        N.check(N.lib().ipt_shadow_hit_host(self.handle, n, o.ctypes.data_as(N.fp), d.ctypes.data_as(N.fp),
                                            tg.ctypes.data_as(ip), sr.ctypes.data_as(ip), t.ctypes.data_as(N.fp),
                                            idx.ctypes.data_as(ip)), "shadow_hit")
        return t, idx

    # ---------------------------------------------------------- host-memory renders
    def render_samples(self, width, height, spp, max_bounces=None, seed=0, row_begin=0, row_end=None, row_step=1):
        p = N.make_params(width, height, spp, max_bounces, seed, row_begin, row_end, row_step)
        out = np.zeros((p.rows * width * spp, 3), np.float32)
        N.check(N.lib().ipt_render_samples_host(self.handle, C.byref(p), out.ctypes.data_as(N.fp)), "render_samples")
        return out

    def render(self, width, height, spp, max_bounces=None, seed=0, row_begin=0, row_end=None, ldr=False, row_step=1):
        """HDR image (rows, W, 3) = per-pixel mean of the samples (+ 8-bit tonemap)."""
        p = N.make_params(width, height, spp, max_bounces, seed, row_begin, row_end, row_step)
        rows = p.rows
        hdr = np.zeros((rows, width, 3), np.float32)
        u8 = np.zeros((rows, width, 3), np.uint8) if ldr else None
        N.check(N.lib().ipt_render_host(self.handle, C.byref(p), hdr.ctypes.data_as(N.fp),
                                        u8.ctypes.data_as(N.u8p) if ldr else None), "render")
        return (hdr, u8) if ldr else hdr

    def adjoint(self, adj, width, height, spp, max_bounces, seed=0, row_begin=0, row_end=None, row_step=1):
        """d(sum(adj * I))/dKd as (nT, 3) float64; adj is (H, W, 3)."""
        p = N.make_params(width, height, spp, max_bounces, seed, row_begin, row_end, row_step)
        adj = np.ascontiguousarray(np.asarray(adj, np.float32).reshape(height, width, 3))
        g = np.zeros((self.nT, 3), np.float64)
        N.check(N.lib().ipt_adjoint_host(self.handle, C.byref(p), adj.ctypes.data_as(N.fp),
                                         g.ctypes.data_as(N.dp)), "adjoint")
        return g

    def graph(self, target, width, height, spp, max_bounces=None, seed=0, row_begin=0, row_end=None, row_step=1):
        """createGraph: returns (acc[(nT+1)*nT, 8] float64, data[(nT+1)*nT*7] float32)."""
        p = N.make_params(width, height, spp, max_bounces, seed, row_begin, row_end, row_step)
        target = np.ascontiguousarray(np.asarray(target, np.uint8).reshape(height, width, 3))
        acc = np.zeros(((self.nT + 1) * self.nT, N.ACC_WIDTH), np.float64)
        data = np.zeros((self.nT + 1) * self.nT * 7, np.float32)
        N.check(N.lib().ipt_graph_host(self.handle, C.byref(p), target.ctypes.data_as(N.u8p),
                                       acc.ctypes.data_as(N.dp), data.ctypes.data_as(N.fp)), "graph")
        return acc, data


def compress(nT: int, acc: np.ndarray) -> np.ndarray:
    """DataWrapper::compress (inv_scene.h:87-115) of fp64 bins."""
    acc = np.ascontiguousarray(acc, np.float64)
    data = np.zeros((nT + 1) * nT * 7, np.float32)
    N.check(N.lib().ipt_compress(nT, acc.ctypes.data_as(N.dp), data.ctypes.data_as(N.fp)), "compress")
    return data


def unpack_graph(nT: int, data: np.ndarray):
    """Split createGraph output like generate_data (ipt_cuda.py:153-163)."""
    size = (nT + 1) * nT
    data = np.asarray(data).astype(np.float64)
    w = data[:size].reshape(nT + 1, nT)
    pixel = data[size:size * 4].reshape(nT + 1, nT, 3)
    light = data[size * 4:].reshape(nT + 1, nT, 3)
    return w, pixel, light


def png_write(path: str, rgb: np.ndarray):
    rgb = np.ascontiguousarray(rgb, np.uint8)
    H, W = rgb.shape[:2]
    N.check(N.lib().ipt_png_write(path.encode(), W, H, rgb.ctypes.data_as(N.u8p)), "png_write")


def png_read(path: str) -> np.ndarray:
    w, h = C.c_int(0), C.c_int(0)
    N.check(N.lib().ipt_png_read(path.encode(), C.byref(w), C.byref(h), None, 0), "png_read")
    out = np.zeros((h.value, w.value, 3), np.uint8)
    N.check(N.lib().ipt_png_read(path.encode(), C.byref(w), C.byref(h), out.ctypes.data_as(N.u8p), out.size),
            "png_read")
    return out
