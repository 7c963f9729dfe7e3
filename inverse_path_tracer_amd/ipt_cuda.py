"""Module surface of the reference's ipt_cuda.py, as a thin shim.

Callers of /root/reference/ipt_cuda.py (ipt.py:7,139) find the same names,
signatures, return values and buffer layouts here:

* constants: ``lib_ipt``/``lib_pt`` (ipt_cuda.py:7-8; both are the MI355X
  library lib/libipt_amd.so, which exports all six reference symbols), the
  shape tags ``Cube, Sphere, Cornell, Other`` and ``c_int_p``/``c_float_p``;
* scene text: ``rand_mtl``, ``to_string``, ``from_string``, ``load_params``,
  ``ObjParams``, ``dereference`` (ipt_cuda.py:14-107) -- the parsing and
  formatting live in ``scene.py``; this module only packs the results into
  the ctypes records the legacy ``loadScene`` takes;
* the three workflow calls ``generate_files``, ``generate_data`` and
  ``render_with_materials`` (ipt_cuda.py:115-183), which drive the legacy C
  symbols (createImage / createGraph render the configuration set by
  ``ipt_legacy_config``, default 500x500, 100 spp, unbounded, time seed).

Differences, all deliberate: a failing native call raises
``NativeError`` (the reference's library exit(1)s or silently writes
nothing); ``render_with_materials`` also accepts a numpy array.
"""
import os
from ctypes import POINTER, Structure, c_char_p, c_float, c_int, c_void_p, cdll, pointer

import numpy as np

from . import _native
from .scene import format_object_block, inline_kd, parse_object_block, parse_scene_text

try:  # the reference shows a progress bar while generating scenes
    from tqdm import tqdm as _progress
except Exception:  # pragma: no cover
    def _progress(it):
        return it

_native.lib()  # no library -> NativeError here (there is no fallback)
lib_ipt = cdll.LoadLibrary(_native.LIB_PATH)
lib_pt = lib_ipt
Cube, Sphere, Cornell, Other = range(4)
c_int_p = POINTER(c_int)
c_float_p = POINTER(c_float)

# shape tag -> (OBJ, fixed MTL or None = a random inline diffuse material)
_SHAPES = {
    Cube: ("./shapes/cube.obj", None),
    Sphere: ("./shapes/sphere.obj", None),
    Cornell: ("./CornellBox/CornellBox-Empty-CO.obj", "./CornellBox/CornellBox-Empty-CO.mtl"),
}


def rand_mtl():
    """Inline material with three uniform draws from numpy's global RNG."""
    return inline_kd([np.random.uniform() for _ in range(3)])


def to_string(shp=None, pos=None, ori=None, scl=None, obj_file=None, mtl_file=None):
    """One OBJECT block's text; a shape tag fixes the OBJ (and MTL) path."""
    if shp in _SHAPES:
        obj_file, fixed = _SHAPES[shp]
        if fixed is not None:
            mtl_file = fixed
        elif mtl_file is None:
            mtl_file = rand_mtl()
    assert obj_file is not None and mtl_file is not None
    return format_object_block(obj_file, mtl_file, pos, ori, scl)


class ObjParams(Structure):
    """ctypes record of one object (field layout of the reference's ObjParams)."""

    _fields_ = [("shp", c_int), ("pos", c_float * 3), ("ori", c_float * 3), ("scl", c_float * 3),
                ("obj_file", c_char_p), ("mtl_file", c_char_p)]

    def __init__(self, pos, ori, scl, obj_file, mtl_file):
        super().__init__()
        for name, v in (("pos", pos), ("ori", ori), ("scl", scl)):
            setattr(self, name, (c_float * 3)(*v))
        self.obj_file = c_char_p(obj_file.encode("utf-8"))
        self.mtl_file = c_char_p(mtl_file.encode("utf-8"))


def _record(spec):
    return ObjParams(spec.pos, spec.ori, spec.scl, spec.obj_file, spec.mtl_file)


def from_string(string):
    try:
        spec = parse_object_block(string)
    except ValueError as e:  # the reference asserts
        raise AssertionError(str(e))
    return _record(spec)


def dereference(py_objects):
    """Parallel pointer arrays + count: loadScene's first six arguments."""
    objs = list(py_objects)
    n = len(objs)

    def column(ctype, field):
        return (ctype * n)(*[getattr(o, field) for o in objs])

    return (column(c_float_p, "pos"), column(c_float_p, "ori"), column(c_float_p, "scl"),
            column(c_char_p, "obj_file"), column(c_char_p, "mtl_file"), n)


def load_params(filename):
    with open(filename, "r") as f:
        specs = parse_scene_text(f.read())
    return dereference([_record(s) for s in specs])


def _checked(what, rc=None):
    err = _native.last_error()
    if err or (rc is not None and rc < 0):
        raise _native.NativeError("%s failed: %s" % (what, err or "error"))
    return rc


def load_scene(scenefile):
    """(nT, scene handle) of a scene file; paths resolve against the CWD."""
    handle = c_void_p(0)
    _native.lib().ipt_clear_error()
    n_t = _checked("loadScene", lib_pt.loadScene(*load_params(scenefile), pointer(handle)))
    return n_t, handle


def _create_image(handle, png_path):
    """createImage + freeScene, raising if the render or the PNG write failed."""
    _native.lib().ipt_clear_error()
    lib_pt.createImage(handle, c_char_p(png_path.encode("utf-8")))
    err = _native.last_error()
    lib_ipt.freeScene(handle)
    if err:
        raise _native.NativeError("createImage(%s) failed: %s" % (png_path, err))


def generate_files(n):
    """scenes/{i}.txt (Cornell box + a cube with a random diffuse colour) and
    imgs/{i}.png, its legacy-configuration render, for i < n."""
    os.makedirs("scenes", exist_ok=True)
    os.makedirs("imgs", exist_ok=True)
    for i in _progress(range(n)):
        text = ("OBJECT\n" + to_string(shp=Cornell, pos=np.array([0, 0, 4]), scl=np.ones(3) * 2) +
                "OBJECT\n" + to_string(shp=Cube, pos=np.array([0, -1.5, 4])))
        path = "scenes/%d.txt" % i
        with open(path, "w") as f:
            f.write(text)
        _, handle = load_scene(path)
        _create_image(handle, "imgs/%d.png" % i)


def generate_data(scenefile, imgfile):
    """createGraph against imgfile + getMaterials: (w (nT+1, nT),
    pixel (nT+1, nT, 3), light (nT+1, nT, 3), labels (nT, 3)), float64."""
    n_t, handle = load_scene(scenefile)
    rows = (n_t + 1) * n_t
    flat = np.zeros(rows * 7, np.float32)
    labels = np.zeros(n_t * 3, np.float32)
    _native.lib().ipt_clear_error()
    lib_ipt.createGraph(handle, c_char_p(imgfile.encode("utf-8")), flat.ctypes.data_as(c_float_p))
    err = _native.last_error()
    lib_ipt.getMaterials(handle, labels.ctypes.data_as(c_float_p))
    lib_ipt.freeScene(handle)
    if err:
        raise _native.NativeError("createGraph failed: %s" % err)
    w, pixel, light = np.split(flat.astype(np.float64), [rows, 4 * rows])
    pixel = pixel.reshape(n_t + 1, n_t, 3)
    assert not np.isnan(pixel).any()
    return w.reshape(n_t + 1, n_t), pixel, light.reshape(n_t + 1, n_t, 3), labels.astype(np.float64).reshape(n_t, 3)


def render_with_materials(scenefile, imgfile, materials):
    """Legacy-configuration render of scenefile with per-triangle diffuse
    albedo `materials` (nT, 3) (torch tensor or array) written to imgfile."""
    _, handle = load_scene(scenefile)
    kd = materials.detach().cpu().numpy() if hasattr(materials, "detach") else np.asarray(materials)
    kd = np.ascontiguousarray(kd, np.float32)
    lib_ipt.setMaterials(handle, kd.ctypes.data_as(c_float_p))
    err = _native.last_error()
    if err:
        lib_ipt.freeScene(handle)
        raise _native.NativeError("setMaterials failed: %s" % err)
    _create_image(handle, imgfile)
