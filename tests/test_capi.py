"""The drop-in boundary: the C-ABI library loads without a GPU and exports
every symbol include/ipt.h declares; the reference-named copies exist; the
ipt_cuda mirror keeps the reference's module surface and scene format."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ASSETS, ROOT, TESTS

HEADER = os.path.join(ROOT, "include", "ipt.h")
LEGACY = ["loadScene", "freeScene", "createImage", "createGraph", "getMaterials", "setMaterials"]


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", text)
    return sorted(set(n for n in names if n not in ("sizeof",)))


def test_header_declares_reference_symbols():
    names = declared_functions()
    for s in LEGACY:
        assert s in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    from inverse_path_tracer_amd import _native as N

    L = N.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
        assert name in N.SIGNATURES, "python binding lacks %s" % name
    assert L.ipt_abi_version() == 5


@pytest.mark.parametrize("soname", ["libpt.so", "libipt.so"])
def test_reference_sonames(soname):
    """ipt_cuda.py:7-8 loads ./build/libipt.so and ./build/libpt.so."""
    path = os.path.join(ROOT, "build", soname)
    assert os.path.exists(path), "run __graft_entry__.build()"
    L = C.CDLL(path)
    for s in LEGACY:
        assert hasattr(L, s)


def test_ipt_cuda_surface():
    from inverse_path_tracer_amd import ipt_cuda as M

    for name in ["rand_mtl", "to_string", "from_string", "ObjParams", "dereference", "load_params", "load_scene",
                 "generate_files", "generate_data", "render_with_materials", "lib_ipt", "lib_pt", "Cube", "Sphere",
                 "Cornell", "Other", "c_float_p", "c_int_p"]:
        assert hasattr(M, name), name
    assert (M.Cube, M.Sphere, M.Cornell, M.Other) == (0, 1, 2, 3)


def test_scene_text_roundtrip():
    from inverse_path_tracer_amd import ipt_cuda as M
    from inverse_path_tracer_amd.scene import parse_scene_text

    s = M.to_string(shp=M.Cornell, pos=np.array([0, 0, 4]), scl=np.ones(3) * 2)
    assert s == ("POS 0 0 4\nSCL 2.0 2.0 2.0\nOBJ ./CornellBox/CornellBox-Empty-CO.obj\n"
                 "MTL ./CornellBox/CornellBox-Empty-CO.mtl\n")
    o = M.from_string(s)
    assert list(o.pos) == [0, 0, 4] and list(o.ori) == [0, 0, 0] and list(o.scl) == [2, 2, 2]
    assert o.obj_file == b"./CornellBox/CornellBox-Empty-CO.obj"
    cube = M.to_string(shp=M.Cube, pos=np.array([0, -1.5, 4]))
    assert re.match(r"POS 0.0 -1.5 4.0\nOBJ ./shapes/cube.obj\nMTL \*Kd \S+ \S+ \S+\*\n$", cube)
    with open(os.path.join(ASSETS, "scenes", "0.txt")) as f:
        text = f.read()
    objs = parse_scene_text(text)
    assert len(objs) == 2 and objs[1].mtl_file.startswith("*Kd 0.904")
    poss, oris, scls, objf, mtlf, n = M.load_params(os.path.join(ASSETS, "scenes", "0.txt"))
    assert n == 2 and list(poss[1][:3]) == [0.0, -1.5, 4.0] and mtlf[1] == objs[1].mtl_file.encode()
    with pytest.raises(AssertionError):
        M.from_string("POS 1 2 3\n")


def test_png_roundtrip_and_decode_reference_png(tmp_path):
    from PIL import Image

    from inverse_path_tracer_amd import png_read, png_write

    img = np.random.RandomState(0).randint(0, 256, (37, 53, 3)).astype(np.uint8)
    p = str(tmp_path / "x.png")
    png_write(p, img)
    assert np.array_equal(png_read(p), img)
    assert np.array_equal(np.asarray(Image.open(p).convert("RGB")), img)
    ref = os.path.join(TESTS, "golden", "preds_0_true.png")
    assert np.array_equal(png_read(ref), np.asarray(Image.open(ref).convert("RGB")))
    for mode in ("L", "RGBA", "P"):
        q = str(tmp_path / ("m_%s.png" % mode))
        Image.fromarray(img).convert(mode).save(q)
        assert np.array_equal(png_read(q), np.asarray(Image.open(q).convert("RGB")))


def test_png_errors(tmp_path):
    from inverse_path_tracer_amd import NativeError, png_read

    bad = tmp_path / "bad.png"
    bad.write_bytes(b"not a png")
    with pytest.raises(NativeError, match="not a PNG"):
        png_read(str(bad))
    with pytest.raises(NativeError):
        png_read(str(tmp_path / "missing.png"))


def test_compress_matches_oracle(oracle):
    from inverse_path_tracer_amd import compress

    nT = 30
    acc = np.random.RandomState(5).uniform(0, 10, ((nT + 1) * nT, 8))
    acc[::7] = 0.0
    assert np.array_equal(compress(nT, acc).view(np.uint32), oracle.compress(nT, acc).view(np.uint32))


def test_shard_rows_partition():
    from inverse_path_tracer_amd.distributed import frame_seed, shard_rows

    for H in (1, 7, 512, 1024, 1000):
        for W in (1, 2, 3, 8):
            bands = [shard_rows(H, W, r) for r in range(W)]
            assert bands[0][0] == 0 and bands[-1][1] == H
            assert all(b[1] == c[0] for b, c in zip(bands, bands[1:]))
            assert max(e - b for b, e in bands) - min(e - b for b, e in bands) <= 1
    assert frame_seed(0, 2, 512, 512, 64) == 2 * 512 * 512 * 64


def test_interleaved_shares_partition_rows():
    from inverse_path_tracer_amd import _native as N
    from inverse_path_tracer_amd.distributed import shard_rows_interleaved

    for H in (1, 7, 512, 1024, 1000):
        for W in (1, 2, 3, 8, 13):
            rows = []
            for r in range(W):
                b, e, s = shard_rows_interleaved(H, W, r)
                rows += list(range(b, e, s))
                assert N.make_params(16, H, 1, 2, 0, b, e, s).rows == len(range(b, e, s))
            assert sorted(rows) == list(range(H))
