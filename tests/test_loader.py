"""Scene ingest: the product's C++ loader (host-only handle, no GPU) against
the oracle's C restatement of tinyobjloader/MTL/Mesh/Triangle, bit for bit."""
import os

import numpy as np
import pytest

from conftest import ASSETS, CORNELL, CUBE_KD, SCENE0, SPHERE_OBJ, product_scene


def _bits(a):
    return np.asarray(a, np.float32).view(np.uint32)


def _same(records, oracle):
    p = product_scene(records, device=False)
    q = oracle.OracleScene(records)
    assert (p.nT, p.nE) == (q.nT, q.nE)
    assert np.array_equal(_bits(p.triangles()), _bits(q.triangles()))
    assert np.array_equal(_bits(p.camera()), _bits(q.camera()))
    return p, q


def test_scene0_and_cornell(oracle):
    p, _ = _same(SCENE0, oracle)
    assert p.nT == 30 and p.nE == 2
    p, _ = _same(CORNELL, oracle)
    assert p.nT == 18


def test_sphere_with_rotation_scale_and_vertex_normals(oracle):
    rec = [((0.1, -0.2, 3.0), (0.3, -0.2, 0.7), (1.0, 2.0, 0.5), SPHERE_OBJ, "*Kd 0.5 0.25 0.125*")]
    p, _ = _same(rec, oracle)
    assert p.nT == 1280
    tri = p.triangles()
    assert not np.allclose(tri[:, 9:12], tri[:, 18:21])  # smooth normals kept


def test_all_scene_files_parse(oracle):
    from inverse_path_tracer_amd.scene import parse_scene_text

    for i in range(0, 100, 11):
        with open(os.path.join(ASSETS, "scenes", "%d.txt" % i)) as f:
            objs = parse_scene_text(f.read())
        recs = [(o.pos, o.ori, o.scl, os.path.join(ASSETS, o.obj_file), o.mtl_file if o.mtl_file.startswith("*")
                 else os.path.join(ASSETS, o.mtl_file)) for o in objs]
        p, _ = _same(recs, oracle)
        assert p.nT == 30


OBJ_TEXT = """# synthetic: quads, n-gons, negative indices, v/vt/vn, groups, materials
mtllib whatever.mtl
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0
v 2 0 0.5
v 2.5 1 0.25
v 1.5 1.5 0.5
vt 0 0
vt 1 0
vn 0 0 1
g first
usemtl red
f 1 2 3 4
f 2/1 5/2 6/1 7/2 3/1
usemtl missing
f -4 -3 -1
o second
usemtl blue
f 1//1 3//1 4//1
usemtl red
f 2 5 6 7 3 4
g
f 1 2 5
"""
MTL_TEXT = """newmtl red
  Kd 0.8 0.1 0.1
  Ks 0.25 0.25 0.25
  Ns 12.5
newmtl blue
Kd .1 .2 +.9e0
Ke 1e-1 0 0
newmtl red
Kd 0 1 0
"""


def test_synthetic_obj_semantics(oracle, tmp_path):
    obj = tmp_path / "m.obj"
    mtl = tmp_path / "m.mtl"
    obj.write_bytes(OBJ_TEXT.replace("\n", "\r\n").encode())
    mtl.write_text(MTL_TEXT)
    p, q = _same([((0, 0, 0), (0, 0, 0), (1, 1, 1), str(obj), str(mtl))], oracle)
    tri = p.triangles()
    kd = tri[:, 25:28]
    assert np.allclose(kd[0], [0.8, 0.1, 0.1])           # quad 1 -> 2 tris, red
    assert np.allclose(tri[0, 28:31], 0.25) and tri[0, 34] == 12.5
    assert np.allclose(kd[5], 0.0)                        # usemtl missing -> default
    assert np.allclose(kd[6], [0.1, 0.2, 0.9])            # blue (parsed '.1', '+.9e0')
    assert p.nE == 1 and tri[6, 56] == 0                  # Ke 0.1 makes blue emissive
    assert p.nT == 2 + 3 + 1 + 1 + 4 + 1


def test_inline_material_and_no_mtl(oracle, tmp_path):
    obj = tmp_path / "t.obj"
    obj.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3\n")
    p, _ = _same([((0, 0, 1), (0, 0, 0), (1, 1, 1), str(obj), "*Kd 0.3 0.4 0.5\nKs 1 1 1*")], oracle)
    tri = p.triangles()
    assert np.allclose(tri[0, 25:28], [0.3, 0.4, 0.5])
    assert np.allclose(tri[0, 28:31], 0.0)  # only Kd is read from an inline material (scene_basics.h:261)
    assert tri[0, 34] == 1.0                # InitMaterial shininess


def test_missing_obj_raises_not_exits(tmp_path):
    from inverse_path_tracer_amd import NativeError

    with pytest.raises(NativeError, match="Object File was not able to be opened"):
        product_scene([((0, 0, 0), (0, 0, 0), (1, 1, 1), str(tmp_path / "nope.obj"), CUBE_KD)], device=False)


def test_zero_face_index_raises(tmp_path):
    from inverse_path_tracer_amd import NativeError

    obj = tmp_path / "bad.obj"
    obj.write_text("v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n")
    with pytest.raises(NativeError, match="zero face index"):
        product_scene([((0, 0, 0), (0, 0, 0), (1, 1, 1), str(obj), CUBE_KD)], device=False)


def test_materials_roundtrip_host_only():
    s = product_scene(SCENE0, device=False)
    kd = s.materials
    assert kd.shape == (30, 3)
    new = np.random.RandomState(0).uniform(0, 1, (30, 3)).astype(np.float32)
    s.materials = new
    assert np.array_equal(s.materials, new)


def test_host_only_scene_refuses_render():
    from inverse_path_tracer_amd import NativeError

    s = product_scene(SCENE0, device=False)
    with pytest.raises(NativeError, match="host-only"):
        s.render(8, 8, 1, 2, 0)
    with pytest.raises(NativeError):
        s.adjoint(np.zeros((8, 8, 3), np.float32), 8, 8, 1, 2, 0)


def _num(rs):
    """A decimal in one of the spellings tryParseDouble accepts (utils.h:70-200):
    signs, leading/trailing dots, e/E exponents with signs, long mantissas."""
    m = rs.uniform(-3, 3)
    k = rs.randint(8)
    if k == 0:
        return "%d" % int(round(m * 3))
    if k == 1:
        return ("%.9f" % m).rstrip("0")
    if k == 2:
        return ("+" if m >= 0 else "") + "%.6g" % m
    if k == 3:
        s = "%.5f" % abs(m)
        return ("-" if m < 0 else "") + (s[1:] if s.startswith("0.") else s)  # ".123"
    if k == 4:
        return "%.4e" % m
    if k == 5:
        return ("%.3E" % (m * 1e-3)).replace("E-0", "E-")
    if k == 6:
        return "%.22f" % m  # more digits than a double holds
    return "%de%+d" % (int(m * 1000), rs.randint(-4, 2))


def _random_obj(rs):
    nv = rs.randint(4, 12)
    lines = ["# fuzz", "mtllib fuzz.mtl"]
    for _ in range(nv):
        lines.append("v %s %s %s" % (_num(rs), _num(rs), _num(rs)))
    nvn = rs.randint(0, 3)
    for _ in range(nvn):
        lines.append("vn %s %s %s" % (_num(rs), _num(rs), _num(rs)))
    lines.append("vt 0 0")
    mats = ["a", "b", "nope"]
    for f in range(rs.randint(1, 6)):
        if rs.randint(3) == 0:
            lines.append("usemtl " + mats[rs.randint(3)])
        n = rs.randint(3, min(7, nv + 1))
        idx = rs.choice(nv, size=n, replace=False) + 1
        toks = []
        use_n = nvn > 0 and rs.randint(2) == 0
        for i in idx:
            vi = str(i) if rs.randint(4) else str(i - nv - 1)  # negative (relative) indices
            if use_n:
                toks.append("%s//%d" % (vi, rs.randint(nvn) + 1))
            elif rs.randint(4) == 0:
                toks.append("%s/1" % vi)
            else:
                toks.append(vi)
        lines.append("f " + " ".join(toks))
    return "\n".join(lines) + "\n"


MTL_FUZZ = """newmtl a
Kd 0.5 .25 1e-1
Ke 0 0 0
newmtl b
Kd 0.9 0.1 0.3
Ks 0.2 0.2 0.2
Ns 7
"""


@pytest.mark.parametrize("seed", range(200))
def test_fuzzed_obj_files_bitwise(oracle, tmp_path, seed):
    """Random OBJ texts (number spellings, polygons up to 6 sides, negative
    indices, v//vn and v/vt faces, material switches) through a random object
    transform: the product's loader equals the oracle's bit for bit."""
    rs = np.random.RandomState(1000 + seed)
    obj = tmp_path / "fuzz.obj"
    mtl = tmp_path / "fuzz.mtl"
    obj.write_text(_random_obj(rs))
    mtl.write_text(MTL_FUZZ)
    pos = tuple(float(x) for x in rs.uniform(-2, 2, 3))
    ori = tuple(float(x) for x in rs.uniform(-1.5, 1.5, 3)) if seed % 3 else (0.0, 0.0, 0.0)
    scl = tuple(float(x) for x in rs.uniform(0.3, 2.5, 3))
    _same([(pos, ori, scl, str(obj), str(mtl))], oracle)


def _random_mtl(rs, names):
    keys = ["Kd", "Ks", "Ke", "Ka", "Tf"]
    out = ["# fuzzed materials"]
    for nm in names + [names[rs.randint(len(names))]]:  # one name defined twice
        out.append(("\t" if rs.randint(3) == 0 else "") + "newmtl " + nm)
        for _ in range(rs.randint(1, 6)):
            k = rs.randint(8)
            ind = " " * rs.randint(3)
            if k < 5:
                v = [_num(rs).lstrip("-") for _ in range(3)]  # colours >= 0
                out.append("%s%s %s" % (ind, keys[k], " ".join(v if rs.randint(4) else v[:1])))
            elif k == 5:
                out.append("%sNs %s" % (ind, _num(rs).lstrip("-")))
            elif k == 6:
                out.append("%sillum %d" % (ind, rs.randint(3)))
            else:
                out.append("%sd %s" % (ind, _num(rs).lstrip("-")))
        if rs.randint(3) == 0:
            out.append("")
    return ("\r\n" if rs.randint(2) else "\n").join(out) + "\n"


@pytest.mark.parametrize("seed", range(60))
def test_fuzzed_mtl_files_bitwise(oracle, tmp_path, seed):
    """Random MTL texts (Kd/Ks/Ke with one or three values, Ns, unknown keys,
    indentation, CRLF, a material defined twice) under a fixed mesh: the
    product's materials equal the oracle's bit for bit."""
    rs = np.random.RandomState(5000 + seed)
    obj = tmp_path / "m.obj"
    mtl = tmp_path / "m.mtl"
    obj.write_text("mtllib m.mtl\nv 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nv 0 0 1\n"
                   "usemtl a\nf 1 2 3\nusemtl b\nf 1 3 4\nusemtl c\nf 1 2 5\nf 2 3 5 4\n")
    mtl.write_text(_random_mtl(rs, ["a", "b", "c"]))
    _same([((0, 0, 3), (0, 0, 0), (1, 1, 1), str(obj), str(mtl))], oracle)
