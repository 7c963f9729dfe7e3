"""A/B timing of kernel variants (lib/variants/libipt_*.so) in ONE process,
interleaved rounds (cdna_hip_programming.md §5.4 rule 24).  Each variant is
checked bit-exact against the default library on a small frame first."""
import ctypes as C
import glob
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inverse_path_tracer_amd import _native as N  # noqa: E402

A = os.path.join(ROOT, "assets")
SCENES = {
    "cornell": [(A + "/CornellBox/CornellBox-Empty-CO.obj", A + "/CornellBox/CornellBox-Empty-CO.mtl", (0, 0, 4), (0, 0, 0), (2, 2, 2))],
}
SCENES["scene0"] = SCENES["cornell"] + [(A + "/shapes/cube.obj", "*Kd 0.9041462985304743 0.5854651848798454 0.007022117649276849*",
                                          (0, -1.5, 4), (0, 0, 0), (1, 1, 1))]
if os.environ.get("IPT_VB_SPHERE"):  # large scene: BVH instance (triangle BVH + large-triangle pre-pass)
    SCENES["sphere"] = SCENES["cornell"] + [(A + "/shapes/sphere.obj", "*Kd 0.2 0.6 0.3*", (0.3, -1.2, 4.2), (0.0, 0.4, 0.0),
                                             (1.2, 1.2, 1.2))]
if os.environ.get("IPT_VB_CLUTTER"):  # the 4-object scene of tests/test_bvh.py (2590 triangles)
    SCENES["clutter"] = SCENES["cornell"] + [
        (A + "/shapes/sphere.obj", "*Kd 0.2 0.6 0.3*", (0.3, -1.2, 4.2), (0.0, 0.4, 0.0), (1.2, 1.2, 1.2)),
        (A + "/shapes/cube.obj", "*Kd 0.5 0.5 0.5*", (-0.9, -1.4, 3.9), (0.2, 0.7, 0.1), (0.7, 0.7, 0.7)),
        (A + "/shapes/sphere.obj", "*Kd 0.9 0.1 0.1*", (0.8, 0.9, 4.6), (0.0, 0.0, 0.5), (0.5, 0.5, 0.5))]
if os.environ.get("IPT_VB_NORTHSTAR"):  # BASELINE configs[2]: scenes/0.txt + sphere (1310 triangles)
    SCENES["northstar"] = SCENES["scene0"] + [(A + "/shapes/sphere.obj", "*Kd 0.2 0.6 0.3*", (-1.2, -1.35, 4.6),
                                               (0.0, 0.0, 0.0), (1.2, 1.2, 1.2))]
if os.environ.get("IPT_VB_PHONG"):  # scenes/0.txt with a Phong cube (bench.py c3_phong): the SPEC instances
    SCENES["phong"] = SCENES["cornell"] + [(A + "/phong/cube_phong.obj", A + "/phong/cube_phong.mtl", (0, -1.5, 4),
                                            (0, 0, 0), (1, 1, 1))]
if os.environ.get("IPT_VB_ONLY"):  # comma-separated scene names
    SCENES = {k: v for k, v in SCENES.items() if k in os.environ["IPT_VB_ONLY"].split(",")}


def load(path):
    L = C.CDLL(path, mode=os.RTLD_LOCAL)
    for name, (res, args) in N.SIGNATURES.items():
        if not hasattr(L, name):  # older variant builds lack newer symbols
            continue
        f = getattr(L, name)
        f.restype, f.argtypes = res, args
    return L


def scene(L, recs):
    n = len(recs)
    pos = np.array([r[2] for r in recs], np.float32)
    ori = np.array([r[3] for r in recs], np.float32)
    scl = np.array([r[4] for r in recs], np.float32)
    objs = (C.c_char_p * n)(*[r[0].encode() for r in recs])
    mtls = (C.c_char_p * n)(*[r[1].encode() for r in recs])
    h = C.c_void_p(0)
    assert L.ipt_load_scene(n, pos.ctypes.data_as(N.fp), ori.ctypes.data_as(N.fp), scl.ctypes.data_as(N.fp), objs,
                            mtls, C.byref(h)) > 0
    if os.environ.get("IPT_VB_ACCEL") == "bvh":  # force the BVH instance (ablations on small scenes)
        assert L.ipt_scene_set_accel(h, N.ACCEL_BVH) == 0
    return h


def main():
    names = sys.argv[1:] or sorted(os.path.basename(p)[7:-3] for p in glob.glob(os.path.join(ROOT, "inverse_path_tracer_amd/lib/variants/libipt_*.so")))
    libs = {n: load(os.path.join(ROOT, "inverse_path_tracer_amd/lib/variants/libipt_%s.so" % n)) for n in names}
    ref = load(N.LIB_PATH)
    libs["cur"] = ref  # the default build is timed next to the variants
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for sname, recs in SCENES.items():
        hs = {n: scene(L, recs) for n, L in libs.items()}
        href = hs["cur"]
        # correctness: small frame bit-exact vs default library
        p = N.make_params(64, 64, 8, 4, 123)
        want = np.zeros((64 * 64 * 8, 3), np.float32)
        assert ref.ipt_render_samples_host(href, C.byref(p), want.ctypes.data_as(N.fp)) == 0
        for n, L in libs.items():
            got = np.zeros_like(want)
            assert L.ipt_render_samples_host(hs[n], C.byref(p), got.ctypes.data_as(N.fp)) == 0
            print(sname, n, "bit-exact" if np.array_equal(got.view(np.uint32), want.view(np.uint32)) else "MISMATCH", flush=True)
        # adjoint: fp64 sums, equal to the default library's up to summation order
        adj_s = np.random.RandomState(5).uniform(-1, 1, (64, 64, 3)).astype(np.float32)
        nt = ref.ipt_scene_num_triangles(href)
        gw = np.zeros((nt, 3), np.float64)
        assert ref.ipt_adjoint_host(href, C.byref(p), adj_s.ctypes.data_as(N.fp), gw.ctypes.data_as(N.dp)) == 0
        for n, L in libs.items():
            gg = np.zeros_like(gw)
            assert L.ipt_adjoint_host(hs[n], C.byref(p), adj_s.ctypes.data_as(N.fp), gg.ctypes.data_as(N.dp)) == 0
            err = float(np.max(np.abs(gg - gw)) / max(np.max(np.abs(gw)), 1e-300))
            print(sname, n, "adjoint max rel diff %.2e" % err, "OK" if err < 1e-9 else "MISMATCH", flush=True)
        p = N.make_params(512, 512, 64, 4, 0)
        buf = torch.empty((512 * 512 * 64, 3), device=dev)
        adj = torch.ones((512, 512, 3), device=dev)
        g = torch.zeros((8192, 3), dtype=torch.float64, device=dev)
        pb = N.make_params(512, 512, 64, 4, 0, 192, 256)  # one 64-row band: a small launch (the 8-GPU share)
        pr8 = N.make_params(512, 512, 64, 4, 0, 0, 512, 8)  # one interleaved 1/8 share (the bench's tile split)
        hdr = torch.empty((512 * 512, 3), device=dev)
        pu = N.make_params(512, 512, 64, None, 0)  # the reference's own estimator (no bounce cap)
        # adj5: the bounded adjoint with IPT_ADJW=0 (the 5-wave instance; the
        # library reads the variable at each launch)
        kinds = ("fwd", "fsm", "adj", "band", "render", "render8", "adj8", "adju", "renderu", "adj5")
        times = {n: {k: [] for k in kinds} for n in libs}
        for rnd in range(6):
            for n, L in libs.items():
                for kind in kinds:
                    if kind == "fsm" and not hasattr(L, "ipt_render_samples_sm_dev"):
                        continue
                    if kind == "adj5":
                        os.environ["IPT_ADJW"] = "0"
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(3):
                        if kind == "fwd":
                            assert L.ipt_render_samples_dev(hs[n], C.byref(p), None, buf.data_ptr(), st) == 0
                        elif kind == "fsm":
                            assert L.ipt_render_samples_sm_dev(hs[n], C.byref(p), None, buf.data_ptr(), st) == 0
                        elif kind == "band":
                            assert L.ipt_render_samples_sm_dev(hs[n], C.byref(pb), None, buf.data_ptr(), st) == 0
                        elif kind in ("render", "render8", "renderu"):
                            pp = {"render": p, "render8": pr8, "renderu": pu}[kind]
                            assert L.ipt_render_dev(hs[n], C.byref(pp), None, hdr.data_ptr(), None, st) == 0
                        elif kind == "adju":
                            assert L.ipt_adjoint_dev(hs[n], C.byref(pu), None, adj.data_ptr(), g.data_ptr(), st) == 0
                        elif kind == "adj8":
                            assert L.ipt_adjoint_dev(hs[n], C.byref(pr8), None, adj.data_ptr(), g.data_ptr(), st) == 0
                        else:
                            assert L.ipt_adjoint_dev(hs[n], C.byref(p), None, adj.data_ptr(), g.data_ptr(), st) == 0
                    e1.record()
                    torch.cuda.synchronize()
                    os.environ.pop("IPT_ADJW", None)
                    if rnd > 0:
                        times[n][kind].append(e0.elapsed_time(e1) / 3)
        for n in libs:
            f, a = np.median(times[n]["fwd"]), np.median(times[n]["adj"])
            fs = np.median(times[n]["fsm"]) if times[n]["fsm"] else float("nan")
            out[sname + ":" + n] = {"fwd_ms": round(f, 4), "fsm_ms": round(fs, 4), "adj_ms": round(a, 4),
                                    "band_ms": round(float(np.median(times[n]["band"])), 4),
                                    "render_ms": round(float(np.median(times[n]["render"])), 4),
                                    "render8_ms": round(float(np.median(times[n]["render8"])), 4),
                                    "adj8_ms": round(float(np.median(times[n]["adj8"])), 4),
                                    "adju_ms": round(float(np.median(times[n]["adju"])), 4),
                                    "renderu_ms": round(float(np.median(times[n]["renderu"])), 4),
                                    "adj5_ms": round(float(np.median(times[n]["adj5"])), 4),
                                    "fwd_Msps": round(512 * 512 * 64 / f / 1e3, 1), "adj_Msps": round(512 * 512 * 64 / a / 1e3, 1)}
            print(sname, n, out[sname + ":" + n], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
