"""Per-scene throughput of the forward and adjoint integrators on one GPU,
brute-force loop vs BVH (A/B for DESIGN.md §5.2 and profiles/).

    python tools/bench_scenes.py [--size 512] [--spp 64] [--bounces 4] [--steps 5]

One JSON line per (scene, accel): Msamples/s forward, grad-Msamples/s adjoint
(all-ones adjoint image), kernel ms (HIP events on the launch stream).
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from inverse_path_tracer_amd import _native as N  # noqa: E402
from inverse_path_tracer_amd.scene import ObjectSpec, Scene  # noqa: E402

A = os.path.join(ROOT, "assets")
CORNELL = (os.path.join(A, "CornellBox", "CornellBox-Empty-CO.obj"), os.path.join(A, "CornellBox", "CornellBox-Empty-CO.mtl"),
           (0, 0, 4), (0, 0, 0), (2, 2, 2))
CUBE0 = (os.path.join(A, "shapes", "cube.obj"), "*Kd 0.9041462985304743 0.5854651848798454 0.007022117649276849*",
         (0, -1.5, 4), (0, 0, 0), (1, 1, 1))
SPHERE = (os.path.join(A, "shapes", "sphere.obj"), "*Kd 0.2 0.6 0.3*", (0.3, -1.2, 4.2), (0.0, 0.4, 0.0), (1.2, 1.2, 1.2))
CUBE2 = (os.path.join(A, "shapes", "cube.obj"), "*Kd 0.5 0.5 0.5*", (-0.9, -1.4, 3.9), (0.2, 0.7, 0.1), (0.7, 0.7, 0.7))
SPHERE2 = (os.path.join(A, "shapes", "sphere.obj"), "*Kd 0.9 0.1 0.1*", (0.8, 0.9, 4.6), (0.0, 0.0, 0.5), (0.5, 0.5, 0.5))
SCENES = {
    "cornell": [CORNELL],
    "scene0": [CORNELL, CUBE0],
    "sphere": [CORNELL, SPHERE],
    "clutter": [CORNELL, SPHERE, CUBE2, SPHERE2],
    # BASELINE configs[2] as the north_star names it (assets/northstar.txt): 1310 triangles
    "northstar": [CORNELL, CUBE0, (os.path.join(A, "shapes", "sphere.obj"), "*Kd 0.2 0.6 0.3*", (-1.2, -1.35, 4.6),
                                   (0.0, 0.0, 0.0), (1.2, 1.2, 1.2))],
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--scenes", default="cornell,scene0,sphere,clutter")
    ap.add_argument("--brute-max-tris", type=int, default=4000, help="skip brute force above this size")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    L = N.lib()
    W = H = args.size
    stream = torch.cuda.current_stream(dev)
    st = stream.cuda_stream
    samples = torch.empty((W * H * args.spp, 3), device=dev)
    adj = torch.full((H, W, 3), 1.0, device=dev)
    for name in args.scenes.split(","):
        scene = Scene([ObjectSpec(o, m, p, r, s) for (o, m, p, r, s) in SCENES[name]])
        grad = torch.zeros((scene.nT, 3), device=dev, dtype=torch.float64)
        info = scene.bvh_info()
        modes = [("auto", N.ACCEL_AUTO)]
        if info["has_bvh"]:
            modes = [("bvh", N.ACCEL_BVH)]
            if scene.nT <= args.brute_max_tris:
                modes.append(("brute", N.ACCEL_BRUTE))
        for label, mode in modes:
            scene.set_accel(mode)
            p = N.make_params(W, H, args.spp, args.bounces, 0)

            def fwd():
                N.check(L.ipt_render_samples_sm_dev(scene.handle, C.byref(p), None, samples.data_ptr(), st))

            def bwd():
                N.check(L.ipt_adjoint_dev(scene.handle, C.byref(p), None, adj.data_ptr(), grad.data_ptr(), st))

            res = {}
            for key, fn in (("fwd", fwd), ("adj", bwd)):
                fn()
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(args.steps):
                    fn()
                e1.record(stream)
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / args.steps
                res[key + "_ms"] = round(ms, 4)
                res[key + "_Msamples_s"] = round(W * H * args.spp / ms / 1e3, 2)
            out = {"scene": name, "triangles": scene.nT, "accel": label, "size": W, "spp": args.spp,
                   "bounces": args.bounces, **res}
            if info["has_bvh"]:
                out["bvh"] = {k: info[k] for k in ("nodes", "pairs", "depth")}
            print(json.dumps(out), flush=True)
        scene.set_accel(N.ACCEL_AUTO)


if __name__ == "__main__":
    main()
