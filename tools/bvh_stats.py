"""BVH work counters of a profiling build (make variant V=stats
DEFS=-DIPT_BVH_STATS): per cast, inner-node visits and leaf pair tests,
and the shadow early-out rate, on the forward of a large scene.

    IPT_AMD_LIB=inverse_path_tracer_amd/lib/variants/libipt_stats.so \
        python tools/bvh_stats.py [--scene sphere] [--size 512] [--spp 64]

Prints one JSON line: the "tests actually executed" that the roofline of a
BVH scene charges.
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from bench_scenes import SCENES  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402
from inverse_path_tracer_amd.scene import ObjectSpec, Scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="sphere")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bounces", type=int, default=4)
    args = ap.parse_args()
    L = N.lib()
    stats = L.ipt_debug_bvh_stats
    stats.argtypes = [C.POINTER(C.c_ulonglong)]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    scene = Scene([ObjectSpec(o, m, p, r, s) for (o, m, p, r, s) in SCENES[args.scene]])
    W = H = args.size
    samples = torch.empty((W * H * args.spp, 3), device=dev)
    p = N.make_params(W, H, args.spp, args.bounces, 0)
    buf = (C.c_ulonglong * 4)()
    stats(buf)  # reset
    N.check(L.ipt_render_samples_sm_dev(scene.handle, C.byref(p), None, samples.data_ptr(), None))
    torch.cuda.synchronize()
    stats(buf)
    casts, nodes, pairs, occluded = list(buf)
    n = W * H * args.spp
    print(json.dumps({"scene": args.scene, "triangles": scene.nT, "samples": n, "casts": casts,
                      "casts_per_sample": casts / n, "nodes_per_cast": nodes / casts,
                      "pair_tests_per_cast": pairs / casts, "tri_tests_per_cast": 2 * pairs / casts,
                      "shadow_early_out": occluded, "bvh": scene.bvh_info()}), flush=True)


if __name__ == "__main__":
    main()
