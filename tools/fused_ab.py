"""A/B of the render: the pixel mean fused into the trace kernel (default)
against the two-kernel form (IPT_RENDER_TWO_KERNEL=1: sample buffer +
pixel_mean_sm_kernel), in one process, interleaved rounds, HIP events on the
launch stream.  Scenes: Cornell (C2), scenes/0.txt (C3), the north-star BVH
scene; shares: the whole 512x512x64 frame and one interleaved 1/8 share (the
8-GPU tile split's per-rank launch).

    python tools/fused_ab.py [--reps 10] [--rounds 6]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import CORNELL, NORTHSTAR, SCENE0, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--scenes", default="cornell,scene0,northstar")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    L = N.lib()
    stream = torch.cuda.current_stream()
    st = stream.cuda_stream
    W = H = 512
    spp, mb = 64, 4
    hdr = torch.empty((W * H, 3), device="cuda")
    recs = {"cornell": CORNELL, "scene0": SCENE0, "northstar": NORTHSTAR}
    out = {}
    for name in args.scenes.split(","):
        sc = product_scene(recs[name])
        for share in (1, 8):
            p = N.make_params(W, H, spp, mb, 0, 0, H, share)
            ref = None
            for mode in ("fused", "two_kernel"):  # bitwise equal first
                if mode == "two_kernel":
                    os.environ["IPT_RENDER_TWO_KERNEL"] = "1"
                N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, hdr.data_ptr(), None, st))
                os.environ.pop("IPT_RENDER_TWO_KERNEL", None)
                img = hdr.cpu().numpy().view(np.uint32).copy()
                if ref is None:
                    ref = img
                else:
                    print(name, share, "fused == two_kernel:", bool(np.array_equal(img, ref)), flush=True)
            times = {"fused": [], "two_kernel": []}
            for rnd in range(args.rounds):
                for mode in ("fused", "two_kernel"):
                    if mode == "two_kernel":
                        os.environ["IPT_RENDER_TWO_KERNEL"] = "1"
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.reps):
                        N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, hdr.data_ptr(), None, st))
                    e1.record(stream)
                    torch.cuda.synchronize()
                    os.environ.pop("IPT_RENDER_TWO_KERNEL", None)
                    if rnd > 0:
                        times[mode].append(e0.elapsed_time(e1) / args.reps)
            rec = {k: round(float(np.median(v)), 4) for k, v in times.items()}
            out["%s:1/%d" % (name, share)] = rec
            print(name, "1/%d" % share, rec, flush=True)
        sc.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
