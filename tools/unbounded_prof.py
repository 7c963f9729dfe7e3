"""Launch driver for rocprofv3 passes over the reference's own estimator (no
bounce cap): the fused render and the unbounded adjoint (MODE_ADJU) of
scenes/0.txt (C3) at 512x512x64, and the legacy createImage configuration
(500x500, 100 spp).  Each leg runs --steps times after one warm-up.

    rocprofv3 --kernel-trace --stats -d OUT -- python3 tools/unbounded_prof.py
"""
import argparse
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import SCENE0, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    L = N.lib()
    st = torch.cuda.current_stream().cuda_stream
    sc = product_scene(SCENE0)
    legs = []
    for W, H, spp in ((512, 512, 64), (500, 500, 100)):
        p = N.make_params(W, H, spp, None, 0)
        hdr = torch.empty((W * H, 3), device="cuda")
        ldr = torch.empty((W * H, 3), device="cuda", dtype=torch.uint8)
        adj = torch.full((H, W, 3), 1.0 / (3 * W * H), device="cuda")
        g = torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda")
        legs.append(lambda p=p, hdr=hdr, ldr=ldr: N.check(
            L.ipt_render_dev(sc.handle, C.byref(p), None, hdr.data_ptr(), ldr.data_ptr(), st)))
        if spp == 64:
            legs.append(lambda p=p, adj=adj, g=g: N.check(
                L.ipt_adjoint_dev(sc.handle, C.byref(p), None, adj.data_ptr(), g.data_ptr(), st)))
    for leg in legs:
        for _ in range(args.steps + 1):
            leg()
    torch.cuda.synchronize()
    sc.close()


if __name__ == "__main__":
    main()
