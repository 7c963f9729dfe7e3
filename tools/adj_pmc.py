"""Launch driver for per-instance rocprofv3 passes of the C2 headline's two
kernels: the fused render (trace_kernel<4>) and the bounded adjoint -- the
6-wave instance (trace_kernel<5>, the default for full-size launches) or,
with IPT_ADJW=0 in the environment, the 5-wave one (trace_kernel<1>).
IPT_AMD_LIB selects another build (a `make variant` library), so the same
counters can be read for each form in its own process:

    rocprofv3 --kernel-trace --pmc FETCH_SIZE -d OUT -- python3 tools/adj_pmc.py
    IPT_ADJW=0 rocprofv3 ... -- python3 tools/adj_pmc.py --no-fwd

Each leg runs --steps launches after one warm-up, one stream, synchronised
(launches alone, no frames in flight)."""
import argparse
import ctypes as C
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import CORNELL, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--no-fwd", action="store_true")
    args = ap.parse_args()
    torch.cuda.set_device(0)
    L = N.lib()
    st = torch.cuda.current_stream().cuda_stream
    sc = product_scene(CORNELL)
    W = H = 512
    p = N.make_params(W, H, 64, 4, 0)
    hdr = torch.empty((W * H, 3), device="cuda")
    adj = torch.full((H, W, 3), 1.0 / (3 * W * H), device="cuda")
    g = torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda")
    legs = [lambda: N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p), None, adj.data_ptr(), g.data_ptr(), st))]
    if not args.no_fwd:
        legs.insert(0, lambda: N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, hdr.data_ptr(), None, st)))
    for leg in legs:
        leg()
        torch.cuda.synchronize()
        for _ in range(args.steps):
            leg()
            torch.cuda.synchronize()
    sc.close()


if __name__ == "__main__":
    main()
