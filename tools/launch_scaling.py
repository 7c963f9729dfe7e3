"""Fixed cost of a launch: the C2 forward and adjoint on 1/1 ... 1/64 of the
frame's rows (interleaved shares, as one rank of an N-GPU tile split traces
them), timed alone with HIP events.  A fit t(n) = a + b * n over the shares
separates the per-launch fixed cost a (start-up, tail, the memset and the
per-pixel mean) from the per-sample cost b.

    python tools/launch_scaling.py [--reps 20]
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
from conftest import CORNELL, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    L = N.lib()
    stream = torch.cuda.current_stream()
    st = stream.cuda_stream
    sc = product_scene(CORNELL)
    W = H = 512
    spp, mb = 64, 4
    samples = torch.empty((W * H * spp, 3), device="cuda")
    hdr = torch.empty((W * H, 3), device="cuda")
    adj = torch.full((H, W, 3), 1.0, device="cuda")
    grad = torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda")
    rows = []
    for share in (1, 2, 4, 8, 16, 32, 64):
        p = N.make_params(W, H, spp, mb, 0, 0, H, share)  # rows 0, share, 2 share, ...
        npix = (H // share) * W

        def trace():
            N.check(L.ipt_render_samples_sm_dev(sc.handle, C.byref(p), None, samples.data_ptr(), st))

        def render():
            N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, hdr.data_ptr(), None, st))

        def adjoint():
            N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p), None, adj.data_ptr(), grad.data_ptr(), st))

        rec = {"share": share, "samples": npix * spp}
        for name, fn in (("trace_ms", trace), ("render_ms", render), ("adjoint_ms", adjoint)):
            fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                fn()
            e1.record(stream)
            torch.cuda.synchronize()
            rec[name] = round(e0.elapsed_time(e1) / args.reps, 4)
        print(json.dumps(rec), flush=True)
        rows.append(rec)
    n = np.array([r["samples"] for r in rows], np.float64)
    fit = {}
    for key in ("trace_ms", "render_ms", "adjoint_ms"):
        b, a = np.polyfit(n, [r[key] for r in rows], 1)
        fit[key] = {"fixed_ms": round(float(a), 4), "ns_per_Msample": round(float(b) * 1e6, 3)}
    print(json.dumps({"fit": fit, "rows": rows}), flush=True)


if __name__ == "__main__":
    main()
