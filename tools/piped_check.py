"""Frames in flight on two streams must be the frames rendered one after
another: renders steps 0..K-1 of the bench headline (C2, per-step seeds)
alternating between two streams into per-step images, then each step again
alone on one stream, and compares bitwise (render and adjoint); prints the
two timings.

    python tools/piped_check.py [--steps K]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import CORNELL, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=8)
    a = ap.parse_args()
    torch.cuda.set_device(0)
    L = N.lib()
    W = H = 512
    sc = product_scene(CORNELL)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    main_st = torch.cuda.current_stream()
    K = a.steps
    imgs = [torch.empty((W * H, 3), device="cuda") for _ in range(K)]
    ref = [torch.empty((W * H, 3), device="cuda") for _ in range(K)]
    grads = [torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda") for _ in range(K)]
    gref = [torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda") for _ in range(K)]
    adj = torch.full((H, W, 3), 1.0 / (3 * W * H), device="cuda")
    ps = [N.make_params(W, H, 64, 4, 1000 + 77 * i) for i in range(K)]
    out = {}
    for kind in ("render", "adjoint"):
        def launch(i, st, dst):
            if kind == "render":
                N.check(L.ipt_render_dev(sc.handle, C.byref(ps[i]), None, dst[i].data_ptr(), None, st.cuda_stream))
            else:
                N.check(L.ipt_adjoint_dev(sc.handle, C.byref(ps[i]), None, adj.data_ptr(), dst[i].data_ptr(),
                                          st.cuda_stream))
        dst, rdst = (imgs, ref) if kind == "render" else (grads, gref)
        for rep in range(3):  # warm-up rounds (first use of a stream: its chunk counters)
            for i in range(K):
                launch(i, streams[i % 2], dst)
        torch.cuda.synchronize()
        for g in grads + gref:
            g.zero_()
        for d in imgs + ref:
            d.fill_(float("nan"))
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(main_st)
        for s in streams:
            s.wait_event(e0)
        for i in range(K):
            launch(i, streams[i % 2], dst)
        for s in streams:
            main_st.wait_stream(s)
        e1.record(main_st)
        torch.cuda.synchronize()
        piped = e0.elapsed_time(e1) / K
        t0 = time.perf_counter()
        for i in range(K):
            launch(i, main_st, rdst)
        torch.cuda.synchronize()
        serial = (time.perf_counter() - t0) * 1e3 / K
        if kind == "render":
            same = [bool(torch.equal(dst[i].view(torch.int32), rdst[i].view(torch.int32))) for i in range(K)]
        else:  # fp64 atomics in another order: equal to ~1e-15
            same = [float(((dst[i] - rdst[i]).abs().max() / rdst[i].abs().max()).item()) for i in range(K)]
        out[kind] = {"piped_ms": round(piped, 4), "serial_ms_wall": round(serial, 4),
                     "bitwise_equal" if kind == "render" else "max_rel_diff": same}
        print(kind, json.dumps(out[kind]), flush=True)
    # the bench's order: adjoint and render launches sharing each stream (and
    # its chunk counters), alternating streams; then every frame alone
    for d in imgs + ref:
        d.fill_(float("nan"))
    for rep in range(2):
        for i in range(K):
            st = streams[i % 2]
            N.check(L.ipt_adjoint_dev(sc.handle, C.byref(ps[i]), None, adj.data_ptr(), grads[i].data_ptr(),
                                      st.cuda_stream))
            N.check(L.ipt_render_dev(sc.handle, C.byref(ps[i]), None, imgs[i].data_ptr(), None, st.cuda_stream))
    for i in range(K):
        N.check(L.ipt_render_dev(sc.handle, C.byref(ps[i]), None, ref[i].data_ptr(), None, main_st.cuda_stream))
    torch.cuda.synchronize()
    same = [bool(torch.equal(imgs[i].view(torch.int32), ref[i].view(torch.int32))) for i in range(K)]
    print("mixed", json.dumps({"render_bitwise_equal": same}), flush=True)
    sc.close()


if __name__ == "__main__":
    main()
