"""Timing of createGraph's integrator (trace_kernel<MODE_GRAPH>) next to the
forward at the same size: scenes/0.txt and the Cornell box, 512x512x64, 4
bounces, and the reference's own configuration (500x500x100, unbounded)."""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import CORNELL, SCENE0, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402


def timed(fn, reps=3):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    torch.cuda.set_device(0)
    L = N.lib()
    st = torch.cuda.current_stream().cuda_stream
    out = []
    for name, recs in (("cornell", CORNELL), ("scene0", SCENE0)):
        P = product_scene(recs)
        for W, spp, mb in ((512, 64, 4), (500, 100, None)):
            p = N.make_params(W, W, spp, mb, 0)
            tgt = torch.randint(0, 256, (W, W, 3), dtype=torch.uint8, device="cuda")
            acc = torch.zeros(((P.nT + 1) * P.nT, N.ACC_WIDTH), dtype=torch.float64, device="cuda")
            smp = torch.empty((W * W * spp, 3), device="cuda")
            g = timed(lambda: N.check(L.ipt_graph_dev(P.handle, C.byref(p), tgt.data_ptr(), acc.data_ptr(), st)))
            f = timed(lambda: N.check(L.ipt_render_samples_sm_dev(P.handle, C.byref(p), None, smp.data_ptr(), st)))
            r = {"scene": name, "size": W, "spp": spp, "bounces": mb, "graph_ms": round(g, 3), "fwd_ms": round(f, 3),
                 "graph_Msamples_s": round(W * W * spp / g / 1e3, 1)}
            print(json.dumps(r), flush=True)
            out.append(r)
        P.close()


if __name__ == "__main__":
    main()
