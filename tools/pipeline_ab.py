"""Consecutive frames on one stream (each launch waits for the previous one's
tail) against frames alternating between two streams (one frame's tail
overlaps the next frame's start): C2 render and adjoint, the whole frame and
an interleaved 1/8 share (the 8-GPU tile split's per-rank launch).  Images
of both forms are compared bitwise.

    python tools/pipeline_ab.py [--steps 40] [--rounds 5]
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
from conftest import CORNELL, SCENE0, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402
from inverse_path_tracer_amd.distributed import frame_seed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    L = N.lib()
    main_s = torch.cuda.current_stream()
    side = [torch.cuda.Stream(), torch.cuda.Stream()]
    W = H = 512
    spp, mb = 64, 4
    out = {}
    for name, recs in (("cornell", CORNELL), ("scene0", SCENE0)):
        sc = product_scene(recs)
        for share in (1, 8):
            npix = (H // share) * W
            hdr = [torch.empty((npix, 3), device="cuda") for _ in range(2)]
            adj = torch.full((H, W, 3), 1.0 / (3 * W * H), device="cuda")
            grad = [torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda") for _ in range(2)]

            def params(i):
                return N.make_params(W, H, spp, mb, frame_seed(0, i, W, H, spp), 0, H, share)

            def fwd(i, st):
                N.check(L.ipt_render_dev(sc.handle, C.byref(params(i)), None, hdr[i % 2].data_ptr(), None,
                                         st.cuda_stream))

            def adjoint(i, st):
                with torch.cuda.stream(st):
                    grad[i % 2].zero_()
                N.check(L.ipt_adjoint_dev(sc.handle, C.byref(params(i)), None, adj.data_ptr(), grad[i % 2].data_ptr(),
                                          st.cuda_stream))

            def run(kind, piped):
                fn = fwd if kind == "fwd" else adjoint
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(main_s)
                for s in side:
                    s.wait_event(e0)
                for i in range(args.steps):
                    fn(i, side[i % 2] if piped else side[0])
                for s in side:
                    main_s.wait_stream(s)
                e1.record(main_s)
                torch.cuda.synchronize()
                return e0.elapsed_time(e1) / args.steps

            # bitwise: frame 1 of each form
            run("fwd", False)
            a = hdr[1].cpu().numpy().view(np.uint32).copy()
            run("fwd", True)
            b = hdr[1].cpu().numpy().view(np.uint32).copy()
            print(name, share, "frames bitwise equal:", bool(np.array_equal(a, b)), flush=True)
            t = {(k, p): [] for k in ("fwd", "adj") for p in (False, True)}
            for _ in range(args.rounds):
                for k in ("fwd", "adj"):
                    for p in (False, True):
                        t[(k, p)].append(run(k, p))
            rec = {"%s_%s" % (k, "two_streams" if p else "one_stream"): round(float(np.median(v)), 4)
                   for (k, p), v in t.items()}
            out["%s:1/%d" % (name, share)] = rec
            print(name, "1/%d" % share, rec, flush=True)
        sc.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
