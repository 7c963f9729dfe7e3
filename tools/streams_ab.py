"""Frames in flight: consecutive C2 frames (render and adjoint, whole frame and
an interleaved 1/8 share) dealt round-robin over 1, 2, 3 or 4 HIP streams,
each stream with its own output buffers.  With k streams a frame's tail (its
last long paths on a few waves per CU) overlaps the next k-1 frames' starts.
Frames of every form are compared bitwise with frames rendered alone.

    python tools/streams_ab.py [--steps 40] [--rounds 5] [--streams 1,2,3,4]
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
from inverse_path_tracer_amd.distributed import frame_seed  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--streams", default="1,2,3,4")
    args = ap.parse_args()
    counts = [int(x) for x in args.streams.split(",")]
    torch.cuda.set_device(0)
    L = N.lib()
    main_s = torch.cuda.current_stream()
    side = [torch.cuda.Stream() for _ in range(max(counts))]
    W = H = 512
    spp, mb = 64, 4
    sc = product_scene(CORNELL)
    out = {}
    for share in (1, 8):
        npix = (H // share) * W
        hdr = [torch.empty((npix, 3), device="cuda") for _ in side]
        adj = torch.full((H, W, 3), 1.0 / (3 * W * H), device="cuda")
        grad = [torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda") for _ in side]

        def params(i):
            return N.make_params(W, H, spp, mb, frame_seed(0, i, W, H, spp), 0, H, share)

        def fwd(i, k):
            N.check(L.ipt_render_dev(sc.handle, C.byref(params(i)), None, hdr[k].data_ptr(), None,
                                     side[k].cuda_stream))

        def adjoint(i, k):
            with torch.cuda.stream(side[k]):
                grad[k].zero_()
            N.check(L.ipt_adjoint_dev(sc.handle, C.byref(params(i)), None, adj.data_ptr(), grad[k].data_ptr(),
                                      side[k].cuda_stream))

        def run(kind, n):
            fn = fwd if kind == "fwd" else adjoint
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            for s in side:
                s.wait_event(e0)
            for i in range(args.steps):
                fn(i, i % n)
            for s in side:
                main_s.wait_stream(s)
            e1.record(main_s)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) / args.steps

        # bitwise: the last frame on each stream vs the same frame alone
        ok = {}
        for n in counts:
            run("fwd", n)
            got = {(args.steps - 1 - j) % n: (args.steps - 1 - j, hdr[(args.steps - 1 - j) % n].clone())
                   for j in range(n)}
            eq = True
            for k, (i, g) in got.items():
                fwd(i, 0)
                torch.cuda.synchronize()
                eq = eq and bool(torch.equal(g.view(torch.int32), hdr[0].view(torch.int32)))
            ok[n] = eq
        t = {(k, n): [] for k in ("fwd", "adj") for n in counts}
        for _ in range(args.rounds):
            for n in counts:
                for k in ("fwd", "adj"):
                    t[(k, n)].append(run(k, n))
        res = {"bitwise_equal_alone": {str(n): ok[n] for n in counts}}
        for (k, n), v in t.items():
            res["%s_ms_%dstreams" % (k, n)] = round(float(np.median(v)), 4)
        out["share_1_of_%d" % share] = res
        print(share, json.dumps(res), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
