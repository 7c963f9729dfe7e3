"""Timing of the C5 scene batch against single-scene launches of the same
work: scenes/0.txt geometry, 256x256, 32 spp, 4 bounces, 13 material sets --
one batched launch, 13 single launches, and one single launch of 13x the
samples (a 256x(256*13) frame) as the per-sample reference rate."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from inverse_path_tracer_amd import _native as N  # noqa: E402
from inverse_path_tracer_amd.scene import Scene  # noqa: E402


def main():
    torch.cuda.set_device(0)
    L = N.lib()
    st = torch.cuda.current_stream().cuda_stream
    sc = Scene.from_file(os.path.join(ROOT, "assets", "scenes", "0.txt"))
    S, W, H, spp, mb = 13, 256, 256, 32, 4
    kd = torch.from_numpy(np.random.RandomState(0).uniform(0, 1, (S, sc.nT, 3)).astype(np.float32)).cuda()
    hdr = torch.empty((S, H, W, 3), device="cuda")
    adj = torch.ones((S, H, W, 3), device="cuda") / (S * H * W * 3)
    g = torch.zeros((S, sc.nT, 3), device="cuda", dtype=torch.float64)
    p = N.make_params(W, H, spp, mb, 0)
    pbig = N.make_params(W, H * S, spp, mb, 0)
    big = torch.empty((H * S, W, 3), device="cuda")
    adjbig = torch.ones((H * S, W, 3), device="cuda")

    def batch_fwd():
        N.check(L.ipt_render_batch_dev(sc.handle, C.byref(p), S, W * H * spp, kd.data_ptr(), hdr.data_ptr(), st))

    def batch_adj():
        N.check(L.ipt_adjoint_batch_dev(sc.handle, C.byref(p), S, W * H * spp, kd.data_ptr(), adj.data_ptr(),
                                        g.data_ptr(), st))

    def singles_fwd():
        for b in range(S):
            q = N.make_params(W, H, spp, mb, b * W * H * spp)
            N.check(L.ipt_render_dev(sc.handle, C.byref(q), kd[b].data_ptr(), hdr[b].data_ptr(), None, st))

    def singles_adj():
        for b in range(S):
            q = N.make_params(W, H, spp, mb, b * W * H * spp)
            N.check(L.ipt_adjoint_dev(sc.handle, C.byref(q), kd[b].data_ptr(), adj[b].data_ptr(), g[b].data_ptr(), st))

    p416 = N.make_params(W, H, spp * S, mb, 0)
    p512 = N.make_params(512, 512, 64, mb, 0)
    o512 = torch.empty((512, 512, 3), device="cuda")
    a512 = torch.ones((512, 512, 3), device="cuda")

    def deep_fwd():
        N.check(L.ipt_render_dev(sc.handle, C.byref(p416), kd[0].data_ptr(), hdr[0].data_ptr(), None, st))

    def deep_adj():
        N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p416), kd[0].data_ptr(), adj[0].data_ptr(), g[0].data_ptr(), st))

    def c3_fwd():
        N.check(L.ipt_render_dev(sc.handle, C.byref(p512), kd[0].data_ptr(), o512.data_ptr(), None, st))

    def c3_adj():
        N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p512), kd[0].data_ptr(), a512.data_ptr(), g[0].data_ptr(), st))

    def tall_fwd():
        N.check(L.ipt_render_dev(sc.handle, C.byref(pbig), kd[0].data_ptr(), big.data_ptr(), None, st))

    def tall_adj():
        N.check(L.ipt_adjoint_dev(sc.handle, C.byref(pbig), kd[0].data_ptr(), adjbig.data_ptr(), g[0].data_ptr(), st))

    def batch_s(nsets, sppx, same_kd=False):
        q = N.make_params(W, H, sppx, mb, 0)
        k = kd[:1].expand(nsets, -1, -1).contiguous() if same_kd else kd[:nsets].contiguous()
        def f():
            N.check(L.ipt_render_batch_dev(sc.handle, C.byref(q), nsets, W * H * sppx, k.data_ptr(), hdr.data_ptr(), st))
        def b():
            N.check(L.ipt_adjoint_batch_dev(sc.handle, C.byref(q), nsets, W * H * sppx, k.data_ptr(), adj.data_ptr(),
                                            g.data_ptr(), st))
        return f, b

    extra = []
    for nsets, sppx in [(1, 416), (2, 208), (4, 104), (8, 52)]:
        f, b = batch_s(nsets, sppx)
        extra += [("batch%d_fwd" % nsets, f), ("batch%d_adj" % nsets, b)]
    f, b = batch_s(13, 32, True)
    extra += [("batch13same_fwd", f), ("batch13same_adj", b)]
    out = {}
    for name, fn in [("batch_fwd", batch_fwd), ("singles_fwd", singles_fwd), ("tall_fwd", tall_fwd),
                     ("deep_fwd", deep_fwd), ("c3_fwd_16.8M", c3_fwd),
                     ("batch_adj", batch_adj), ("singles_adj", singles_adj), ("tall_adj", tall_adj),
                     ("deep_adj", deep_adj), ("c3_adj_16.8M", c3_adj)] + extra:
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(e0.elapsed_time(e1) / 10, 4)
        print(name, out[name], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
