"""A/B of the BVH large-triangle threshold (bvh.cpp kBigFrac, overridden by
IPT_BVH_BIGFRAC at scene load) on the BVH scenes: the same library, the scene
loaded once per threshold, interleaved timing rounds; every variant's frame
checked bit-exact against the default threshold first."""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("IPT_VB_NORTHSTAR", "1")
os.environ.setdefault("IPT_VB_SPHERE", "1")
import variant_bench as VB  # noqa: E402

N = VB.N


def main():
    fracs = sys.argv[1:] or ["0.03125", "0.015625", "0.0078125", "0.00390625"]
    L = VB.load(N.LIB_PATH)
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for sname in ("northstar", "sphere"):
        recs = VB.SCENES[sname]
        hs = {}
        for f in fracs:
            os.environ["IPT_BVH_BIGFRAC"] = f
            hs[f] = VB.scene(L, recs)
        os.environ.pop("IPT_BVH_BIGFRAC")
        p = N.make_params(64, 64, 8, 4, 123)
        want = None
        for f in fracs:
            got = np.zeros((64 * 64 * 8, 3), np.float32)
            assert L.ipt_render_samples_host(hs[f], C.byref(p), got.ctypes.data_as(N.fp)) == 0
            want = got if want is None else want
            print(sname, f, "bit-exact" if np.array_equal(got.view(np.uint32), want.view(np.uint32)) else "MISMATCH",
                  flush=True)
        p = N.make_params(512, 512, 64, 4, 0)
        buf = torch.empty((512 * 512 * 64, 3), device=dev)
        adj = torch.ones((512, 512, 3), device=dev)
        g = torch.zeros((8192, 3), dtype=torch.float64, device=dev)
        times = {f: {"fwd": [], "adj": []} for f in fracs}
        for rnd in range(5):
            for f in fracs:
                for kind in ("fwd", "adj"):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    for _ in range(3):
                        if kind == "fwd":
                            assert L.ipt_render_samples_sm_dev(hs[f], C.byref(p), None, buf.data_ptr(), st) == 0
                        else:
                            assert L.ipt_adjoint_dev(hs[f], C.byref(p), None, adj.data_ptr(), g.data_ptr(), st) == 0
                    e1.record()
                    torch.cuda.synchronize()
                    if rnd:
                        times[f][kind].append(e0.elapsed_time(e1) / 3)
        for f in fracs:
            out["%s:%s" % (sname, f)] = {k: round(float(np.median(v)), 4) for k, v in times[f].items()}
            print(sname, f, out["%s:%s" % (sname, f)], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
