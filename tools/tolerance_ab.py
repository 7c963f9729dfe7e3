"""Tolerance check of a non-exact kernel variant (e.g. the fast-cast build,
make variant V=fastcast DEFS=-DIPT_FAST_CAST=1) against the exact library
(which equals the CPU oracle bit for bit, tests/test_gpu_full.py) on the
C2 and C3 frames, with SURVEY.md §8(c)'s tolerances: >= 99.9% of per-sample
radiances within rtol 1e-4 / atol 1e-6, image-mean relative error <= 1e-3,
adjoint gradient rtol 1e-3.

    python tools/tolerance_ab.py fastcast
"""
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import variant_bench as VB  # noqa: E402

N = VB.N


def main():
    name = sys.argv[1]
    L = VB.load(os.path.join(VB.ROOT, "inverse_path_tracer_amd/lib/variants/libipt_%s.so" % name))
    ref = VB.load(N.LIB_PATH)
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for sname in ("cornell", "scene0"):
        recs = VB.SCENES[sname]
        hv, hr = VB.scene(L, recs), VB.scene(ref, recs)
        p = N.make_params(512, 512, 64, 4, 0)
        a = torch.empty((512 * 512 * 64, 3), device=dev)
        b = torch.empty_like(a)
        assert L.ipt_render_samples_dev(hv, C.byref(p), None, a.data_ptr(), st) == 0
        assert ref.ipt_render_samples_dev(hr, C.byref(p), None, b.data_ptr(), st) == 0
        torch.cuda.synchronize()
        close = torch.isclose(a, b, rtol=1e-4, atol=1e-6).all(dim=1)
        frac = float(close.float().mean())
        mean_rel = float((a.double().mean(0) - b.double().mean(0)).abs().max() / b.double().mean(0).abs().max())
        adj = torch.from_numpy(np.random.RandomState(1).uniform(-1, 1, (512, 512, 3)).astype(np.float32)).to(dev)
        nT = 18 if sname == "cornell" else 30
        ga = torch.zeros((nT, 3), dtype=torch.float64, device=dev)
        gb = torch.zeros_like(ga)
        assert L.ipt_adjoint_dev(hv, C.byref(p), None, adj.data_ptr(), ga.data_ptr(), st) == 0
        assert ref.ipt_adjoint_dev(hr, C.byref(p), None, adj.data_ptr(), gb.data_ptr(), st) == 0
        torch.cuda.synchronize()
        grel = float(((ga - gb).abs() / gb.abs().clamp_min(1e-3 * float(gb.abs().max()))).max())
        r = {"samples_within_rtol1e-4": round(frac, 6), "samples_bit_identical": round(float((a == b).all(1).float().mean()), 6),
             "image_mean_rel_err": mean_rel, "grad_max_rel_err": grel,
             "pass": frac >= 0.999 and mean_rel <= 1e-3 and grel <= 1e-3}
        out[sname] = r
        print(sname, json.dumps(r), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
