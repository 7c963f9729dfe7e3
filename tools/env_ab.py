"""A/B of launch-time switches read from the environment (one process,
interleaved rounds, HIP events on the launch stream): each mode is a name and
a set of environment variables applied around its launches, e.g.

    python tools/env_ab.py fused: two_kernel:IPT_RENDER_TWO_KERNEL=1 g0:IPT_GUIDED_TAIL=0

Legs per scene (Cornell = C2, scenes/0.txt = C3, the north-star BVH scene):
the render (ipt_render_dev) and the adjoint (ipt_adjoint_dev) of the whole
512x512x64 frame and of one interleaved 1/8 share (the 8-GPU tile split's
per-rank launch).  The first mode's image and gradient are the reference:
every other mode must reproduce the image bitwise and the gradient to 1e-12.
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
from conftest import CORNELL, NORTHSTAR, SCENE0, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402


def parse_mode(m):
    name, _, rest = m.partition(":")
    env = dict(kv.split("=", 1) for kv in rest.split(",") if kv)
    return name, env


class Env:
    def __init__(self, env):
        self.env, self.old = env, {}

    def __enter__(self):
        for k, v in self.env.items():
            self.old[k] = os.environ.get(k)
            os.environ[k] = v

    def __exit__(self, *a):
        for k, v in self.old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("modes", nargs="+")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--scenes", default="cornell,scene0,northstar")
    ap.add_argument("--legs", default="fwd,adj")
    ap.add_argument("--scene-env", action="store_true",
                    help="load each mode's own copy of the scene under its environment (scene-load switches, "
                         "e.g. IPT_WIDE_LEAF_TRIS)")
    args = ap.parse_args()
    modes = [parse_mode(m) for m in args.modes]
    torch.cuda.set_device(0)
    L = N.lib()
    stream = torch.cuda.current_stream()
    st = stream.cuda_stream
    W = H = 512
    spp, mb = 64, 4
    hdr = torch.empty((W * H, 3), device="cuda")
    adj = torch.full((H, W, 3), 1.0 / (3 * W * H), device="cuda")
    recs = {"cornell": CORNELL, "scene0": SCENE0, "northstar": NORTHSTAR}
    out = {}
    for name in args.scenes.split(","):
        scs = {}
        for mname, env in modes:
            if args.scene_env or not scs:
                with Env(env if args.scene_env else {}):
                    scs[mname] = product_scene(recs[name])
            else:
                scs[mname] = next(iter(scs.values()))
        nT = next(iter(scs.values())).nT
        grad = torch.zeros((nT, 3), dtype=torch.float64, device="cuda")
        for share in (1, 8):
            p = N.make_params(W, H, spp, mb, 0, 0, H, share)
            pu = N.make_params(W, H, spp, None, 0, 0, H, share)  # the reference's own estimator (no bounce cap)

            def mode_calls(sc):
                return {"fwd": lambda: N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, hdr.data_ptr(), None, st)),
                        "adj": lambda: N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p), None, adj.data_ptr(),
                                                                 grad.data_ptr(), st)),
                        "fwdu": lambda: N.check(L.ipt_render_dev(sc.handle, C.byref(pu), None, hdr.data_ptr(), None,
                                                                 st)),
                        "adju": lambda: N.check(L.ipt_adjoint_dev(sc.handle, C.byref(pu), None, adj.data_ptr(),
                                                                  grad.data_ptr(), st))}
            mcalls = {mname: mode_calls(scs[mname]) for mname, _ in modes}
            legs = args.legs.split(",")
            ref = {}
            for mname, env in modes:  # correctness against the first mode
                calls = mcalls[mname]
                with Env(env):
                    for leg in legs:
                        grad.zero_()
                        calls[leg]()
                        torch.cuda.synchronize()
                        fwd = leg.startswith("fwd")
                        v = hdr.cpu().numpy().view(np.uint32).copy() if fwd else grad.cpu().numpy().copy()
                        if leg not in ref:
                            ref[leg] = v
                        elif fwd:
                            print(name, share, mname, "image bitwise:", bool(np.array_equal(v, ref[leg])), flush=True)
                        else:
                            err = float(np.max(np.abs(v - ref[leg])) / max(np.max(np.abs(ref[leg])), 1e-300))
                            print(name, share, mname, "gradient max rel diff %.1e" % err, flush=True)
            times = {(m, leg): [] for m, _ in modes for leg in legs}
            for rnd in range(args.rounds):
                for mname, env in modes:
                    calls = mcalls[mname]
                    with Env(env):
                        for leg in legs:
                            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                            e0.record(stream)
                            for _ in range(args.reps):
                                calls[leg]()
                            e1.record(stream)
                            torch.cuda.synchronize()
                            if rnd > 0:
                                times[(mname, leg)].append(e0.elapsed_time(e1) / args.reps)
            for (mname, leg), v in times.items():
                key = "%s:1/%d:%s:%s" % (name, share, leg, mname)
                out[key] = round(float(np.median(v)), 4)
                print(key, out[key], flush=True)
        for sc in {id(v): v for v in scs.values()}.values():
            sc.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
