"""createGraph's integrator (trace_kernel<MODE_GRAPH>, inv_path_trace.cu:152-208)
at the reference's own configuration -- scenes/0.txt, 500x500, 100 spp, no
bounce cap, target preds/0_true.png -- K back-to-back launches, for
rocprofv3 --kernel-trace --stats (tools/gpu.sh graphprof).  Prints the HIP
event time per launch."""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import SCENE0, product_scene  # noqa: E402
from inverse_path_tracer_amd import _native as N, png_read  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    L = N.lib()
    st = torch.cuda.current_stream()
    P = product_scene(SCENE0)
    tgt = torch.from_numpy(png_read(os.path.join(ROOT, "tests", "golden", "preds_0_true.png"))).cuda()
    acc = torch.zeros(((P.nT + 1) * P.nT, N.ACC_WIDTH), dtype=torch.float64, device="cuda")
    p = N.make_params(500, 500, 100, None, 0)

    def step():
        acc.zero_()
        N.check(L.ipt_graph_dev(P.handle, C.byref(p), tgt.data_ptr(), acc.data_ptr(), st.cuda_stream))

    step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(args.steps):
        step()
    e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    print(json.dumps({"workload": "createGraph scenes/0.txt 500x500x100 unbounded, target preds/0_true.png",
                      "ms_per_launch": round(ms, 4), "Msamples_s": round(500 * 500 * 100 / ms / 1e3, 1)}))


if __name__ == "__main__":
    main()
