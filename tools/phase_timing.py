"""Per-phase cycle breakdown of trace_kernel from the IPT_PHASE_TIMING build
(lib/variants/libipt_phase.so): s_memtime deltas summed over waves.
Phases: 0 refill, 1 path cast, 2 shade+draws, 3 shadow cast, 4 emitter eval,
5 finalise (+ adjoint sweep).  Also loop iterations and mean active lanes."""
import ctypes as C
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import variant_bench as VB  # noqa: E402

N = VB.N
NAMES = ["refill", "path_cast", "shade", "shadow_cast", "emitter_eval", "finalise"]


def main():
    for lib in os.environ.get("IPT_PHASE_LIBS", "phase").split(","):
        run(lib)


def run(lib):
    L = VB.load(os.path.join(VB.ROOT, "inverse_path_tracer_amd/lib/variants/libipt_%s.so" % lib))
    L.ipt_debug_phase_cycles.argtypes = [C.POINTER(C.c_ulonglong)]
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream().cuda_stream
    out = {}
    for sname, recs in VB.SCENES.items():
        h = VB.scene(L, recs)
        p = N.make_params(512, 512, 64, 4, 0)
        buf = torch.empty((512 * 512 * 64, 3), device=dev)
        adj = torch.ones((512, 512, 3), device=dev)
        g = torch.zeros((8192, 3), dtype=torch.float64, device=dev)
        cyc = (C.c_ulonglong * 8)()
        for kind in ("fwd", "adj"):
            for rep in range(2):
                L.ipt_debug_phase_cycles(cyc)
                if kind == "fwd":
                    assert L.ipt_render_samples_sm_dev(h, C.byref(p), None, buf.data_ptr(), st) == 0
                else:
                    assert L.ipt_adjoint_dev(h, C.byref(p), None, adj.data_ptr(), g.data_ptr(), st) == 0
                torch.cuda.synchronize()
                L.ipt_debug_phase_cycles(cyc)
            v = list(cyc)
            tot = sum(v[:6])
            res = {n: round(v[i] / tot, 4) for i, n in enumerate(NAMES)}
            res["iterations_per_wave_total"] = v[6]
            res["mean_active_lanes"] = round(v[7] / max(1, v[6]), 2)
            res["cycles_total"] = tot
            out["%s:%s:%s" % (lib, sname, kind)] = res
            print(lib, sname, kind, json.dumps(res), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
