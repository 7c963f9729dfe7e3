"""Per-phase cycle breakdown of trace_kernel from the IPT_PHASE_TIMING build
(lib/variants/libipt_phase.so): s_memtime deltas summed over waves.
Phases: 0 refill, 1 path cast, 2 shade+draws, 3 shadow cast, 4 emitter eval,
5 finalise (+ adjoint sweep); tree_path / tree_shadow: the coop_cast part of
phases 1 and 3 (BVH scenes).  Also loop iterations and mean active lanes,
and per phase the mean number of lanes that take part in it when a wave runs
it (`lanes`: refill = lanes refilled, path_cast = active lanes, shade /
finalise = lanes at a path vertex, shadow_cast = lanes casting a shadow ray,
emitter_eval = lanes whose shadow ray reached the emitter, sweep = valid
tasks per round) and `runs` = the fraction of wave iterations that run it;
`lane_use` = the cycle-weighted mean of lanes/64 over the six phases (the
finalise phase weighted by its own lanes, the adjoint sweep not split out),
an estimate of the lane-slots the phases' instructions use; chain: the
adjoint sweep's chain steps per round and the fraction of them that a lane
still needs."""
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
        pu = N.make_params(512, 512, 64, None, 0)
        hdr = torch.empty((512 * 512, 3), device=dev)
        adj = torch.ones((512, 512, 3), device=dev)
        g = torch.zeros((8192, 3), dtype=torch.float64, device=dev)
        cyc = (C.c_ulonglong * 26)()
        for kind in ("fwd", "adj", "fwdu", "adju"):  # the render (fused mean for brute-force scenes), the adjoint
            for rep in range(2):
                L.ipt_debug_phase_cycles(cyc)
                q = pu if kind.endswith("u") else p
                if kind.startswith("fwd"):
                    assert L.ipt_render_dev(h, C.byref(q), None, hdr.data_ptr(), None, st) == 0
                else:
                    assert L.ipt_adjoint_dev(h, C.byref(q), None, adj.data_ptr(), g.data_ptr(), st) == 0
                torch.cuda.synchronize()
                L.ipt_debug_phase_cycles(cyc)
            v = list(cyc)
            tot = sum(v[:6])
            res = {n: round(v[i] / tot, 4) for i, n in enumerate(NAMES)}
            res["tree_path"] = round(v[8] / tot, 4)
            res["tree_shadow"] = round(v[9] / tot, 4)
            res["iterations_per_wave_total"] = v[6]
            res["mean_active_lanes"] = round(v[7] / max(1, v[6]), 2)
            res["cycles_total"] = tot
            it = max(1, v[6])
            lanes = {"refill": (v[10], v[11]), "path_cast": (v[7], v[6]), "shade": (v[12], v[13]),
                     "shadow_cast": (v[14], v[15]), "emitter_eval": (v[16], v[17]), "finalise": (v[18], v[19])}
            res["lanes"] = {k: round(a / max(1, b), 2) for k, (a, b) in lanes.items()}
            res["runs"] = {k: round(b / it, 4) for k, (a, b) in lanes.items()}
            res["lane_use"] = round(sum(v[i] / tot * (a / max(1, b)) / 64 for i, (k, (a, b)) in
                                        enumerate(lanes.items())), 4)
            if v[21]:
                res["sweep"] = {"rounds_per_iteration": round(v[21] / it, 4), "tasks_per_round": round(v[20] / v[21], 2),
                                "chain_steps_per_round": round(v[22] / v[21], 3),
                                "chain_lane_use": round(v[24] / max(1, 64 * v[22]), 4)}
            out["%s:%s:%s" % (lib, sname, kind)] = res
            print(lib, sname, kind, json.dumps(res), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
