"""BVH work counters of a profiling build (make variant V=stats
DEFS=-DIPT_BVH_STATS) over the forward and the adjoint of large scenes at the
C2/C3 size: the "tests actually executed" that the roofline of a BVH scene
charges.

    IPT_AMD_LIB=inverse_path_tracer_amd/lib/variants/libipt_stats.so \\
        python tools/bvh_stats.py [--scenes northstar,sphere] [--size 512] [--spp 64]

Writes profiles/bvh_stats.json: per scene and integrator the raw counters
(ipt_device.h kBvhStats) and per sample: triangle tests (large-triangle
pre-pass + shadow target + leaf), box tests (root + 8 per 8-wide node visit),
and the algorithmic FLOP per sample = 38 * triangle tests + 12 * box tests
(a slab test is 6 FMA; its min/max are not counted).
"""
import argparse
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from bench_scenes import SCENES  # noqa: E402
from inverse_path_tracer_amd import _native as N  # noqa: E402
from inverse_path_tracer_amd.scene import ObjectSpec, Scene  # noqa: E402

NAMES = ["tree_rays", "node_visits", "leaf_visits", "shadow_occluded_in_tree", "leaf_tri_tests", "coop_calls",
         "coop_rounds", "casts", "prepass_tri_tests", "shadow_target_tests", "shadow_decided_before_tree", "unused",
         "cull_shadow_lanes", "cull_target_accepted", "cull_wave_calls", "cull_wave_pair_tests",
         "cull_lane_pair_tests", "cull_lane_box_tests", "pcull_casts", "pcull_lane_pair_tests", "pcull_lane_box_tests", "pcull_wave_calls",
         "pcull_wave_trips"]


def derive(c, n):
    tri = c["prepass_tri_tests"] + c["shadow_target_tests"] + c["leaf_tri_tests"]
    roots = c["casts"] - c["shadow_decided_before_tree"]
    box = roots + 8 * c["node_visits"]
    if c["casts"]:  # BVH scene: its culled shadow pre-pass (pair boxes + marked pair tests) too
        tri += 2 * c["cull_lane_pair_tests"]
        box += c["cull_lane_box_tests"]
    return {"samples": n, "casts_per_sample": c["casts"] / n, "tri_tests_per_sample": tri / n,
            "box_tests_per_sample": box / n, "flop_per_sample": (38 * tri + 12 * box) / n,
            "tree_rays_per_cast": c["tree_rays"] / max(1, c["casts"]),
            "nodes_per_tree_ray": c["node_visits"] / max(1, c["tree_rays"]),
            "leaf_tris_per_tree_ray": c["leaf_tri_tests"] / max(1, c["tree_rays"]),
            "rays_per_coop_round": c["tree_rays"] / max(1, c["coop_rounds"]),
            "rounds_per_coop_call": c["coop_rounds"] / max(1, c["coop_calls"]),
            "cull_target_accepted_frac": c["cull_target_accepted"] / max(1, c["cull_shadow_lanes"]),
            "cull_lanes_per_wave_call": c["cull_shadow_lanes"] / max(1, c["cull_wave_calls"]),
            "cull_pairs_tested_per_wave_call": c["cull_wave_pair_tests"] / max(1, c["cull_wave_calls"]),
            "cull_shadow_casts_per_sample": c["cull_shadow_lanes"] / n,
            "cull_tri_tests_per_sample": (c["cull_shadow_lanes"] + 2 * c["cull_lane_pair_tests"]) / n,
            "cull_box_tests_per_sample": c["cull_lane_box_tests"] / n,
            "pcull_casts_per_sample": c.get("pcull_casts", 0) / n,
            "pcull_tri_tests_per_sample": 2 * c.get("pcull_lane_pair_tests", 0) / n,
            "pcull_pairs_per_cast": c.get("pcull_lane_pair_tests", 0) / max(1, c.get("pcull_casts", 0)),
            "pcull_box_tests_per_sample": c.get("pcull_lane_box_tests", 0) / n,
            "pcull_lanes_per_wave_call": c.get("pcull_casts", 0) / max(1, c.get("pcull_wave_calls", 0)),
            "pcull_trips_per_wave_call": c.get("pcull_wave_trips", 0) / max(1, c.get("pcull_wave_calls", 0))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default="northstar,sphere,cornell,scene0")
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "bvh_stats.json"))
    args = ap.parse_args()
    L = N.lib()
    stats = L.ipt_debug_bvh_stats
    stats.argtypes = [C.POINTER(C.c_ulonglong)]
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    W = H = args.size
    n = W * H * args.spp
    samples = torch.empty((n, 3), device=dev)
    adj = torch.ones((H, W, 3), device=dev)
    buf = (C.c_ulonglong * len(NAMES))()
    out = {}
    for name in args.scenes.split(","):
        scene = Scene([ObjectSpec(o, m, p, r, s) for (o, m, p, r, s) in SCENES[name]])
        grad = torch.zeros((scene.nT, 3), device=dev, dtype=torch.float64)
        p = N.make_params(W, H, args.spp, args.bounces, 0)
        for kind in ("fwd", "adj"):
            stats(buf)  # reset
            if kind == "fwd":
                N.check(L.ipt_render_samples_sm_dev(scene.handle, C.byref(p), None, samples.data_ptr(), None))
            else:
                N.check(L.ipt_adjoint_dev(scene.handle, C.byref(p), None, adj.data_ptr(), grad.data_ptr(), None))
            torch.cuda.synchronize()
            stats(buf)
            c = dict(zip(NAMES, list(buf)))
            out["%s_%s" % (name, kind)] = {"triangles": scene.nT, "config": [W, H, args.spp, args.bounces, 0],
                                           "counters": c, "derived": derive(c, n), "bvh": scene.bvh_info()}
            print(name, kind, json.dumps(out["%s_%s" % (name, kind)]["derived"]), flush=True)
        scene.close()
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
