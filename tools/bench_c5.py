"""C5 (BASELINE.json configs[4]): batch material recovery over scenes/*.txt,
256x256, 32 spp, 4 bounces, Adam on per-scene Kd in PyTorch-ROCm
(inverse_path_tracer_amd.optimize).  One GPU runs its scene-parallel share
(--scenes 13 = ceil(100/8), the per-GPU load of the 8-GPU configuration).

    python tools/bench_c5.py [--scenes 13] [--steps 20] [--warmup 3] [--total 300]

One persistent optimiser: `warmup` untimed steps, `steps` timed steps (HIP
events around whole steps: batched render + loss + backward (batched adjoint)
+ Adam + clamp), then more steps up to `total` for the convergence record.
Prints one JSON line with the step rate, the forward+adjoint sample rate, and
the cube's observability-masked Kd error before and after.
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from inverse_path_tracer_amd.optimize import MaterialOptimizer, build_tasks, observable_mask  # noqa: E402


def masked_err(tasks, masks):
    return sum(float((t.kd.detach() - t.truth)[18:][m].abs().mean()) for t, m in zip(tasks, masks)) / len(tasks)


def run(scenes=13, steps=20, warmup=3, total=300, size=256, spp=32, target_spp=1024, bounces=4, lr=1e-2):
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    files = [os.path.join(ROOT, "assets", "scenes", "%d.txt" % i) for i in range(scenes)]
    t0 = time.perf_counter()
    tasks = build_tasks(files, size, size, target_spp, bounces, 0.5, dev)
    torch.cuda.synchronize()
    t_targets = time.perf_counter() - t0
    masks = observable_mask(tasks, size, size, 64, bounces)
    err0 = masked_err(tasks, masks)
    opt = MaterialOptimizer(tasks, size, size, spp, bounces, lr=lr)
    opt.run(warmup)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        opt.step()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    opt.run(max(0, total - warmup - steps))
    err1 = masked_err(tasks, masks)
    samples = scenes * size * size * spp
    return {
        "workload": "C5: scenes/0..%d, %dx%d, %d spp, %d bounces, Adam lr %g on per-scene Kd (1 GPU's share), "
                    "one batched forward + one batched adjoint launch per step" % (scenes - 1, size, size, spp,
                                                                                  bounces, lr),
        "ms_per_step": round(ms, 3), "steps_per_s": round(1e3 / ms, 2),
        "scene_iterations_per_s": round(scenes * 1e3 / ms, 1),
        "fwd_plus_adj_Msamples_s": round(2 * samples / ms / 1e3, 1),
        "targets_s": round(t_targets, 2), "steps_total": opt.step_count,
        "observable_tris_per_scene": [int(m.sum()) for m in masks],
        "cube_kd_masked_abs_err_before": round(err0, 4), "cube_kd_masked_abs_err_after": round(err1, 4),
        "loss_first_last": [tasks[0].history[0], tasks[0].history[-1]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=13)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--total", type=int, default=300)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--target-spp", type=int, default=1024)
    a = ap.parse_args()
    print(json.dumps(run(a.scenes, a.steps, a.warmup, a.total, a.size, a.spp, a.target_spp)), flush=True)


if __name__ == "__main__":
    main()
