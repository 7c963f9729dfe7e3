"""C5 (BASELINE.json configs[4]): batch material recovery over scenes/*.txt,
256x256, 32 spp, 4 bounces, Adam on per-scene Kd in PyTorch-ROCm
(inverse_path_tracer_amd.optimize).  One GPU runs its scene-parallel share
(--scenes 13 = ceil(100/8), the per-GPU load of the 8-GPU configuration).

    python tools/bench_c5.py [--scenes 13] [--steps 20] [--warmup 2]

Prints one JSON line: optimisation steps/s over all of this GPU's scenes, the
scene-iterations/s, and the forward+adjoint sample rate inside the loop
(HIP events around whole steps: render + loss + backward + Adam + clamp).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from inverse_path_tracer_amd.optimize import build_tasks, optimize  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", type=int, default=13)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--target-spp", type=int, default=1024)
    args = ap.parse_args()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    files = [os.path.join(ROOT, "assets", "scenes", "%d.txt" % i) for i in range(args.scenes)]
    t0 = time.perf_counter()
    tasks = build_tasks(files, args.size, args.size, args.target_spp, 4, 0.5, dev)
    torch.cuda.synchronize()
    t_targets = time.perf_counter() - t0
    optimize(tasks, args.size, args.size, args.spp, 4, args.warmup, lr=1e-2)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    optimize(tasks, args.size, args.size, args.spp, 4, args.steps, lr=1e-2, seed=10**6)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    err0 = sum(float((t.kd.detach() - t.truth).abs()[18:].mean()) for t in tasks) / len(tasks)
    samples = args.scenes * args.size * args.size * args.spp
    print(json.dumps({
        "workload": "C5: scenes/0..%d, %dx%d, %d spp, 4 bounces, Adam lr 1e-2 on per-scene Kd (1 GPU's share)" % (
            args.scenes - 1, args.size, args.size, args.spp),
        "ms_per_step": round(ms, 3), "steps_per_s": round(1e3 / ms, 2),
        "scene_iterations_per_s": round(args.scenes * 1e3 / ms, 1),
        "fwd_plus_adj_Msamples_s": round(2 * samples / ms / 1e3, 1),
        "targets_s": round(t_targets, 2), "cube_kd_mean_abs_err_after": round(err0, 4),
        "loss_first_last": [tasks[0].history[0], tasks[0].history[-1]]}), flush=True)


if __name__ == "__main__":
    main()
