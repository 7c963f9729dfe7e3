"""Material recovery by gradient descent (BASELINE.json configs[4], "C5").

The reference recovers per-triangle albedo by regressing a GCN on transport
graphs (ipt.py:86-140).  With the adjoint integrator the same unknowns are
optimised directly: per scene, Kd (nT, 3) starts at a constant and Adam
minimises the L2 distance between the rendered HDR image and a target render
(the reference's imgs/*.png are not shipped; targets are forward renders at
the ground-truth Kd with many more samples).

Scene-parallel: scene i belongs to rank i % world; per-scene parameters need
no collective.  ``tie_shared=True`` additionally treats the Cornell-box
triangles (identical in every scenes/*.txt) as ONE parameter set shared by all
scenes -- their gradient is then summed across scenes and ranks with a single
RCCL all-reduce per step.

    python -m inverse_path_tracer_amd.optimize --scenes assets/scenes --n 4 --steps 50
"""
from __future__ import annotations

import argparse
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional

import torch

from . import torch_ops
from .distributed import allreduce_, world
from .scene import Scene


@dataclass
class SceneTask:
    path: str
    scene: Scene
    truth: torch.Tensor           # ground-truth Kd (nT, 3)
    target: torch.Tensor          # target HDR image (H, W, 3)
    kd: torch.Tensor              # parameters (nT, 3), requires_grad
    history: List[float] = field(default_factory=list)


def _scene_files(root: str, n: int) -> List[str]:
    return [os.path.join(root, "%d.txt" % i) for i in range(n)]


def build_tasks(files: List[str], width: int, height: int, target_spp: int, max_bounces: int, init: float,
                device: torch.device, seed: int = 7) -> List[SceneTask]:
    tasks = []
    for f in files:
        sc = Scene.from_file(f)
        truth = torch.tensor(sc.materials, device=device)
        with torch.no_grad():
            target = torch_ops.render(sc, truth, width, height, target_spp, max_bounces, seed=seed + 10**9)
        kd = torch.full_like(truth, init).requires_grad_(True)
        tasks.append(SceneTask(f, sc, truth, target, kd))
    return tasks


def optimize(tasks: List[SceneTask], width: int, height: int, spp: int, max_bounces: int, steps: int,
             lr: float = 1e-2, tie_shared: Optional[int] = None, seed: int = 0, log_every: int = 0):
    """Adam on every task's kd.  tie_shared = number of leading triangles whose
    Kd is shared by all scenes (18 = the Cornell box), or None."""
    W, R = world()
    shared = None
    if tie_shared:
        shared = tasks[0].kd.detach()[:tie_shared].clone().requires_grad_(True) if tasks else None
        if shared is None:
            shared = torch.full((tie_shared, 3), 0.5, device="cuda", requires_grad=True)
    params = [t.kd for t in tasks] + ([shared] if shared is not None else [])
    opt = torch.optim.Adam(params, lr=lr)
    pending = []  # (task, loss tensor) in step order
    for step in range(steps):
        opt.zero_grad(set_to_none=False)
        for i, t in enumerate(tasks):
            kd = t.kd
            if shared is not None:
                kd = torch.cat([shared, t.kd[tie_shared:]], dim=0)
            img = torch_ops.render(t.scene, kd, width, height, spp, max_bounces,
                                   seed=seed + (step * 1009 + i) * width * height * spp)
            loss = ((img - t.target) ** 2).mean()
            loss.backward()
            pending.append((t, loss.detach()))  # no host sync per scene: read back once per step
        if shared is not None:
            if shared.grad is None:
                shared.grad = torch.zeros_like(shared)
            allreduce_(shared.grad)  # the only exchange: one nT_shared*3 all-reduce
        opt.step()
        with torch.no_grad():
            for p in params:
                p.clamp_(0.0, 1.0)
        if log_every and step % log_every == 0 and R == 0:
            _flush_losses(pending)
            print("step %d loss %.6g" % (step, sum(t.history[-1] for t in tasks) / max(1, len(tasks))), flush=True)
    _flush_losses(pending)
    return shared


def _flush_losses(pending):
    """Move the step losses to the tasks' histories with one device->host copy."""
    if pending:
        vals = torch.stack([l for _, l in pending]).float().cpu().tolist()
        for (t, _), v in zip(pending, vals):
            t.history.append(v)
        pending.clear()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default=os.path.join(os.path.dirname(os.path.dirname(__file__)), "assets", "scenes"))
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--target-spp", type=int, default=1024)
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--tie", action="store_true")
    args = ap.parse_args()
    import torch.distributed as dist

    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if ws > 1:
        dist.init_process_group("nccl", device_id=dev)
    files = [f for i, f in enumerate(_scene_files(args.scenes, args.n)) if i % ws == rank]
    t0 = time.time()
    tasks = build_tasks(files, args.width, args.height, args.target_spp, args.bounces, 0.5, dev)
    torch.cuda.synchronize()
    t1 = time.time()
    optimize(tasks, args.width, args.height, args.spp, args.bounces, args.steps, args.lr,
             tie_shared=18 if args.tie else None, log_every=10)
    torch.cuda.synchronize()
    t2 = time.time()
    err = [float((t.kd.detach() - t.truth).abs()[18:].mean()) for t in tasks]
    if rank == 0:
        print("scenes/rank %d  targets %.2fs  optimise %.2fs  mean |Kd - truth| (cube) %.4f" % (
            len(tasks), t1 - t0, t2 - t1, sum(err) / max(1, len(err))))
    if ws > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
