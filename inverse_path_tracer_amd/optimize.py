"""Material recovery by gradient descent (BASELINE.json configs[4], "C5").

The reference recovers per-triangle albedo by regressing a GCN on transport
graphs (ipt.py:86-140).  With the adjoint integrator the same unknowns are
optimised directly: per scene, Kd (nT, 3) starts at a constant and Adam
minimises the L2 distance between the rendered HDR image and a target render
(the reference's imgs/*.png are not shipped; targets are forward renders at
the ground-truth Kd with many more samples).

* Scene batches: scenes/0..99.txt share their geometry and differ only in the
  cube's Kd (ipt_cuda.py:115-134 writes them that way), so the scenes of a rank
  form ONE batch over one loaded geometry: each step is one batched forward
  launch and one batched adjoint launch (torch_ops.render_batch) for all of
  them, instead of two launches and an autograd graph per scene.  Scenes whose
  geometry differs fall back to per-scene renders.
* Unbiased gradients: the adjoint of step t traces an independent sample
  stream (``adjoint_seed``), so the residual I - T of the forward is not
  correlated with the derivative (same-stream replay biases Adam towards
  darker albedo by O(1/spp)).
* Scene-parallel: rank r owns a contiguous block of the scenes
  (``shard_scenes``); per-scene parameters need no collective.  Every sample
  stream is keyed on the GLOBAL scene index and the global scene count (the
  target render of scene i, the forward / adjoint frames of step t), so a
  split over ranks traces exactly the samples of the one-rank run: images
  bitwise, gradients to fp64 summation order (tests/test_gpu_multirank.py).  ``tie_shared=k`` additionally treats the first k triangles
  (18 = the Cornell box, identical in every scene) as ONE parameter set shared
  by all scenes -- their gradient is summed across scenes and ranks with a
  single RCCL all-reduce per step.

    python -m inverse_path_tracer_amd.optimize --scenes assets/scenes --n 13 --steps 200
"""
from __future__ import annotations

import argparse
import os
import time
from dataclasses import dataclass, field
from typing import List, Optional

import numpy as np
import torch

from . import torch_ops
from .distributed import allreduce_, world
from .scene import Scene

# ipt_scene_export_triangles columns holding the diffuse Kd (everything else
# is geometry / other material fields that must agree for a batch)
_KD_COLS = slice(25, 28)


@dataclass
class SceneTask:
    path: str
    scene: Scene                  # geometry handle (shared by the tasks of one batch)
    truth: torch.Tensor           # ground-truth Kd (nT, 3)
    target: torch.Tensor          # target HDR image (H, W, 3)
    kd: torch.Tensor              # parameters (nT, 3)
    history: List[float] = field(default_factory=list)
    index: int = 0                # global scene index (keys the task's sample streams)


def _scene_files(root: str, n: int) -> List[str]:
    return [os.path.join(root, "%d.txt" % i) for i in range(n)]


def shard_scenes(n: int, world: int, rank: int):
    """Contiguous block [begin, end) of the n scenes owned by `rank` (balanced:
    sizes differ by at most one).  Contiguous, so a rank's scenes of one
    geometry are ONE batch whose sample streams continue the global ones."""
    base, rem = divmod(n, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def _runs(idx: List[int], tasks: List[SceneTask], limit: int):
    """Split task positions into runs of consecutive global indices (<= limit each)."""
    runs, cur = [], []
    for i in idx:
        if cur and (tasks[i].index != tasks[cur[-1]].index + 1 or len(cur) >= limit):
            runs.append(cur)
            cur = []
        cur.append(i)
    if cur:
        runs.append(cur)
    return runs


def _geometry_key(sc: Scene) -> bytes:
    t = sc.triangles()
    return np.concatenate([t[:, :_KD_COLS.start], t[:, _KD_COLS.stop:]], axis=1).tobytes()


def build_tasks(files: List[str], width: int, height: int, target_spp: int, max_bounces: int, init: float,
                device: torch.device, seed: int = 7, target_chunk: int = 16, first_index: int = 0) -> List[SceneTask]:
    """Load the scenes (one device geometry per distinct geometry), render the
    targets in batches of `target_chunk`, and create the parameters.  files[i]
    is global scene first_index + i: its target render traces the samples of
    seed + 10^9 + (first_index + i) * W*H*target_spp, whichever rank loads it."""
    groups = {}  # geometry key -> device Scene
    tasks = []
    for k, f in enumerate(files):
        host = Scene.from_file(f, device=False)
        key = _geometry_key(host)
        if key not in groups:
            groups[key] = Scene.from_file(f)
        truth = torch.tensor(host.materials, device=device)
        host.close()
        tasks.append(SceneTask(f, groups[key], truth, None, torch.full_like(truth, init).requires_grad_(True),
                               index=first_index + k))
    stride = width * height * target_spp
    with torch.no_grad():
        for sc in groups.values():
            mine = [i for i, t in enumerate(tasks) if t.scene is sc]
            for idx in _runs(mine, tasks, target_chunk):
                kd = torch.stack([tasks[i].truth for i in idx])
                img = torch_ops.render_batch(sc, kd, width, height, target_spp, max_bounces,
                                             seed=seed + 10**9 + tasks[idx[0]].index * stride, seed_stride=stride)
                for j, i in enumerate(idx):
                    tasks[i].target = img[j].clone()
    return tasks


class MaterialOptimizer:
    """Persistent Adam state over every task's kd (nT, 3).  Each group of
    tasks sharing a geometry is one batch: a (S, nT, 3) parameter whose rows
    the tasks' kd become views of, rendered by one batched forward and one
    batched adjoint launch per step.  tie_shared = number of leading
    triangles whose Kd is shared by all scenes (18 = the Cornell box), or
    None.  Losses reach the tasks' histories with one device->host copy every
    `flush_every` steps (on every rank) and at the end of each run().

    Sample streams: step t of the whole job (n_total scenes over all ranks,
    default max(task index) + 1) traces frames [2 t n_total, 2 (t + 1) n_total) of the
    sample-index space, scene i's forward in frame 2 t n_total + i and its
    adjoint n_total frames later -- so each rank of a scene-parallel split
    traces exactly the one-rank run's samples for its scenes.  A batch is
    one geometry's tasks with consecutive global indices (seed_stride = one
    frame between its sets)."""

    def __init__(self, tasks: List[SceneTask], width: int, height: int, spp: int, max_bounces: int,
                 lr: float = 1e-2, tie_shared: Optional[int] = None, seed: int = 0, flush_every: int = 16,
                 decorrelate: bool = True, n_total: Optional[int] = None):
        self.tasks, self.W, self.H, self.spp, self.mb = tasks, width, height, spp, max_bounces
        self.tie, self.seed, self.flush_every, self.decorrelate = tie_shared, seed, flush_every, decorrelate
        # the job's scene count: the caller's, else max(index) + 1 (a rank
        # given only the tasks of global scenes b .. b+k-1 must pass the job's n)
        idx = [t.index for t in tasks]
        if len(set(idx)) != len(idx):
            raise ValueError("MaterialOptimizer: task indices must be unique (build_tasks(first_index=...))")
        self.n_total = (max(idx) + 1 if idx else 0) if n_total is None else int(n_total)
        if idx and max(idx) >= self.n_total:
            raise ValueError("MaterialOptimizer: task index %d >= n_total %d" % (max(idx), self.n_total))
        self.frame = width * height * spp
        self.batches = []  # (scene, tasks)
        for t in tasks:
            b = self.batches[-1] if self.batches else None
            if b is not None and b[0] is t.scene and t.index == b[1][-1].index + 1:
                b[1].append(t)
            else:
                self.batches.append((t.scene, [t]))
        self.leaves, self.targets, self.offsets = [], [], []
        for sc, ts in self.batches:
            leaf = torch.stack([t.kd.detach() for t in ts]).clone().requires_grad_(True)
            tgt = torch.stack([t.target for t in ts])
            for j, t in enumerate(ts):
                t.kd, t.target = leaf[j], tgt[j]
            self.offsets.append(ts[0].index)  # global index of the batch's first scene
            self.leaves.append(leaf)
            self.targets.append(tgt)
        self.shared = None
        if tie_shared:
            self.shared = tasks[0].kd.detach()[:tie_shared].clone().requires_grad_(True) if tasks else \
                torch.full((tie_shared, 3), 0.5, device="cuda", requires_grad=True)
        self.params = self.leaves + ([self.shared] if self.shared is not None else [])
        self.opt = torch.optim.Adam(self.params, lr=lr)
        self.step_count = 0
        self.pending = []  # (tasks, per-scene loss tensor) in step order

    def step(self):
        """One Adam step over every scene (no host synchronisation)."""
        self.opt.zero_grad(set_to_none=False)
        step = self.step_count
        for (sc, ts), leaf, target, n_before in zip(self.batches, self.leaves, self.targets, self.offsets):
            kd = leaf
            if self.shared is not None:
                kd = torch.cat([self.shared.unsqueeze(0).expand(len(ts), -1, -1), leaf[:, self.tie:]], dim=1)
            # step t uses 2T frames of the sample-index space: the T forward frames, then the T adjoint frames
            T = self.n_total
            base = self.seed + (2 * step * T + n_before) * self.frame
            img = torch_ops.render_batch(sc, kd, self.W, self.H, self.spp, self.mb, seed=base, seed_stride=self.frame,
                                         adjoint_seed=(base + T * self.frame) if self.decorrelate else None)
            per_scene = ((img - target) ** 2).mean(dim=(1, 2, 3))
            per_scene.sum().backward()  # each scene's loss only reaches its own parameters
            self.pending.append((ts, per_scene.detach()))
        if self.shared is not None:
            if self.shared.grad is None:
                self.shared.grad = torch.zeros_like(self.shared)
            allreduce_(self.shared.grad)  # the only exchange: one nT_shared*3 all-reduce
        self.opt.step()
        with torch.no_grad():
            for p in self.params:
                p.clamp_(0.0, 1.0)
        self.step_count += 1
        if self.flush_every and self.step_count % self.flush_every == 0:
            _flush_losses(self.pending)

    def run(self, steps: int, log_every: int = 0):
        _, R = world()
        for i in range(steps):
            self.step()
            if log_every and i % log_every == 0:
                _flush_losses(self.pending)
                if R == 0:
                    print("step %d loss %.6g" % (self.step_count - 1, sum(t.history[-1] for t in self.tasks) /
                                                 max(1, len(self.tasks))), flush=True)
        _flush_losses(self.pending)
        return self


def optimize(tasks: List[SceneTask], width: int, height: int, spp: int, max_bounces: int, steps: int,
             lr: float = 1e-2, tie_shared: Optional[int] = None, seed: int = 0, log_every: int = 0,
             flush_every: int = 16, decorrelate: bool = True, n_total: Optional[int] = None):
    """`steps` Adam steps of a fresh MaterialOptimizer; returns the shared
    (tied) parameter or None."""
    m = MaterialOptimizer(tasks, width, height, spp, max_bounces, lr, tie_shared, seed, flush_every, decorrelate,
                          n_total)
    m.run(steps, log_every)
    return m.shared


def _flush_losses(pending):
    """Move the pending per-scene losses to the tasks' histories (one copy)."""
    if pending:
        vals = torch.cat([l for _, l in pending]).float().cpu().tolist()
        k = 0
        for ts, _ in pending:
            for t in ts:
                t.history.append(vals[k])
                k += 1
        pending.clear()


def observable_mask(tasks: List[SceneTask], width: int, height: int, spp: int, max_bounces: int, seed: int = 5,
                    frac: float = 0.25, first: int = 18):
    """Per task, the triangles >= `first` whose Kd the image constrains: |dL/dKd|
    at the start above `frac` of the largest (the cube's back and bottom faces
    never reach the camera and cannot be recovered)."""
    masks = []
    for t in tasks:
        kd = t.kd.detach().clone().requires_grad_(True)
        img = torch_ops.render(t.scene, kd, width, height, spp, max_bounces, seed=seed)
        ((img - t.target) ** 2).mean().backward()
        g = kd.grad.abs().sum(1)[first:]
        masks.append(g > frac * float(g.max()))
    return masks


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scenes", default=os.path.join(os.path.dirname(os.path.dirname(__file__)), "assets", "scenes"))
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--width", type=int, default=256)
    ap.add_argument("--height", type=int, default=256)
    ap.add_argument("--spp", type=int, default=32)
    ap.add_argument("--target-spp", type=int, default=1024)
    ap.add_argument("--bounces", type=int, default=4)
    ap.add_argument("--steps", type=int, default=200)
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
    b, e = shard_scenes(args.n, ws, rank)
    files = _scene_files(args.scenes, args.n)[b:e]
    t0 = time.time()
    tasks = build_tasks(files, args.width, args.height, args.target_spp, args.bounces, 0.5, dev, first_index=b)
    torch.cuda.synchronize()
    t1 = time.time()
    m = MaterialOptimizer(tasks, args.width, args.height, args.spp, args.bounces, args.lr,
                          tie_shared=18 if args.tie else None, n_total=args.n)
    m.run(args.steps, log_every=10)
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
