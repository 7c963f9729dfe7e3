"""Multi-GPU sharding of the path tracer (one process per GPU, torch.distributed).

The reference has no multi-GPU path.  The work shards with no
data-path exchange because every sample's RNG is seeded by its GLOBAL index
(path_trace.cu:151-153): any partition of the sample space reproduces the
single-GPU result bit-for-bit (forward) or up to fp64 summation order
(adjoint, graph).

* Strong scaling (one image, C2 / C4): each rank traces a share of the rows.
  ``shard_rows`` gives contiguous bands; ``shard_rows_interleaved`` gives rank
  r the rows r, r + world, ... (row_step = world), which balances the cost:
  at C4 the contiguous bands differ by 7.6% (max/mean: the light and the cube
  sit in particular bands), interleaved shares by < 1% (bench.py
  ``bands_*``).  The forward needs no collective (``gather_rows`` only if a
  rank wants the whole image); the adjoint's only exchange is ONE all-reduce
  of the nT*3 fp64 gradient (``allreduce_``), 720 B for 30 triangles --
  latency-bound on xGMI, no bucketing needed.
* createGraph (G3) across ranks (``graph_sharded``): per-rank fp64 bins of
  the rank's interleaved rows (as the forward and adjoint legs), ONE
  all-reduce of the (nT+1)*nT*8 bins (59.5 KB for nT = 30), then
  DataWrapper::compress on every rank.
* Weak scaling (bench.py): every rank renders its own frame of the same
  configuration; frame f uses the seed offset ``frame_seed`` so the global
  sample index space stays disjoint across frames.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_rows(height: int, world: int, rank: int):
    """Contiguous, balanced row band [begin, end) of `rank` out of `world`."""
    base, rem = divmod(height, world)
    begin = rank * base + min(rank, rem)
    return begin, begin + base + (1 if rank < rem else 0)


def shard_rows_interleaved(height: int, world: int, rank: int):
    """(row_begin, row_end, row_step) of `rank`'s interleaved share: rows
    rank, rank + world, ... < height (the C ABI's row_step)."""
    return min(rank, height), height, max(1, world)


def frame_seed(seed: int, frame: int, width: int, height: int, spp: int) -> int:
    """Seed of frame `frame`: its sample indices follow frame-1's (disjoint RNG streams)."""
    return (int(seed) + int(frame) * width * height * spp) & 0xFFFFFFFFFFFFFFFF


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def allreduce_(t: torch.Tensor) -> torch.Tensor:
    """Sum a per-rank partial (gradient or graph bins) in place across ranks."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return t


def gather_rows(band: torch.Tensor, height: int, interleaved: bool = False) -> torch.Tensor:
    """All-gather the ranks' rows (shard_rows or shard_rows_interleaved
    layout) into the full (H, W, C) image."""
    W, R = world()
    if W == 1:
        return band
    counts = [len(range(*shard_rows_interleaved(height, W, r))) if interleaved else
              (lambda be: be[1] - be[0])(shard_rows(height, W, r)) for r in range(W)]
    pad = torch.zeros((max(counts),) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
    pad[: band.shape[0]] = band
    out = [torch.empty_like(pad) for _ in range(W)]
    dist.all_gather(out, pad)
    if not interleaved:
        return torch.cat([o[:n] for o, n in zip(out, counts)], dim=0)
    full = torch.empty((height,) + tuple(band.shape[1:]), dtype=band.dtype, device=band.device)
    for r, (o, n) in enumerate(zip(out, counts)):
        full[r::W] = o[:n]
    return full


def graph_sharded(scene, target, width: int, height: int, spp: int, max_bounces=None, seed: int = 0,
                  device=None):
    """createGraph (inv_path_trace.cu:195-208) sharded by interleaved rows
    (rank r traces rows r, r + world, ...: shard_rows_interleaved, the same
    split as the forward and adjoint legs; contiguous bands differ in cost by
    up to 7.6%): returns the compressed (nT+1)*nT*7 floats, identical on every
    rank and equal to the single-GPU result up to fp64 summation order.
    `scene` is a Scene (or any object with .nT and .graph(target, W, H, spp,
    mb, seed, row_begin, row_end, row_step) returning (bins, data)).
    `device` is where the all-reduce runs: default CPU under gloo, the
    current GPU under nccl (RCCL)."""
    import numpy as np

    from .scene import compress

    W, R = world()
    b, e, st = shard_rows_interleaved(height, W, R)
    bins, _ = scene.graph(target, width, height, spp, max_bounces, seed, b, e, st)
    t = torch.from_numpy(np.ascontiguousarray(bins, np.float64))
    if device is None and W > 1 and dist.get_backend() == "nccl":
        device = torch.device("cuda", torch.cuda.current_device())  # RCCL reduces device tensors only
    if device is not None:
        t = t.to(device)
    allreduce_(t)
    return compress(scene.nT, t.cpu().numpy())
