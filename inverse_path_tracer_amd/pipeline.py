"""The reference's end-to-end workflow (ipt.py:85-150 with ipt_cuda.py's
generate_files / generate_data / render_with_materials), sharded over ranks.

    python -m inverse_path_tracer_amd.pipeline all --root OUT --n 100
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        -m inverse_path_tracer_amd.pipeline all --root OUT --n 100

Stages (each rank takes scenes i = rank, rank + world, ...; no data-path
collective, one barrier between stages):

* ``files`` -- generate_files (ipt_cuda.py:115-134): ``scenes/{i}.txt`` =
  Cornell box at (0,0,4) scaled 2 + cube at (0,-1.5,4) with a uniform random
  inline Kd, then ``imgs/{i}.png`` = createImage (tonemapped mean of the
  forward render).  The reference draws Kd from the unseeded global numpy RNG
  and seeds its renders with time(NULL); here both are seeded per scene
  (``--seed``), so the dataset does not depend on the number of ranks.
* ``data`` -- generate_data (ipt_cuda.py:136-165) for every scene: createGraph
  against ``imgs/{i}.png`` and getMaterials, saved as ``data/{i}.npz`` (w,
  pixel, light, labels; numpy, not a pickle).
* ``train`` -- ipt.py:104-124 on rank 0: the DGL-free GCN (gcn.py), Adam.
* ``preds`` -- ipt.py:126-138: ``preds/{i}_true.png`` (copy of the target) and
  ``preds/{i}_pred.png`` = createImage with the predicted materials.

Defaults are the reference's compile-time render configuration (scene.h:3-13:
500x500, 100 spp, unbounded paths).
"""
from __future__ import annotations

import argparse
import os
import shutil
from typing import Callable, List, Optional, Sequence

import numpy as np

CORNELL_OBJ = "./CornellBox/CornellBox-Empty-CO.obj"
CORNELL_MTL = "./CornellBox/CornellBox-Empty-CO.mtl"
CUBE_OBJ = "./shapes/cube.obj"


def my_scenes(n: int, world: int, rank: int) -> List[int]:
    """Scenes of `rank`: round-robin, so every rank gets n/world of them."""
    return list(range(rank, n, world))


def cube_kd(seed: int, i: int) -> np.ndarray:
    """rand_mtl (ipt_cuda.py:14-15) for scene i: three uniforms in [0, 1)."""
    return np.random.RandomState((int(seed) * 1000003 + int(i)) & 0xFFFFFFFF).uniform(size=3)


def scene_text(kd: Sequence[float]) -> str:
    """The scene file generate_files writes (ipt_cuda.py:120-127 via to_string)."""
    return ("OBJECT\n"
            "POS 0 0 4\nSCL 2.0 2.0 2.0\nOBJ %s\nMTL %s\n"
            "OBJECT\n"
            "POS 0.0 -1.5 4.0\nOBJ %s\nMTL *Kd %r %r %r*\n"
            % (CORNELL_OBJ, CORNELL_MTL, CUBE_OBJ, float(kd[0]), float(kd[1]), float(kd[2])))


def scene_seed(seed: int, i: int, width: int, height: int, spp: int) -> int:
    """Render seed of scene i: disjoint per-sample RNG streams across scenes."""
    from .distributed import frame_seed

    return frame_seed(seed, i, width, height, spp)


def _paths(root: str, i: int):
    return (os.path.join(root, "scenes", "%d.txt" % i), os.path.join(root, "imgs", "%d.png" % i),
            os.path.join(root, "data", "%d.npz" % i))


ASSETS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "assets")


def _load(root: str, i: int):
    """loadScene of scene i; ./CornellBox and ./shapes resolve against the
    repo's assets (the reference resolves them against its checkout)."""
    from .scene import Scene

    return Scene.from_file(_paths(root, i)[0], root=ASSETS)


def generate_files(root: str, indices: Sequence[int], width=500, height=500, spp=100, max_bounces=None, seed=0,
                   render: bool = True, renderer: Optional[Callable] = None):
    """Write scenes/{i}.txt and render imgs/{i}.png for the given scenes.
    `renderer(scene_file, i) -> uint8 (H, W, 3)` replaces the GPU render (tests)."""
    for sub in ("scenes", "imgs"):
        os.makedirs(os.path.join(root, sub), exist_ok=True)
    for i in indices:
        sfile, ifile, _ = _paths(root, i)
        tmp = sfile + ".tmp"
        with open(tmp, "w") as f:
            f.write(scene_text(cube_kd(seed, i)))
        os.replace(tmp, sfile)
        if not render:
            continue
        if renderer is not None:
            ldr = renderer(sfile, i)
        else:
            sc = _load(root, i)
            _, ldr = sc.render(width, height, spp, max_bounces, scene_seed(seed, i, width, height, spp), ldr=True)
            sc.close()
        from .scene import png_write

        png_write(ifile, ldr)


def generate_data(root: str, indices: Sequence[int], width=500, height=500, spp=100, max_bounces=None, seed=0):
    """generate_data for the given scenes: data/{i}.npz with the createGraph
    split (w (nT+1, nT), pixel / light (nT+1, nT, 3)) and labels (nT, 3)."""
    from .scene import png_read, unpack_graph

    os.makedirs(os.path.join(root, "data"), exist_ok=True)
    for i in indices:
        _, ifile, dfile = _paths(root, i)
        target = png_read(ifile)
        if target.shape[:2] != (height, width):
            raise ValueError("%s is %dx%d, the graph integrator needs %dx%d" % (ifile, target.shape[1],
                                                                                   target.shape[0], width, height))
        sc = _load(root, i)
        _, data = sc.graph(target, width, height, spp, max_bounces,
                           scene_seed(seed, i, width, height, spp) ^ 0x5bd1e995)
        labels = sc.materials.astype(np.float64)
        nT = sc.nT
        sc.close()
        w, pixel, light = unpack_graph(nT, data)
        assert not np.isnan(pixel).any()  # ipt_cuda.py:162
        tmp = dfile + ".tmp.npz"
        np.savez(tmp, w=w, pixel=pixel, light=light, labels=labels)
        os.replace(tmp, dfile)


def load_data(root: str, indices: Sequence[int]):
    out = []
    for i in indices:
        with np.load(_paths(root, i)[2]) as z:  # allow_pickle stays False
            out.append((z["w"], z["pixel"], z["light"], z["labels"]))
    return out


def train_and_predict(root: str, indices: Sequence[int], epochs: int, lr=1e-4, device=None, split: Optional[int] = None,
                      width=500, height=500, spp=100, max_bounces=None, seed=0, log_every=0, render_preds=True):
    """ipt.py:102-138: train on the first `split` graphs, then predict every
    scene's materials and render preds/{i}_pred.png next to preds/{i}_true.png.
    Returns (model, per-scene L1 error of the prediction)."""
    import torch

    from .gcn import build_graph, train
    from .scene import png_write

    data = load_data(root, indices)
    graphs = [build_graph(w, pixel, light) for w, pixel, light, _ in data]
    labels = [torch.tensor(l) for *_, l in data]
    split = len(graphs) if split is None else split
    model = train(graphs[:split], labels[:split], epochs, lr=lr, device=device, log_every=log_every, seed=seed)
    errs = []
    os.makedirs(os.path.join(root, "preds"), exist_ok=True)
    dev = next(model.parameters()).device
    for i, g, y in zip(indices, graphs, labels):
        with torch.no_grad():
            pred = model(g.to(dev)).cpu()
        errs.append(float((pred.double() - y).abs().mean()))
        if not render_preds:
            continue
        shutil.copy(_paths(root, i)[1], os.path.join(root, "preds", "%d_true.png" % i))
        sc = _load(root, i)
        sc.materials = pred.numpy().astype(np.float32)
        _, ldr = sc.render(width, height, spp, max_bounces, scene_seed(seed, i, width, height, spp), ldr=True)
        sc.close()
        png_write(os.path.join(root, "preds", "%d_pred.png" % i), ldr)
    return model, errs


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("stage", choices=["files", "data", "train", "all"])
    ap.add_argument("--root", required=True)
    ap.add_argument("--n", type=int, default=100)
    ap.add_argument("--width", type=int, default=500)
    ap.add_argument("--height", type=int, default=500)
    ap.add_argument("--spp", type=int, default=100)
    ap.add_argument("--max-bounces", type=int, default=-1, help="-1: unbounded, the reference")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--epochs", type=int, default=1000)
    ap.add_argument("--lr", type=float, default=1e-4)
    ap.add_argument("--split", type=int, default=None, help="training scenes (default: all)")
    a = ap.parse_args(argv)
    mb = None if a.max_bounces < 0 else a.max_bounces

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    os.makedirs(a.root, exist_ok=True)
    mine = my_scenes(a.n, world, rank)
    cfg = dict(width=a.width, height=a.height, spp=a.spp, max_bounces=mb, seed=a.seed)
    if a.stage in ("files", "all"):
        generate_files(a.root, mine, **cfg)
    if world > 1:
        dist.barrier()
    if a.stage in ("data", "all"):
        generate_data(a.root, mine, **cfg)
    if world > 1:
        dist.barrier()
    if a.stage in ("train", "all") and rank == 0:
        _, errs = train_and_predict(a.root, list(range(a.n)), a.epochs, lr=a.lr, device="cuda", split=a.split,
                                    log_every=max(1, a.epochs // 10), **cfg)
        print("mean L1 material error per scene: %.4f" % float(np.mean(errs)))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
