"""One rank of the product's N-rank path, started as a fresh child process by
tests/test_gpu_multirank.py (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in
the environment; every rank on device 0, gloo -- the one-GPU rehearsal of the
driver's one-rank-per-GPU RCCL run, same code path above the collective).

    python tests/multirank_worker.py tile OUTDIR
        interleaved row shares of one frame (distributed.shard_rows_interleaved):
        fused forward through torch_ops.render_into -> gather_rows; bounded and
        unbounded adjoints through torch_ops.adjoint_into -> allreduce_; the
        differentiable torch_ops.render with row_step + backward -> allreduce_;
        createGraph through distributed.graph_sharded.  Rank 0 writes tile.pt.
    python tests/multirank_worker.py rccl OUTDIR   (IPT_DIST_BACKEND=nccl, world 1)
        the product's collectives through RCCL on its own device tensors.
    python tests/multirank_worker.py optimize OUTDIR
        C5's scene-parallel split (optimize.shard_scenes): a contiguous block of
        the scenes per rank, MaterialOptimizer(n_total=all scenes) for a few
        Adam steps.  Every rank writes opt_<rank>.pt.
    python tests/multirank_worker.py c5 OUTDIR   (world 8)
        C5 as configured: scenes/0..99.txt over 8 ranks, 256x256, 32 spp, 240
        Adam steps.  Every rank writes c5_<rank>.pt.

Sizes and seeds are shared with the test through CONFIG.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE):
    if p not in sys.path:
        sys.path.insert(0, p)

# tile: a ragged frame (61 rows do not split evenly) of scenes/0.txt; the
# north-star scene (BVH, two-kernel render) on a smaller one
CONFIG = {"W": 64, "H": 61, "spp": 16, "mb": 4, "seed": 4242, "ns_W": 48, "ns_H": 37, "ns_spp": 8,
          "opt_n": 4, "opt_size": 32, "opt_spp": 8, "opt_target_spp": 64, "opt_steps": 3,
          # c5: BASELINE configs[4] as configured -- 100 scenes over 8 ranks
          "c5_n": 100, "c5_world": 8, "c5_size": 256, "c5_spp": 32, "c5_target_spp": 1024, "c5_steps": 240}


def inputs(H, W, device):
    """The adjoint image and the createGraph target of the tile test (deterministic)."""
    import numpy as np
    import torch

    adj = torch.from_numpy(np.random.RandomState(11).uniform(-1, 1, (H, W, 3)).astype(np.float32)).to(device)
    target = np.random.RandomState(12).randint(0, 256, (H, W, 3)).astype(np.uint8)
    return adj, target


def tile(out):
    import torch

    from conftest import NORTHSTAR, SCENE0, product_scene
    from inverse_path_tracer_amd import _native as N
    from inverse_path_tracer_amd import torch_ops
    from inverse_path_tracer_amd.distributed import allreduce_, gather_rows, graph_sharded, shard_rows_interleaved, world

    c = CONFIG
    Wd, R = world()
    dev = torch.device("cuda", 0)
    W, H, spp, mb, seed = c["W"], c["H"], c["spp"], c["mb"], c["seed"]
    b, e, st = shard_rows_interleaved(H, Wd, R)
    sc = product_scene(SCENE0)
    res = {"rows": (b, e, st)}
    adj, target = inputs(H, W, dev)
    # forward: the rank's rows, gathered into the full image
    p = N.make_params(W, H, spp, mb, seed, b, e, st)
    hdr = torch.empty((p.rows, W, 3), device=dev, dtype=torch.float32)
    torch_ops.render_into(sc, p, None, hdr)
    torch.cuda.synchronize()
    res["img"] = gather_rows(hdr.cpu(), H, interleaved=True)
    # adjoints (bounded: LDS records; unbounded: the reference's estimator, global ring): one all-reduce each
    for key, bounces in (("g_bounded", mb), ("g_unbounded", None)):
        q = N.make_params(W, H, spp, bounces, seed, b, e, st)
        g = torch.zeros((sc.nT, 3), device=dev, dtype=torch.float64)
        torch_ops.adjoint_into(sc, q, None, adj.data_ptr(), g)
        torch.cuda.synchronize()
        res[key] = allreduce_(g.cpu())
    # the differentiable op with row_step: forward of the share, backward through the adjoint kernel
    kd = torch.tensor(sc.materials, device=dev, requires_grad=True)
    img = torch_ops.render(sc, kd, W, H, spp, mb, seed, row_begin=b, row_end=e, row_step=st)
    (img * adj[b:e:st]).sum().backward()
    torch.cuda.synchronize()
    res["g_autograd"] = allreduce_(kd.grad.detach().double().cpu())
    # createGraph: interleaved rows, one all-reduce of the fp64 bins, compress on every rank
    res["graph"] = torch.from_numpy(graph_sharded(sc, target, W, H, spp, None, seed))
    sc.close()
    # the BVH scene (cooperative traversal, two-kernel render): forward and adjoint shares
    ns = product_scene(NORTHSTAR)
    nW, nH, nspp = c["ns_W"], c["ns_H"], c["ns_spp"]
    b2, e2, s2 = shard_rows_interleaved(nH, Wd, R)
    p2 = N.make_params(nW, nH, nspp, mb, seed, b2, e2, s2)
    h2 = torch.empty((p2.rows, nW, 3), device=dev, dtype=torch.float32)
    torch_ops.render_into(ns, p2, None, h2)
    adj2 = adj[:nH, :nW].contiguous()
    g2 = torch.zeros((ns.nT, 3), device=dev, dtype=torch.float64)
    torch_ops.adjoint_into(ns, p2, None, adj2.data_ptr(), g2)
    torch.cuda.synchronize()
    res["ns_img"] = gather_rows(h2.cpu(), nH, interleaved=True)
    res["ns_g"] = allreduce_(g2.cpu())
    ns.close()
    if R == 0:
        torch.save(res, os.path.join(out, "tile.pt"))


def optimize(out):
    import torch

    from inverse_path_tracer_amd.distributed import world
    from inverse_path_tracer_amd.optimize import MaterialOptimizer, _scene_files, build_tasks, shard_scenes

    c = CONFIG
    Wd, R = world()
    dev = torch.device("cuda", 0)
    b, e = shard_scenes(c["opt_n"], Wd, R)
    files = _scene_files(os.path.join(ROOT, "assets", "scenes"), c["opt_n"])[b:e]
    s = c["opt_size"]
    tasks = build_tasks(files, s, s, c["opt_target_spp"], c["mb"], 0.5, dev, first_index=b)
    m = MaterialOptimizer(tasks, s, s, c["opt_spp"], c["mb"], lr=1e-2, n_total=c["opt_n"])
    m.run(c["opt_steps"])
    torch.cuda.synchronize()
    torch.save({t.index: {"kd": t.kd.detach().cpu(), "target": t.target.cpu(), "history": list(t.history)}
                for t in tasks}, os.path.join(out, "opt_%d.pt" % R))


def c5(out):
    """BASELINE configs[4] as configured, one rank of 8: this rank's contiguous
    block of scenes/0..99.txt (12-13 scenes), 256x256, 32 spp, 4 bounces,
    Adam lr 1e-2, C5_STEPS steps, n_total = 100 (the sample streams of the
    one-rank run).  Records per scene the parameters, target, loss history and
    the observable cube-Kd error before / after, plus this rank's wall times."""
    import time

    import torch

    from inverse_path_tracer_amd.distributed import world
    from inverse_path_tracer_amd.optimize import MaterialOptimizer, _scene_files, build_tasks, observable_mask, shard_scenes

    c = CONFIG
    Wd, R = world()
    dev = torch.device("cuda", 0)
    n, s = c["c5_n"], c["c5_size"]
    b, e = shard_scenes(n, Wd, R)
    files = _scene_files(os.path.join(ROOT, "assets", "scenes"), n)[b:e]
    t0 = time.time()
    tasks = build_tasks(files, s, s, c["c5_target_spp"], c["mb"], 0.5, dev, first_index=b)
    masks = observable_mask(tasks, s, s, 64, c["mb"])
    err = [lambda t=t, m=m: float((t.kd.detach() - t.truth)[18:][m].abs().mean()) for t, m in zip(tasks, masks)]
    e0 = [f() for f in err]
    torch.cuda.synchronize()
    t1 = time.time()
    m = MaterialOptimizer(tasks, s, s, c["c5_spp"], c["mb"], lr=1e-2, n_total=n)
    m.run(c["c5_steps"])
    torch.cuda.synchronize()
    t2 = time.time()
    e1 = [f() for f in err]
    torch.save({"rank": R, "scenes": [b, e], "setup_s": t1 - t0, "optimise_s": t2 - t1,
                "tasks": {t.index: {"kd": t.kd.detach().cpu(), "target": t.target.cpu(), "history": list(t.history),
                                    "err0": a, "err1": z, "observable": int(mk.sum())}
                          for t, mk, a, z in zip(tasks, masks, e0, e1)}},
               os.path.join(out, "c5_%d.pt" % R))


def rccl(out):
    """One rank on RCCL (backend "nccl" on ROCm; a GPU takes one RCCL rank, so
    the one-GPU box runs world 1): the collectives the product issues at N
    ranks -- the fp64 gradient's all-reduce (torch_ops.adjoint_into's output),
    the fp64 createGraph bins' all-reduce, an all-gather of an image band --
    executed through RCCL on the product's own device tensors.  At world 1
    they must return their inputs unchanged."""
    import torch
    import torch.distributed as dist

    from conftest import SCENE0, product_scene
    from inverse_path_tracer_amd import _native as N
    from inverse_path_tracer_amd import torch_ops

    c = CONFIG
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    dev = torch.device("cuda", 0)
    W, H, spp, mb, seed = c["W"], c["H"], c["spp"], c["mb"], c["seed"]
    sc = product_scene(SCENE0)
    adj, target = inputs(H, W, dev)
    g = torch.zeros((sc.nT, 3), device=dev, dtype=torch.float64)
    torch_ops.adjoint_into(sc, N.make_params(W, H, spp, mb, seed), None, adj.data_ptr(), g)
    g0 = g.clone()
    dist.all_reduce(g, op=dist.ReduceOp.SUM)
    bins, _ = sc.graph(target, W, H, spp, None, seed)
    b = torch.from_numpy(bins).to(dev)
    b0 = b.clone()
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    hdr = torch.empty((H, W, 3), device=dev, dtype=torch.float32)
    torch_ops.render_into(sc, N.make_params(W, H, spp, mb, seed), None, hdr)
    outs = [torch.empty_like(hdr)]
    dist.all_gather(outs, hdr)
    torch.cuda.synchronize()
    res = {"grad_equal": bool(torch.equal(g, g0)), "bins_equal": bool(torch.equal(b, b0)),
           "gather_equal": bool(torch.equal(outs[0].view(torch.int32), hdr.view(torch.int32))),
           "grad_nonzero": bool(g0.abs().max().item() > 0)}
    torch.save(res, os.path.join(out, "rccl.pt"))
    sc.close()


def main():
    import torch
    import torch.distributed as dist

    mode, out = sys.argv[1], sys.argv[2]
    torch.cuda.set_device(0)
    backend = os.environ.get("IPT_DIST_BACKEND", "gloo")
    if backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    else:
        dist.init_process_group(backend)
    try:
        {"tile": tile, "optimize": optimize, "rccl": rccl, "c5": c5}[mode](out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
