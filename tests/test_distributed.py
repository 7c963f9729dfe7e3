"""N>1 path on CPU: two gloo ranks shard rows (shard_rows), render their
bands, all-gather the image and all-reduce the gradient -- exactly the
exchange the GPU path does over RCCL.  The per-rank compute here is the CPU
oracle (no GPU in this container); the GPU ranks call the HIP kernels with
the same row bands (tests/test_gpu.py::test_row_band_sharding_*)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import SCENE0

W, H, SPP, MB, SEED = 16, 13, 2, 3, 99


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out, interleaved=False):
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.dirname(here))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_lib
    from inverse_path_tracer_amd.distributed import allreduce_, gather_rows, shard_rows, shard_rows_interleaved

    oracle_lib.lib().oro_set_threads(1)
    sc = oracle_lib.OracleScene(SCENE0)
    if interleaved:  # rows rank, rank + world, ... (the C ABI's row_step)
        rows = list(range(*shard_rows_interleaved(H, world, rank)))
    else:
        rows = list(range(*shard_rows(H, world, rank)))
    adj = np.random.RandomState(7).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    g = torch.from_numpy(sum(sc.adjoint(W, H, SPP, MB, SEED, adj, row_begin=r, row_end=r + 1) for r in rows))
    allreduce_(g)
    s = np.concatenate([sc.render_samples(W, H, SPP, MB, SEED, r * W * SPP, (r + 1) * W * SPP)[0] for r in rows])
    hdr, _ = oracle_lib.pixel_mean(s, len(rows) * W, SPP)
    img = gather_rows(torch.from_numpy(hdr.reshape(len(rows), W, 3)), H, interleaved=interleaved)
    b, e = shard_rows(H, world, rank)
    # createGraph: per-rank bins of the row band, one all-reduce, compress
    from inverse_path_tracer_amd.distributed import graph_sharded

    class _OracleGraph:  # the Scene.graph calling convention over the oracle
        nT = sc.nT

        def graph(self, target, w, h, spp, mb, seed, rb, re, step=1):
            # the rank's rows rb, rb + step, ... (the oracle traces contiguous bands: one per row)
            acc = sum(sc.graph(w, h, spp, mb, seed, target, r, r + 1)[0] for r in range(rb, re, step))
            return acc, None

    target = np.random.RandomState(3).randint(0, 256, (H, W, 3)).astype(np.uint8)
    data = torch.from_numpy(graph_sharded(_OracleGraph(), target, W, H, SPP, MB, SEED))
    if rank == 0:
        torch.save({"g": g, "img": img, "graph": data}, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,interleaved", [(2, False), (3, False), (3, True)])
def test_row_band_sharding_gloo(oracle, tmp_path, world, interleaved):
    out = str(tmp_path / "r0.pt")
    mp.spawn(_worker, args=(world, _free_port(), out, interleaved), nprocs=world, join=True)
    res = torch.load(out, weights_only=True)
    sc = oracle.OracleScene(SCENE0)
    adj = np.random.RandomState(7).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    g_full = sc.adjoint(W, H, SPP, MB, SEED, adj)
    hdr_full, _, _ = sc.render(W, H, SPP, MB, SEED)
    # forward: bit-identical (samples are seeded by their global index)
    assert np.array_equal(res["img"].numpy().view(np.uint32), hdr_full.view(np.uint32))
    # gradient: equal up to fp64 summation order
    np.testing.assert_allclose(res["g"].numpy(), g_full, rtol=1e-11, atol=1e-14)
    # graph: bins summed across ranks then compressed == the single-rank result
    target = np.random.RandomState(3).randint(0, 256, (H, W, 3)).astype(np.uint8)
    acc_full, data_full = sc.graph(W, H, SPP, MB, SEED, target)
    np.testing.assert_allclose(res["graph"].numpy(), data_full, rtol=1e-6, atol=1e-7)
