"""Benchmark: Msamples/s (forward) + grad-Msamples/s (adjoint), 512x512 Cornell
box, 64 spp, 4 bounces (BASELINE.json configs[1]) on N MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step is one frame of the configuration: every sample of every pixel traced
(per-sample radiance kernel + per-pixel mean kernel).  Weak scaling: each rank
renders its own frame (disjoint sample-index ranges via frame_seed), so the
forward has no collective; the adjoint step adds the one exchange the path has,
an RCCL all-reduce of the per-material gradient vector.  Inputs are resident
in HBM before the timed region; timing is HIP events on the launch stream,
bracketed by barrier + synchronize, max over ranks.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from inverse_path_tracer_amd import _native as N  # noqa: E402
from inverse_path_tracer_amd.distributed import frame_seed  # noqa: E402
from inverse_path_tracer_amd.scene import ObjectSpec, Scene  # noqa: E402

W = H = 512
SPP = 64
BOUNCES = 4
ASSETS = os.path.join(ROOT, "assets")
CORNELL = [ObjectSpec(os.path.join(ASSETS, "CornellBox", "CornellBox-Empty-CO.obj"),
                      os.path.join(ASSETS, "CornellBox", "CornellBox-Empty-CO.mtl"), (0, 0, 4), (0, 0, 0), (2, 2, 2))]
# C3 (BASELINE.json configs[2]): scenes/0.txt = Cornell + the cube with its inline Kd
SCENE0 = CORNELL + [ObjectSpec(os.path.join(ASSETS, "shapes", "cube.obj"),
                               "*Kd 0.9041462985304743 0.5854651848798454 0.007022117649276849*", (0, -1.5, 4),
                               (0, 0, 0), (1, 1, 1))]
# the north_star's "+ sphere.obj" scene (not a shipped scene file): 1298 triangles, BVH
SPHERE = CORNELL + [ObjectSpec(os.path.join(ASSETS, "shapes", "sphere.obj"), "*Kd 0.2 0.6 0.3*", (0.3, -1.2, 4.2),
                               (0.0, 0.4, 0.0), (1.2, 1.2, 1.2))]
# casts/sample counted by the CPU oracle over the full C2
# frame (tools/count_casts.py -> profiles/casts_per_sample.json)
CASTS_PER_SAMPLE = 5.694442272186279
N_TRIANGLES = 18
FLOP_PER_TEST = 38          # F1 test with hoisted edge planes
PEAK_FP32_TFLOPS = 157.3    # MI355X FP32 vector (= FP32 MFMA) peak, MI355X_MICROARCH.md
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_fwd_trace_kernel.json")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the C3/C4/BVH-scene lines (profiling runs: keeps the C2 kernel's statistics pure)")
    return ap.parse_args()


def cpu_baseline(fwd_seconds=8.0, one_core_seconds=3.0, adj_seconds=4.0):
    """The CPU oracle (test infrastructure, oracle/ipt_oracle.c -O2 OpenMP) on
    bounded samples of the same C2 workload: whole frames (consecutive frame
    seeds) on this rank's allowed cores (capped at 16) until fwd_seconds, the
    first rows on ONE core, and the adjoint on the first rows."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    cores = min(16, len(os.sched_getaffinity(0)))
    L = oracle_lib.lib()
    recs = [(o.pos, o.ori, o.scl, o.obj_file, o.mtl_file) for o in CORNELL]
    sc = oracle_lib.OracleScene(recs)

    def rows_for(seconds, fn):
        rows, done, secs = 4, 0, 0.0
        while secs < seconds and done < H:
            r = min(rows, H - done)
            t0 = time.perf_counter()
            fn(done, done + r)
            secs += time.perf_counter() - t0
            done += r
            rows *= 2
        return done, secs

    L.oro_set_threads(cores)
    frames, secs = 0, 0.0
    while secs < fwd_seconds and frames < 16:
        t0 = time.perf_counter()
        sc.render_samples(W, H, SPP, BOUNCES, frame_seed(0, frames, W, H, SPP))
        secs += time.perf_counter() - t0
        frames += 1
    fwd = frames * W * H * SPP / secs / 1e6
    adj = np.ones((H, W, 3), np.float32)
    arows, asecs = rows_for(adj_seconds, lambda b, e: sc.adjoint(W, H, SPP, BOUNCES, 0, adj, b, e))
    L.oro_set_threads(1)
    orows, osecs = rows_for(one_core_seconds,
                            lambda b, e: sc.render_samples(W, H, SPP, BOUNCES, 0, b * W * SPP, e * W * SPP))
    L.oro_set_threads(cores)
    return {"value": round(fwd, 3), "unit": "Msamples/s", "cores": cores, "kind": "port",
            "sample": "CPU oracle (oracle/ipt_oracle.c, -O2 OpenMP) on %d whole C2 frame(s) (%d samples, %.1f s); "
                      "adjoint on rows [0,%d) (%.1f s); 1 core on rows [0,%d) (%.1f s)" % (
                          frames, frames * W * H * SPP, secs, arows, asecs, orows, osecs),
            "grad_value": round(arows * W * SPP / asecs / 1e6, 3),
            "value_1core": round(orows * W * SPP / osecs / 1e6, 3)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
    scene = Scene(CORNELL)
    stream = torch.cuda.current_stream(dev)
    st = stream.cuda_stream
    L = N.lib()
    npix = W * H
    samples = torch.empty((npix * SPP, 3), device=dev, dtype=torch.float32)
    hdr = torch.empty((H, W, 3), device=dev, dtype=torch.float32)
    adj = torch.full((H, W, 3), 1.0 / (3 * npix), device=dev, dtype=torch.float32)
    grad = torch.zeros((scene.nT, 3), device=dev, dtype=torch.float64)

    def params(step):
        return N.make_params(W, H, SPP, BOUNCES, frame_seed(args.seed, rank * 100003 + step, W, H, SPP))

    def fwd(step, ev=None):
        p = params(step)
        if ev is not None:
            ev[0].record(stream)
        N.check(L.ipt_render_samples_sm_dev(scene.handle, C.byref(p), None, samples.data_ptr(), st))
        if ev is not None:
            ev[1].record(stream)
        N.check(L.ipt_pixel_mean_sm_dev(samples.data_ptr(), npix, SPP, hdr.data_ptr(), None, st))

    def bwd(step):
        p = params(step)
        grad.zero_()
        N.check(L.ipt_adjoint_dev(scene.handle, C.byref(p), None, adj.data_ptr(), grad.data_ptr(), st))
        if world > 1:
            dist.all_reduce(grad)  # the per-material gradient vector, nT*3 fp64

    def barrier():
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    for i in range(args.warmup):
        fwd(10**6 + i)
        bwd(10**6 + i)
    # ---------------------------------------------------------------- forward
    kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier()
    t_wall = time.perf_counter()
    e0.record(stream)
    for i in range(args.steps):
        fwd(i, kev[i])
    e1.record(stream)
    barrier()
    wall_fwd = time.perf_counter() - t_wall
    fwd_ms = max_over_ranks(e0.elapsed_time(e1))
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in kev]))
    # ---------------------------------------------------------------- adjoint
    barrier()
    e0.record(stream)
    for i in range(args.steps):
        bwd(i)
    e1.record(stream)
    barrier()
    bwd_ms = max_over_ranks(e0.elapsed_time(e1))
    # ------------------------------------------- secondary workloads (info)
    extra = {}
    for key, objs, kind in (() if args.no_secondary else (("c3_grad", SCENE0, "adj"), ("bvh_fwd", SPHERE, "fwd"))):
        sc = Scene(objs)
        g2 = torch.zeros((sc.nT, 3), device=dev, dtype=torch.float64)

        def run(step):
            p = params(step)
            if kind == "adj":
                g2.zero_()
                N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p), None, adj.data_ptr(), g2.data_ptr(), st))
                if world > 1:
                    dist.all_reduce(g2)
            else:
                N.check(L.ipt_render_samples_sm_dev(sc.handle, C.byref(p), None, samples.data_ptr(), st))

        k = max(1, min(args.steps, 5))
        run(10**6)
        barrier()
        e0.record(stream)
        for i in range(k):
            run(i)
        e1.record(stream)
        barrier()
        ms = max_over_ranks(e0.elapsed_time(e1)) / k
        extra[key] = {"value": round(world * W * H * SPP / ms / 1e3, 2),
                      "unit": "grad-Msamples/s" if kind == "adj" else "Msamples/s", "ms_per_step": round(ms, 4),
                      "triangles": sc.nT, "accel": sc.bvh_info()["accel"],
                      "workload": ("C3: scenes/0.txt (Cornell + cube), 512x512, 64 spp, 4 bounces, adjoint dL/dKd "
                                   "+ all-reduce" if kind == "adj" else
                                   "Cornell + sphere.obj (north_star scene), 512x512, 64 spp, 4 bounces, forward")}
        sc.close()
    # C4 (BASELINE.json configs[3]): scenes/0.txt, 1024x1024, 256 spp, 8 bounces,
    # rank k traces row band k of 8 (the 8-GPU sharding); forward + adjoint
    # with the one gradient all-reduce.  At N < 8 only bands 0..N-1 run.
    if world <= 8 and not args.no_secondary:
        from inverse_path_tracer_amd.distributed import shard_rows
        W4, S4, B4 = 1024, 256, 8
        b4, e4 = shard_rows(W4, 8, rank)
        sc = Scene(SCENE0)
        g4 = torch.zeros((sc.nT, 3), device=dev, dtype=torch.float64)
        adj4 = torch.full((W4, W4, 3), 1.0 / (3 * W4 * W4), device=dev, dtype=torch.float32)
        smp4 = torch.empty(((e4 - b4) * W4 * S4, 3), device=dev, dtype=torch.float32)
        p4 = N.make_params(W4, W4, S4, B4, args.seed, b4, e4)
        res4 = {}
        for kind in ("fwd", "adj"):
            def run4():
                if kind == "fwd":
                    N.check(L.ipt_render_samples_sm_dev(sc.handle, C.byref(p4), None, smp4.data_ptr(), st))
                else:
                    g4.zero_()
                    N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p4), None, adj4.data_ptr(), g4.data_ptr(), st))
                    if world > 1:
                        dist.all_reduce(g4)
            run4()
            barrier()
            e0.record(stream)
            for _ in range(2):
                run4()
            e1.record(stream)
            barrier()
            res4[kind] = max_over_ranks(e0.elapsed_time(e1)) / 2
        n4 = world * (e4 - b4) * W4 * S4
        extra["c4"] = {"value": round(n4 / res4["fwd"] / 1e3, 2), "unit": "Msamples/s",
                       "grad_value": round(n4 / res4["adj"] / 1e3, 2), "grad_unit": "grad-Msamples/s",
                       "fwd_ms": round(res4["fwd"], 3), "adj_ms": round(res4["adj"], 3), "bands": "%d of 8" % world,
                       "workload": "C4: scenes/0.txt, 1024x1024, 256 spp, 8 bounces; rank k = row band k of 8 "
                                   "(forward, adjoint + all-reduce)"}
        sc.close()
        del smp4

    samples_per_frame = W * H * SPP
    value = world * args.steps * samples_per_frame / (fwd_ms / 1e3) / 1e6
    grad_value = world * args.steps * samples_per_frame / (bwd_ms / 1e3) / 1e6
    # roofline of the dominant kernel (trace_kernel<FWD>), SURVEY.md §8(d)
    flop_per_launch = samples_per_frame * CASTS_PER_SAMPLE * N_TRIANGLES * FLOP_PER_TEST
    achieved = flop_per_launch / (kernel_ms / 1e3) / 1e12
    traffic = None
    if os.path.exists(PMC_FILE):
        with open(PMC_FILE) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
    # SURVEY.md §8(d) "HBM fraction": PMC-measured bytes of the same kernel
    # (profiles/, FETCH x2 + WRITE) over this run's kernel time, vs 8 TB/s
    hbm = None
    if traffic:
        gbs = traffic / (kernel_ms / 1e3) / 1e9
        hbm = {"bytes_per_launch": traffic, "achieved_GBps": round(gbs, 1), "peak_GBps": 8000.0,
               "frac": round(gbs / 8000.0, 4), "algorithmic_bytes_per_launch": samples_per_frame * 12,
               "source": os.path.relpath(PMC_FILE, ROOT)}
    roofline = {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": traffic,
                "kernel": "trace_kernel<MODE_FWD>", "kernel_ms": round(kernel_ms, 4),
                "flop_per_launch": flop_per_launch,
                "formula": "samples*C_bar(%.4f)*nT(%d)*38 FLOP / kernel time; peak = FP32 vector peak (equal to "
                           "the FP32 MFMA peak on gfx950)" % (CASTS_PER_SAMPLE, N_TRIANGLES)}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()
    if rank == 0:
        out = {
            "metric": "Msamples/sec fwd + grad-Msamples/sec, 512² Cornell 64spp, 1/2/4/8 GPU",
            "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(fwd_ms / args.steps, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "C2: CornellBox-Empty-CO.obj, 512x512, 64 spp, max_bounces=4, one frame per "
                                   "rank per step (fwd); adjoint dL/dKd per frame + RCCL all-reduce (grad)",
                       "width": W, "height": H, "spp": SPP, "max_bounces": BOUNCES, "triangles": scene.nT,
                       "parallelism": "frame-parallel x%d" % world},
            "grad_value": round(grad_value, 2), "grad_unit": "grad-Msamples/s",
            "grad_ms_per_step": round(bwd_ms / args.steps, 4),
            "wall_s_fwd_region": round(wall_fwd, 4),
            "roofline": roofline, "hbm": hbm, "cpu_baseline": cpu, "secondary": extra,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
