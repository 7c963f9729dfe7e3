"""Benchmark: Msamples/s (forward) + grad-Msamples/s (adjoint), 512x512 Cornell
box, 64 spp, 4 bounces (BASELINE.json configs[1]) on N MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

A step is one C2 frame, tiled across the ranks exactly as the north_star asks
("image tiles shard across the GPUs, RCCL reduce on the per-material gradient
vector only"): rank r traces rows r, r + N, ... of the SAME frame
(shard_rows_interleaved -- contiguous bands differ in cost by up to 7.6%,
see `bands_*`; sample seeds are global indices, so the shares are the
single-GPU frame's samples);
the forward needs no collective, the adjoint step ends with ONE all-reduce of
the nT*3 fp64 gradient.  Consecutive steps go round-robin over NSTREAMS = 3
HIP streams (three frames in flight, each with its own image / gradient
buffer), so one frame's tail overlaps the next frames' starts; `secondary.serial` is the same
run on one stream.  Strong scaling: value = frame samples * K / (max
over ranks of the time of K steps).  Inputs are resident in HBM before the
timed region; timing is HIP events on the launch stream, bracketed by barrier
+ synchronize.

Secondary lines (JSON `secondary`): weak scaling (a whole frame per rank),
a sustained >= 0.5 s run of each leg, the per-band cost table of C2 and C4 (N =
1: predicts the 8-GPU critical path), C3, the north_star sphere scene, C4's
band and C5 (scene batch + Adam).
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
from inverse_path_tracer_amd.distributed import frame_seed, shard_rows, shard_rows_interleaved  # noqa: E402
from inverse_path_tracer_amd.scene import ObjectSpec, Scene  # noqa: E402

W = H = 512
SPP = 64
BOUNCES = 4
# frames in flight of the headline: consecutive steps are dealt round-robin
# over this many HIP streams (tools/streams_ab.py, profiles/r05/streams_ab_r05q.log:
# C2 forward per frame 1.568 / 1.513 / 1.507 / 1.522 ms and adjoint 1.853 /
# 1.780 / 1.758 / 1.782 ms on 1 / 2 / 3 / 4 streams -- the fourth shares a
# hardware queue with torch's own)
NSTREAMS = 3
ASSETS = os.path.join(ROOT, "assets")
CORNELL = [ObjectSpec(os.path.join(ASSETS, "CornellBox", "CornellBox-Empty-CO.obj"),
                      os.path.join(ASSETS, "CornellBox", "CornellBox-Empty-CO.mtl"), (0, 0, 4), (0, 0, 0), (2, 2, 2))]
# C3 (BASELINE.json configs[2]): scenes/0.txt = Cornell + the cube with its inline Kd
CUBE = ObjectSpec(os.path.join(ASSETS, "shapes", "cube.obj"),
                  "*Kd 0.9041462985304743 0.5854651848798454 0.007022117649276849*", (0, -1.5, 4), (0, 0, 0),
                  (1, 1, 1))
SCENE0 = CORNELL + [CUBE]
# scenes/0.txt with the cube given a Phong lobe (Ks 0.5, shininess 20; assets/phong/scene0_phong.txt):
# the reference's BSDF supports Ks != 0 (path_trace.cu:10-28, 91-109); the SPEC kernel instances run it
SCENE0_PHONG = CORNELL + [ObjectSpec(os.path.join(ASSETS, "phong", "cube_phong.obj"),
                                     os.path.join(ASSETS, "phong", "cube_phong.mtl"), (0, -1.5, 4), (0, 0, 0), (1, 1, 1))]
# BASELINE configs[2] as the north_star names it: scenes/0.txt + sphere.obj (assets/northstar.txt), 1310 triangles
NORTHSTAR = SCENE0 + [ObjectSpec(os.path.join(ASSETS, "shapes", "sphere.obj"), "*Kd 0.2 0.6 0.3*", (-1.2, -1.35, 4.6),
                                 (0.0, 0.0, 0.0), (1.2, 1.2, 1.2))]
# the round-1 "+ sphere.obj" scene (Cornell + sphere, no cube): 1298 triangles, BVH
SPHERE = CORNELL + [ObjectSpec(os.path.join(ASSETS, "shapes", "sphere.obj"), "*Kd 0.2 0.6 0.3*", (0.3, -1.2, 4.2),
                               (0.0, 0.4, 0.0), (1.2, 1.2, 1.2))]
# casts/sample counted by the CPU oracle over the full C2
# frame (tools/count_casts.py -> profiles/casts_per_sample.json; re-derived
# by tests/test_gpu_full.py::test_c2_forward_full_frame_bit_exact)
CASTS_PER_SAMPLE = 5.694429993629456
N_TRIANGLES = 18
FLOP_PER_TEST = 38          # F1 test with hoisted edge planes
PEAK_FP32_TFLOPS = 157.3    # MI355X FP32 vector (= FP32 MFMA) peak, MI355X_MICROARCH.md
PMC_FILE = os.path.join(ROOT, "profiles", "pmc_fwd_trace_kernel.json")
# algorithmic FLOP per sample of the other lines: brute force
# = C_bar * nT * 38 (C3's C_bar from tools/count_casts.py); BVH scenes = the
# tests actually executed, counted by the IPT_BVH_STATS build
# (tools/bvh_stats.py -> profiles/bvh_stats.json: 38 per triangle test + 12
# per slab test)
CASTS_PER_SAMPLE_C3 = 5.61258190870285
CASTS_PER_SAMPLE_PHONG = 5.586285471916199  # C3 with the Phong cube (tools/count_casts.py C3_phong_512x512x64_b4)
# createGraph's integrator at the reference's configuration (scenes/0.txt,
# 500x500, 100 spp, no bounce cap): tools/count_casts.py with the oracle
CASTS_PER_SAMPLE_GRAPH = 7.1221032
GRAPH_TARGET = os.path.join(ROOT, "tests", "golden", "preds_0_true.png")  # the reference's preds/0_true.png
BVH_STATS_FILE = os.path.join(ROOT, "profiles", "bvh_stats.json")


def executed_flop_per_sample(name, c_bar, n_tri):
    """Small scenes: the tests the culled casts actually execute
    (profiles/bvh_stats.json, IPT_BVH_STATS build): the path casts' pair
    tests of the pairs each lane's ray enters, the shadow casts' target tests
    and the pair tests some lane needed, x 38, plus 12 per slab (box) test.
    None without the stats file."""
    if not os.path.exists(BVH_STATS_FILE):
        return None
    with open(BVH_STATS_FILE) as f:
        st = json.load(f)
    d = st.get(name + "_fwd", {}).get("derived")
    if not d or "cull_shadow_casts_per_sample" not in d:
        return None
    if d.get("pcull_casts_per_sample"):  # culled path casts: the pair tests and box tests they issue
        path_flop = 38 * d["pcull_tri_tests_per_sample"] + 12 * d["pcull_box_tests_per_sample"]
    else:
        path_flop = 38 * (c_bar - d["cull_shadow_casts_per_sample"]) * n_tri
    return path_flop + 38 * d["cull_tri_tests_per_sample"] + 12 * d["cull_box_tests_per_sample"]


def flop_per_sample(key):
    if key == "c3":
        return CASTS_PER_SAMPLE_C3 * 30 * FLOP_PER_TEST, "C_bar(C3) * 30 * 38"
    if key == "c3_phong":
        return CASTS_PER_SAMPLE_PHONG * 30 * FLOP_PER_TEST, "C_bar(C3 Phong cube) * 30 * 38"
    name = {"c3_northstar": "northstar", "bvh_sphere": "sphere"}.get(key)
    if name and os.path.exists(BVH_STATS_FILE):
        with open(BVH_STATS_FILE) as f:
            st = json.load(f)
        if name + "_fwd" in st:
            return st[name + "_fwd"]["derived"]["flop_per_sample"], "executed BVH tests (profiles/bvh_stats.json)"
    return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true",
                    help="skip the secondary lines (profiling runs: keeps the C2 kernel's statistics pure)")
    return ap.parse_args()


# ----------------------------------------------------------------- CPU baseline
def cpu_baseline(seconds_per_leg=1.5):
    """The CPU oracle (test infrastructure, oracle/ipt_oracle.c) on bounded
    samples of C1, C2 and the C3 adjoint: rows of the frame until each leg has
    run `seconds_per_leg`, with the parity build (-O2 -ffp-contract=off) and
    the fast build (-O3 x86-64-v3, FMA contraction), on this rank's share of
    the host cores and on one core."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS") or affinity)
    cores = max(1, min(share, affinity))
    recs = {"cornell": [(o.pos, o.ori, o.scl, o.obj_file, o.mtl_file) for o in CORNELL],
            "scene0": [(o.pos, o.ori, o.scl, o.obj_file, o.mtl_file) for o in SCENE0]}
    legs = {"c1_fwd": ("cornell", 128, 128, 8, 2, "fwd"), "c2_fwd": ("cornell", W, H, SPP, BOUNCES, "fwd"),
            "c3_adj": ("scene0", W, H, SPP, BOUNCES, "adj"), "graph": ("scene0", 500, 500, 100, None, "graph")}
    from inverse_path_tracer_amd import png_read
    target = png_read(GRAPH_TARGET)
    out = {}
    # every CPU in the affinity mask ("all host cores"), for
    # the fast build's C2 forward and C3 adjoint -- the job's own share
    # (OMP_NUM_THREADS, 16 on the GPU box) is the primary figure
    allc = max(cores, affinity)
    for fast in (False, True):
        scenes = {k: oracle_lib.OracleScene(v, fast=fast) for k, v in recs.items()}
        L = oracle_lib.lib(fast)
        for threads in ((cores, 1, allc) if fast and allc > cores else (cores, 1)):
            L.oro_set_threads(threads)
            for leg, (sc_name, w, h, spp, mb, kind) in legs.items():
                if threads == allc and threads != cores and leg not in ("c2_fwd", "c3_adj"):
                    continue
                sc = scenes[sc_name]
                adj = np.ones((h, w, 3), np.float32)
                rows, row, total, secs = 2, 0, 0, 0.0
                while secs < seconds_per_leg and total < 64 * h:  # rows in frame order, wrapping (C1 is small)
                    r = min(rows, h - row)
                    t0 = time.perf_counter()
                    if kind == "fwd":
                        sc.render_samples(w, h, spp, mb, 0, row * w * spp, (row + r) * w * spp)
                    elif kind == "graph":
                        sc.graph(w, h, spp, mb, 0, target, row, row + r)
                    else:
                        sc.adjoint(w, h, spp, mb, 0, adj, row, row + r)
                    secs += time.perf_counter() - t0
                    total += r
                    row = (row + r) % h
                    rows *= 2
                key = "%s_%s_%s" % (leg, "fast" if fast else "parity",
                                    "1core" if threads == 1 else ("all" if threads == cores else "allcores"))
                out[key] = {"Msamples_s": round(total * w * spp / secs / 1e6, 3), "rows": total, "s": round(secs, 2),
                            "threads": threads}
        L.oro_set_threads(cores)
    c2 = out["c2_fwd_fast_all"]
    quota = None  # the job's cgroup CPU quota (cpu.max "max_us period_us"), in CPUs
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    ac = {}
    if "c2_fwd_fast_allcores" in out:
        ac = {"value_allcores": out["c2_fwd_fast_allcores"]["Msamples_s"],
              "grad_value_allcores": out["c3_adj_fast_allcores"]["Msamples_s"], "cores_allcores": allc}
    else:  # the job's share is already every CPU it may use
        ac = {"value_allcores": c2["Msamples_s"], "grad_value_allcores": out["c3_adj_fast_all"]["Msamples_s"],
              "cores_allcores": cores}
    return {"value": c2["Msamples_s"], "unit": "Msamples/s", "cores": cores, "kind": "port", **ac,
            "sample": "CPU oracle (oracle/ipt_oracle.c) fast build (-O3 x86-64-v3 -fopenmp) on %d rows of the "
                      "C2 frame (%.1f s); legs: C1/C2 forward and C3 adjoint, parity and fast builds, %d cores and "
                      "1 core, >= %.1f s each (table in `legs`)" % (c2["rows"], c2["s"], cores, seconds_per_leg),
            "grad_value": out["c3_adj_fast_all"]["Msamples_s"], "value_1core": out["c2_fwd_fast_1core"]["Msamples_s"],
            "graph_value": out["graph_fast_all"]["Msamples_s"],
            "cores_note": "%d = this job's CPU share (OMP_NUM_THREADS on the GPU box; %d CPUs in the affinity mask, "
                          "%d in the machine); value_allcores / grad_value_allcores: the same fast-build C2 forward "
                          "and C3 adjoint legs on all %d CPUs of the affinity mask (cgroup CPU quota: %s CPUs -- "
                          "threads beyond it time-share the quota)"
                          % (cores, affinity, os.cpu_count() or 0, allc, "none" if quota is None else quota),
            "cgroup_cpu_quota": quota,
            "legs": out}


# ----------------------------------------------------------------- GPU timing helpers
class Ctx:
    def __init__(self, dev, world, rank):
        self.dev, self.world, self.rank = dev, world, rank
        self.stream = torch.cuda.current_stream(dev)
        self.st = self.stream.cuda_stream
        self.L = N.lib()

    def barrier(self):
        torch.cuda.synchronize(self.dev)
        if self.world > 1:
            dist.barrier()
        torch.cuda.synchronize(self.dev)

    def max_over_ranks(self, x):
        if self.world == 1:
            return x
        t = torch.tensor([x], device=self.dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def timed(self, fn, k, streams=()):
        """ms for k calls of fn(i) (barrier-bracketed, max over ranks).  With
        `streams`, fn(i) launches on streams[i % len(streams)]: they start after
        the region's start event and the region ends when all have drained."""
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        self.barrier()
        e0.record(self.stream)
        for s in streams:
            s.wait_event(e0)
        for i in range(k):
            fn(i)
        for s in streams:
            self.stream.wait_stream(s)
        e1.record(self.stream)
        self.barrier()
        return self.max_over_ranks(e0.elapsed_time(e1))

    def sustained(self, fn, seconds=0.5):
        """Back-to-back calls until >= `seconds` of GPU time: (calls, ms)."""
        k, ms = 4, 0.0
        while True:
            ms = self.timed(fn, k)
            if ms >= seconds * 1e3 or k >= 1 << 16:
                return k, ms
            k = max(k * 2, int(k * seconds * 1e3 / max(ms, 1e-3) * 1.1) + 1)


class Leg:
    """One workload on one scene: forward (HDR image, pixel mean fused into
    the trace kernel) and adjoint (+ gradient all-reduce) over rows [b, e)."""

    def __init__(self, cx, objs, w, h, spp, mb, b=0, e=None, seed=0, step=1, streams=None):
        self.cx, self.w, self.h, self.spp, self.mb, self.seed = cx, w, h, spp, mb, seed
        self.b, self.e, self.step = b, (h if e is None else e), step
        self.rows = len(range(self.b, self.e, self.step))
        self.sc = Scene(objs)
        dev = cx.dev
        npix = self.rows * w
        self.npix = npix
        self.hdr = torch.empty((npix, 3), device=dev, dtype=torch.float32)
        self.adj = torch.full((h, w, 3), 1.0 / (3 * w * h), device=dev, dtype=torch.float32)
        self.grad = torch.zeros((self.sc.nT, 3), device=dev, dtype=torch.float64)
        # frames in flight (piped=True): consecutive steps go round-robin over
        # NSTREAMS streams, each with its own output image and gradient, so one
        # frame's tail overlaps the next frames' starts (the chunk counters are per stream)
        # (the headline's Leg is the process's first: HIP maps streams onto a
        # few hardware queues in creation order, and two streams sharing one
        # run in order; measured per-share overlap: tools/pipeline_ab.py)
        # (streams: reuse another Leg's streams -- the per-share pipelined table
        # runs on the headline's streams, the process's first)
        self.streams = list(streams) if streams else [torch.cuda.Stream(dev) for _ in range(NSTREAMS)]
        ns = len(self.streams)
        self.hdr2 = [self.hdr] + [torch.empty_like(self.hdr) for _ in range(ns - 1)]
        self.grad2 = [self.grad] + [torch.zeros_like(self.grad) for _ in range(ns - 1)]
        self.kev = []

    def params(self, step):
        return N.make_params(self.w, self.h, self.spp, self.mb, frame_seed(self.seed, step, self.w, self.h, self.spp),
                             self.b, self.e, self.step)

    def fwd(self, step, ev=None, piped=False):
        """The HDR image of the rank's rows: ONE launch of the trace kernel with
        the per-pixel mean fused in (brute-force scenes; BVH scenes render
        through the sample buffer + pixel_mean_sm_kernel inside the same call)."""
        cx, p = self.cx, self.params(step)
        k = step % len(self.streams)
        st, hdr = (self.streams[k], self.hdr2[k]) if piped else (cx.stream, self.hdr)
        if ev is not None:
            ev[0].record(st)
        N.check(cx.L.ipt_render_dev(self.sc.handle, C.byref(p), None, hdr.data_ptr(), None, st.cuda_stream))
        if ev is not None:
            ev[1].record(st)

    def adjoint(self, step, reduce=True, piped=False):
        cx, p = self.cx, self.params(step)
        k = step % len(self.streams)
        st, grad = (self.streams[k], self.grad2[k]) if piped else (cx.stream, self.grad)
        with torch.cuda.stream(st):
            grad.zero_()
            N.check(cx.L.ipt_adjoint_dev(self.sc.handle, C.byref(p), None, self.adj.data_ptr(), grad.data_ptr(),
                                         st.cuda_stream))
            if reduce and cx.world > 1:
                dist.all_reduce(grad)  # the per-material gradient vector, nT*3 fp64 (720 B for 30 triangles)

    def samples_per_call(self):
        return self.rows * self.w * self.spp

    def close(self):
        self.sc.close()


def band_table(cx, objs, w, h, spp, mb, n=8, reps=2, interleaved=False):
    """Each of the n row shares of one frame timed alone (forward, adjoint):
    the critical path of an n-GPU tile split is the slowest share."""
    rows = []
    for r in range(n):
        b, e, st = shard_rows_interleaved(h, n, r) if interleaved else shard_rows(h, n, r) + (1,)
        leg = Leg(cx, objs, w, h, spp, mb, b, e, step=st)
        leg.fwd(10**6)
        leg.adjoint(10**6, reduce=False)
        f = cx.timed(lambda i: leg.fwd(i), reps) / reps
        a = cx.timed(lambda i: leg.adjoint(i, reduce=False), reps) / reps
        rows.append({"rows": [b, e, st], "fwd_ms": round(f, 4), "adj_ms": round(a, 4)})
        leg.close()
    fw = [x["fwd_ms"] for x in rows]
    ad = [x["adj_ms"] for x in rows]
    return {"bands": rows, "fwd_max_over_mean": round(max(fw) / np.mean(fw), 4),
            "adj_max_over_mean": round(max(ad) / np.mean(ad), 4)}


def band_table_piped(cx, objs, w, h, spp, mb, streams, n=8, reps=20):
    """Each interleaved 1/n share of one frame with frames in flight, the
    headline's form (consecutive steps round-robin over its streams), on the
    headline's own streams: HIP maps streams onto its few hardware queues in
    creation order, and two streams created late can share one and run in
    order.  Per share: ms per step over `reps` steps (forward, adjoint) and a
    bitwise check that the last pipelined frame equals the same frame rendered
    alone."""
    rows = []
    for r in range(n):
        b, e, st = shard_rows_interleaved(h, n, r)
        leg = Leg(cx, objs, w, h, spp, mb, b, e, step=st, streams=streams)
        for i in range(2):
            leg.fwd(10**6 + i, piped=True)
            leg.adjoint(10**6 + i, reduce=False, piped=True)
        f = cx.timed(lambda i: leg.fwd(i, piped=True), reps, leg.streams) / reps
        a = cx.timed(lambda i: leg.adjoint(i, reduce=False, piped=True), reps, leg.streams) / reps
        last = leg.hdr2[(reps - 1) % len(leg.streams)].clone()
        ref = torch.empty_like(last)
        p = leg.params(reps - 1)
        N.check(cx.L.ipt_render_dev(leg.sc.handle, C.byref(p), None, ref.data_ptr(), None, cx.st))
        torch.cuda.synchronize(cx.dev)
        same = bool(torch.equal(last.view(torch.int32), ref.view(torch.int32)))
        rows.append({"rows": [b, e, st], "fwd_ms": round(f, 4), "adj_ms": round(a, 4), "bitwise_equal": same})
        leg.close()
    fw = [x["fwd_ms"] for x in rows]
    ad = [x["adj_ms"] for x in rows]
    return {"bands": rows, "reps": reps, "fwd_max_ms": max(fw), "adj_max_ms": max(ad),
            "fwd_max_over_mean": round(max(fw) / np.mean(fw), 4), "adj_max_over_mean": round(max(ad) / np.mean(ad), 4),
            "all_bitwise_equal": all(x["bitwise_equal"] for x in rows),
            "workload": "interleaved 1/%d shares of the C2 frame, frames in flight on the headline's HIP "
                        "streams; ms per step" % n}


def graph_line(cx, seed=0, reps=5):
    """createGraph's integrator (hot path #2, inv_path_trace.cu:152-208) at
    the reference's own configuration: scenes/0.txt, 500x500, 100 spp, no
    bounce cap, the reference's target preds/0_true.png; this rank's
    interleaved rows + one RCCL all-reduce of the fp64 bins.  The host
    compress (O(nT^2), inv_scene.h:87-115) is not timed."""
    from inverse_path_tracer_amd import png_read

    gw = gh = 500
    gspp = 100
    b, e, st = shard_rows_interleaved(gh, cx.world, cx.rank)
    sc = Scene(SCENE0)
    tgt = torch.from_numpy(png_read(GRAPH_TARGET)).to(cx.dev)
    acc = torch.zeros(((sc.nT + 1) * sc.nT, N.ACC_WIDTH), device=cx.dev, dtype=torch.float64)
    p = N.make_params(gw, gh, gspp, None, seed, b, e, st)

    def step(i):
        acc.zero_()
        N.check(cx.L.ipt_graph_dev(sc.handle, C.byref(p), tgt.data_ptr(), acc.data_ptr(), cx.st))
        if cx.world > 1:
            dist.all_reduce(acc)

    step(0)
    ms = cx.timed(step, reps) / reps
    frame = gw * gh * gspp
    flop = frame * CASTS_PER_SAMPLE_GRAPH * sc.nT * FLOP_PER_TEST
    out = {"value": round(frame / ms / 1e3, 2), "unit": "Msamples/s", "ms_per_step": round(ms, 4),
           "workload": "createGraph: scenes/0.txt (30 triangles), 500x500, 100 spp, unbounded, target "
                       "preds/0_true.png; interleaved rows over %d rank(s) + all-reduce of the (nT+1)*nT*8 fp64 "
                       "bins" % cx.world,
           "roofline": {"bound": "valu", "unit": "TFLOP/s", "peak": PEAK_FP32_TFLOPS,
                        "flop_per_sample": round(CASTS_PER_SAMPLE_GRAPH * sc.nT * FLOP_PER_TEST, 1),
                        "formula": "C_bar(graph, %.4f) * nT(30) * 38, brute-force-equivalent" % CASTS_PER_SAMPLE_GRAPH,
                        "achieved": round(flop / (ms / 1e3) / 1e12, 3),
                        "frac": round(flop / (ms / 1e3) / 1e12 / PEAK_FP32_TFLOPS, 4)}}
    sc.close()
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # IPT_BENCH_DEVICE / IPT_DIST_BACKEND: rehearse the N-rank path on a
    # one-GPU box (every rank on device 0, gloo); the driver's runs use the
    # defaults (rank i on GPU LOCAL_RANK, RCCL)
    local = int(os.environ.get("IPT_BENCH_DEVICE", local))
    backend = os.environ.get("IPT_DIST_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)  # RCCL over xGMI
        else:
            dist.init_process_group(backend)
    cx = Ctx(dev, world, rank)
    b, e, rs = shard_rows_interleaved(H, world, rank)
    head = Leg(cx, CORNELL, W, H, SPP, BOUNCES, b, e, seed=args.seed, step=rs)
    for i in range(args.warmup):
        head.fwd(10**6 + i)
        head.adjoint(10**6 + i)
        head.fwd(10**6 + i, piped=True)
        head.adjoint(10**6 + i, piped=True)
    # ---------------------------------------------------------- headline: tile-split C2 frame
    # (1) frames one after another on one stream: each launch's own time
    # (HIP events around it: the roofline's kernel time) and the serial rate
    kev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    fwd_serial_ms = cx.timed(lambda i: head.fwd(i, kev[i]), args.steps)
    kernel_ms = float(np.mean([a.elapsed_time(z) for a, z in kev]))
    bwd_serial_ms = cx.timed(lambda i: head.adjoint(i), args.steps)
    # (2) the headline: consecutive frames round-robin over NSTREAMS streams
    # (frames in flight: one frame's tail -- its last paths, a few waves per
    # CU -- overlaps the next frame's start), the same K frames of work
    t_wall = time.perf_counter()
    fwd_ms = cx.timed(lambda i: head.fwd(i, piped=True), args.steps, head.streams)
    wall_fwd = time.perf_counter() - t_wall
    # the last NSTREAMS frames in flight, re-rendered alone: bitwise the same images
    last = list(range(max(0, args.steps - len(head.streams)), args.steps))
    got = {i: head.hdr2[i % len(head.streams)].clone() for i in last}  # (hdr2[0] is head.hdr, which fwd(i) overwrites)
    piped_ok = []
    for i in last:
        head.fwd(i)
        torch.cuda.synchronize()
        piped_ok.append(bool(torch.equal(got[i].view(torch.int32), head.hdr.view(torch.int32))))
    if not all(piped_ok):
        # a headline that rendered different images is not a measurement of
        # this frame: fall back to the one-stream rate and say so in the line
        print("bench: frames in flight differ from frames rendered alone: %s" % piped_ok, file=sys.stderr)
        fwd_ms = fwd_serial_ms
    # (gloo, the one-GPU rehearsal backend, stages every all-reduce through the
    # host: there the adjoint steps stay on one stream)
    piped_adj = world == 1 or backend == "nccl"
    bwd_ms = cx.timed(lambda i: head.adjoint(i, piped=piped_adj), args.steps, head.streams if piped_adj else ())
    # ... and the last NSTREAMS gradients in flight against the same adjoints
    # alone on one stream: equal to fp64 summation order (the atomics' order)
    gots = {i: head.grad2[i % len(head.streams)].clone() for i in last} if piped_adj else {}
    adj_ok = []
    for i in gots:
        head.adjoint(i)
        torch.cuda.synchronize()
        g, w = gots[i].cpu().numpy(), head.grad.cpu().numpy()
        adj_ok.append(bool(np.allclose(g, w, rtol=1e-9, atol=1e-12 * max(np.abs(w).max(), 1e-300))))
    if not all(adj_ok):
        print("bench: adjoints in flight differ from adjoints alone: %s" % adj_ok, file=sys.stderr)
        bwd_ms = bwd_serial_ms
    frame = W * H * SPP
    value = args.steps * frame / (fwd_ms / 1e3) / 1e6
    grad_value = args.steps * frame / (bwd_ms / 1e3) / 1e6

    extra = {"serial": {"value": round(args.steps * frame / (fwd_serial_ms / 1e3) / 1e6, 2),
                        "grad_value": round(args.steps * frame / (bwd_serial_ms / 1e3) / 1e6, 2),
                        "ms_per_step": round(fwd_serial_ms / args.steps, 4),
                        "grad_ms_per_step": round(bwd_serial_ms / args.steps, 4),
                        "workload": "the headline's frames one after another on ONE stream (no frame overlap)"},
             "piped_frames_bitwise_equal_alone": piped_ok,
             "headline_forward_form": ("%d frames in flight" % len(head.streams) if all(piped_ok) else
                                       "INVALID in flight (frames differed from frames rendered alone): "
                                       "value is the one-stream rate"),
             "piped_gradients_equal_alone": adj_ok,
             "headline_adjoint_form": (("%d adjoints in flight" % len(head.streams) if all(adj_ok) else
                                        "INVALID in flight (gradients differed from adjoints alone beyond fp64 "
                                        "summation order): grad_value is the one-stream rate")
                                       if piped_adj else "one stream (gloo)")}
    if not args.no_secondary:
        # sustained rates (>= 0.5 s of back-to-back steps per leg; DVFS-steady)
        k, ms = cx.sustained(lambda i: head.fwd(i))
        ka, msa = cx.sustained(lambda i: head.adjoint(i))
        extra["sustained"] = {"fwd_Msamples_s": round(k * frame / ms / 1e3, 2), "fwd_steps": k, "fwd_s": round(ms / 1e3, 3),
                              "grad_Msamples_s": round(ka * frame / msa / 1e3, 2), "adj_steps": ka,
                              "adj_s": round(msa / 1e3, 3)}
        # weak scaling: every rank traces a whole frame of its own
        weak = Leg(cx, CORNELL, W, H, SPP, BOUNCES, seed=args.seed + (rank + 1) * 7919 * frame)
        kw = max(4, min(args.steps, 40))
        wf = cx.timed(lambda i: weak.fwd(i), kw)
        wa = cx.timed(lambda i: weak.adjoint(i), kw)
        extra["weak"] = {"value": round(world * kw * frame / wf / 1e3, 2), "grad_value": round(world * kw * frame / wa / 1e3, 2),
                         "unit": "Msamples/s", "workload": "C2, one whole frame per rank per step (frame-parallel)"}
        weak.close()
        # other configurations, this rank's band of an N-way tile split
        for key, objs, w, h, spp, mb, desc in (
                ("c3", SCENE0, W, H, SPP, BOUNCES, "C3: scenes/0.txt (Cornell + cube, 30 triangles), 512x512, 64 spp, 4 bounces"),
                ("c3_phong", SCENE0_PHONG, W, H, SPP, BOUNCES, "C3 with a Phong cube (Ks 0.5, shininess 20; "
                 "assets/phong/scene0_phong.txt): the SPEC kernel instances, 512x512, 64 spp, 4 bounces"),
                ("c3_unbounded", SCENE0, W, H, SPP, None, "C3 with the reference's own estimator (no bounce cap: "
                 "Russian roulette only), scenes/0.txt, 512x512, 64 spp; fused render (slot ring); adjoint = global "
                 "record ring + chunk replay"),
                ("legacy_create_image", SCENE0, 500, 500, 100, None, "the reference's createImage configuration "
                 "(path_trace.cu:200-234, scene.h:8-10): scenes/0.txt, 500x500, 100 spp, no bounce cap; fused render "
                 "(no per-sample buffer)"),
                ("c3_northstar", NORTHSTAR, W, H, SPP, BOUNCES, "C3 as the north_star names it: Cornell + cube + "
                 "sphere.obj (assets/northstar.txt, 1310 triangles, BVH), 512x512, 64 spp, 4 bounces"),
                ("c3_northstar_unbounded", NORTHSTAR, W, H, SPP, None, "the north-star scene (1310 triangles, BVH) with "
                 "the reference's own estimator (no bounce cap), 512x512, 64 spp; two-kernel render; adjoint = record "
                 "ring in LDS + per-wave chunk pools + chunk replay"),
                ("bvh_sphere", SPHERE, W, H, SPP, BOUNCES, "Cornell + sphere.obj (1298 triangles, BVH), 512x512, 64 spp, 4 bounces"),
                ("c4", SCENE0, 1024, 1024, 256, 8, "C4: scenes/0.txt, 1024x1024, 256 spp, 8 bounces")):
            if key != "c4":
                bb, ee, ss = shard_rows_interleaved(h, world, rank)
            else:  # C4: 8 interleaved shares, one per rank; ranks past 8 run none
                bb, ee, ss = shard_rows_interleaved(h, 8, rank) if rank < 8 else (0, 0, 1)
            leg = Leg(cx, objs, w, h, spp, mb, bb, ee, step=ss)
            leg.fwd(10**6)
            leg.adjoint(10**6)
            reps = 2 if key == "c4" else 5
            f = cx.timed(lambda i: leg.fwd(i), reps) / reps
            a = cx.timed(lambda i: leg.adjoint(i), reps) / reps
            n = leg.samples_per_call() * world
            fps, how = flop_per_sample(key)
            if fps:  # per rank: this rank's samples over its own kernel time
                extra[key + "_roofline"] = {
                    "bound": "valu", "unit": "TFLOP/s", "peak": PEAK_FP32_TFLOPS, "flop_per_sample": round(fps, 2),
                    "flop_source": how,
                    "fwd_frac": round(leg.samples_per_call() * fps / (f / 1e3) / 1e12 / PEAK_FP32_TFLOPS, 4),
                    "adj_frac": round(leg.samples_per_call() * fps / (a / 1e3) / 1e12 / PEAK_FP32_TFLOPS, 4)}
                ex = executed_flop_per_sample("scene0", CASTS_PER_SAMPLE_C3, 30) if key == "c3" else None
                if ex:
                    extra[key + "_roofline"]["executed"] = {
                        "flop_per_sample": round(ex, 1),
                        "fwd_frac": round(leg.samples_per_call() * ex / (f / 1e3) / 1e12 / PEAK_FP32_TFLOPS, 4),
                        "adj_frac": round(leg.samples_per_call() * ex / (a / 1e3) / 1e12 / PEAK_FP32_TFLOPS, 4)}
            extra[key] = {"value": round(n / f / 1e3, 2), "unit": "Msamples/s", "grad_value": round(n / a / 1e3, 2),
                          "grad_unit": "grad-Msamples/s", "fwd_ms": round(f, 4), "adj_ms": round(a, 4),
                          "triangles": leg.sc.nT, "accel": leg.sc.bvh_info()["accel"],
                          "workload": desc + ("; rank k = interleaved share k of 8 (rows k, k+8, ...; %d of 8 "
                                              "shares run)" % min(world, 8) if key == "c4" else
                                              "; interleaved rows over %d rank(s)" % world)}
            leg.close()
        if world == 1:
            extra["bands_c2"] = band_table(cx, CORNELL, W, H, SPP, BOUNCES, reps=4)
            extra["bands_c2_interleaved"] = band_table(cx, CORNELL, W, H, SPP, BOUNCES, reps=4, interleaved=True)
            extra["bands_c2_piped"] = band_table_piped(cx, CORNELL, W, H, SPP, BOUNCES, head.streams)
            extra["bands_c4"] = band_table(cx, SCENE0, 1024, 1024, 256, 8, reps=1)
            extra["bands_c4_interleaved"] = band_table(cx, SCENE0, 1024, 1024, 256, 8, reps=1, interleaved=True)
            sys.path.insert(0, os.path.join(ROOT, "tools"))
            import bench_c5
            extra["c5"] = bench_c5.run(scenes=13, steps=20, warmup=3, total=240)  # 240 steps: the convergence record (~2 s)
        extra["graph"] = graph_line(cx)
    # ---------------------------------------------------------- roofline of the dominant kernel
    band_samples = head.samples_per_call()
    flop_per_launch = band_samples * CASTS_PER_SAMPLE * N_TRIANGLES * FLOP_PER_TEST
    achieved = flop_per_launch / (kernel_ms / 1e3) / 1e12
    # the adjoint kernel over the same casts (its step also holds the gradient memset + all-reduce)
    grad_achieved = flop_per_launch / (bwd_serial_ms / args.steps / 1e3) / 1e12  # the launch's own time
    traffic = grad_traffic = None
    if os.path.exists(PMC_FILE):
        with open(PMC_FILE) as f:
            pmc = json.load(f)
        if "trace_kernel<4" in pmc.get("kernel", ""):  # counters of the kernel timed here (the fused render)
            traffic = pmc.get("hbm_bytes_per_launch")
        if "trace_kernel<5" in pmc.get("grad_kernel", ""):  # and of the 6-wave adjoint the gradient leg runs
            grad_traffic = pmc.get("grad_hbm_bytes_per_launch")
        if world > 1:  # the counters were taken on the whole frame
            traffic = traffic * band_samples / frame if traffic else traffic
            grad_traffic = grad_traffic * band_samples / frame if grad_traffic else grad_traffic
    hbm = None
    if traffic:
        gbs = traffic / (kernel_ms / 1e3) / 1e9
        hbm = {"bytes_per_launch": traffic, "achieved_GBps": round(gbs, 1), "peak_GBps": 8000.0,
               "frac": round(gbs / 8000.0, 4), "algorithmic_bytes_per_launch": head.npix * 12,
               "algorithmic": "the 12 B/pixel HDR output (compulsory)",
               "source": os.path.relpath(PMC_FILE, ROOT)}
        if grad_traffic:
            hbm["grad_bytes_per_launch"] = grad_traffic
            hbm["grad_achieved_GBps"] = round(grad_traffic / (bwd_serial_ms / args.steps / 1e3) / 1e9, 1)
            hbm["grad_algorithmic"] = "the 12 B/pixel adjoint image read once (%d B)" % (head.npix * 12)
    roofline = {"bound": "valu", "achieved": round(achieved, 3), "peak": PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": round(achieved / PEAK_FP32_TFLOPS, 4), "traffic": traffic, "grad_traffic": grad_traffic,
                # SURVEY.md 8(d) fixes `frac`'s formula (brute-force-equivalent tests, judge and builder
                # alike); the same number under its descriptive name, and `executed_frac` below
                "brute_force_equivalent_frac": round(achieved / PEAK_FP32_TFLOPS, 4),
                "kernel": "trace_kernel<MODE_FWDM> (forward + fused per-pixel mean, the step's only kernel)",
                "kernel_ms": round(kernel_ms, 4),
                "flop_per_launch": flop_per_launch,
                "grad_achieved": round(grad_achieved, 3), "grad_frac": round(grad_achieved / PEAK_FP32_TFLOPS, 4),
                "basis": "brute-force-equivalent work (SURVEY.md 8(d) fixed formula): every cast is charged all "
                         "nT triangle tests, although the culled casts execute ~1/4 of them -- `executed_frac` "
                         "is the hardware-use figure",
                "formula": "samples*C_bar(%.4f)*nT(%d)*38 FLOP / kernel time; peak = FP32 vector peak (equal to "
                           "the FP32 MFMA peak on gfx950)" % (CASTS_PER_SAMPLE, N_TRIANGLES)}
    ex = executed_flop_per_sample("cornell", CASTS_PER_SAMPLE, N_TRIANGLES)
    if ex:  # the culled casts skip pairs no ray can accept: the work actually issued is smaller
        ea = band_samples * ex / (kernel_ms / 1e3) / 1e12
        roofline["executed_frac"] = round(ea / PEAK_FP32_TFLOPS, 4)
        roofline["executed_grad_frac"] = round(band_samples * ex / (bwd_serial_ms / args.steps / 1e3) / 1e12 /
                                               PEAK_FP32_TFLOPS, 4)
        roofline["executed"] = {"flop_per_sample": round(ex, 1), "achieved": round(ea, 3),
                                "source": "triangle tests (x38) and slab tests (x12) actually executed, "
                                          "profiles/bvh_stats.json (IPT_BVH_STATS build)"}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline()
    if rank == 0:
        out = {
            "metric": "Msamples/sec fwd + grad-Msamples/sec, 512² Cornell 64spp, 1/2/4/8 GPU",
            "value": round(value, 2), "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(fwd_ms / args.steps, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "C2: CornellBox-Empty-CO.obj, 512x512, 64 spp, max_bounces=4; one frame per step "
                                   "tiled over the ranks as interleaved rows (fwd); adjoint dL/dKd of the rank's rows "
                                   "+ RCCL all-reduce of the gradient (grad); %d frames in flight (consecutive steps "
                                   "round-robin over %d HIP streams; one stream: secondary.serial)" % (NSTREAMS, NSTREAMS),
                       "streams": NSTREAMS if piped_adj else "%d (fwd) / 1 (grad: gloo)" % NSTREAMS,
                       "width": W, "height": H, "spp": SPP, "max_bounces": BOUNCES, "triangles": head.sc.nT,
                       "parallelism": "interleaved row tiles x%d" % world, "rank0_rows": [b, e, rs]},
            "grad_value": round(grad_value, 2), "grad_unit": "grad-Msamples/s",
            "grad_ms_per_step": round(bwd_ms / args.steps, 4),
            "wall_s_fwd_region": round(wall_fwd, 4),
            "roofline": roofline, "hbm": hbm, "cpu_baseline": cpu, "secondary": extra,
        }
        print(json.dumps(out), flush=True)
    head.close()
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
