"""GPU parity tests (run with -m gpu on an MI355X).

Every compute call goes through the C ABI of lib/libipt_amd.so.  Bars:
  * forward per-sample radiance and per-pixel HDR: BIT-IDENTICAL to the CPU
    oracle on the same seeds (canonical arithmetic);
  * adjoint gradient and graph bins: fp64 sums whose order differs (atomics),
    so rtol 1e-9 against the oracle; the compressed createGraph floats are
    compared at rtol 1e-6;
  * at the BASELINE.json sizes (oracle too slow): size-independent properties
    -- row-band sharding reproduces the full frame bit-for-bit, the adjoint is
    linear in the adjoint image and matches central finite differences of the
    GPU forward, and the reference's golden render statistics hold.
"""
import ctypes as C
import json
import os

import numpy as np
import pytest

from conftest import CORNELL, CUBE_OBJ, SCENE0, SPHERE_OBJ, TESTS, product_scene

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    from inverse_path_tracer_amd import _native

    assert _native.device_count() >= 1
    yield


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def scenes(oracle):
    return {
        "cornell": (product_scene(CORNELL), oracle.OracleScene(CORNELL)),
        "scene0": (product_scene(SCENE0), oracle.OracleScene(SCENE0)),
    }


# ------------------------------------------------------------- forward
@pytest.mark.parametrize("name,W,H,spp,mb,seed", [
    ("cornell", 128, 128, 8, 2, 0),          # BASELINE config C1 (the CPU plumbing config)
    ("cornell", 64, 48, 16, 4, 1),
    ("scene0", 64, 64, 16, None, 7),         # reference semantics: unbounded
    ("scene0", 40, 30, 8, 0, 3),             # direct lighting only
    ("scene0", 33, 17, 5, 8, 2**33 + 5),     # odd sizes, 64-bit seed
    ("scene0", 1, 1, 1, 4, 0),               # single sample
])
def test_forward_samples_bit_exact(scenes, name, W, H, spp, mb, seed):
    P, Q = scenes[name]
    got = P.render_samples(W, H, spp, mb, seed)
    want, _ = Q.render_samples(W, H, spp, mb, seed)
    assert np.array_equal(bits(got), bits(want))


def test_forward_hdr_and_tonemap_bit_exact(scenes, oracle):
    P, Q = scenes["scene0"]
    hdr, u8 = P.render(48, 40, 12, 4, 5, ldr=True)
    s, _ = Q.render_samples(48, 40, 12, 4, 5)
    hq, uq = oracle.pixel_mean(s, 48 * 40, 12)
    assert np.array_equal(bits(hdr.reshape(-1, 3)), bits(hq))
    assert np.array_equal(u8.reshape(-1, 3), uq)


def test_sphere_scene_bit_exact(oracle):
    recs = CORNELL + [((0.3, -1.2, 4.2), (0.0, 0.4, 0.0), (1.2, 1.2, 1.2), SPHERE_OBJ, "*Kd 0.2 0.6 0.3*")]
    P, Q = product_scene(recs), oracle.OracleScene(recs)
    assert P.nT == 18 + 1280
    got = P.render_samples(24, 24, 4, 3, 9)
    want, _ = Q.render_samples(24, 24, 4, 3, 9)
    assert np.array_equal(bits(got), bits(want))


def test_specular_material_bit_exact(oracle, tmp_path):
    mtl = tmp_path / "s.mtl"
    mtl.write_text("newmtl shiny\nKd 0.3 0.3 0.3\nKs 0.5 0.4 0.3\nNs 20\n")
    obj = tmp_path / "s.obj"
    obj.write_text(open(CUBE_OBJ).read().replace("f 1 2 3", "mtllib s.mtl\nusemtl shiny\nf 1 2 3", 1))
    recs = CORNELL + [((0, -1.5, 4), (0, 0.3, 0), (1, 1, 1), str(obj), str(mtl))]
    P, Q = product_scene(recs), oracle.OracleScene(recs)
    assert np.any(P.triangles()[:, 28:31] > 0)
    got = P.render_samples(32, 32, 8, 4, 4)
    want, _ = Q.render_samples(32, 32, 8, 4, 4)
    assert np.array_equal(bits(got), bits(want))
    adj = np.random.RandomState(0).uniform(-1, 1, (32, 32, 3)).astype(np.float32)
    np.testing.assert_allclose(P.adjoint(adj, 32, 32, 8, 4, 4), Q.adjoint(32, 32, 8, 4, 4, adj), rtol=1e-9, atol=1e-12)


def test_phong_scene_fused_render_and_unbounded_adjoint(oracle):
    """The bench's c3_phong scene (assets/phong: the cube with Ks 0.5,
    shininess 20) through the SPEC instances the other Phong test does not
    reach: the fused render (HDR = the oracle's toneMap, bitwise, bounded and
    unbounded paths) and the unbounded adjoint (rtol 1e-9)."""
    import oracle_lib
    from conftest import ASSETS

    recs = CORNELL + [((0, -1.5, 4), (0, 0, 0), (1, 1, 1), os.path.join(ASSETS, "phong", "cube_phong.obj"),
                       os.path.join(ASSETS, "phong", "cube_phong.mtl"))]
    P, Q = product_scene(recs), oracle.OracleScene(recs)
    assert np.any(P.triangles()[:, 28:31] > 0)
    W, H, spp, seed = 40, 24, 16, 6
    for mb in (4, None):
        hdr = P.render(W, H, spp, mb, seed)
        s, _ = Q.render_samples(W, H, spp, mb, seed)
        hq, _ = oracle_lib.pixel_mean(s, W * H, spp)
        assert np.array_equal(bits(hdr.reshape(-1, 3)), bits(hq)), mb
    adj = np.random.RandomState(1).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    np.testing.assert_allclose(P.adjoint(adj, W, H, spp, None, seed), Q.adjoint(W, H, spp, None, seed, adj),
                               rtol=1e-9, atol=1e-12)
    P.close()


def test_phong_sphere_bvh_instances(oracle, tmp_path):
    """The SPEC x BVH kernel instances (a Phong material in a scene large
    enough for the triangle BVH): the north-star scene with the sphere given
    Ks 0.4, shininess 30.  Forward samples bit-exact (bounded and unbounded),
    bounded and unbounded adjoints rtol 1e-9 against the oracle."""
    from conftest import SCENE0

    mtl = tmp_path / "shiny.mtl"
    mtl.write_text("newmtl shiny\nKd 0.2 0.6 0.3\nKs 0.4 0.4 0.4\nNs 30\n")
    src = open(SPHERE_OBJ).read()
    i = src.index("\nf ") + 1
    obj = tmp_path / "sphere_shiny.obj"
    obj.write_text(src[:i] + "mtllib shiny.mtl\nusemtl shiny\n" + src[i:])
    recs = SCENE0 + [((-1.2, -1.35, 4.6), (0, 0, 0), (1.2, 1.2, 1.2), str(obj), str(mtl))]
    P, Q = product_scene(recs), oracle.OracleScene(recs)
    assert P.nT > 1000 and np.any(P.triangles()[:, 28:31] > 0)
    W, H, spp, seed = 32, 24, 8, 12
    adj = np.random.RandomState(3).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    for mb in (4, None):
        got = P.render_samples(W, H, spp, mb, seed)
        want, _ = Q.render_samples(W, H, spp, mb, seed)
        assert np.array_equal(bits(got), bits(want)), mb
        np.testing.assert_allclose(P.adjoint(adj, W, H, spp, mb, seed), Q.adjoint(W, H, spp, mb, seed, adj),
                                   rtol=1e-9, atol=1e-12, err_msg=str(mb))
    P.close()


def test_no_emitters_is_black_not_nan(oracle):
    recs = [((0, -1.5, 4), (0, 0, 0), (1, 1, 1), CUBE_OBJ, "*Kd 0.5 0.5 0.5*")]
    P, Q = product_scene(recs), oracle.OracleScene(recs)
    assert P.nE == 0
    got = P.render_samples(16, 16, 4, None, 0)
    want, _ = Q.render_samples(16, 16, 4, None, 0)
    assert np.array_equal(bits(got), bits(want)) and np.all(got == 0)


def test_empty_band_and_bad_params(scenes):
    from inverse_path_tracer_amd import NativeError

    P, _ = scenes["scene0"]
    assert P.render(16, 16, 2, 2, 0, row_begin=5, row_end=5).shape == (0, 16, 3)
    with pytest.raises(NativeError):
        P.render(16, 16, 0, 2, 0)
    with pytest.raises(NativeError):
        P.render(16, 16, 2, 2, 0, row_begin=3, row_end=20)
    with pytest.raises(NativeError, match="max_bounces"):
        P.adjoint(np.zeros((8, 8, 3), np.float32), 8, 8, 1, 63, 0)


# ------------------------------------------------------------- sharding (C2/C4 sizes)
@pytest.mark.parametrize("W,H,spp,mb,world", [(512, 512, 64, 4, 8), (1024, 1024, 32, 8, 8), (512, 512, 64, 4, 3)])
def test_row_band_sharding_bit_exact(scenes, W, H, spp, mb, world):
    from inverse_path_tracer_amd.distributed import shard_rows, shard_rows_interleaved

    P, _ = scenes["scene0"]
    full = P.render(W, H, spp, mb, 0)
    bands = [P.render(W, H, spp, mb, 0, *shard_rows(H, world, r)) for r in range(world)]
    assert np.array_equal(bits(np.concatenate(bands)), bits(full))
    for r in range(world):  # interleaved shares (the bench's tile split)
        b, e, st = shard_rows_interleaved(H, world, r)
        assert np.array_equal(bits(P.render(W, H, spp, mb, 0, b, e, row_step=st)), bits(full[b:e:st]))


# ------------------------------------------------------------- adjoint
@pytest.mark.parametrize("name,W,H,spp,mb,seed", [
    ("scene0", 64, 64, 8, 4, 3), ("scene0", 31, 23, 4, 8, 1), ("cornell", 48, 48, 8, 2, 6), ("scene0", 16, 16, 4, 0, 2),
    # spp not a power of two (the weight division path), long paths (many sweep tasks per lane)
    ("scene0", 20, 12, 3, 5, 5), ("cornell", 24, 16, 5, 20, 7),
    # the reference's own estimator (no cap): ring records + chunk replays of paths longer than the ring
    ("scene0", 64, 64, 8, None, 3), ("cornell", 33, 21, 16, None, 9),
    # unbounded with spp not a power of two and a 64-bit seed
    ("scene0", 19, 13, 7, None, 2**33 + 11)])
def test_adjoint_matches_oracle(scenes, name, W, H, spp, mb, seed):
    P, Q = scenes[name]
    adj = np.random.RandomState(seed % 2**32).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    g = P.adjoint(adj, W, H, spp, mb, seed)
    want = Q.adjoint(W, H, spp, mb, seed, adj)
    np.testing.assert_allclose(g, want, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("name,W,H,spp,mb,seed", [("scene0", 64, 64, 8, 4, 3), ("cornell", 48, 48, 8, 2, 6)])
def test_adjoint_six_wave_instance_matches_oracle(scenes, monkeypatch, name, W, H, spp, mb, seed):
    """MODE_ADJW (the bounded adjoint at 6 waves/SIMD, chosen for launches
    of >= 8 M samples) forced onto small launches: same gradient."""
    monkeypatch.setenv("IPT_ADJW", "1")
    P, Q = scenes[name]
    adj = np.random.RandomState(seed).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    g = P.adjoint(adj, W, H, spp, mb, seed)
    want = Q.adjoint(W, H, spp, mb, seed, adj)
    np.testing.assert_allclose(g, want, rtol=1e-9, atol=1e-12)


def test_back_to_back_launches_with_ragged_chunks(scenes):
    """Launches on one stream share the chunk counters, which the launch's
    last grab zeroes (ipt_hip.hip grab_failed, TraceArgs::grabs: the host's
    count of the launch's grabs).  509 x 97 pixels:
    the fused render's last 8-pixel chunk holds 5 (more than its 4-pixel
    small chunk) and the adjoint's 789 968 samples leave 80 (more than 64)
    past the last full 128-item chunk, with more chunks than waves -- round
    4's host-side count of the grabs (and round 5's) has to match the
    kernel's enumeration exactly, or later launches skip or re-trace chunks."""
    P, Q = scenes["scene0"]
    W, H, spp, mb, seed = 509, 97, 16, 4, 21
    adj = np.random.RandomState(8).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    P.render(W, H, spp, mb, seed)             # fused render (ragged pixel chunks)
    g1 = P.adjoint(adj, W, H, spp, mb, seed)  # ragged sample chunks
    g2 = P.adjoint(adj, W, H, spp, mb, seed)
    hdr = P.render(W, H, spp, mb, seed)
    want = Q.adjoint(W, H, spp, mb, seed, adj)
    np.testing.assert_allclose(g1, want, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(g2, want, rtol=1e-9, atol=1e-12)
    s, _ = Q.render_samples(W, H, spp, mb, seed)
    import oracle_lib

    hq, _ = oracle_lib.pixel_mean(s, W * H, spp)
    assert np.array_equal(bits(hdr.reshape(-1, 3)), bits(hq))


def test_new_stream_behind_busy_null_stream():
    """A stream's chunk counters are created (and zeroed) at its first
    launch.  Zeroed with a blocking hipMemset they were ordered on the null
    stream, which a non-blocking torch stream does not wait for: behind queued
    null-stream work the zeroing landed after the new stream's first launch
    had advanced the counter, and every later launch on that stream rendered
    part of its frame (bench.py's frames in flight).  Now zeroed on the launch
    stream: launches on a fresh stream behind a busy null stream are bitwise
    the null stream's."""
    import torch

    from inverse_path_tracer_amd import _native as N

    L = N.lib()
    hip = C.CDLL("libamdhip64.so")
    sc = product_scene(CORNELL)
    raws = []
    try:
        W = H = 256
        ps = [N.make_params(W, H, 64, 4, 5 + i) for i in range(3)]
        null = torch.cuda.current_stream()
        ref = [torch.empty((W * H, 3), device="cuda") for _ in ps]
        for p, r in zip(ps, ref):
            N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, r.data_ptr(), None, null.cuda_stream))
        torch.cuda.synchronize()
        for trial in range(3):
            busy = torch.empty((W * H, 3), device="cuda")
            for _ in range(6):  # queued null-stream work
                N.check(L.ipt_render_dev(sc.handle, C.byref(ps[0]), None, busy.data_ptr(), None, null.cuda_stream))
            # a raw non-blocking stream never used before (torch's stream pool
            # may hand back one whose counters already exist)
            raw = C.c_void_p()
            assert hip.hipStreamCreateWithFlags(C.byref(raw), 1) == 0  # hipStreamNonBlocking
            raws.append(raw)
            st = torch.cuda.ExternalStream(raw.value)
            got = [torch.full((W * H, 3), float("nan"), device="cuda") for _ in ps]
            torch.cuda.synchronize()
            for _ in range(6):
                N.check(L.ipt_render_dev(sc.handle, C.byref(ps[0]), None, busy.data_ptr(), None, null.cuda_stream))
            for p, g in zip(ps, got):
                N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, g.data_ptr(), None, st.cuda_stream))
            torch.cuda.synchronize()
            for g, r in zip(got, ref):
                assert torch.equal(g.view(torch.int32), r.view(torch.int32)), trial
    finally:
        torch.cuda.synchronize()
        sc.close()  # (frees the scene's per-stream counters)
        for raw in raws:
            hip.hipStreamDestroy(raw)


def _stream(hip):
    import torch

    raw = C.c_void_p()
    assert hip.hipStreamCreateWithFlags(C.byref(raw), 1) == 0  # hipStreamNonBlocking
    return raw, torch.cuda.ExternalStream(raw.value)


@pytest.mark.parametrize("nstreams", [3, 4])
def test_frames_in_flight_equal_frames_alone(nstreams):
    """bench.py's headline form: consecutive C2 frames (per-step seeds) dealt
    round-robin over `nstreams` fresh non-blocking streams, each stream with
    its own image and gradient, no synchronisation between them -- the fused
    render of every frame bitwise equal to the frame rendered alone, the
    adjoint's fp64 gradient equal to the lone launch's to summation order."""
    import torch

    from inverse_path_tracer_amd import _native as N
    from inverse_path_tracer_amd.distributed import frame_seed

    L = N.lib()
    hip = C.CDLL("libamdhip64.so")
    sc = product_scene(CORNELL)
    W = H = 128
    spp, mb, frames = 64, 4, 9
    ps = [N.make_params(W, H, spp, mb, frame_seed(0, i, W, H, spp)) for i in range(frames)]
    adj = torch.full((H, W, 3), 1.0 / (3 * W * H), device="cuda")
    streams = [_stream(hip) for _ in range(nstreams)]
    try:
        null = torch.cuda.current_stream().cuda_stream
        alone_img, alone_g = [], []
        for p in ps:
            img = torch.empty((W * H, 3), device="cuda")
            g = torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda")
            N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, img.data_ptr(), None, null))
            N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p), None, adj.data_ptr(), g.data_ptr(), null))
            alone_img.append(img)
            alone_g.append(g)
        torch.cuda.synchronize()
        imgs = [torch.full((W * H, 3), float("nan"), device="cuda") for _ in ps]
        gs = [torch.zeros((sc.nT, 3), dtype=torch.float64, device="cuda") for _ in ps]
        torch.cuda.synchronize()
        for i, p in enumerate(ps):
            st = streams[i % nstreams][1].cuda_stream
            N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, imgs[i].data_ptr(), None, st))
            N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p), None, adj.data_ptr(), gs[i].data_ptr(), st))
        torch.cuda.synchronize()
        for i in range(frames):
            assert torch.equal(imgs[i].view(torch.int32), alone_img[i].view(torch.int32)), i
            np.testing.assert_allclose(gs[i].cpu().numpy(), alone_g[i].cpu().numpy(), rtol=1e-12, atol=1e-18)
    finally:
        torch.cuda.synchronize()
        sc.close()
        for raw, _ in streams:
            hip.hipStreamDestroy(raw)


def test_mixed_launch_kinds_share_one_stream(scenes):
    """Every kind of launch may follow any other on a stream: single-set
    renders, 8-set scene batches (as many counter words as a single launch
    has), adjoints and createGraph, interleaved on one fresh stream -- each
    result equals the same launch alone on its own fresh stream (round 4's
    counters, keyed by word count with per-word host bases, gave an 8-set
    batch after a single render stale bases for sets 1..7: ADVICE r4)."""
    import torch

    from inverse_path_tracer_amd import _native as N

    L = N.lib()
    hip = C.CDLL("libamdhip64.so")
    P, _ = scenes["scene0"]
    W, H, spp, mb, seed = 96, 64, 16, 4, 77
    S, stride = 8, W * H * spp
    kd = torch.from_numpy(np.random.RandomState(5).uniform(0, 1, (S, P.nT, 3)).astype(np.float32)).cuda()
    adj = torch.from_numpy(np.random.RandomState(6).uniform(-1, 1, (S, H, W, 3)).astype(np.float32)).cuda()
    tgt = torch.from_numpy(np.random.RandomState(7).randint(0, 255, (H, W, 3)).astype(np.uint8)).cuda()
    p = N.make_params(W, H, spp, mb, seed)
    pu = N.make_params(W, H, spp, -1, seed + 1)
    nacc = (P.nT + 1) * P.nT * 8

    def run(kind, st):
        if kind == "render":
            o = torch.empty((H * W, 3), device="cuda")
            N.check(L.ipt_render_dev(P.handle, C.byref(p), kd[3].data_ptr(), o.data_ptr(), None, st))
        elif kind == "batch":
            o = torch.empty((S, H * W, 3), device="cuda")
            N.check(L.ipt_render_batch_dev(P.handle, C.byref(p), S, stride, kd.data_ptr(), o.data_ptr(), st))
        elif kind == "adjoint":
            o = torch.zeros((P.nT, 3), device="cuda", dtype=torch.float64)
            N.check(L.ipt_adjoint_dev(P.handle, C.byref(p), kd[1].data_ptr(), adj[1].data_ptr(), o.data_ptr(), st))
        elif kind == "adjoint_u":
            o = torch.zeros((P.nT, 3), device="cuda", dtype=torch.float64)
            N.check(L.ipt_adjoint_dev(P.handle, C.byref(pu), kd[2].data_ptr(), adj[2].data_ptr(), o.data_ptr(), st))
        elif kind == "adjoint_batch":
            o = torch.zeros((S, P.nT, 3), device="cuda", dtype=torch.float64)
            N.check(L.ipt_adjoint_batch_dev(P.handle, C.byref(p), S, stride, kd.data_ptr(), adj.data_ptr(),
                                            o.data_ptr(), st))
        else:  # graph
            o = torch.zeros(nacc, device="cuda", dtype=torch.float64)
            N.check(L.ipt_graph_dev(P.handle, C.byref(pu), tgt.data_ptr(), o.data_ptr(), st))
        return o

    kinds = ["render", "batch", "batch", "adjoint", "render", "adjoint_batch", "graph", "batch", "adjoint_u",
             "render", "adjoint_batch", "batch"]
    raws = []
    try:
        want = {}
        for k in sorted(set(kinds)):  # each kind alone on a fresh stream
            raw, st = _stream(hip)
            raws.append(raw)
            want[k] = run(k, st.cuda_stream)
        torch.cuda.synchronize()
        raw, st = _stream(hip)
        raws.append(raw)
        got = [run(k, st.cuda_stream) for k in kinds]
        torch.cuda.synchronize()
        for k, g in zip(kinds, got):
            w = want[k]
            if k in ("render", "batch"):
                assert torch.equal(g.view(torch.int32), w.view(torch.int32)), k
            else:  # fp64 sums: only the order of the atomics differs
                np.testing.assert_allclose(g.cpu().numpy(), w.cpu().numpy(), rtol=1e-9, atol=1e-13, err_msg=k)
    finally:
        torch.cuda.synchronize()
        for raw in raws:
            hip.hipStreamDestroy(raw)


def test_counter_grow_with_concurrent_launches_on_one_stream(scenes):
    """The chunk-counter buffer of a (scene, stream) is replaced by a larger
    one when a launch needs more words than it has (a scene batch of more
    than 16 sets).  Two host threads launch on ONE stream at once -- single
    renders and 20-set batches (ctypes releases the GIL, so the calls
    interleave) -- after a single render sized the buffer at 16 words: the
    replaced buffer stays alive for launches that took it before the grow
    (ADVICE r5), and every result equals the same launch alone."""
    import threading

    import torch

    from inverse_path_tracer_amd import _native as N

    L = N.lib()
    hip = C.CDLL("libamdhip64.so")
    P = product_scene(SCENE0)
    W, H, spp, mb, seed = 64, 48, 16, 4, 19
    S, stride = 20, W * H * spp
    kd = torch.from_numpy(np.random.RandomState(8).uniform(0, 1, (S, P.nT, 3)).astype(np.float32)).cuda()
    p = N.make_params(W, H, spp, mb, seed)
    raws = []
    try:
        def single(st):
            o = torch.empty((H * W, 3), device="cuda")
            N.check(L.ipt_render_dev(P.handle, C.byref(p), kd[5].data_ptr(), o.data_ptr(), None, st))
            return o

        def batch(st):
            o = torch.empty((S, H * W, 3), device="cuda")
            N.check(L.ipt_render_batch_dev(P.handle, C.byref(p), S, stride, kd.data_ptr(), o.data_ptr(), st))
            return o

        raw, st = _stream(hip)
        raws.append(raw)
        want_single, want_batch = single(st.cuda_stream), batch(st.cuda_stream)
        torch.cuda.synchronize()
        raw, st = _stream(hip)
        raws.append(raw)
        s = st.cuda_stream
        first = single(s)  # sizes this stream's counters at 16 words
        outs = {"a": [], "b": []}
        errs = []

        def worker(key, fn, n):
            try:
                for _ in range(n):
                    outs[key].append(fn(s))
            except Exception as e:  # noqa: BLE001 (re-raised below)
                errs.append(e)

        ths = [threading.Thread(target=worker, args=("a", single, 8)),
               threading.Thread(target=worker, args=("b", batch, 3))]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        torch.cuda.synchronize()
        assert not errs, errs
        for o in [first] + outs["a"]:
            assert torch.equal(o.view(torch.int32), want_single.view(torch.int32))
        for o in outs["b"]:
            assert torch.equal(o.view(torch.int32), want_batch.view(torch.int32))
    finally:
        torch.cuda.synchronize()
        P.close()
        for raw in raws:
            hip.hipStreamDestroy(raw)


def test_counter_reset_over_launch_shapes(scenes, oracle):
    """The chunk counters reset themselves only if the host's count of a
    launch's grabs (ipt_hip.hip launch_grabs) equals what the kernel's waves
    do.  Launches of many shapes -- ragged frames, tiny and wide, fused
    renders with 1..16-pixel groups, the unfused fallbacks (spp > 256, < 32
    samples per group), row shares, bounded and unbounded adjoints, the BVH
    instance's guided chunks -- run back to back on ONE stream into
    NaN-filled buffers, each equal to the same launch on a fresh stream: a
    counter left non-zero would make the next launch skip chunks."""
    import torch

    from conftest import NORTHSTAR
    from inverse_path_tracer_amd import _native as N

    L = N.lib()
    hip = C.CDLL("libamdhip64.so")
    ns = product_scene(NORTHSTAR)
    objs = {"cornell": scenes["cornell"][0], "scene0": scenes["scene0"][0], "northstar": ns}
    shapes = [("cornell", 1, 1, 1, 4), ("cornell", 7, 3, 5, 2), ("scene0", 33, 17, 64, 4), ("scene0", 100, 9, 100, None),
              ("cornell", 13, 31, 256, 4), ("scene0", 5, 4, 300, 4), ("cornell", 16, 8, 2, 4), ("scene0", 64, 64, 16, 8),
              ("northstar", 21, 19, 16, 4), ("northstar", 40, 8, 64, None), ("cornell", 129, 1, 3, 4),
              ("scene0", 2, 77, 33, None), ("northstar", 3, 3, 1, 2)]
    raws = []
    try:
        raw, st_shared = _stream(hip)
        raws.append(raw)
        runs = []
        for name, W, H, spp, mb in shapes:
            for rows in ((0, H, 1), (H // 3, H, 2)):
                p = N.make_params(W, H, spp, mb, 11 + W, *rows)
                np_ = ((rows[1] - rows[0] + rows[2] - 1) // rows[2]) * W
                adj = torch.from_numpy(np.random.RandomState(W).uniform(-1, 1, (H, W, 3)).astype(np.float32)).cuda()
                for kind in ("render", "adjoint"):
                    def go(st, kind=kind, p=p, np_=np_, adj=adj, sc=objs[name]):
                        if kind == "render":
                            o = torch.full((max(np_, 1), 3), float("nan"), device="cuda")
                            N.check(L.ipt_render_dev(sc.handle, C.byref(p), None, o.data_ptr(), None, st))
                        else:
                            o = torch.zeros((sc.nT, 3), device="cuda", dtype=torch.float64)
                            N.check(L.ipt_adjoint_dev(sc.handle, C.byref(p), None, adj.data_ptr(), o.data_ptr(), st))
                        return o
                    runs.append(((name, W, H, spp, mb, rows, kind), go, np_))
        got = [go(st_shared.cuda_stream) for _, go, _ in runs]
        torch.cuda.synchronize()
        for (key, go, np_), g in zip(runs, got):
            raw, st = _stream(hip)
            raws.append(raw)
            w = go(st.cuda_stream)
            torch.cuda.synchronize()
            if key[-1] == "render":
                assert not torch.isnan(g[:np_]).any(), key
                assert torch.equal(g.view(torch.int32), w.view(torch.int32)), key
            else:
                np.testing.assert_allclose(g.cpu().numpy(), w.cpu().numpy(), rtol=1e-9, atol=1e-13, err_msg=str(key))
    finally:
        torch.cuda.synchronize()
        ns.close()
        for raw in raws:
            hip.hipStreamDestroy(raw)


def test_failed_launch_leaves_the_stream_usable(scenes):
    """A launch that fails after its chunk counters and scratch are allocated
    (ipt_debug_fail_launches: the error comes just before the kernel is
    enqueued) changes nothing a later launch on the stream depends on: the
    next render, adjoint and unbounded adjoint on the same stream (the host
    wrappers' null stream) equal the oracle."""
    import oracle_lib
    from inverse_path_tracer_amd import _native as N

    L = N.lib()
    P, Q = scenes["scene0"]
    W, H, spp, mb, seed = 64, 48, 8, 4, 31
    adj = np.random.RandomState(2).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    for kind in ("render", "adjoint", "adjoint_u"):
        b = None if kind == "adjoint_u" else mb
        L.ipt_debug_fail_launches(1)
        try:
            with pytest.raises(N.NativeError, match="on request"):
                if kind == "render":
                    P.render(W, H, spp, b, seed)
                else:
                    P.adjoint(adj, W, H, spp, b, seed)
        finally:
            L.ipt_debug_fail_launches(0)
        if kind == "render":
            hdr = P.render(W, H, spp, b, seed)
            s, _ = Q.render_samples(W, H, spp, b, seed)
            hq, _ = oracle_lib.pixel_mean(s, W * H, spp)
            assert np.array_equal(bits(hdr.reshape(-1, 3)), bits(hq))
        else:
            g = P.adjoint(adj, W, H, spp, b, seed)
            want = Q.adjoint(W, H, spp, b, seed, adj)
            np.testing.assert_allclose(g, want, rtol=1e-9, atol=1e-12)


_TINY_POOL_WANT = {}


@pytest.mark.parametrize("pool,lds", [(1, 1), (2, 1), (3, 2), (1, 4)])
def test_unbounded_adjoint_with_tiny_record_pools(scenes, oracle, pool, lds):
    """The unbounded adjoint's ring forced small with
    ipt_debug_adju_ring: `pool` 16-slot chunks per wave and `lds` LDS slots
    per lane.  Lanes then find the pool empty and make their current slot
    count their ring size (1 or 17 slots...), so long paths replay from their
    camera rays chunk by chunk -- paths the default sizes almost never take.
    The gradient equals the oracle's (rtol 1e-9), on scenes/0 and the
    north-star (BVH instance)."""
    from inverse_path_tracer_amd import _native as N

    from conftest import NORTHSTAR

    L = N.lib()
    adj = np.random.RandomState(4).uniform(-1, 1, (40, 48, 3)).astype(np.float32)
    if "northstar" not in scenes:
        scenes["northstar"] = (product_scene(NORTHSTAR), oracle.OracleScene(NORTHSTAR))
    for name in ("scene0", "northstar"):
        P, Q = scenes[name]
        L.ipt_debug_adju_ring(pool, lds)
        try:
            g = P.adjoint(adj, 48, 40, 8, None, 77)
        finally:
            L.ipt_debug_adju_ring(0, 0)
        if name not in _TINY_POOL_WANT:
            _TINY_POOL_WANT[name] = Q.adjoint(48, 40, 8, None, 77, adj)
        np.testing.assert_allclose(g, _TINY_POOL_WANT[name], rtol=1e-9, atol=1e-12, err_msg=name)


def test_adjoint_row_bands_sum_to_full(scenes):
    from inverse_path_tracer_amd.distributed import shard_rows

    P, _ = scenes["scene0"]
    adj = np.random.RandomState(4).uniform(-1, 1, (128, 128, 3)).astype(np.float32)
    full = P.adjoint(adj, 128, 128, 16, 4, 0)
    parts = sum(P.adjoint(adj, 128, 128, 16, 4, 0, *shard_rows(128, 4, r)) for r in range(4))
    np.testing.assert_allclose(parts, full, rtol=1e-10)


def _loss(P, kd, adj, W, H, spp, mb, seed):
    P.materials = kd
    return float((adj.astype(np.float64) * P.render(W, H, spp, mb, seed).astype(np.float64)).sum())


def test_adjoint_fd_at_c3_size(scenes):
    """BASELINE config C3 (scenes/0.txt, 512x512x64, 4 bounces): gradient vs
    central differences of the GPU forward under common random numbers."""
    P, _ = scenes["scene0"]
    W = H = 512
    spp, mb, seed = 64, 4, 0
    kd0 = P.materials
    adj = np.ones((H, W, 3), np.float32)
    g = P.adjoint(adj, W, H, spp, mb, seed)
    h = 1e-2
    for t, c in [(0, 0), (8, 1), (12, 2), (14, 0), (19, 1), (25, 0)]:
        kp, km = kd0.copy(), kd0.copy()
        kp[t, c] += h
        km[t, c] -= h
        fd = (_loss(P, kp, adj, W, H, spp, mb, seed) - _loss(P, km, adj, W, H, spp, mb, seed)) / (2 * h)
        assert abs(fd - g[t, c]) <= 1e-3 * abs(g[t, c]) + 1e-2, (t, c, fd, g[t, c])
    P.materials = kd0


def test_adjoint_linear_in_adjoint_image(scenes):
    P, _ = scenes["scene0"]
    a1 = np.random.RandomState(1).uniform(-1, 1, (256, 256, 3)).astype(np.float32)
    a2 = np.random.RandomState(2).uniform(-1, 1, (256, 256, 3)).astype(np.float32)
    g1 = P.adjoint(a1, 256, 256, 16, 4, 0)
    g2 = P.adjoint(a2, 256, 256, 16, 4, 0)
    g12 = P.adjoint(a1 + a2, 256, 256, 16, 4, 0)
    np.testing.assert_allclose(g12, g1 + g2, rtol=1e-4, atol=1e-6 * np.abs(g1).max())


def test_torch_autograd_op(scenes, oracle):
    from inverse_path_tracer_amd import torch_ops

    P, Q = scenes["scene0"]
    kd = torch.tensor(P.materials, device="cuda", requires_grad=True)
    img = torch_ops.render(P, kd, 40, 40, 8, 4, 12)
    s, _ = Q.render_samples(40, 40, 8, 4, 12)
    hq, _ = oracle.pixel_mean(s, 1600, 8)
    assert np.array_equal(bits(img.detach().cpu().numpy().reshape(-1, 3)), bits(hq))
    adj = torch.rand((40, 40, 3), device="cuda") - 0.5
    (img * adj).sum().backward()
    np.testing.assert_allclose(kd.grad.double().cpu().numpy(), Q.adjoint(40, 40, 8, 4, 12, adj.cpu().numpy()),
                               rtol=1e-5, atol=1e-9)
    # band render through autograd
    kd2 = torch.tensor(P.materials, device="cuda", requires_grad=True)
    band = torch_ops.render(P, kd2, 40, 40, 8, 4, 12, 10, 25)
    (band * adj[10:25]).sum().backward()
    want = Q.adjoint(40, 40, 8, 4, 12, adj.cpu().numpy(), 10, 25)
    np.testing.assert_allclose(kd2.grad.double().cpu().numpy(), want, rtol=1e-5, atol=1e-9)


# ------------------------------------------------------------- graph
@pytest.mark.parametrize("W,H,spp,mb,seed", [(64, 64, 8, None, 5), (50, 40, 4, 3, 1)])
def test_graph_matches_oracle(scenes, W, H, spp, mb, seed):
    P, Q = scenes["scene0"]
    tgt = np.random.RandomState(seed).randint(0, 256, (H, W, 3)).astype(np.uint8)
    acc, data = P.graph(tgt, W, H, spp, mb, seed)
    acc_q, data_q = Q.graph(W, H, spp, mb, seed, tgt)
    np.testing.assert_allclose(acc, acc_q, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(data, data_q, rtol=1e-6, atol=1e-7)


# ------------------------------------------------------------- legacy drop-in
def test_legacy_ipt_cuda_pipeline(oracle, tmp_path, monkeypatch):
    """generate_data / render_with_materials through the reference's module
    surface, at a small legacy configuration."""
    from inverse_path_tracer_amd import _native as N
    from inverse_path_tracer_amd import ipt_cuda as M
    from inverse_path_tracer_amd import png_read, png_write

    assets = os.path.join(os.path.dirname(TESTS), "assets")
    monkeypatch.chdir(assets)  # scene files hold CWD-relative paths, like the reference
    N.lib().ipt_legacy_config(64, 64, 8, -1, 77)
    try:
        tgt = np.random.RandomState(3).randint(0, 256, (64, 64, 3)).astype(np.uint8)
        tpath = str(tmp_path / "t.png")
        png_write(tpath, tgt)
        w, pixel, light, labels = M.generate_data("scenes/0.txt", tpath)
        Q = oracle.OracleScene(SCENE0)
        _, data_q = Q.graph(64, 64, 8, None, 77, tgt)
        size = 31 * 30
        np.testing.assert_allclose(w, data_q[:size].reshape(31, 30), rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(pixel, data_q[size:4 * size].reshape(31, 30, 3), rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(labels, Q.get_materials())
        kd = np.random.RandomState(4).uniform(0, 1, (30, 3)).astype(np.float32)
        out = str(tmp_path / "r.png")
        M.render_with_materials("scenes/0.txt", out, torch.from_numpy(kd))
        Q.set_materials(kd)
        _, u8, _ = Q.render(64, 64, 8, None, 77)
        assert np.array_equal(png_read(out), u8)
        with pytest.raises(N.NativeError, match="expected 64x64"):
            small = str(tmp_path / "small.png")
            png_write(small, tgt[:32])
            M.generate_data("scenes/0.txt", small)
    finally:
        N.lib().ipt_legacy_config(500, 500, 100, -1, -1)


def test_statistical_kat_full_reference_config(scenes):
    """The reference's own configuration (500x500, 100 spp, unbounded) vs
    preds/0_true.png: region means within 1 level, mean |diff| at the MC-noise
    level of two independent reference renders (3.5)."""
    from inverse_path_tracer_amd import png_read

    P, _ = scenes["scene0"]
    _, u8 = P.render(500, 500, 100, None, 31337, ldr=True)
    g = json.load(open(os.path.join(TESTS, "golden", "preds_0_true_stats.json")))
    from test_oracle import region_means

    for k, v in region_means(u8, 1.0).items():
        assert np.abs(v - np.array(g["regions"][k])).max() < (1.0 if k != "cube_front" else 1.5), k
    ref = png_read(os.path.join(TESTS, "golden", "preds_0_true.png")).astype(np.float64)
    noise = np.abs(u8.astype(np.float64) - ref).mean()
    assert abs(noise - g["noise_mean_abs_true_vs_pred"]) < 0.3
    blocks = u8.astype(np.float64).reshape(50, 10, 50, 10, 3).mean(axis=(1, 3))
    assert np.abs(blocks - np.array(g["block10_means"])).mean() < 0.6


def test_sample_major_buffer_and_mean(scenes, oracle):
    """ipt_render_dev's internal layout: [s][pixel][3] samples, coalesced mean."""
    from inverse_path_tracer_amd import _native as N

    P, Q = scenes["scene0"]
    W, H, spp = 40, 24, 8
    p = N.make_params(W, H, spp, 4, 17, 4, 20)
    npix = (p.row_end - p.row_begin) * W
    buf = torch.empty((spp, npix, 3), device="cuda")
    hdr = torch.empty((npix, 3), device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    N.check(N.lib().ipt_render_samples_sm_dev(P.handle, C.byref(p), None, buf.data_ptr(), st))
    N.check(N.lib().ipt_pixel_mean_sm_dev(buf.data_ptr(), npix, spp, hdr.data_ptr(), None, st))
    torch.cuda.synchronize()
    want, _ = Q.render_samples(W, H, spp, 4, 17, 4 * W * spp, 20 * W * spp)
    got = buf.permute(1, 0, 2).contiguous().cpu().numpy().reshape(-1, 3)
    assert np.array_equal(bits(got), bits(want))
    hq, _ = oracle.pixel_mean(want, npix, spp)
    assert np.array_equal(bits(hdr.cpu().numpy()), bits(hq))


@pytest.mark.parametrize("W,H,spp,rows", [(512, 512, 64, None), (333, 97, 7, (13, 90))])
def test_sample_major_equals_pixel_major_at_c2_size(scenes, W, H, spp, rows):
    """The two sample layouts hold the same bits (work enumeration does not
    change any sample), at the bench's full C2 size and on an odd band."""
    from inverse_path_tracer_amd import _native as N

    P, _ = scenes["cornell"]
    p = N.make_params(W, H, spp, 4, 99, *(rows or (0, H)))
    npix = (p.row_end - p.row_begin) * W
    a = torch.empty((npix, spp, 3), device="cuda")
    b = torch.empty((spp, npix, 3), device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    N.check(N.lib().ipt_render_samples_dev(P.handle, C.byref(p), None, a.data_ptr(), st))
    N.check(N.lib().ipt_render_samples_sm_dev(P.handle, C.byref(p), None, b.data_ptr(), st))
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int32), b.permute(1, 0, 2).contiguous().view(torch.int32))


def test_material_recovery_c5_small():
    """C5 in miniature: Adam through the adjoint recovers the cube's albedo."""
    import os

    from inverse_path_tracer_amd import torch_ops
    from inverse_path_tracer_amd.optimize import build_tasks, optimize

    assets = os.path.join(os.path.dirname(TESTS), "assets", "scenes")
    tasks = build_tasks([os.path.join(assets, "0.txt"), os.path.join(assets, "1.txt")], 64, 64, 256, 4, 0.5,
                        torch.device("cuda"))
    # only triangles the image constrains can be recovered (the cube's back and
    # bottom faces never reach the camera): observability = |dL/dKd| at the start
    masks = []
    for t in tasks:
        img = torch_ops.render(t.scene, t.kd, 64, 64, 64, 4, seed=5)
        ((img - t.target) ** 2).mean().backward()
        g = t.kd.grad.abs().sum(1)[18:]
        masks.append(g > 0.25 * float(g.max()))
        t.kd.grad = None
    err0 = [float((t.kd.detach() - t.truth)[18:][m].abs().mean()) for t, m in zip(tasks, masks)]
    optimize(tasks, 64, 64, 16, 4, steps=60, lr=2e-2)
    for t, e0, m in zip(tasks, err0, masks):
        assert int(m.sum()) >= 2
        assert t.history[-1] < 0.5 * t.history[0]
        err = float((t.kd.detach() - t.truth)[18:][m].abs().mean())
        assert err < 0.5 * e0, (err, e0)


def test_math_cores_bit_exact_on_device():
    """The in-range sqrt/division cores used by the kernels equal the IEEE
    operations bit for bit across their whole operand ranges (csrc
    math_selftest_kernel: 2^24 random operand sets per test)."""
    from inverse_path_tracer_amd import _native as N

    counts = (C.c_uint64 * 8)()
    N.check(N.lib().ipt_selftest_math(1 << 24, 12345, counts))
    c = list(counts)
    names = ["sqrt_core", "dsqrt_core", "div_inrange", "div_hit_range", "div3_core", "unit", "unit_fast_hits",
             "div_camera"]
    bad = {n: v for n, v in zip(names, c) if v and n != "unit_fast_hits"}
    assert not bad, bad
    assert 0.2 * (1 << 24) < c[6] < 0.95 * (1 << 24)  # both unit() paths exercised


def test_c1_golden_vectors_on_device():
    """BASELINE config C1 on the GPU equals the committed oracle golden vectors
    bit for bit (HDR and tonemapped u8)."""
    g = np.load(os.path.join(TESTS, "golden", "c1_cornell_128x128x8_b2_seed0.npz"))
    P = product_scene(CORNELL)
    hdr, u8 = P.render(128, 128, 8, 2, 0, ldr=True)
    assert np.array_equal(bits(hdr), bits(g["hdr"]))
    assert np.array_equal(u8, g["ldr"])


def _one_triangle_obj(tmp_path, name="tri.obj", z=0.0):
    p = tmp_path / name
    p.write_text("v -0.4 -0.3 %g\nv 0.5 -0.2 %g\nv 0.1 0.45 %g\nf 1 2 3\n" % (z, z + 0.1, z - 0.05))
    return str(p)


@pytest.mark.parametrize("extra_cubes", [0, 2])
def test_odd_triangle_counts_bit_exact(oracle, tmp_path, extra_cubes):
    """Odd nT exercises the zero-triangle padding of the last TriPair: nT = 19
    (unrolled small-scene loop) and nT = 43 (generic pair loop, LDS tables)."""
    recs = CORNELL + [((0.2, -0.6, 3.6), (0.3, 0.2, 0.1), (1, 1, 1), _one_triangle_obj(tmp_path), "*Kd 0.7 0.2 0.4*")]
    for i in range(extra_cubes):
        recs.append(((-0.5 + i, -1.5, 4.2 + 0.3 * i), (0, 0.4 * i, 0), (0.5, 0.5, 0.5), CUBE_OBJ, "*Kd 0.3 0.8 0.5*"))
    P, Q = product_scene(recs), oracle.OracleScene(recs)
    assert P.nT == 19 + 12 * extra_cubes and P.nT % 2 == 1
    got = P.render_samples(40, 32, 6, 4, 21)
    want, _ = Q.render_samples(40, 32, 6, 4, 21)
    assert np.array_equal(bits(got), bits(want))
    adj = np.random.RandomState(5).uniform(-1, 1, (32, 40, 3)).astype(np.float32)
    np.testing.assert_allclose(P.adjoint(adj, 40, 32, 6, 4, 21), Q.adjoint(40, 32, 6, 4, 21, adj), rtol=1e-9,
                               atol=1e-12)


def test_large_scene_adjoint_and_graph(oracle):
    """nT = 1298 (sphere): no LDS kd tables (nT > 512) in the adjoint sweep and
    global-memory graph bins (> 64 KB)."""
    recs = CORNELL + [((0.3, -1.2, 4.2), (0.0, 0.4, 0.0), (1.2, 1.2, 1.2), SPHERE_OBJ, "*Kd 0.2 0.6 0.3*")]
    P, Q = product_scene(recs), oracle.OracleScene(recs)
    W = H = 12
    adj = np.random.RandomState(8).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    np.testing.assert_allclose(P.adjoint(adj, W, H, 3, 3, 4), Q.adjoint(W, H, 3, 3, 4, adj), rtol=1e-9, atol=1e-12)
    tgt = np.random.RandomState(9).randint(0, 256, (H, W, 3)).astype(np.uint8)
    acc, data = P.graph(tgt, W, H, 2, 3, 4)
    acc_q, data_q = Q.graph(W, H, 2, 3, 4, tgt)
    np.testing.assert_allclose(acc, acc_q, rtol=1e-9, atol=1e-12)
    np.testing.assert_allclose(data, data_q, rtol=1e-6, atol=1e-7)


# ------------------------------------------------------------- triangle BVH
def _bvh_scene(recs):
    from test_bvh import CLUTTER_SCENE, SPHERE_SCENE  # noqa: F401

    P = product_scene(recs)
    assert P.bvh_info()["accel"] == "bvh"
    return P


def _rays(P, n_adv, n_rand, seed):
    from test_bvh import _adversarial_rays

    tris = P.triangles()
    cam_origin = P.camera()[:3, 3].astype(np.float64)
    rng = np.random.RandomState(seed)
    O, D = _adversarial_rays(tris, cam_origin, rng, n_adv)
    v = tris[:, 0:9].reshape(-1, 3)
    lo, hi = v.min(0), v.max(0)
    Or = rng.uniform(lo, hi, (n_rand, 3)).astype(np.float32)
    Dr = rng.normal(size=(n_rand, 3))
    Dr = (Dr / np.linalg.norm(Dr, axis=1, keepdims=True)).astype(np.float32)
    return np.concatenate([O, Or]), np.concatenate([D, Dr])


@pytest.mark.parametrize("which", ["sphere", "clutter"])
def test_bvh_closest_hit_equals_brute_force(oracle, which):
    """The device BVH cast returns the brute-force loop's hit bit-for-bit
    (index and t) on adversarial + random rays, and both equal the oracle."""
    from inverse_path_tracer_amd import _native as N
    from test_bvh import CLUTTER_SCENE, SPHERE_SCENE

    recs = SPHERE_SCENE if which == "sphere" else CLUTTER_SCENE
    P = _bvh_scene(recs)
    O, D = _rays(P, 20000, 400000, 3 if which == "sphere" else 4)
    P.set_accel(N.ACCEL_BVH)
    tb, ib = P.closest_hit(O, D)
    P.set_accel(N.ACCEL_BRUTE)
    tf, i_f = P.closest_hit(O, D)
    P.set_accel(N.ACCEL_AUTO)
    assert np.array_equal(ib, i_f)
    assert np.array_equal(bits(tb), bits(tf))
    assert (ib >= 0).mean() > 0.5
    Q = oracle.OracleScene(recs)
    tq, iq = Q.closest_hit(O[:60000], D[:60000])
    assert np.array_equal(iq, ib[:60000])
    hit = iq >= 0
    assert np.array_equal(bits(tq[hit]), bits(tb[:60000][hit]))


def test_bvh_shadow_query_equals_brute_force():
    """Shadow rays (target = an emitter triangle): the BVH's early-out answer
    "closest hit is the target, at t" equals the full brute-force search."""
    from inverse_path_tracer_amd import _native as N
    from test_bvh import SPHERE_SCENE

    P = _bvh_scene(SPHERE_SCENE)
    tris = P.triangles()
    emit = np.nonzero(tris[:, 56] >= 0)[0]
    assert len(emit) == 2
    rng = np.random.RandomState(12)
    n = 300000
    v = tris[:, 0:9].reshape(-1, 3, 3)
    src = rng.randint(0, P.nT, n)
    a, b = rng.uniform(0, 1, (2, n))
    flip = a + b > 1
    a[flip], b[flip] = 1 - a[flip], 1 - b[flip]
    O = v[src, 0] + a[:, None] * (v[src, 1] - v[src, 0]) + b[:, None] * (v[src, 2] - v[src, 0])
    tg = emit[rng.randint(0, 2, n)]
    a2, b2 = rng.uniform(0, 1, (2, n))
    flip = a2 + b2 > 1
    a2[flip], b2[flip] = 1 - a2[flip], 1 - b2[flip]
    pt = v[tg, 0] + a2[:, None] * (v[tg, 1] - v[tg, 0]) + b2[:, None] * (v[tg, 2] - v[tg, 0])
    D = pt - O
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    O, D = O.astype(np.float32), D.astype(np.float32)
    P.set_accel(N.ACCEL_BVH)
    tb, ib = P.closest_hit(O, D, targets=tg)
    P.set_accel(N.ACCEL_BRUTE)
    tf, i_f = P.closest_hit(O, D)
    P.set_accel(N.ACCEL_AUTO)
    vis_b, vis_f = ib == tg, i_f == tg
    assert np.array_equal(vis_b, vis_f)
    assert 0.05 < vis_f.mean() < 0.95
    assert np.array_equal(bits(tb[vis_b]), bits(tf[vis_f]))


def test_bvh_renders_equal_brute_force_and_oracle(oracle):
    """Forward samples, adjoint and graph of the clutter scene (3 objects,
    2 spheres): BVH == brute force bit-for-bit, and == the oracle."""
    from inverse_path_tracer_amd import _native as N
    from test_bvh import CLUTTER_SCENE

    P = _bvh_scene(CLUTTER_SCENE)
    Q = oracle.OracleScene(CLUTTER_SCENE)
    W, H, spp, mb, seed = 48, 40, 4, 4, 77
    got = P.render_samples(W, H, spp, mb, seed)
    want, _ = Q.render_samples(W, H, spp, mb, seed)
    assert np.array_equal(bits(got), bits(want))
    P.set_accel(N.ACCEL_BRUTE)
    big_f = P.render_samples(160, 128, 8, 4, 5)
    P.set_accel(N.ACCEL_BVH)
    big_b = P.render_samples(160, 128, 8, 4, 5)
    assert np.array_equal(bits(big_f), bits(big_b))
    adj = np.random.RandomState(3).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    np.testing.assert_allclose(P.adjoint(adj, W, H, spp, mb, seed), Q.adjoint(W, H, spp, mb, seed, adj),
                               rtol=1e-9, atol=1e-12)
    P.set_accel(N.ACCEL_AUTO)


@pytest.mark.parametrize("which", ["cornell", "scene0"])
def test_culled_shadow_query_equals_brute_force(which):
    """Small scenes: the megakernel's culled shadow cast (target first, pairs
    skipped by acceptance box over [1e-2, t_target]) answers "closest hit is
    the target, at t" exactly as the full brute-force loop, for shadow rays
    from points on every triangle (grazing ones included) and from random
    points inside the scene box, towards points on the emitters (edges and
    corners included)."""
    P = product_scene(CORNELL if which == "cornell" else SCENE0)
    tris = P.triangles()
    emit = np.nonzero(tris[:, 56] >= 0)[0]
    assert len(emit) >= 1
    rng = np.random.RandomState(21)
    n = 400000
    v = tris[:, 0:9].reshape(-1, 3, 3)

    def on_tri(idx, a, b):
        flip = a + b > 1
        a, b = np.where(flip, 1 - a, a), np.where(flip, 1 - b, b)
        return v[idx, 0] + a[:, None] * (v[idx, 1] - v[idx, 0]) + b[:, None] * (v[idx, 2] - v[idx, 0])

    src = rng.randint(0, P.nT, n)
    O = on_tri(src, *rng.uniform(0, 1, (2, n)))
    box = v.reshape(-1, 3)
    inside = rng.uniform(0, 1, n) < 0.2
    O[inside] = rng.uniform(box.min(0), box.max(0), (int(inside.sum()), 3))
    tg = emit[rng.randint(0, len(emit), n)]
    ab = rng.uniform(0, 1, (2, n))
    edge = rng.uniform(0, 1, n) < 0.3  # targets on or next to the emitter's edges and corners
    ab[:, edge] = np.round(ab[:, edge] * 4) / 4 + rng.normal(0, 1e-6, (2, int(edge.sum())))
    pt = on_tri(tg, np.clip(ab[0], 0, 1), np.clip(ab[1], 0, 1))
    D = pt - O
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    O, D = O.astype(np.float32), D.astype(np.float32)
    tc, ic = P.closest_hit(O, D, targets=tg)
    tf, i_f = P.closest_hit(O, D)
    vis_c, vis_f = ic == tg, i_f == tg
    assert np.array_equal(vis_c, vis_f)
    assert 0.05 < vis_f.mean() < 0.98
    assert np.array_equal(bits(tc[vis_c]), bits(tf[vis_f]))
    P.close()


@pytest.mark.parametrize("which", ["cornell", "scene0"])
def test_culled_path_cast_equals_brute_force(oracle, which):
    """Small scenes: the megakernel's culled path cast (a lane tests only the
    pairs whose acceptance box its ray enters, per-lane from the LDS copy)
    returns the full brute-force loop's hit bit-for-bit (index and t), and the
    oracle's: rays from points on every triangle in all directions (grazing
    included), adversarial rays at vertices and edges from the camera, and
    random rays inside the scene box."""
    recs = CORNELL if which == "cornell" else SCENE0
    P = product_scene(recs)
    tris = P.triangles()
    rng = np.random.RandomState(31)
    n = 300000
    v = tris[:, 0:9].reshape(-1, 3, 3)
    src = rng.randint(0, P.nT, n)
    a, b = rng.uniform(0, 1, (2, n))
    flip = a + b > 1
    a[flip], b[flip] = 1 - a[flip], 1 - b[flip]
    O = v[src, 0] + a[:, None] * (v[src, 1] - v[src, 0]) + b[:, None] * (v[src, 2] - v[src, 0])
    D = rng.normal(size=(n, 3))
    nrm = np.cross(v[src, 1] - v[src, 0], v[src, 2] - v[src, 0])
    graze = rng.uniform(0, 1, n) < 0.2  # directions within ~1e-3 of the triangle's plane
    Dg = D - (np.sum(D * nrm, 1) / np.sum(nrm * nrm, 1))[:, None] * nrm
    D[graze] = Dg[graze] + rng.normal(0, 1e-3, (int(graze.sum()), 3))
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    Oa, Da = _rays(P, 20000, 60000, 5)
    O = np.concatenate([O.astype(np.float32), Oa])
    D = np.concatenate([D.astype(np.float32), Da])
    tg = np.full(len(O), -1, np.int32)
    tc, ic = P.closest_hit(O, D, targets=tg)
    tf, i_f = P.closest_hit(O, D)
    assert np.array_equal(ic, i_f)
    assert np.array_equal(bits(tc), bits(tf))
    assert (ic >= 0).mean() > 0.4  # the Cornell box is open at the front
    Q = oracle.OracleScene(recs)
    tq, iq = Q.closest_hit(O[:60000], D[:60000])
    assert np.array_equal(iq, ic[:60000])
    hit = iq >= 0
    assert np.array_equal(bits(tq[hit]), bits(tc[:60000][hit]))
    P.close()


@pytest.mark.parametrize("which", ["northstar", "clutter"])
def test_tree_entry_culls_equal_brute_force(which):
    """BVH scenes: the tree's entry tests (bvh.cpp tree_cull) -- the bounding
    sphere of its triangles' acceptance regions and the source-plane skip of
    rays leaving a triangle with every tree triangle behind its plane (the
    sphere's own faces) -- return the full brute-force loop's hit bit-for-bit:
    bounce rays (targets -1) from points on every triangle, in all
    directions, grazing ones within 1e-3 of the plane and a fifth near the
    skip's threshold; rays from the room towards points just outside and
    inside the tree's bounding sphere; shadow rays with their source."""
    from inverse_path_tracer_amd import _native as N
    from conftest import NORTHSTAR
    from test_bvh import CLUTTER_SCENE, _shadow_rays

    P = product_scene(NORTHSTAR if which == "northstar" else CLUTTER_SCENE)
    assert P.bvh_info()["accel"] == "bvh"
    tris = P.triangles()
    v = tris[:, 0:9].reshape(-1, 3, 3).astype(np.float64)
    rng = np.random.RandomState(41)
    n = 300000
    src = rng.randint(0, P.nT, n)
    a, b = rng.uniform(0, 1, (2, n))
    flip = a + b > 1
    a[flip], b[flip] = 1 - a[flip], 1 - b[flip]
    O = v[src, 0] + a[:, None] * (v[src, 1] - v[src, 0]) + b[:, None] * (v[src, 2] - v[src, 0])
    nrm = np.cross(v[src, 1] - v[src, 0], v[src, 2] - v[src, 0])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    D = rng.normal(size=(n, 3))
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    kind = rng.uniform(0, 1, n)
    graze = kind < 0.25  # within ~1e-3 of the plane, either side
    Dg = D - np.sum(D * nrm, 1)[:, None] * nrm
    D[graze] = Dg[graze] + rng.normal(0, 1e-3, (int(graze.sum()), 3))
    near = (kind >= 0.25) & (kind < 0.45)  # cos to the face normal near the skip's threshold (~0.02-0.05)
    c = rng.uniform(0.0, 0.08, int(near.sum()))
    Dt = Dg[near] / np.maximum(np.linalg.norm(Dg[near], axis=1, keepdims=True), 1e-30)
    D[near] = Dt * np.sqrt(1 - c * c)[:, None] + nrm[near] * c[:, None]
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    # rays from the room aimed at points on and just off the objects (not the
    # Cornell box's 18 triangles): silhouettes and the bounding sphere's rim
    m = 100000
    box = v.reshape(-1, 3)
    Or = rng.uniform(box.min(0), box.max(0), (m, 3))
    k = rng.randint(18, P.nT, m)
    a2, b2 = rng.uniform(0, 1, (2, m))
    flip = a2 + b2 > 1
    a2[flip], b2[flip] = 1 - a2[flip], 1 - b2[flip]
    aim = v[k, 0] + a2[:, None] * (v[k, 1] - v[k, 0]) + b2[:, None] * (v[k, 2] - v[k, 0])
    aim += rng.normal(0, 0.03, (m, 3))
    Dr = aim - Or
    Dr /= np.linalg.norm(Dr, axis=1, keepdims=True)
    # rays from points on every triangle towards points on the objects, in
    # either hemisphere of the source: from faces with the whole tree behind
    # them, the backward ones do reach it (the skip needs dot(n_s, d) > 0)
    q = 60000
    s2 = rng.randint(0, P.nT, q)
    a3, b3 = rng.uniform(0, 1, (2, q))
    flip = a3 + b3 > 1
    a3[flip], b3[flip] = 1 - a3[flip], 1 - b3[flip]
    O2 = v[s2, 0] + a3[:, None] * (v[s2, 1] - v[s2, 0]) + b3[:, None] * (v[s2, 2] - v[s2, 0])
    k2 = rng.randint(18, P.nT, q)
    D2 = v[k2].mean(1) - O2
    D2 /= np.maximum(np.linalg.norm(D2, axis=1, keepdims=True), 1e-30)
    O = np.concatenate([O, Or, O2]).astype(np.float32)
    D = np.concatenate([D, Dr, D2]).astype(np.float32)
    S = np.concatenate([src, np.full(m, -1), s2]).astype(np.int32)
    tg = np.full(len(O), -1, np.int32)
    tc, ic = P.shadow_hit(O, D, tg, S)  # the megakernel's BVH path cast with the source triangle
    P.set_accel(N.ACCEL_BRUTE)
    tf, i_f = P.closest_hit(O, D)
    P.set_accel(N.ACCEL_AUTO)
    assert np.array_equal(ic, i_f)
    assert np.array_equal(bits(tc), bits(tf))
    # shadow rays with their source triangle (the sphere's faces towards the light included)
    Os, Ds, tgs, srcs, _, _ = _shadow_rays(tris, 300000, np.random.RandomState(43))
    tc, ic = P.shadow_hit(Os, Ds, tgs, srcs)
    P.set_accel(N.ACCEL_BRUTE)
    tf, i_f = P.closest_hit(Os, Ds)
    P.set_accel(N.ACCEL_AUTO)
    vis_c, vis_f = ic == tgs, i_f == tgs
    assert np.array_equal(vis_c, vis_f)
    assert np.array_equal(bits(tc[vis_c]), bits(tf[vis_f]))
    P.close()


@pytest.mark.parametrize("scale", [0.5, 3.0])
@pytest.mark.parametrize("which", ["northstar", "clutter", "scene0"])
def test_closest_hit_with_non_unit_directions(which, scale):
    """ipt_closest_hit / ipt_shadow_hit take caller directions of any length
    (ADVICE r5): the BVH scenes' tree-entry culls assume |d| = 1 (the
    megakernel's rays), so for other lengths the cast keeps only the box test
    and still returns the brute-force loop's hit bit-for-bit; small scenes'
    culled path cast likewise.  Rays from points on every triangle in all
    directions (with their source triangle) and rays from the room at the
    objects, directions scaled by 0.5 and 3."""
    from inverse_path_tracer_amd import _native as N
    from conftest import NORTHSTAR
    from test_bvh import CLUTTER_SCENE

    P = product_scene({"northstar": NORTHSTAR, "clutter": CLUTTER_SCENE, "scene0": SCENE0}[which])
    tris = P.triangles()
    v = tris[:, 0:9].reshape(-1, 3, 3).astype(np.float64)
    rng = np.random.RandomState(53)
    n = 200000
    src = rng.randint(0, P.nT, n)
    a, b = rng.uniform(0, 1, (2, n))
    flip = a + b > 1
    a[flip], b[flip] = 1 - a[flip], 1 - b[flip]
    O = v[src, 0] + a[:, None] * (v[src, 1] - v[src, 0]) + b[:, None] * (v[src, 2] - v[src, 0])
    D = rng.normal(size=(n, 3))
    m = 100000
    box = v.reshape(-1, 3)
    Or = rng.uniform(box.min(0), box.max(0), (m, 3))
    k = rng.randint(min(18, P.nT - 1), P.nT, m)
    Dr = v[k].mean(1) + rng.normal(0, 0.03, (m, 3)) - Or
    O = np.concatenate([O, Or]).astype(np.float32)
    D = np.concatenate([D, Dr])
    D = (D / np.linalg.norm(D, axis=1, keepdims=True) * scale).astype(np.float32)
    S = np.concatenate([src, np.full(m, -1)]).astype(np.int32)
    tg = np.full(len(O), -1, np.int32)
    if P.bvh_info()["accel"] == "bvh":
        tc, ic = P.shadow_hit(O, D, tg, S)  # the megakernel's path cast with its source triangle
        P.set_accel(N.ACCEL_BVH)
        tb, ib = P.closest_hit(O, D)
        P.set_accel(N.ACCEL_BRUTE)
        tf, i_f = P.closest_hit(O, D)
        P.set_accel(N.ACCEL_AUTO)
        assert np.array_equal(ib, i_f)
        assert np.array_equal(bits(tb), bits(tf))
    else:
        tc, ic = P.closest_hit(O, D, targets=tg)  # the culled path cast
        tf, i_f = P.closest_hit(O, D)
    assert np.array_equal(ic, i_f)
    assert np.array_equal(bits(tc), bits(tf))
    assert (i_f >= 0).mean() > 0.4
    P.close()


@pytest.mark.parametrize("which", ["cornell", "scene0", "northstar"])
def test_masked_shadow_query_equals_brute_force(which):
    """The megakernel's shadow cast with the static potential-occluder mask of
    its (source triangle, emitter) answers "closest hit is the target, at t"
    exactly as the full brute-force loop: origins on every triangle (shadow
    rays along the light's own plane included), targets on the emitters near
    their edges and corners (ties with the coplanar ceiling)."""
    from inverse_path_tracer_amd import _native as N
    from conftest import NORTHSTAR
    from test_bvh import _shadow_rays

    P = product_scene({"cornell": CORNELL, "scene0": SCENE0, "northstar": NORTHSTAR}[which])
    O, D, tg, src, _, _ = _shadow_rays(P.triangles(), 400000, np.random.RandomState(23))
    src[::7] = -1  # no mask for some: the plain culled cast
    tc, ic = P.shadow_hit(O, D, tg, src)  # BVH scenes: the large-triangle pre-pass with the masks
    P.set_accel(N.ACCEL_BRUTE)
    tf, i_f = P.closest_hit(O, D)
    P.set_accel(N.ACCEL_AUTO)
    vis_c, vis_f = ic == tg, i_f == tg
    assert np.array_equal(vis_c, vis_f)
    assert 0.05 < vis_f.mean() < 0.98
    assert np.array_equal(bits(tc[vis_c]), bits(tf[vis_f]))
    P.close()
