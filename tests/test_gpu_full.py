"""GPU parity at the BASELINE.json configurations themselves (run with -m gpu).

The CPU oracle (oracle/ipt_oracle.c, OpenMP) renders a whole C2 frame in ~2 s
on the box's 16 cores, so the configurations are checked at full size against
it instead of through self-consistency properties:

  * C2 forward (Cornell, 512x512, 64 spp, 4 bounces): every per-sample
    radiance bit-identical to the oracle;
  * C3 adjoint (scenes/0.txt, 512x512, 64 spp, 4 bounces): dL/dKd for a
    U(-1,1) adjoint image and an all-ones one, rtol 1e-9 (fp64 sums, order);
  * createGraph at the reference's own configuration (500x500, 100 spp,
    unbounded; scene.h:8-11, ipt_cuda.py:136-165) against the reference's
    golden target preds/0_true.png: fp64 bins rtol 1e-9, compressed floats
    rtol 1e-6;
  * C4 (scenes/0.txt, 1024x1024, 256 spp, 8 bounces, 8 row bands): every band
    bit-identical to the full frame, band 3 bit-identical to the oracle per
    sample, the 8 band adjoints summing to the full adjoint (the single-GPU
    emulation of the RCCL gradient reduce) and band 3's adjoint equal to the
    oracle's;
  * C5 (scenes/0..12.txt, 256x256, 32 spp, 4 bounces, Adam, one GPU's share of
    8): the scene batch equals per-scene launches, and >= 200 steps of one
    persistent optimiser recover the observable cube albedo.
"""
import os

import numpy as np
import pytest

from conftest import CORNELL, SCENE0, TESTS, product_scene

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
ROOT = os.path.dirname(TESTS)


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    yield


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def scene0(oracle):
    return product_scene(SCENE0), oracle.OracleScene(SCENE0)


# ------------------------------------------------------------- C2 / C3
def test_c2_forward_full_frame_bit_exact(oracle):
    P, Q = product_scene(CORNELL), oracle.OracleScene(CORNELL)
    got = P.render_samples(512, 512, 64, 4, 0)
    want, casts = Q.render_samples(512, 512, 64, 4, 0)
    assert got.shape == (512 * 512 * 64, 3)
    assert np.array_equal(bits(got), bits(want))
    # the roofline's casts/sample constant (profiles/casts_per_sample.json) is this frame's count
    assert abs(casts / (512 * 512 * 64) - 5.694429993629456) < 1e-9


@pytest.mark.parametrize("kind", ["uniform", "ones"])
def test_c3_adjoint_full_frame_matches_oracle(scene0, kind):
    P, Q = scene0
    W = H = 512
    adj = (np.random.RandomState(1).uniform(-1, 1, (H, W, 3)) if kind == "uniform" else np.ones((H, W, 3)))
    adj = adj.astype(np.float32)
    g = P.adjoint(adj, W, H, 64, 4, 0)
    want = Q.adjoint(W, H, 64, 4, 0, adj)
    np.testing.assert_allclose(g, want, rtol=1e-9, atol=1e-12 * np.abs(want).max())


def test_c3_unbounded_adjoint_full_frame_matches_oracle(scene0):
    """The adjoint of the reference's own estimator (scenes/0.txt, 512x512,
    64 spp, NO bounce cap: path_trace.cu:172-181) at full size."""
    P, Q = scene0
    adj = np.random.RandomState(3).uniform(-1, 1, (512, 512, 3)).astype(np.float32)
    g = P.adjoint(adj, 512, 512, 64, None, 0)
    want = Q.adjoint(512, 512, 64, None, 0, adj)
    np.testing.assert_allclose(g, want, rtol=1e-9, atol=1e-12 * np.abs(want).max())


def test_unbounded_adjoint_through_autograd_matches_fd(scene0):
    """torch_ops.render(max_bounces=None) backward vs central differences of
    the GPU forward under common random numbers."""
    from inverse_path_tracer_amd import torch_ops

    P, _ = scene0
    W = H = 64
    spp, seed = 16, 77
    kd0 = torch.tensor(P.materials, device="cuda")
    adj = torch.from_numpy(np.random.RandomState(9).uniform(-1, 1, (H, W, 3)).astype(np.float32)).cuda()
    kd = kd0.clone().requires_grad_(True)
    (torch_ops.render(P, kd, W, H, spp, None, seed) * adj).sum().backward()

    def loss(k):
        with torch.no_grad():
            return float((torch_ops.render(P, k, W, H, spp, None, seed).double() * adj.double()).sum())

    h = 1e-2
    for t, c in [(0, 0), (8, 1), (12, 2), (14, 0), (19, 1), (25, 0)]:
        kp, km = kd0.clone(), kd0.clone()
        kp[t, c] += h
        km[t, c] -= h
        fd = (loss(kp) - loss(km)) / (2 * h)
        assert abs(fd - float(kd.grad[t, c])) <= 2e-3 * max(1.0, abs(fd)), (t, c, fd, float(kd.grad[t, c]))


def test_graph_legacy_config_matches_oracle(scene0):
    """createGraph's configuration: 500x500, 100 spp, unbounded paths, the
    reference's own target image."""
    from inverse_path_tracer_amd import png_read

    P, Q = scene0
    tgt = png_read(os.path.join(TESTS, "golden", "preds_0_true.png"))
    acc, data = P.graph(tgt, 500, 500, 100, None, 31337)
    acc_q, data_q = Q.graph(500, 500, 100, None, 31337, tgt)
    np.testing.assert_allclose(acc, acc_q, rtol=1e-9, atol=1e-12 * np.abs(acc_q).max())
    np.testing.assert_allclose(data, data_q, rtol=1e-6, atol=1e-7)
    assert not np.isnan(data).any()


# ------------------------------------------------------------- C4
C4 = dict(W=1024, H=1024, spp=256, mb=8, seed=0)


def _bands(n=8):
    from inverse_path_tracer_amd.distributed import shard_rows

    return [shard_rows(C4["H"], n, r) for r in range(n)]


def test_c4_bands_equal_full_frame(scene0):
    P, _ = scene0
    a = (C4["W"], C4["H"], C4["spp"], C4["mb"], C4["seed"])
    full = P.render(*a)
    bands = [P.render(*a, b, e) for b, e in _bands()]
    assert [x.shape[0] for x in bands] == [128] * 8
    assert np.array_equal(bits(np.concatenate(bands)), bits(full))


def test_c4_band_samples_bit_exact_vs_oracle(scene0):
    P, Q = scene0
    b, e = _bands()[3]
    W, spp = C4["W"], C4["spp"]
    got = P.render_samples(W, C4["H"], spp, C4["mb"], C4["seed"], b, e)
    want, _ = Q.render_samples(W, C4["H"], spp, C4["mb"], C4["seed"], b * W * spp, e * W * spp)
    assert got.shape == (128 * 1024 * 256, 3)
    assert np.array_equal(bits(got), bits(want))


def test_c4_band_adjoints_sum_to_full_and_match_oracle(scene0):
    P, Q = scene0
    W, H = C4["W"], C4["H"]
    a = (W, H, C4["spp"], C4["mb"], C4["seed"])
    adj = np.random.RandomState(2).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    full = P.adjoint(adj, *a)
    parts = [P.adjoint(adj, *a, b, e) for b, e in _bands()]
    scale = np.abs(full).max()
    np.testing.assert_allclose(sum(parts), full, rtol=1e-10, atol=1e-10 * scale)
    b, e = _bands()[3]
    want = Q.adjoint(W, H, C4["spp"], C4["mb"], C4["seed"], adj, b, e)
    np.testing.assert_allclose(parts[3], want, rtol=1e-9, atol=1e-12 * np.abs(want).max())


def test_c4_interleaved_shares_equal_full_frame_and_sum_to_full_adjoint(scene0):
    """The bench's tile split: rank r traces rows r, r+8, ... (row_step = 8)."""
    P, _ = scene0
    W, H = C4["W"], C4["H"]
    a = (W, H, C4["spp"], C4["mb"], C4["seed"])
    full = P.render(*a)
    adj = np.random.RandomState(5).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    g_full = P.adjoint(adj, *a)
    g = 0
    for r in range(8):
        share = P.render(*a, r, H, row_step=8)
        assert share.shape == (128, W, 3)
        assert np.array_equal(bits(share), bits(full[r::8])), r
        g = g + P.adjoint(adj, *a, r, H, row_step=8)
    np.testing.assert_allclose(g, g_full, rtol=1e-10, atol=1e-10 * np.abs(g_full).max())


def test_interleaved_rows_through_autograd_match_oracle(scene0):
    """torch_ops.render with row_step: forward rows == the oracle's, and the
    backward (adjoint image scattered to global rows) == the oracle's adjoint
    summed over those rows."""
    from inverse_path_tracer_amd import torch_ops

    P, Q = scene0
    W, H, spp, mb, seed = 40, 37, 8, 4, 21
    rows = list(range(2, H, 3))
    kd = torch.tensor(P.materials, device="cuda", requires_grad=True)
    img = torch_ops.render(P, kd, W, H, spp, mb, seed, 2, H, row_step=3)
    assert img.shape == (len(rows), W, 3)
    full, _, _ = Q.render(W, H, spp, mb, seed)
    assert np.array_equal(bits(img.detach().cpu().numpy()), bits(full[rows]))
    adj = np.random.RandomState(6).uniform(-1, 1, (H, W, 3)).astype(np.float32)
    (img * torch.from_numpy(adj[rows]).cuda()).sum().backward()
    want = sum(Q.adjoint(W, H, spp, mb, seed, adj, r, r + 1) for r in rows)
    np.testing.assert_allclose(kd.grad.double().cpu().numpy(), want, rtol=1e-5, atol=1e-9)


# ------------------------------------------------------------- C5 scene batch
def test_scene_batch_equals_single_launches(scene0, oracle):
    """ipt_render_batch_dev / ipt_adjoint_batch_dev: set b == the single-scene
    launch with kd[b] and seed + b*stride (images bitwise, gradients rtol 1e-9),
    and one set == the oracle."""
    from inverse_path_tracer_amd import torch_ops

    P, Q = scene0
    W, H, spp, mb, seed = 48, 40, 8, 4, 123
    S, stride = 5, W * H * spp
    kd = torch.from_numpy(np.random.RandomState(0).uniform(0, 1, (S, P.nT, 3)).astype(np.float32)).cuda()
    kd.requires_grad_(True)
    adj = torch.from_numpy(np.random.RandomState(1).uniform(-1, 1, (S, H, W, 3)).astype(np.float32)).cuda()
    img = torch_ops.render_batch(P, kd, W, H, spp, mb, seed=seed, seed_stride=stride)
    (img * adj).sum().backward()
    for b in range(S):
        k1 = kd.detach()[b].clone().requires_grad_(True)
        one = torch_ops.render(P, k1, W, H, spp, mb, seed=seed + b * stride)
        assert torch.equal(one.view(torch.int32), img[b].detach().view(torch.int32)), b
        (one * adj[b]).sum().backward()
        np.testing.assert_allclose(kd.grad[b].double().cpu().numpy(), k1.grad.double().cpu().numpy(), rtol=1e-6,
                                   atol=1e-9)
    Q.set_materials(kd.detach()[2].cpu().numpy())
    hq, _, _ = Q.render(W, H, spp, mb, seed + 2 * stride)
    assert np.array_equal(bits(img[2].detach().cpu().numpy()), bits(hq))
    gq = Q.adjoint(W, H, spp, mb, seed + 2 * stride, adj[2].cpu().numpy())
    Q.set_materials(P.materials)
    # kd.grad is float32 (the op returns the parameter's dtype); compare at that precision
    np.testing.assert_allclose(kd.grad[2].double().cpu().numpy(), gq, rtol=1e-6, atol=1e-9)


def test_scene_batch_adjoint_fp64_matches_oracle(scene0):
    """The batched adjoint's fp64 output (before any cast) vs the oracle at rtol 1e-9."""
    import ctypes as C

    from inverse_path_tracer_amd import _native as N
    from inverse_path_tracer_amd import torch_ops  # noqa: F401

    P, Q = scene0
    W, H, spp, mb, seed = 64, 64, 16, 4, 9
    S, stride = 3, W * H * spp
    kd = np.random.RandomState(3).uniform(0, 1, (S, P.nT, 3)).astype(np.float32)
    adj = np.random.RandomState(4).uniform(-1, 1, (S, H, W, 3)).astype(np.float32)
    kd_t, adj_t = torch.from_numpy(kd).cuda(), torch.from_numpy(adj).cuda()
    g = torch.zeros((S, P.nT, 3), device="cuda", dtype=torch.float64)
    p = N.make_params(W, H, spp, mb, seed)
    N.check(N.lib().ipt_adjoint_batch_dev(P.handle, C.byref(p), S, stride, kd_t.data_ptr(), adj_t.data_ptr(),
                                          g.data_ptr(), torch.cuda.current_stream().cuda_stream))
    g = g.cpu().numpy()
    for b in range(S):
        Q.set_materials(kd[b])
        want = Q.adjoint(W, H, spp, mb, seed + b * stride, adj[b])
        np.testing.assert_allclose(g[b], want, rtol=1e-9, atol=1e-12 * np.abs(want).max())
    Q.set_materials(P.materials)


def test_c5_recovery_at_config():
    """BASELINE config C5 on one GPU's share (13 of 100 scenes): 256x256, 32 spp,
    4 bounces, Adam lr 1e-2, 240 steps of ONE persistent optimiser, adjoint on
    an independent sample stream.  The observable cube albedo error (triangles
    the image constrains) must drop by >= 50% in every scene, and the loss too."""
    from inverse_path_tracer_amd.optimize import MaterialOptimizer, build_tasks, observable_mask

    files = [os.path.join(ROOT, "assets", "scenes", "%d.txt" % i) for i in range(13)]
    tasks = build_tasks(files, 256, 256, 1024, 4, 0.5, torch.device("cuda"))
    assert len({id(t.scene) for t in tasks}) == 1  # one geometry: one batch
    masks = observable_mask(tasks, 256, 256, 64, 4)

    def err(t, m):
        return float((t.kd.detach() - t.truth)[18:][m].abs().mean())

    e0 = [err(t, m) for t, m in zip(tasks, masks)]
    opt = MaterialOptimizer(tasks, 256, 256, 32, 4, lr=1e-2)
    opt.run(240)
    for t, m, a in zip(tasks, masks, e0):
        assert int(m.sum()) >= 2
        assert len(t.history) == 240
        assert np.mean(t.history[-20:]) < 0.5 * t.history[0], t.path
        assert err(t, m) < 0.5 * a, (t.path, err(t, m), a)


def test_decorrelated_gradient_is_unbiased_at_low_spp():
    """with the adjoint on the forward's own samples the L2 gradient
    is E[(I-T) dI/dKd] = (E[I]-T) E[dI/dKd] + Cov(I, dI/dKd): the covariance
    term is a bias (positive: it pushes Kd down).  With an independent adjoint
    stream (adjoint_seed) the expected gradient is exactly (E[I]-T) E[dI/dKd].
    At the true albedo, 4 spp, 256 trials per estimator, observable cube
    triangles of scenes/0.txt: the decorrelated mean equals that expectation
    (estimated at 2^20 spp, independent seeds) within 4 standard errors; the
    same-stream mean does not."""
    from inverse_path_tracer_amd import torch_ops
    from inverse_path_tracer_amd.optimize import build_tasks, observable_mask

    W = H = 64
    spp, mb, trials, big = 4, 4, 256, 1 << 20
    (t,) = build_tasks([os.path.join(ROOT, "assets", "scenes", "0.txt")], W, H, big, mb, 0.5, torch.device("cuda"))
    t.kd = t.truth.clone()
    (m,) = observable_mask([t], W, H, 256, mb)
    # the expectation both estimators target: 2/N sum (E[I]-T) E[dI], from independent high-spp renders
    with torch.no_grad():
        ibar = torch_ops.render(t.scene, t.truth, W, H, big, mb, seed=(1 << 31) + 12345)
    kd = t.truth.clone().requires_grad_(True)
    img = torch_ops.render(t.scene, kd, W, H, 1 << 14, mb, seed=(3 << 30) + 777)
    (img * (2.0 * (ibar - t.target) / img.numel())).sum().backward()
    expect = float(kd.grad[18:][m].sum())
    stats = {}
    for dec in (True, False):
        vals = []
        for i in range(trials):
            kd = t.truth.clone().requires_grad_(True)
            seed = (i + 1) * W * H * spp
            img = torch_ops.render(t.scene, kd, W, H, spp, mb, seed=seed,
                                   adjoint_seed=seed + (trials + 1) * W * H * spp if dec else None)
            ((img - t.target) ** 2).mean().backward()
            vals.append(float(kd.grad[18:][m].sum()))
        v = np.array(vals)
        stats[dec] = (v.mean(), v.std(ddof=1) / np.sqrt(trials))
    print("gradient at the truth (observable cube Kd): expectation %.3e; decorrelated %.3e +- %.1e, "
          "same-stream %.3e +- %.1e" % ((expect,) + stats[True] + stats[False]))
    mu, se = stats[True]
    assert abs(mu - expect) < 4 * se
    mu_s, se_s = stats[False]
    assert mu_s - expect > 4 * se_s  # the bias the fix removes
