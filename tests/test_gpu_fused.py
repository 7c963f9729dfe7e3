"""The forward with the pixel mean fused into the trace kernel (gpu_render,
MODE_FWDM): each wave keeps a ring of one-pixel LDS slots and sums a pixel's
samples in sample order once its last one is in, so the HDR image (and its
8-bit tonemap) must be bit-identical to the oracle's toneMap over the
oracle's per-sample radiances (path_trace.cu:186-198) and to the unfused
two-kernel render (ipt_render_samples_sm_dev into a sample buffer +
ipt_pixel_mean_sm_dev).

Cases cover the group shapes gpu_render picks (p pixels per group, p * spp
<= 256, the ring holding 2 groups for <= 8 bounces and 4 otherwise): spp a
power of two (16-B LDS reads, multiply by 1/spp), spp not a power of two
(IEEE division), spp = 256 (one pixel per group), partial last groups (the
division path of the item split), long bounded paths and the reference's
own unbounded estimator (long Russian-roulette paths hold their pixel's slot
while the ring moves on), row bands and interleaved shares, the BVH
instance (two-kernel render) and the unfused fallback (spp > 256)."""
import numpy as np
import pytest

from conftest import CORNELL, NORTHSTAR, SCENE0, product_scene

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")


@pytest.fixture(scope="module", autouse=True)
def _device():
    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.set_device(0)
    yield


def bits(a):
    return np.ascontiguousarray(a, np.float32).view(np.uint32)


@pytest.fixture(scope="module")
def scenes(oracle):
    return {n: (product_scene(r), oracle.OracleScene(r)) for n, r in
            (("cornell", CORNELL), ("scene0", SCENE0), ("northstar", NORTHSTAR))}


def two_kernel(P, W, H, spp, mb, seed, row_begin=0, row_end=None):
    """The unfused render of the same rows: the per-sample kernel into a
    sample-major buffer, then the toneMap kernel (flattened HDR image)."""
    import ctypes as C

    from inverse_path_tracer_amd import _native as N

    L = N.lib()
    p = N.make_params(W, H, spp, mb, seed, row_begin, row_end)
    rows = (H if row_end is None else row_end) - row_begin
    samples = torch.empty((spp * rows * W, 3), device="cuda")
    hdr = torch.empty((rows * W, 3), device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    N.check(L.ipt_render_samples_sm_dev(P.handle, C.byref(p), None, samples.data_ptr(), st))
    N.check(L.ipt_pixel_mean_sm_dev(samples.data_ptr(), rows * W, spp, hdr.data_ptr(), None, st))
    return hdr.cpu().numpy().reshape(-1)


@pytest.mark.parametrize("name,W,H,spp,mb,seed", [
    ("cornell", 33, 17, 5, 4, 7),       # p = 16, spp odd (division); last chunk 1 pixel
    ("scene0", 31, 7, 64, 4, 3),        # p = 4 (the C2 shape); last chunk 1 pixel
    ("scene0", 37, 3, 48, 16, 2),       # 16 bounces (long paths: 4 groups in the ring); last group 3 pixels
    ("scene0", 29, 11, 48, 40, 12),     # 40 bounces
    ("scene0", 20, 10, 100, 2, 9),      # the reference's 100 spp: p = 2
    ("scene0", 9, 5, 256, 8, 1),        # p = 1
    ("northstar", 24, 20, 16, 4, 11),   # BVH instance, p = 16
    ("scene0", 16, 8, 2, 4, 4),         # unfused fallback: 8 pixels x 2 spp < 32 samples per group
    ("scene0", 16, 8, 8, None, 4),      # unbounded paths (the reference's estimator)
    ("cornell", 45, 23, 64, None, 6),   # unbounded, 64 spp: 8 slots, 2-pixel groups
    ("scene0", 31, 13, 100, None, 8),   # unbounded, the reference's 100 spp: 5 slots, 1-pixel groups
    ("scene0", 7, 3, 300, 4, 2),        # unfused fallback: spp > 256
])
def test_fused_render_equals_oracle_tonemap(scenes, oracle, name, W, H, spp, mb, seed):
    P, Q = scenes[name]
    hdr, u8 = P.render(W, H, spp, mb, seed, ldr=True)
    s, _ = Q.render_samples(W, H, spp, mb, seed)
    hq, uq = oracle.pixel_mean(s, W * H, spp)
    assert np.array_equal(bits(hdr.reshape(-1, 3)), bits(hq))
    assert np.array_equal(u8.reshape(-1, 3), uq)


def test_fused_c2_frame_equals_oracle_and_unfused(scenes, oracle):
    """The headline configuration (Cornell, 512x512, 64 spp, 4 bounces) at full
    size: the fused HDR frame == the oracle's toneMap == the two-kernel frame;
    the interleaved 1/8 share (the bench's tile split) == its rows."""
    P, Q = scenes["cornell"]
    hdr = P.render(512, 512, 64, 4, 0)
    want, _, _ = Q.render(512, 512, 64, 4, 0)
    assert np.array_equal(bits(hdr), bits(want))
    assert np.array_equal(bits(two_kernel(P, 512, 512, 64, 4, 0)), bits(hdr).reshape(-1))
    for r in (0, 5):
        share = P.render(512, 512, 64, 4, 0, r, 512, row_step=8)
        assert np.array_equal(bits(share), bits(hdr[r::8]))


def test_fused_unbounded_reference_config_equals_oracle(scenes, oracle):
    """The legacy createImage configuration (scenes/0.txt, 500x500, 100 spp,
    no bounce cap, path_trace.cu:200-234) through the fused ring: == the
    oracle's toneMap bitwise (HDR and 8-bit), with no per-sample buffer."""
    P, Q = scenes["scene0"]
    hdr, u8 = P.render(500, 500, 100, None, 77, ldr=True)
    want, uq, _ = Q.render(500, 500, 100, None, 77)
    assert np.array_equal(bits(hdr), bits(want))
    assert np.array_equal(u8, uq)


def test_fused_band_of_c4_shape(scenes):
    """C4's sample count per pixel (256 spp, 8 bounces: one pixel per chunk) on
    a band of a 1024-wide frame: fused == unfused, bitwise."""
    P, _ = scenes["scene0"]
    a = (1024, 1024, 256, 8, 0, 512, 520)
    assert np.array_equal(bits(P.render(*a)).reshape(-1), bits(two_kernel(P, *a)))


def test_fused_render_batch_equals_single(scenes):
    """ipt_render_batch_dev through the fused kernel: set b == the single-scene
    fused launch with that kd and seed (each set writes its own HDR image)."""
    from inverse_path_tracer_amd import torch_ops

    P, _ = scenes["scene0"]
    W, H, spp, mb, seed, stride = 40, 24, 32, 4, 17, 1 << 20
    kd0 = torch.tensor(P.materials, device="cuda:0")
    kd = torch.stack([kd0 * (0.5 + 0.25 * b) for b in range(3)])
    img = torch_ops.render_batch(P, kd, W, H, spp, mb, seed=seed, seed_stride=stride)
    for b in range(3):
        one = torch_ops.render(P, kd[b].clone(), W, H, spp, mb, seed=seed + b * stride)
        assert torch.equal(img[b], one)
