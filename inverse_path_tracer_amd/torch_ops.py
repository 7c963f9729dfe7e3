"""PyTorch-ROCm autograd op over the HIP kernels.

``render(scene, kd, ...)`` returns the HDR image (rows, W, 3) rendered with
per-triangle diffuse albedo ``kd`` (nT, 3) on the GPU; its backward runs the
adjoint kernel (path replay under common random numbers) and
returns dLoss/dkd.  PyTorch only provides device memory and the stream; all
compute is libipt_amd.so (there is no fallback).
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _native as N
from .scene import Scene


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def render_into(scene: Scene, params: N.Params, kd: torch.Tensor, hdr: torch.Tensor):
    """Forward kernels on torch's current stream, into a preallocated image."""
    N.check(N.lib().ipt_render_dev(scene.handle, C.byref(params), kd.data_ptr() if kd is not None else None,
                                   hdr.data_ptr(), None, _stream(hdr.device)), "ipt_render_dev")
    return hdr


def adjoint_into(scene: Scene, params: N.Params, kd: torch.Tensor, adj_full: torch.Tensor, grad: torch.Tensor):
    """Accumulate d(sum adj*I)/dkd (fp64, nT*3) for rows [row_begin,row_end).
    ``adj_full`` is indexed by global pixel: pass the full (H, W, 3) image or a
    band pointer offset by row_begin*W*3 (see adjoint_band)."""
    N.check(N.lib().ipt_adjoint_dev(scene.handle, C.byref(params), kd.data_ptr() if kd is not None else None,
                                    adj_full, grad.data_ptr(), _stream(grad.device)), "ipt_adjoint_dev")
    return grad


def adjoint_band(scene: Scene, params: N.Params, kd, adj_band: torch.Tensor, grad: torch.Tensor):
    """Adjoint for a launch whose adjoint image holds only its own rows."""
    adj_band = adj_band.contiguous()
    if params.row_step > 1:  # interleaved rows: scatter into a full-frame image
        full = torch.zeros((params.height, params.width, 3), device=adj_band.device, dtype=torch.float32)
        full[params.row_begin:params.row_end:params.row_step] = adj_band
        return adjoint_into(scene, params, kd, full.data_ptr(), grad)
    base = adj_band.data_ptr() - params.row_begin * params.width * 3 * 4  # global-pixel indexing
    return adjoint_into(scene, params, kd, base, grad)


class _RenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kd, scene, params, adjoint_seed):
        kd_c = kd.detach().contiguous().float()
        hdr = torch.empty((params.rows, params.width, 3), device=kd.device, dtype=torch.float32)
        render_into(scene, params, kd_c, hdr)
        ctx.scene, ctx.params, ctx.adjoint_seed = scene, params, adjoint_seed
        ctx.save_for_backward(kd_c)
        return hdr

    @staticmethod
    def backward(ctx, grad_hdr):
        (kd_c,) = ctx.saved_tensors
        g = torch.zeros(kd_c.shape, device=kd_c.device, dtype=torch.float64)
        adjoint_band(ctx.scene, _replay_params(ctx.params, ctx.adjoint_seed), kd_c, grad_hdr.float(), g)
        return g.to(kd_c.dtype), None, None, None


def _replay_params(p: N.Params, adjoint_seed):
    """The adjoint's parameters: the forward's (common random numbers: the
    exact derivative of the returned image), or the same configuration on an
    independent sample stream (adjoint_seed: an unbiased estimate of the
    derivative of the expected image, uncorrelated with the forward's noise)."""
    if adjoint_seed is None:
        return p
    return N.Params(p.width, p.height, p.spp, p.max_bounces, int(adjoint_seed) & 0xFFFFFFFFFFFFFFFF, p.row_begin,
                    p.row_end, p.row_step)


def render(scene: Scene, kd: torch.Tensor, width: int, height: int, spp: int, max_bounces=4, seed: int = 0,
           row_begin: int = 0, row_end=None, adjoint_seed=None, row_step: int = 1) -> torch.Tensor:
    """Differentiable render: HDR image of rows row_begin, row_begin + row_step,
    ... < row_end w.r.t. kd.  max_bounces None is the reference's own
    estimator (paths end by Russian roulette or a miss); its adjoint keeps
    the vertex records in an LDS ring and replays long paths chunk by chunk.

    The backward pass replays the forward's paths (adjoint_seed None) or
    traces the same configuration with seed `adjoint_seed`.  The second form
    is what an optimiser of E[loss] wants: with the forward's own samples the
    gradient of (I - T)^2 correlates the residual with the derivative, a bias
    of order 1/spp towards darker albedo.

    Choose `adjoint_seed` so that its samples' seeds (adjoint_seed + global
    sample index) differ from the forward's in the LOW 32 bits, e.g. the
    next frame: seed + W*H*spp.  curand_init's XORWOW set-up hashes the two
    32-bit halves of a seed separately, so seeds equal mod 2^32 share three
    of the five state words and their first draws differ only by a constant
    -- correlated streams (measured: a residual bias of ~14% of the
    same-stream one, tests/test_gpu_full.py)."""
    p = N.make_params(width, height, spp, max_bounces, seed, row_begin, row_end, row_step)
    return _RenderFn.apply(kd, scene, p, adjoint_seed)


class _BatchRenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kd, scene, params, stride, adjoint_seed):
        kd_c = kd.detach().contiguous().float()
        S = kd_c.shape[0]
        hdr = torch.empty((S, params.height, params.width, 3), device=kd.device, dtype=torch.float32)
        N.check(N.lib().ipt_render_batch_dev(scene.handle, C.byref(params), S, stride, kd_c.data_ptr(),
                                             hdr.data_ptr(), _stream(hdr.device)), "ipt_render_batch_dev")
        ctx.scene, ctx.params, ctx.stride, ctx.adjoint_seed = scene, params, stride, adjoint_seed
        ctx.save_for_backward(kd_c)
        return hdr

    @staticmethod
    def backward(ctx, grad_hdr):
        (kd_c,) = ctx.saved_tensors
        g = torch.zeros(kd_c.shape, device=kd_c.device, dtype=torch.float64)
        adj = grad_hdr.float().contiguous()
        p = _replay_params(ctx.params, ctx.adjoint_seed)
        N.check(N.lib().ipt_adjoint_batch_dev(ctx.scene.handle, C.byref(p), kd_c.shape[0], ctx.stride,
                                              kd_c.data_ptr(), adj.data_ptr(), g.data_ptr(), _stream(g.device)),
                "ipt_adjoint_batch_dev")
        return g.to(kd_c.dtype), None, None, None, None


def render_batch(scene: Scene, kd: torch.Tensor, width: int, height: int, spp: int, max_bounces=4, seed: int = 0,
                 seed_stride=None, adjoint_seed=None) -> torch.Tensor:
    """Differentiable render of S material sets over one geometry in one
    launch (ipt_render_batch_dev): kd (S, nT, 3) -> HDR images (S, H, W, 3).
    Set b is ``render(scene, kd[b], ..., seed + b * seed_stride)`` bit for bit
    (default stride: one frame of samples, so the sets' sample streams are
    disjoint); the backward runs ONE batched adjoint launch."""
    if kd.dim() != 3 or kd.shape[1] != scene.nT or kd.shape[2] != 3:
        raise ValueError("kd must be (S, nT=%d, 3), got %s" % (scene.nT, tuple(kd.shape)))
    stride = width * height * spp if seed_stride is None else int(seed_stride)
    p = N.make_params(width, height, spp, max_bounces, seed)
    return _BatchRenderFn.apply(kd, scene, p, stride, adjoint_seed)
