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
    """Adjoint for a row band whose adjoint image holds only rows [row_begin,row_end)."""
    adj_band = adj_band.contiguous()
    base = adj_band.data_ptr() - params.row_begin * params.width * 3 * 4  # global-pixel indexing
    return adjoint_into(scene, params, kd, base, grad)


class _RenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, kd, scene, params):
        kd_c = kd.detach().contiguous().float()
        rows = params.row_end - params.row_begin
        hdr = torch.empty((rows, params.width, 3), device=kd.device, dtype=torch.float32)
        render_into(scene, params, kd_c, hdr)
        ctx.scene, ctx.params = scene, params
        ctx.save_for_backward(kd_c)
        return hdr

    @staticmethod
    def backward(ctx, grad_hdr):
        (kd_c,) = ctx.saved_tensors
        g = torch.zeros(kd_c.shape, device=kd_c.device, dtype=torch.float64)
        adjoint_band(ctx.scene, ctx.params, kd_c, grad_hdr.float(), g)
        return g.to(kd_c.dtype), None, None


def render(scene: Scene, kd: torch.Tensor, width: int, height: int, spp: int, max_bounces=4, seed: int = 0,
           row_begin: int = 0, row_end=None) -> torch.Tensor:
    """Differentiable render: HDR image of rows [row_begin, row_end) w.r.t. kd."""
    if max_bounces is None and kd.requires_grad:
        raise ValueError("the adjoint needs a finite max_bounces (vertex records live in LDS)")
    p = N.make_params(width, height, spp, max_bounces, seed, row_begin, row_end)
    return _RenderFn.apply(kd, scene, p)
