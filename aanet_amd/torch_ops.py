"""``torch.ops.aanet.*``: the hot-path ops as PyTorch custom operators ("Op-level
autograd API": ``torch.ops.aanet.mdcn_forward/backward`` plus an autograd formula).

Each op is a ``torch.library.custom_op`` with a HIP (``cuda`` device type) implementation that
calls the C ABI through ``aanet_amd.ops``, a fake (meta) kernel for shape propagation, and, for
the forward ops, an autograd formula built on the registered backward ops.  There is no CPU
kernel: a CPU tensor reaches the dispatcher with no implementation and raises, as the
reference's CUDA-only DCN does (nets/deform_conv/deform_conv.py:135-136).

    y = torch.ops.aanet.mdcn_forward(x, offset, mask, weight, bias, 1, 2, 2, 1, 2)
    gx, goff, gmask, gw, gb = torch.ops.aanet.mdcn_backward(x, offset, mask, weight, gy, True,
                                                            1, 2, 2, 1, 2)
"""
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import ops

_NS = "aanet"


def _out_size(n, k, s, p, d):
    return (n + 2 * p - (d * (k - 1) + 1)) // s + 1


# ------------------------------------------------------------ modulated deformable conv ---
@torch.library.custom_op(f"{_NS}::mdcn_forward", mutates_args=(), device_types="cuda")
def mdcn_forward(x: Tensor, offset: Tensor, mask: Tensor, weight: Tensor, bias: Optional[Tensor],
                 stride: int, padding: int, dilation: int, groups: int,
                 deformable_groups: int) -> Tensor:
    """deform_conv_cuda.cpp:490-569 (modulated_deform_conv_cuda_forward), functional form."""
    return ops.mdcn_forward(x.contiguous(), offset.contiguous(), mask.contiguous(),
                            weight.contiguous(), None if bias is None else bias.contiguous(),
                            stride, padding, dilation, groups, deformable_groups)


@mdcn_forward.register_fake
def _(x, offset, mask, weight, bias, stride, padding, dilation, groups, deformable_groups):
    N, _, H, W = x.shape
    Co, _, kh, kw = weight.shape
    return x.new_empty((N, Co, _out_size(H, kh, stride, padding, dilation),
                        _out_size(W, kw, stride, padding, dilation)))


@torch.library.custom_op(f"{_NS}::mdcn_backward", mutates_args=(), device_types="cuda")
def mdcn_backward(x: Tensor, offset: Tensor, mask: Tensor, weight: Tensor, grad_out: Tensor,
                  with_bias: bool, stride: int, padding: int, dilation: int, groups: int,
                  deformable_groups: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """deform_conv_cuda.cpp:571-685 -> (gX, gOffset, gMask, gW, gB); gB is empty without bias."""
    gx, goff, gm, gw, gb = ops.mdcn_backward(x.contiguous(), offset.contiguous(),
                                             mask.contiguous(), weight.contiguous(),
                                             grad_out.contiguous(), with_bias, stride, padding,
                                             dilation, groups, deformable_groups)
    return gx, goff, gm, gw, (gb if gb is not None else x.new_empty((0,)))


@mdcn_backward.register_fake
def _(x, offset, mask, weight, grad_out, with_bias, stride, padding, dilation, groups,
      deformable_groups):
    return (torch.empty_like(x), torch.empty_like(offset), torch.empty_like(mask),
            torch.empty_like(weight), x.new_empty((weight.shape[0] if with_bias else 0,)))


def _mdcn_setup(ctx, inputs, output):
    x, offset, mask, weight, bias, stride, padding, dilation, groups, dg = inputs
    ctx.save_for_backward(x, offset, mask, weight)
    ctx.args = (bias is not None, stride, padding, dilation, groups, dg)


def _mdcn_backward_formula(ctx, grad_out):
    x, offset, mask, weight = ctx.saved_tensors
    with_bias, stride, padding, dilation, groups, dg = ctx.args
    gx, goff, gm, gw, gb = mdcn_backward(x, offset, mask, weight, grad_out, with_bias, stride,
                                         padding, dilation, groups, dg)
    return gx, goff, gm, gw, (gb if with_bias else None), None, None, None, None, None


torch.library.register_autograd(f"{_NS}::mdcn_forward", _mdcn_backward_formula,
                                setup_context=_mdcn_setup)


# ------------------------------------------------------------------- cost volumes --------
@torch.library.custom_op(f"{_NS}::corr_volume", mutates_args=(), device_types="cuda")
def corr_volume(left: Tensor, right: Tensor, max_disp: int) -> Tensor:
    """nets/cost.py:40-48 (CostVolume, correlation) -> [B, D, H, W]."""
    return ops.corr_volume(left.contiguous(), right.contiguous(), max_disp)


@corr_volume.register_fake
def _(left, right, max_disp):
    B, _, H, W = left.shape
    return left.new_empty((B, max_disp, H, W))


@torch.library.custom_op(f"{_NS}::corr_volume_backward", mutates_args=(), device_types="cuda")
def corr_volume_backward(left: Tensor, right: Tensor, grad_out: Tensor,
                         max_disp: int) -> Tuple[Tensor, Tensor]:
    from ._lib import call, ptr, require_gpu, stream_of
    left, right, grad_out = left.contiguous(), right.contiguous(), grad_out.contiguous()
    require_gpu(left, right, grad_out, names=("left", "right", "grad_out"))
    gl, gr = torch.empty_like(left), torch.empty_like(right)
    B, C, H, W = left.shape
    call("aanet_corr_volume_bwd_f32", ptr(left), ptr(right), ptr(grad_out), ptr(gl), ptr(gr),
         B, C, H, W, max_disp, stream_of(left))
    return gl, gr


@corr_volume_backward.register_fake
def _(left, right, grad_out, max_disp):
    return torch.empty_like(left), torch.empty_like(right)


def _corr_setup(ctx, inputs, output):
    left, right, max_disp = inputs
    ctx.save_for_backward(left, right)
    ctx.max_disp = max_disp


def _corr_backward_formula(ctx, grad_out):
    left, right = ctx.saved_tensors
    gl, gr = corr_volume_backward(left, right, grad_out, ctx.max_disp)
    return gl, gr, None


torch.library.register_autograd(f"{_NS}::corr_volume", _corr_backward_formula,
                                setup_context=_corr_setup)


# ------------------------------------------------------------ disparity regression ------
@torch.library.custom_op(f"{_NS}::disp_regress", mutates_args=(), device_types="cuda")
def disp_regress(cost: Tensor, negate: bool) -> Tensor:
    """nets/estimation.py:13-30 (soft-argmin) -> [B, H, W]."""
    return ops.disp_regress(cost.contiguous(), negate)


@disp_regress.register_fake
def _(cost, negate):
    B, _, H, W = cost.shape
    return cost.new_empty((B, H, W))


@torch.library.custom_op(f"{_NS}::disp_regress_backward", mutates_args=(), device_types="cuda")
def disp_regress_backward(cost: Tensor, grad_disp: Tensor, negate: bool) -> Tensor:
    from ._lib import call, ptr, require_gpu, stream_of
    cost, grad_disp = cost.contiguous(), grad_disp.contiguous()
    require_gpu(cost, grad_disp, names=("cost", "grad_disp"))
    gc = torch.empty_like(cost)
    B, D, H, W = cost.shape
    call("aanet_disp_regress_bwd_f32", ptr(cost), ptr(grad_disp), ptr(gc), B, D, H, W,
         int(bool(negate)), stream_of(cost))
    return gc


@disp_regress_backward.register_fake
def _(cost, grad_disp, negate):
    return torch.empty_like(cost)


def _regress_setup(ctx, inputs, output):
    cost, negate = inputs
    ctx.save_for_backward(cost)
    ctx.negate = negate


def _regress_backward_formula(ctx, grad_disp):
    (cost,) = ctx.saved_tensors
    return disp_regress_backward(cost, grad_disp, ctx.negate), None


torch.library.register_autograd(f"{_NS}::disp_regress", _regress_backward_formula,
                                setup_context=_regress_setup)

OPS = ("mdcn_forward", "mdcn_backward", "corr_volume", "corr_volume_backward", "disp_regress",
       "disp_regress_backward")
