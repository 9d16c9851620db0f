"""Drop-in for the reference's native module `deform_conv_cuda` (nets/deform_conv/src/
deform_conv_cuda.cpp:687-700), backed by the gfx950 C ABI.

The reference's Python wrapper binds it as `from . import deform_conv_cuda`
(nets/deform_conv/deform_conv.py:9); pointing that import here keeps the wrapper unchanged.
Same argument order and in-place semantics:
  * forward writes `output` in place (cpp:530); `ones` / `columns` are vestigial scratch (the
    reference re-allocates `columns` internally, cpp:532-534) and are ignored here;
  * backward writes grad_input / grad_offset / grad_mask (callers pass zeros,
    deform_conv.py:156-158) and ACCUMULATES into grad_weight / grad_bias (cpp:660-671).
Only stride_h == stride_w, pad_h == pad_w, dilation_h == dilation_w are supported (the only
form deform_conv.py ever passes, :143-147).  The DCNv1 entry points (deform_conv_forward_cuda,
deform_conv_backward_*) are dead code for AANet and raise.
"""
import torch

from . import ops
from ._lib import call, ptr, require_gpu, stream_of


def _sym(a, b, what):
    if a != b:
        raise NotImplementedError(f"asymmetric {what} ({a}, {b})")
    return a


def modulated_deform_conv_cuda_forward(input, weight, bias, ones, offset, mask, output, columns,
                                       kernel_h, kernel_w, stride_h, stride_w, pad_h, pad_w,
                                       dilation_h, dilation_w, group, deformable_group, with_bias):
    s, p, d = _sym(stride_h, stride_w, "stride"), _sym(pad_h, pad_w, "padding"), \
        _sym(dilation_h, dilation_w, "dilation")
    if tuple(weight.shape[2:]) != (kernel_h, kernel_w):
        raise RuntimeError("Input shape and kernel shape wont match")  # cpp:509-511
    if input.shape[1] != weight.shape[1] * group:
        raise RuntimeError("Input shape and kernel channels wont match")  # cpp:512-514
    require_gpu(input, weight, offset, mask, names=("input", "weight", "offset", "mask"))
    N, C, H, W = input.shape
    Co = weight.shape[0]
    Ho = (H + 2 * p - (d * (kernel_h - 1) + 1)) // s + 1
    Wo = (W + 2 * p - (d * (kernel_w - 1) + 1)) // s + 1
    output.resize_(N, Co, Ho, Wo)
    require_gpu(output, names=("output",))
    b = bias if with_bias else None
    call("aanet_mdcn_fwd_f32", ptr(input), ptr(offset.contiguous()), ptr(mask.contiguous()),
         ptr(weight), ptr(b), ptr(output), N, C, H, W, Co, kernel_h, kernel_w, s, p, d, group,
         deformable_group, stream_of(input))


def modulated_deform_conv_cuda_backward(input, weight, bias, ones, offset, mask, columns,
                                        grad_input, grad_weight, grad_bias, grad_offset,
                                        grad_mask, grad_output, kernel_h, kernel_w, stride_h,
                                        stride_w, pad_h, pad_w, dilation_h, dilation_w, group,
                                        deformable_group, with_bias):
    s, p, d = _sym(stride_h, stride_w, "stride"), _sym(pad_h, pad_w, "padding"), \
        _sym(dilation_h, dilation_w, "dilation")
    require_gpu(input, weight, offset, mask, grad_input, grad_weight, grad_offset, grad_mask,
                names=("input", "weight", "offset", "mask", "grad_input", "grad_weight",
                       "grad_offset", "grad_mask"))
    go = grad_output.contiguous()
    if torch.are_deterministic_algorithms_enabled():
        # bit-reproducible form (aanet_mdcn_bwd_det_f32); same in-place / accumulate contract
        gx, goff, gm, gw, gb = ops.mdcn_backward(input, offset, mask, weight, go, with_bias, s, p,
                                                 d, group, deformable_group, deterministic=True)
        grad_input.copy_(gx)
        grad_offset.copy_(goff)
        grad_mask.copy_(gm)
        grad_weight.add_(gw)
        if with_bias:
            grad_bias.add_(gb)
        return
    N, C, H, W = input.shape
    Co = weight.shape[0]
    call("aanet_mdcn_bwd_f32", ptr(input), ptr(offset), ptr(mask), ptr(weight), ptr(go),
         ptr(grad_input), ptr(grad_offset), ptr(grad_mask), ptr(grad_weight),
         ptr(grad_bias) if with_bias else None, N, C, H, W, Co, kernel_h, kernel_w, s, p, d,
         group, deformable_group, stream_of(input))


def _dcn_v1(*_args, **_kw):
    raise NotImplementedError("DCNv1 entry points are not used by AANet (all DeformConv2d use "
                              "modulation=True); use aanet_amd.nets.deform_conv.DeformConv")


deform_conv_forward_cuda = _dcn_v1
deform_conv_backward_input_cuda = _dcn_v1
deform_conv_backward_parameters_cuda = _dcn_v1

__all__ = ["modulated_deform_conv_cuda_forward", "modulated_deform_conv_cuda_backward",
           "deform_conv_forward_cuda", "deform_conv_backward_input_cuda",
           "deform_conv_backward_parameters_cuda", "ops"]
