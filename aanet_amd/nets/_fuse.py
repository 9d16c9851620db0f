"""Eval-mode fusion helpers: fold BatchNorm into the preceding conv (cached per parameter
version) so the inference graph runs conv+BN(+activation) as one op.

Training mode never uses these: modules then run the reference op sequence with autograd.
"""
import torch
import torch.nn.functional as F


def bn_scale_shift(bn):
    """y = x*scale + shift for an eval-mode BatchNorm2d."""
    scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    shift = bn.bias - bn.running_mean * scale
    return scale, shift


def _key(*tensors):
    return tuple((t.data_ptr(), t._version) for t in tensors if t is not None)


def folded(conv, bn):
    """(weight, bias) of conv followed by eval BN, cached on the conv module."""
    key = _key(conv.weight, conv.bias, bn.weight, bn.bias, bn.running_mean, bn.running_var)
    cache = getattr(conv, "_aanet_fold", None)
    if cache is not None and cache[0] == key:
        return cache[1], cache[2]
    with torch.no_grad():
        scale, shift = bn_scale_shift(bn)
        w = (conv.weight * scale.view(-1, 1, 1, 1)).contiguous()
        b = shift if conv.bias is None else conv.bias * scale + shift
        b = b.contiguous()
    conv._aanet_fold = (key, w, b)
    return w, b


def bn_affine(bn):
    """(scale, shift) of an eval BN, cached on the BN module (for kernel epilogues)."""
    key = _key(bn.weight, bn.bias, bn.running_mean, bn.running_var)
    cache = getattr(bn, "_aanet_affine", None)
    if cache is not None and cache[0] == key:
        return cache[1], cache[2]
    with torch.no_grad():
        scale, shift = bn_scale_shift(bn)
        scale, shift = scale.contiguous(), shift.contiguous()
    bn._aanet_affine = (key, scale, shift)
    return scale, shift


def conv_bn_act(x, conv, bn, act=None, inplace_ok=True):
    """conv -> eval BN -> act ('relu' | 'leaky' | None) with BN folded into the conv."""
    w, b = folded(conv, bn)
    y = F.conv2d(x, w, b, conv.stride, conv.padding, conv.dilation, conv.groups)
    if act == "relu":
        y = F.relu_(y) if inplace_ok else F.relu(y)
    elif act == "leaky":
        y = F.leaky_relu_(y, 0.2) if inplace_ok else F.leaky_relu(y, 0.2)
    return y


def use_fused(module, x):
    """Fast path only in eval mode, without autograd, on the HIP device."""
    return (not module.training) and x.is_cuda and not torch.is_grad_enabled() and \
        getattr(module, "aanet_fuse", True)
