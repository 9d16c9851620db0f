"""Drop-in for nets/deform_conv/deform_conv.py (the `deform_conv_cuda` users).

ModulatedDeformConvFunction / modulated_deform_conv / ModulatedDeformConv keep the reference's
argument order, parameter names, init and NotImplementedError-on-CPU behaviour
(deform_conv.py:113-187, 304-351).  DeformConv (DCNv1, dead code for AANet but imported by
nets/deform.py) is provided through the modulated kernel with mask == 1, which is the v1
sampling exactly (kernel.cu:84-115 vs 467-497: same bilinear, no mask multiply; x*1 == x).
"""
import math

import torch
import torch.nn as nn
from torch.nn.modules.utils import _pair, _single

from ..ops import ModulatedDeformConvFunction, modulated_deform_conv  # noqa: F401


def _sym(v, name):
    v = _pair(v)
    if v[0] != v[1]:
        raise NotImplementedError(f"asymmetric {name} {v} is not supported by the gfx950 kernel")
    return v[0]


def deform_conv(input, offset, weight, stride=1, padding=0, dilation=1, groups=1,
                deformable_groups=1, im2col_step=64):
    """DCNv1 (deform_conv.py:186) via the modulated kernel with a unit mask."""
    N, _, H, W = input.shape
    kh, kw = weight.shape[2:]
    s, p, d = _sym(stride, "stride"), _sym(padding, "padding"), _sym(dilation, "dilation")
    Ho = (H + 2 * p - (d * (kh - 1) + 1)) // s + 1
    Wo = (W + 2 * p - (d * (kw - 1) + 1)) // s + 1
    mask = input.new_ones((N, deformable_groups * kh * kw, Ho, Wo))
    return modulated_deform_conv(input, offset, mask, weight, None, s, p, d, groups,
                                 deformable_groups)


class DeformConv(nn.Module):
    """deform_conv.py:190-239 (same parameters and init)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, deformable_groups=1, bias=False):
        super(DeformConv, self).__init__()
        assert not bias
        assert in_channels % groups == 0
        assert out_channels % groups == 0
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = _pair(stride)
        self.padding = _pair(padding)
        self.dilation = _pair(dilation)
        self.groups = groups
        self.deformable_groups = deformable_groups
        self.transposed = False
        self.output_padding = _single(0)
        self.weight = nn.Parameter(torch.Tensor(out_channels, in_channels // self.groups,
                                                *self.kernel_size))
        self.reset_parameters()

    def reset_parameters(self):
        n = self.in_channels
        for k in self.kernel_size:
            n *= k
        stdv = 1. / math.sqrt(n)
        self.weight.data.uniform_(-stdv, stdv)

    def forward(self, x, offset):
        return deform_conv(x, offset, self.weight, self.stride, self.padding, self.dilation,
                           self.groups, self.deformable_groups)


class ModulatedDeformConv(nn.Module):
    """deform_conv.py:304-351 (same parameters, init and forward contract)."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, deformable_groups=1, bias=True):
        super(ModulatedDeformConv, self).__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.kernel_size = _pair(kernel_size)
        self.stride = stride
        self.padding = padding
        self.dilation = dilation
        self.groups = groups
        self.deformable_groups = deformable_groups
        self.with_bias = bias
        self.transposed = False
        self.output_padding = _single(0)
        self.weight = nn.Parameter(torch.Tensor(out_channels, in_channels // groups,
                                                *self.kernel_size))
        if bias:
            self.bias = nn.Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter('bias', None)
        self.reset_parameters()

    def reset_parameters(self):
        n = self.in_channels
        for k in self.kernel_size:
            n *= k
        stdv = 1. / math.sqrt(n)
        self.weight.data.uniform_(-stdv, stdv)
        if self.bias is not None:
            self.bias.data.zero_()

    def forward(self, x, offset, mask):
        return modulated_deform_conv(x, offset, mask, self.weight, self.bias, self.stride,
                                     self.padding, self.dilation, self.groups,
                                     self.deformable_groups)
