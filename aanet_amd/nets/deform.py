"""Drop-in for nets/deform.py (DeformConv2d and the ISA bottlenecks).

Module trees and parameter names are the reference's, so state dicts load unchanged:
  DeformConv2d          nets/deform.py:17-97  (offset_conv + deform_conv)
  DeformBottleneck      nets/deform.py:100-141
  SimpleBottleneck      nets/deform.py:144-184
  DeformSimpleBottleneck nets/deform.py:187-236
Training mode runs the reference op order with autograd (the DCN through the HIP
ModulatedDeformConvFunction).  Eval mode without autograd takes the fused path: BN folded
into the 1x1/3x3 convs, and the deformable conv2 -> bn2 -> ReLU done by ONE kernel that reads
the offset_conv output in place (offset slice + 2*sigmoid(mask logits)) and applies BN+ReLU
in its epilogue.
"""
import contextlib

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ._fuse import (FoldCacheMixin, bn_affine, conv_bn_act, conv_bn_act_s2, folded,
                    halo_input_ok, offset_conv_eval, use_fused)
from .deform_conv import DeformConv, ModulatedDeformConv
from .._lib import is_nhwc
from .._precision import fp32_convs


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    """3x3 convolution with padding (nets/deform.py:6-9)."""
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation,
                     groups=groups, bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    """1x1 convolution (nets/deform.py:12-14)."""
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class DeformConv2d(FoldCacheMixin, nn.Module):
    """A single (modulated) deformable conv layer (nets/deform.py:17-97)."""

    def __init__(self, in_channels, out_channels, kernel_size=3, stride=1, dilation=2, groups=1,
                 deformable_groups=2, modulation=True, double_mask=True, bias=False):
        super(DeformConv2d, self).__init__()
        self.modulation = modulation
        self.deformable_groups = deformable_groups
        self.kernel_size = kernel_size
        self.double_mask = double_mask
        if self.modulation:
            self.deform_conv = ModulatedDeformConv(in_channels, out_channels,
                                                   kernel_size=kernel_size, stride=stride,
                                                   padding=dilation, dilation=dilation,
                                                   groups=groups,
                                                   deformable_groups=deformable_groups, bias=bias)
        else:
            self.deform_conv = DeformConv(in_channels, out_channels, kernel_size=kernel_size,
                                          stride=stride, padding=dilation, dilation=dilation,
                                          groups=groups, deformable_groups=deformable_groups,
                                          bias=bias)
        k = 3 if self.modulation else 2
        offset_out_channels = deformable_groups * k * kernel_size * kernel_size
        # Group-wise offset learning (deform.py:69-72); zero init (deform.py:74-76)
        self.offset_conv = nn.Conv2d(in_channels, offset_out_channels, kernel_size=kernel_size,
                                     stride=stride, padding=dilation, dilation=dilation,
                                     groups=deformable_groups, bias=True)
        nn.init.constant_(self.offset_conv.weight, 0.)
        nn.init.constant_(self.offset_conv.bias, 0.)

    def _offset_conv(self, x):
        """offset_conv (groups = deformable_groups, dilated).  MIOpen has no dilated grouped
        convolution, so torch would fall back to a per-image im2col loop (the largest cost of a
        training step); on the GPU each deformable group runs as its own ungrouped conv."""
        oc = self.offset_conv
        g = oc.groups
        if g == 1 or not x.is_cuda or oc.dilation == (1, 1) or getattr(oc, "_aanet_engine", False):
            return oc(x)  # (train.use_engine_convs: the HIP engine takes grouped dilated convs)
        cin, cout = x.shape[1] // g, oc.out_channels // g
        return torch.cat([F.conv2d(x[:, i * cin:(i + 1) * cin], oc.weight[i * cout:(i + 1) * cout],
                                   oc.bias[i * cout:(i + 1) * cout], oc.stride, oc.padding,
                                   oc.dilation) for i in range(g)], 1)

    @fp32_convs
    def forward(self, x):
        if self.modulation and use_fused(self, x):
            return self.forward_fused(x)
        if self.modulation:
            offset_mask = self._offset_conv(x)
            offset_channel = self.deformable_groups * 2 * self.kernel_size * self.kernel_size
            offset = offset_mask[:, :offset_channel, :, :]
            mask = offset_mask[:, offset_channel:, :, :]
            mask = mask.sigmoid()
            if self.double_mask:
                mask = mask * 2
            return self.deform_conv(x, offset, mask)
        offset = self._offset_conv(x)
        return self.deform_conv(x, offset)

    def forward_fused(self, x, bn=None, act=None):
        """Eval path: offset_conv (HIP conv engine) -> one HIP kernel for DCN (+BN, +act)."""
        dc = self.deform_conv
        offset_mask = offset_conv_eval(x, self.offset_conv)
        ps, psh = bn_affine(bn) if bn is not None else (None, None)
        _, _, wp = folded(dc, None)
        xin = x if is_nhwc(x) else x.contiguous()  # channels-last x: the NHWC window form
        return ops.mdcn_forward_fused(xin, offset_mask.contiguous(), dc.weight,
                                      dc.bias, ps, psh, act, dc.stride, dc.padding, dc.dilation,
                                      self.deformable_groups,
                                      2.0 if self.double_mask else 1.0, packed_weight=wp,
                                      groups=dc.groups)


def _take_post(r, post):
    """(out, csa_out[, post results]) of a tail op -> (out, csa_out) or out, with the post
    stage's results stored in post["result"]."""
    if isinstance(r, tuple) and len(r) == 3:
        post["result"] = r[2]
        return r[0], r[1]
    if post is not None:
        post["result"] = None
    return r


class _BottleneckBase(FoldCacheMixin, nn.Module):
    def _forward_ref(self, x):
        identity = x
        out = self.conv1(x)
        out = self.bn1(out)
        out = self.relu(out)
        out = self.conv2(out)
        out = self.bn2(out)
        out = self.relu(out)
        out = self.conv3(out)
        out = self.bn3(out)
        if self.downsample is not None:
            identity = self.downsample(x)
        out += identity
        out = self.relu(out)
        return out

    def _forward_fused(self, x, deform, conv1_out=None, csa_up=None, before_tail=None, post=None,
                       prep=None):
        """conv1+bn1+relu, then conv2+bn2+relu -> conv3+bn3 (+identity) + relu as ONE HIP kernel
        (the conv3 GEMM runs in conv2's epilogue).  When the tail kernel takes the block, conv1
        writes its output channels-last (NHWC) so that conv2 / offset_conv / the DCN read each
        32-channel chunk of a position as one 128-byte line.  conv1_out: precomputed conv1.
        csa_up: coarser CSA exchange terms of this resolution's output branch; the tail kernel
        then also writes that branch's cross-scale sum, and (out, csa_out) is returned
        (csa_out None when the tail kernel does not take the block).  before_tail: called just
        before the tail kernel is launched (the stream join of the concurrent-scale schedule,
        AdaptiveAggregation: csa_up is produced on the side stream).  post (with csa_up): the
        tail kernel's post stage on the CSA output (ops._post_stage); its results are stored in
        post["result"] (None when the kernel did not take the stage).  prep = (stream, event,
        keep): the deformable block's conv1 and offset_conv run on that side stream once the
        event (its input is written) has fired, beside whatever the current stream does before
        the tail; the tail waits for them (the concurrent-scale schedule, AdaptiveAggregation)."""
        w3, b3, p3 = folded(self.conv3, self.bn3)
        width = self.conv1.weight.shape[0]
        c2 = self.conv2
        if deform:
            pw = c2.modulation and c2.deform_conv.stride == 1 and c2.deform_conv.groups == 1 and \
                width <= 64 and w3.shape[0] <= 64
            cpg = width // c2.deformable_groups  # 32k-channel groups, or pairs of 16-channel ones
            nhwc = pw and width % 32 == 0 and (cpg % 32 == 0 or cpg == 16)
            # no tail kernel (AANetFeature layer3, width 128): a stride-1 modulated DCN still
            # reads conv1's output channels-last -- the grouped offset conv (conv_g3) and the NHWC
            # window form of the DCN
            dc0 = c2.deform_conv
            nhwc = nhwc or (not pw and c2.modulation and dc0.stride in (1, (1, 1)) and
                            dc0.groups == 1 and width % 32 == 0 and cpg % 32 == 0)
        else:
            pw = c2.groups == 1 and width <= 64 and w3.shape[0] <= 64 and \
                c2.stride[0] == c2.stride[1] and c2.padding[0] == c2.padding[1]
            # the ResNet bottlenecks (x4 expansion, no tail kernel): conv1 still writes
            # channels-last when conv2 is a plain 3x3 stride-1 conv, which then stages it on the
            # engine's halo tile (AANetFeature layer1 / layer2)
            nhwc = (pw or halo_input_ok(c2, width)) and width % 32 == 0
        prep = prep if deform and self.conv2.modulation and pw else None
        main = torch.cuda.current_stream(x.device) if prep is not None else None
        if prep is not None:
            prep[0].wait_event(prep[1])
            ctx = torch.cuda.stream(prep[0])
        else:
            ctx = contextlib.nullcontext()
        with ctx:
            if conv1_out is None:
                out = conv_bn_act(x, self.conv1, self.bn1, "relu", out_nhwc=nhwc)
            else:
                out = conv1_out
            # (the non-pw DCN path computes its offsets in forward_fused)
            offset_mask = offset_conv_eval(out, c2.offset_conv) \
                if deform and self.conv2.modulation and pw else None
        if prep is not None:
            main.wait_stream(prep[0])
            prep[2].extend((out, offset_mask))  # written on the side stream, read below
        identity = (self.downsample(x) if self.downsample is not None else x).contiguous()
        if deform and self.conv2.modulation:
            dc = c2.deform_conv
            ps, psh = bn_affine(self.bn2)
            _, _, wp = folded(dc, None)
            if pw:
                if before_tail is not None:
                    before_tail()
                r = ops.mdcn_pw(out, offset_mask, dc.weight, wp, dc.bias, ps, psh, "relu", p3, b3,
                                identity, "relu", dc.stride, dc.padding, dc.dilation,
                                c2.deformable_groups, 2.0 if c2.double_mask else 1.0,
                                csa_up=csa_up, post=post if csa_up is not None else None)
                return _take_post(r, post)
            out = c2.forward_fused(out, self.bn2, act="relu")
        elif deform:
            out = F.relu_(self.bn2(self.conv2(out)))
        else:
            w2, b2, p2 = folded(self.conv2, self.bn2)
            if pw:
                if before_tail is not None:
                    before_tail()
                r = ops.conv2d_pw(out, w2, p2, b2, None, None, "relu", p3, b3, identity, "relu",
                                  c2.stride[0], c2.padding[0], c2.dilation[0], csa_up=csa_up,
                                  post=post if csa_up is not None else None)
                return _take_post(r, post)
            y = conv_bn_act_s2(out, self.conv2, self.bn2, "relu")
            out = y if y is not None else conv_bn_act(out, self.conv2, self.bn2, "relu")
        out = conv_bn_act(out, self.conv3, self.bn3, "relu", residual=identity)
        return out if csa_up is None else (out, None)

    def forward_csa(self, x, csa_up, before_tail=None, conv1_out=None, post=None, prep=None):
        """Eval-only: (block output, its output branch's CSA sum or None); see _forward_fused.
        conv1_out: this block's conv1 output, computed by the previous tail's post stage."""
        deform = isinstance(self, DeformSimpleBottleneck) or isinstance(self, DeformBottleneck)
        r = self._forward_fused(x, deform=deform, csa_up=None if csa_up is None else list(csa_up),
                                before_tail=before_tail, conv1_out=conv1_out, post=post, prep=prep)
        return r if isinstance(r, tuple) else (r, None)


class DeformBottleneck(_BottleneckBase):
    """nets/deform.py:100-141 (feature-extractor block; reuses the HIP DCN)."""
    expansion = 4
    __constants__ = ['downsample']

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super(DeformBottleneck, self).__init__()
        if norm_layer is None:
            norm_layer = nn.BatchNorm2d
        width = int(planes * (base_width / 64.)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = norm_layer(width)
        self.conv2 = DeformConv2d(width, width, stride=stride)
        self.bn2 = norm_layer(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    @fp32_convs
    def forward(self, x):
        if use_fused(self, x):
            return self._forward_fused(x, deform=True)
        return self._forward_ref(x)


class SimpleBottleneck(_BottleneckBase):
    """Simple bottleneck block without channel expansion (nets/deform.py:144-184)."""

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super(SimpleBottleneck, self).__init__()
        if norm_layer is None:
            norm_layer = nn.BatchNorm2d
        width = int(planes * (base_width / 64.)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = norm_layer(width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = norm_layer(width)
        self.conv3 = conv1x1(width, planes)
        self.bn3 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    @fp32_convs
    def forward(self, x):
        if use_fused(self, x):
            return self._forward_fused(x, deform=False)
        return self._forward_ref(x)


class DeformSimpleBottleneck(_BottleneckBase):
    """Used for cost aggregation (nets/deform.py:187-236)."""

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 norm_layer=None, mdconv_dilation=2, deformable_groups=2, modulation=True,
                 double_mask=True):
        super(DeformSimpleBottleneck, self).__init__()
        if norm_layer is None:
            norm_layer = nn.BatchNorm2d
        width = int(planes * (base_width / 64.)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = norm_layer(width)
        self.conv2 = DeformConv2d(width, width, stride=stride, dilation=mdconv_dilation,
                                  deformable_groups=deformable_groups, modulation=modulation,
                                  double_mask=double_mask)
        self.bn2 = norm_layer(width)
        self.conv3 = conv1x1(width, planes)
        self.bn3 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    @fp32_convs
    def forward(self, x):
        if use_fused(self, x):
            return self._forward_fused(x, deform=True)
        return self._forward_ref(x)
