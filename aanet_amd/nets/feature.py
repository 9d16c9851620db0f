"""Feature extractors and pyramids of nets/feature.py, on the drop-in
DCN and the HIP conv engine.

Module trees (attribute names, Sequential indices) are the reference's, so its state dicts load
unchanged.  In eval mode without autograd every plain 2-D conv with its BatchNorm and
ReLU/LeakyReLU(0.2) is one HIP implicit-GEMM kernel (BN folded; residual adds in the epilogue);
transposed convs and 3-D convs stay on PyTorch (MIOpen).  Training runs the reference's op
order with autograd.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from ._fuse import (FusedSequential, conv_bn_act, conv_bn_act_s2, deconv2x_ok, deconv_bn_act,
                    engine_conv, halo_input_ok, use_fused)
from .. import ops
from .deform import DeformConv2d
from .._precision import fp32_convs


def _leaky():
    return nn.LeakyReLU(0.2, inplace=True)


def conv1x1(in_channels, out_channels):
    """feature.py:8-11: 1x1 conv + BN + ReLU."""
    return FusedSequential(nn.Conv2d(in_channels, out_channels, kernel_size=1, bias=False),
                           nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True))


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1, with_bn_relu=False,
            leaky_relu=False):
    """feature.py:15-24: bare 3x3 conv, or conv + BN + (Leaky)ReLU."""
    conv = nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation,
                     groups=groups, bias=False, dilation=dilation)
    if not with_bn_relu:
        return conv
    return FusedSequential(conv, nn.BatchNorm2d(out_planes),
                           _leaky() if leaky_relu else nn.ReLU(inplace=True))


def conv5x5(in_channels, out_channels, stride=2, dilation=1, use_bn=True):
    """feature.py:27-39."""
    conv = nn.Conv2d(in_channels, out_channels, kernel_size=5, stride=stride, padding=2,
                     dilation=dilation, bias=not use_bn)
    mods = [conv] + ([nn.BatchNorm2d(out_channels)] if use_bn else []) + [nn.ReLU(inplace=True)]
    return FusedSequential(*mods)


def convbn(in_planes, out_planes, kernel_size, stride, pad, dilation):
    """feature.py:117-120 (PSMNet): conv + BN; padding = dilation when dilated."""
    return FusedSequential(nn.Conv2d(in_planes, out_planes, kernel_size=kernel_size, stride=stride,
                                     padding=dilation if dilation > 1 else pad,
                                     dilation=dilation, bias=False),
                           nn.BatchNorm2d(out_planes))


def _residual_src(block, x):
    return x if block.downsample is None else block.downsample(x)


class BasicBlock(nn.Module):
    """feature.py:42-76: residual block, LeakyReLU(0.2) by default (StereoNet)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None, leaky_relu=True):
        super(BasicBlock, self).__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self.conv1 = conv3x3(inplanes, planes, stride=stride, dilation=dilation)
        self.bn1 = norm_layer(planes)
        self.relu = _leaky() if leaky_relu else nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes, dilation=dilation)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample
        self.stride = stride

    @fp32_convs
    def forward(self, x):
        if use_fused(self, x) and isinstance(self.bn1, nn.BatchNorm2d):
            act = "leaky" if isinstance(self.relu, nn.LeakyReLU) else "relu"
            out = conv_bn_act(x, self.conv1, self.bn1, act)
            return conv_bn_act(out, self.conv2, self.bn2, act,
                               residual=_residual_src(self, x).contiguous())
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out += _residual_src(self, x)
        return self.relu(out)


class StereoNetFeature(nn.Module):
    """feature.py:79-114: num_downsample 5x5 stride-2 convs, 6 residual blocks, a final conv."""

    def __init__(self, num_downsample=3):
        super(StereoNetFeature, self).__init__()
        self.num_downsample = num_downsample
        self.downsample = nn.Sequential(*[conv5x5(3 if i == 0 else 32, 32)
                                          for i in range(num_downsample)])
        self.residual_blocks = nn.Sequential(*[BasicBlock(32, 32) for _ in range(6)])
        self.final_conv = conv3x3(32, 32)  # no BN / ReLU on the last conv

    @fp32_convs
    def forward(self, img):
        out = self.residual_blocks(self.downsample(img))
        if use_fused(self, out):
            return conv_bn_act(out, self.final_conv)
        return self.final_conv(out)


class PSMNetBasicBlock(nn.Module):
    """feature.py:123-147: conv-BN-ReLU, conv-BN, + shortcut (no ReLU after the add)."""
    expansion = 1

    def __init__(self, inplanes, planes, stride, downsample, pad, dilation):
        super(PSMNetBasicBlock, self).__init__()
        self.conv1 = FusedSequential(convbn(inplanes, planes, 3, stride, pad, dilation),
                                     nn.ReLU(inplace=True))
        self.conv2 = convbn(planes, planes, 3, 1, pad, dilation)
        self.downsample = downsample
        self.stride = stride

    @fp32_convs
    def forward(self, x):
        if use_fused(self, x):
            out = self.conv1(x)
            c, bn = self.conv2[0], self.conv2[1]
            return conv_bn_act(out, c, bn, None, residual=_residual_src(self, x).contiguous())
        out = self.conv2(self.conv1(x))
        out += _residual_src(self, x)
        return out


class FeaturePyrmaid(nn.Module):
    """feature.py:150-179 (sic): 1/1, 1/2, 1/4 pyramid from one feature map."""

    def __init__(self, in_channel=32):
        super(FeaturePyrmaid, self).__init__()

        def level(cin, cout):
            return FusedSequential(
                nn.Conv2d(cin, cout, kernel_size=3, stride=2, padding=1, bias=False),
                nn.BatchNorm2d(cout), _leaky(),
                nn.Conv2d(cout, cout, kernel_size=1, stride=1, padding=0, bias=False),
                nn.BatchNorm2d(cout), _leaky())

        self.out1 = level(in_channel, in_channel * 2)
        self.out2 = level(in_channel * 2, in_channel * 4)

    @fp32_convs
    def forward(self, x):
        out1 = self.out1(x)
        return [x, out1, self.out2(out1)]


class FeaturePyramidNetwork(nn.Module):
    """feature.py:182-231: lateral 1x1 convs, nearest-2x top-down sum, 3x3 conv+BN+ReLU."""

    def __init__(self, in_channels, out_channels=128, num_levels=3):
        super(FeaturePyramidNetwork, self).__init__()
        assert isinstance(in_channels, list)
        self.in_channels = in_channels
        self.lateral_convs = nn.ModuleList(
            [nn.Conv2d(in_channels[i], out_channels, 1) for i in range(num_levels)])
        self.fpn_convs = nn.ModuleList(
            [FusedSequential(nn.Conv2d(out_channels, out_channels, 3, padding=1),
                             nn.BatchNorm2d(out_channels), nn.ReLU(inplace=True))
             for _ in range(num_levels)])
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.xavier_uniform_(m.weight, gain=1)
                nn.init.constant_(m.bias, 0)

    @fp32_convs
    def forward(self, inputs):
        assert len(self.in_channels) == len(inputs)
        n = len(inputs)
        if use_fused(self, inputs[0]):
            # top-down from the coarsest level: each lateral conv adds the upsampled coarser
            # lateral in its epilogue (residual), so no separate add pass
            # The laterals are written channels-last when the 3x3 output convs can stage NHWC
            # input (the engine's halo tile); nearest upsampling keeps channels-last.
            nhwc = all(isinstance(f[0], nn.Conv2d) and
                       halo_input_ok(f[0], f[0].in_channels) for f in self.fpn_convs)
            lat = [None] * n
            lat[n - 1] = conv_bn_act(inputs[n - 1], self.lateral_convs[n - 1], out_nhwc=nhwc)
            for i in range(n - 1, 0, -1):
                up = F.interpolate(lat[i], scale_factor=2, mode='nearest')
                if nhwc:
                    up = up.contiguous(memory_format=torch.channels_last)
                lat[i - 1] = conv_bn_act(inputs[i - 1], self.lateral_convs[i - 1], residual=up,
                                         out_nhwc=nhwc)
            return [self.fpn_convs[i](lat[i]) for i in range(n)]
        lat = [conv(inputs[i]) for i, conv in enumerate(self.lateral_convs)]
        for i in range(n - 1, 0, -1):
            lat[i - 1] += F.interpolate(lat[i], scale_factor=2, mode='nearest')
        return [self.fpn_convs[i](lat[i]) for i in range(n)]


def _psm_layer(owner, block, planes, blocks, stride, pad, dilation):
    """feature.py:271-285 / 472-486 (_make_layer of PSMNet/GCNet features)."""
    downsample = None
    if stride != 1 or owner.inplanes != planes * block.expansion:
        downsample = FusedSequential(
            nn.Conv2d(owner.inplanes, planes * block.expansion, kernel_size=1, stride=stride,
                      bias=False),
            nn.BatchNorm2d(planes * block.expansion))
    layers = [block(owner.inplanes, planes, stride, downsample, pad, dilation)]
    owner.inplanes = planes * block.expansion
    layers += [block(owner.inplanes, planes, 1, None, pad, dilation) for _ in range(1, blocks)]
    return nn.Sequential(*layers)


class PSMNetFeature(nn.Module):
    """feature.py:234-311: SPP feature extractor, [B, 32, H/4, W/4]."""

    def __init__(self):
        super(PSMNetFeature, self).__init__()
        self.inplanes = 32
        self.firstconv = FusedSequential(convbn(3, 32, 3, 2, 1, 1), nn.ReLU(inplace=True),
                                         convbn(32, 32, 3, 1, 1, 1), nn.ReLU(inplace=True),
                                         convbn(32, 32, 3, 1, 1, 1), nn.ReLU(inplace=True))
        self.layer1 = _psm_layer(self, PSMNetBasicBlock, 32, 3, 1, 1, 1)
        self.layer2 = _psm_layer(self, PSMNetBasicBlock, 64, 16, 2, 1, 1)
        self.layer3 = _psm_layer(self, PSMNetBasicBlock, 128, 3, 1, 1, 1)
        self.layer4 = _psm_layer(self, PSMNetBasicBlock, 128, 3, 1, 1, 2)
        for i, k in enumerate((64, 32, 16, 8), start=1):
            setattr(self, f"branch{i}",
                    FusedSequential(nn.AvgPool2d((k, k), stride=(k, k)),
                                    convbn(128, 32, 1, 1, 0, 1), nn.ReLU(inplace=True)))
        self.lastconv = FusedSequential(convbn(320, 128, 3, 1, 1, 1), nn.ReLU(inplace=True),
                                        nn.Conv2d(128, 32, kernel_size=1, padding=0, stride=1,
                                                  bias=False))

    @fp32_convs
    def forward(self, x):
        out = self.layer1(self.firstconv(x))
        raw = self.layer2(out)
        skip = self.layer4(self.layer3(raw))
        size = skip.shape[2:]
        branches = [F.interpolate(getattr(self, f"branch{i}")(skip), size, mode='bilinear',
                                  align_corners=False) for i in (4, 3, 2, 1)]
        return self.lastconv(torch.cat([raw, skip] + branches, 1))


class BasicConv(nn.Module):
    """feature.py:314-339 (GANet): conv / transposed conv (2-D or 3-D) [+ BN] [+ ReLU]."""

    def __init__(self, in_channels, out_channels, deconv=False, is_3d=False, bn=True, relu=True,
                 **kwargs):
        super(BasicConv, self).__init__()
        self.relu = relu
        self.use_bn = bn
        if is_3d:
            conv_t = nn.ConvTranspose3d if deconv else nn.Conv3d
            self.bn = nn.BatchNorm3d(out_channels)
        else:
            conv_t = nn.ConvTranspose2d if deconv else nn.Conv2d
            self.bn = nn.BatchNorm2d(out_channels)
        self.conv = conv_t(in_channels, out_channels, bias=False, **kwargs)

    def fused_deconv(self, x):
        """Eval fast path of a 2-D 4x4 stride-2 transposed conv (ops.deconv2x), or None."""
        return use_fused(self, x) and deconv2x_ok(self.conv)

    @fp32_convs
    def forward(self, x):
        if use_fused(self, x) and engine_conv(self.conv):
            bn, act = self.bn if self.use_bn else None, "relu" if self.relu else None
            y = conv_bn_act_s2(x, self.conv, bn, act) if x.dim() == 4 else None
            return y if y is not None else conv_bn_act(x, self.conv, bn, act)
        if self.fused_deconv(x):
            return deconv_bn_act(x, self.conv, self.bn if self.use_bn else None,
                                 "relu" if self.relu else None)
        x = self.conv(x)
        if self.use_bn:
            x = self.bn(x)
        if self.relu:
            x = F.relu(x, inplace=True)
        return x


class Conv2x(nn.Module):
    """feature.py:342-376: stride-2 (de)conv, then concat (or add) the skip, then a 3x3 conv
    (or the HIP DCN when mdconv)."""

    def __init__(self, in_channels, out_channels, deconv=False, is_3d=False, concat=True, bn=True,
                 relu=True, mdconv=False):
        super(Conv2x, self).__init__()
        self.concat = concat
        kernel = (3, 4, 4) if (deconv and is_3d) else (4 if deconv else 3)
        self.conv1 = BasicConv(in_channels, out_channels, deconv, is_3d, bn=True, relu=True,
                               kernel_size=kernel, stride=2, padding=1)
        if concat and mdconv:
            self.conv2 = DeformConv2d(out_channels * 2, out_channels, kernel_size=3, stride=1)
        else:
            cin = out_channels * 2 if concat else out_channels
            self.conv2 = BasicConv(cin, out_channels, False, is_3d, bn, relu, kernel_size=3,
                                   stride=1, padding=1)

    @fp32_convs
    def forward(self, x, rem, out_nhwc=False):
        """out_nhwc (eval fast path, BasicConv conv2 only): return conv2's output channels-last
        for a consumer that reads NHWC (the refinement's final_conv)."""
        c1 = self.conv1
        if self.concat and c1.fused_deconv(x) and rem.shape[2:] == (2 * x.shape[2], 2 * x.shape[3]):
            # transposed conv + BN + ReLU and the concat: one engine launch + one assembly pass,
            # written channels-last when conv2 stages NHWC input (the halo tile; full-resolution
            # 64 -> 32 conv of the refinement 1136 -> ... us)
            c2 = self.conv2
            nhwc = isinstance(c2, BasicConv) and use_fused(c2, x) and \
                halo_input_ok(c2.conv, c1.conv.out_channels + rem.shape[1])
            x = deconv_bn_act(x, c1.conv, c1.bn if c1.use_bn else None,
                              "relu" if c1.relu else None, rem=rem, out_nhwc=nhwc)
            if out_nhwc and nhwc:
                return conv_bn_act(x, c2.conv, c2.bn if c2.use_bn else None,
                                   "relu" if c2.relu else None, out_nhwc=True)
            return self.conv2(x)
        x = self.conv1(x)
        assert x.size() == rem.size()
        c2 = self.conv2
        if self.concat and isinstance(c2, BasicConv) and use_fused(c2, x) and \
                x.shape[2] % 2 == 0 and x.shape[3] % 2 == 0 and \
                halo_input_ok(c2.conv, x.shape[1] + rem.shape[1]):
            # the concat written channels-last: conv2 stages it on the halo tile
            return c2(ops.concat_nhwc(x, rem))
        x = torch.cat((x, rem), 1) if self.concat else x + rem
        return self.conv2(x)


class GANetFeature(nn.Module):
    """feature.py:379-460 (AANet+): stride-3 stem, two stride-2 hourglass passes, [B,32,H/3,W/3].
    Height and width must be divisible by 48."""

    def __init__(self, feature_mdconv=False):
        super(GANetFeature, self).__init__()
        third = DeformConv2d(32, 32) if feature_mdconv else BasicConv(32, 32, kernel_size=3,
                                                                      padding=1)
        self.conv_start = nn.Sequential(BasicConv(3, 32, kernel_size=3, padding=1),
                                        BasicConv(32, 32, kernel_size=5, stride=3, padding=2),
                                        third)
        self.conv1a = BasicConv(32, 48, kernel_size=3, stride=2, padding=1)
        self.conv2a = BasicConv(48, 64, kernel_size=3, stride=2, padding=1)
        if feature_mdconv:
            self.conv3a = DeformConv2d(64, 96, kernel_size=3, stride=2)
            self.conv4a = DeformConv2d(96, 128, kernel_size=3, stride=2)
        else:
            self.conv3a = BasicConv(64, 96, kernel_size=3, stride=2, padding=1)
            self.conv4a = BasicConv(96, 128, kernel_size=3, stride=2, padding=1)
        chans = (32, 48, 64, 96, 128)
        for sfx in "ab":
            for i in range(4, 0, -1):
                setattr(self, f"deconv{i}{sfx}", Conv2x(chans[i], chans[i - 1], deconv=True))
        self.conv1b = Conv2x(32, 48)
        self.conv2b = Conv2x(48, 64)
        self.conv3b = Conv2x(64, 96, mdconv=feature_mdconv)
        self.conv4b = Conv2x(96, 128, mdconv=feature_mdconv)

    @fp32_convs
    def forward(self, x):
        cs = self.conv_start
        third, c5 = cs[2], cs[1]
        if isinstance(third, DeformConv2d) and third.modulation and use_fused(third, x) and \
                use_fused(c5, x) and engine_conv(c5.conv) and c5.conv.out_channels % 4 == 0:
            # the 5x5 stride-3 conv writes channels-last: the DCN's offset conv stages it on the
            # halo tile and the DCN reads it with the NHWC window form
            y = conv_bn_act(cs[0](x), c5.conv, c5.bn if c5.use_bn else None,
                            "relu" if c5.relu else None, out_nhwc=True)
            return _hourglass2(self, third(y))
        return _hourglass2(self, cs(x))


def _hourglass2(m, x, last_nhwc=False):
    """Shared two-pass hourglass of GANetFeature.forward (feature.py:426-460) and
    HourglassRefinement.forward (refinement.py:160-197): down a, up a, down b, up b.
    last_nhwc: the last block may return its output channels-last (Conv2x out_nhwc)."""
    rem = [x]
    for name in ("conv1a", "conv2a", "conv3a", "conv4a"):
        x = getattr(m, name)(x)
        rem.append(x)
    for i in (4, 3, 2, 1):  # deconv{i}a(x, rem{i-1}); its output replaces rem{i-1}
        x = getattr(m, f"deconv{i}a")(x, rem[i - 1])
        rem[i - 1] = x
    for i in (1, 2, 3):     # conv{i}b(x, rem{i}); its output replaces rem{i}
        x = getattr(m, f"conv{i}b")(x, rem[i])
        rem[i] = x
    x = m.conv4b(x, rem[4])
    for i in (4, 3, 2, 1):
        x = getattr(m, f"deconv{i}b")(x, rem[i - 1], out_nhwc=last_nhwc and i == 1)
    return x


class GCNetFeature(nn.Module):
    """feature.py:463-493: [B, 32, H/2, W/2]."""

    def __init__(self):
        super(GCNetFeature, self).__init__()
        self.inplanes = 32
        self.conv1 = conv5x5(3, 32)
        self.conv2 = _psm_layer(self, PSMNetBasicBlock, 32, 8, 1, 1, 1)
        self.conv3 = conv3x3(32, 32)

    @fp32_convs
    def forward(self, x):
        x = self.conv2(self.conv1(x))
        if use_fused(self, x):
            return conv_bn_act(x, self.conv3)
        return self.conv3(x)
