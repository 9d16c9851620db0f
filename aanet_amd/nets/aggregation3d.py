"""3-D cost aggregators of nets/aggregation.py:62-309: the consumers of the
5-D concat / difference volumes (StereoNet, PSMNet basic + hourglass, GC-Net).

Module trees follow the reference exactly -- including PSMNetBasicAggregation's reuse of ONE
`conv1` block in several Sequentials (shared weights, aggregation.py:101-123), which a
checkpoint load relies on.  The 3-D convs run on PyTorch (MIOpen); the volumes they consume
come from the HIP concat / difference kernels (aanet_amd.nets.cost).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F
from .._precision import fp32_convs


def conv3d(in_channels, out_channels, kernel_size=3, stride=1, dilation=1, groups=1):
    """aggregation.py:8-13: Conv3d + BN3d + LeakyReLU(0.2)."""
    return nn.Sequential(nn.Conv3d(in_channels, out_channels, kernel_size=kernel_size,
                                   stride=stride, padding=dilation, dilation=dilation, bias=False,
                                   groups=groups),
                         nn.BatchNorm3d(out_channels), nn.LeakyReLU(0.2, inplace=True))


def convbn_3d(in_planes, out_planes, kernel_size, stride, pad):
    """aggregation.py:17-20 (PSMNet): Conv3d + BN3d."""
    return nn.Sequential(nn.Conv3d(in_planes, out_planes, kernel_size=kernel_size, padding=pad,
                                   stride=stride, bias=False),
                         nn.BatchNorm3d(out_planes))


def conv3x3_3d(in_planes, out_planes, stride=1, groups=1, dilation=1):
    """aggregation.py:51-56 (GC-Net): 3x3x3 Conv3d + BN3d + ReLU."""
    return nn.Sequential(nn.Conv3d(in_planes, out_planes, kernel_size=3, stride=stride,
                                   padding=dilation, dilation=dilation, groups=groups, bias=False),
                         nn.BatchNorm3d(out_planes), nn.ReLU(inplace=True))


def trans_conv3x3_3d(in_channels, out_channels, stride=1, groups=1, dilation=1):
    """aggregation.py:59-66 (GC-Net): ConvTranspose3d + BN3d + ReLU."""
    return nn.Sequential(nn.ConvTranspose3d(in_channels, out_channels, kernel_size=3,
                                            stride=stride, padding=dilation,
                                            output_padding=dilation, groups=groups,
                                            dilation=dilation, bias=False),
                         nn.BatchNorm3d(out_channels), nn.ReLU(inplace=True))


def _up4(cost):
    """[B,1,D,H,W] -> [B,4D,4H,4W] trilinear (align_corners=False), channel squeezed."""
    return torch.squeeze(F.interpolate(cost, scale_factor=4, mode='trilinear',
                                       align_corners=False), 1)


class StereoNetAggregation(nn.Module):
    """aggregation.py:69-90: four conv3d blocks + a 1-channel Conv3d -> [B, D, H, W]."""

    def __init__(self, in_channels=32):
        super(StereoNetAggregation, self).__init__()
        self.aggregation_layer = nn.Sequential(*[conv3d(in_channels, in_channels)
                                                 for _ in range(4)])
        self.final_conv = nn.Conv3d(in_channels, 1, kernel_size=3, stride=1, padding=1, bias=True)

    @fp32_convs
    def forward(self, cost_volume):
        assert cost_volume.dim() == 5  # [B, C, D, H, W]
        return self.final_conv(self.aggregation_layer(cost_volume)).squeeze(1)


class PSMNetBasicAggregation(nn.Module):
    """aggregation.py:93-138: 12 3-D convs (one shared conv1 block), x4 trilinear upsampling."""

    def __init__(self, max_disp):
        super(PSMNetBasicAggregation, self).__init__()
        self.max_disp = max_disp
        conv0 = convbn_3d(64, 32, 3, 1, 1)
        conv1 = convbn_3d(32, 32, 3, 1, 1)  # shared by every block below (as the reference)
        final_conv = nn.Conv3d(32, 1, kernel_size=3, padding=1, stride=1, bias=False)
        relu = lambda: nn.ReLU(inplace=True)  # noqa: E731
        self.dres0 = nn.Sequential(conv0, relu(), conv1, relu())
        for name in ("dres1", "dres2", "dres3", "dres4"):
            setattr(self, name, nn.Sequential(conv1, relu(), conv1))
        self.classify = nn.Sequential(conv1, relu(), final_conv)

    @fp32_convs
    def forward(self, cost):
        cost0 = self.dres0(cost)
        for name in ("dres1", "dres2", "dres3", "dres4"):
            cost0 = getattr(self, name)(cost0) + cost0
        return [_up4(self.classify(cost0))]


class PSMNetHourglass(nn.Module):
    """aggregation.py:142-189."""

    def __init__(self, inplanes):
        super(PSMNetHourglass, self).__init__()
        c2 = inplanes * 2
        self.conv1 = nn.Sequential(convbn_3d(inplanes, c2, kernel_size=3, stride=2, pad=1),
                                   nn.ReLU(inplace=True))
        self.conv2 = convbn_3d(c2, c2, kernel_size=3, stride=1, pad=1)
        self.conv3 = nn.Sequential(convbn_3d(c2, c2, kernel_size=3, stride=2, pad=1),
                                   nn.ReLU(inplace=True))
        self.conv4 = nn.Sequential(convbn_3d(c2, c2, kernel_size=3, stride=1, pad=1),
                                   nn.ReLU(inplace=True))
        self.conv5 = nn.Sequential(nn.ConvTranspose3d(c2, c2, kernel_size=3, padding=1,
                                                      output_padding=1, stride=2, bias=False),
                                   nn.BatchNorm3d(c2))
        self.conv6 = nn.Sequential(nn.ConvTranspose3d(c2, inplanes, kernel_size=3, padding=1,
                                                      output_padding=1, stride=2, bias=False),
                                   nn.BatchNorm3d(inplanes))

    @fp32_convs
    def forward(self, x, presqu, postsqu):
        pre = self.conv2(self.conv1(x))
        pre = F.relu(pre if postsqu is None else pre + postsqu, inplace=True)
        out = self.conv4(self.conv3(pre))
        post = F.relu(self.conv5(out) + (pre if presqu is None else presqu), inplace=True)
        return self.conv6(post), pre, post


class PSMNetHGAggregation(nn.Module):
    """aggregation.py:192-254: stacked hourglass; three cost outputs in training, one in eval."""

    def __init__(self, max_disp):
        super(PSMNetHGAggregation, self).__init__()
        self.max_disp = max_disp
        self.dres0 = nn.Sequential(convbn_3d(64, 32, 3, 1, 1), nn.ReLU(inplace=True),
                                   convbn_3d(32, 32, 3, 1, 1), nn.ReLU(inplace=True))
        self.dres1 = nn.Sequential(convbn_3d(32, 32, 3, 1, 1), nn.ReLU(inplace=True),
                                   convbn_3d(32, 32, 3, 1, 1))
        self.dres2 = PSMNetHourglass(32)
        self.dres3 = PSMNetHourglass(32)
        self.dres4 = PSMNetHourglass(32)
        for name in ("classif1", "classif2", "classif3"):
            setattr(self, name, nn.Sequential(
                convbn_3d(32, 32, 3, 1, 1), nn.ReLU(inplace=True),
                nn.Conv3d(32, 1, kernel_size=3, padding=1, stride=1, bias=False)))

    @fp32_convs
    def forward(self, cost):
        cost0 = self.dres0(cost)
        cost0 = self.dres1(cost0) + cost0
        out1, pre1, post1 = self.dres2(cost0, None, None)
        out1 = out1 + cost0
        out2, _, post2 = self.dres3(out1, pre1, post1)
        out2 = out2 + cost0
        out3, _, _ = self.dres4(out2, pre1, post2)  # pre1, as the reference (not pre2)
        out3 = out3 + cost0
        cost1 = self.classif1(out1)
        cost2 = self.classif2(out2) + cost1
        cost3 = self.classif3(out3) + cost2
        if self.training:
            return [_up4(cost1), _up4(cost2), _up4(cost3)]
        return [_up4(cost3)]


class GCNetAggregation(nn.Module):
    """aggregation.py:257-309: 3-D encoder-decoder down to 1/32 and back."""

    def __init__(self):
        super(GCNetAggregation, self).__init__()
        self.conv1 = nn.Sequential(conv3x3_3d(64, 32), conv3x3_3d(32, 32))
        for lvl, (cin, cout) in zip((2, 3, 4, 5), ((64, 64), (64, 64), (64, 64), (64, 128))):
            setattr(self, f"conv{lvl}a", conv3x3_3d(cin, cout, stride=2))
            setattr(self, f"conv{lvl}b", nn.Sequential(conv3x3_3d(cout, cout),
                                                       conv3x3_3d(cout, cout)))
        for i, (cin, cout) in enumerate(((128, 64), (64, 64), (64, 64), (64, 32)), start=1):
            setattr(self, f"trans_conv{i}", trans_conv3x3_3d(cin, cout, stride=2))
        self.trans_conv5 = nn.ConvTranspose3d(32, 1, kernel_size=3, stride=2, padding=1, groups=1,
                                              dilation=1, bias=False)

    @fp32_convs
    def forward(self, cost_volume):
        skip1 = self.conv1(cost_volume)
        a, skips = cost_volume, []
        for lvl in (2, 3, 4, 5):
            a = getattr(self, f"conv{lvl}a")(a)
            skips.append(getattr(self, f"conv{lvl}b")(a))
        x = self.trans_conv1(skips[3])
        x = self.trans_conv2(x + skips[2])
        x = self.trans_conv3(x + skips[1])
        x = self.trans_conv4(x + skips[0])
        return torch.squeeze(self.trans_conv5(x + skip1), 1)
