"""AANet's feature extractor (nets/resnet.py): a ResNet-40 stem at 1/3
resolution whose last stage (H/12, C=128 bottlenecks) uses the HIP modulated DCN.

Module tree and initialisation follow resnet.py:104-194, so reference checkpoints load.  In
eval mode without autograd each bottleneck runs on the HIP engine (BN folded, residual + ReLU
in the last conv's epilogue; DeformBottleneck's offset conv and DCN on the HIP kernels).
"""
import torch.nn as nn

from ._fuse import FusedSequential, conv_bn_act, use_fused
from .deform import DeformBottleneck, _BottleneckBase
from .._precision import fp32_convs


def conv3x3(in_planes, out_planes, stride=1, groups=1, dilation=1):
    """resnet.py:6-9."""
    return nn.Conv2d(in_planes, out_planes, kernel_size=3, stride=stride, padding=dilation,
                     groups=groups, bias=False, dilation=dilation)


def conv1x1(in_planes, out_planes, stride=1):
    """resnet.py:12-14."""
    return nn.Conv2d(in_planes, out_planes, kernel_size=1, stride=stride, bias=False)


class BasicBlock(nn.Module):
    """resnet.py:17-55 (ReLU variant; kept for API parity, AANetFeature uses Bottleneck)."""
    expansion = 1
    __constants__ = ['downsample']

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super(BasicBlock, self).__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        if groups != 1 or base_width != 64:
            raise ValueError('BasicBlock only supports groups=1 and base_width=64')
        if dilation > 1:
            raise NotImplementedError("Dilation > 1 not supported in BasicBlock")
        self.conv1 = conv3x3(inplanes, planes, stride)
        self.bn1 = norm_layer(planes)
        self.relu = nn.ReLU(inplace=True)
        self.conv2 = conv3x3(planes, planes)
        self.bn2 = norm_layer(planes)
        self.downsample = downsample
        self.stride = stride

    @fp32_convs
    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        if use_fused(self, x) and isinstance(self.bn1, nn.BatchNorm2d):
            out = conv_bn_act(x, self.conv1, self.bn1, "relu")
            return conv_bn_act(out, self.conv2, self.bn2, "relu", residual=identity.contiguous())
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.bn2(self.conv2(out))
        out += identity
        return self.relu(out)


class Bottleneck(_BottleneckBase):
    """resnet.py:58-101: 1x1 -> 3x3 (stride) -> 1x1 (x4 channels) + shortcut."""
    expansion = 4
    __constants__ = ['downsample']

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64,
                 dilation=1, norm_layer=None):
        super(Bottleneck, self).__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        width = int(planes * (base_width / 64.)) * groups
        self.conv1 = conv1x1(inplanes, width)
        self.bn1 = norm_layer(width)
        self.conv2 = conv3x3(width, width, stride, groups, dilation)
        self.bn2 = norm_layer(width)
        self.conv3 = conv1x1(width, planes * self.expansion)
        self.bn3 = norm_layer(planes * self.expansion)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    @fp32_convs
    def forward(self, x):
        if use_fused(self, x):
            return self._forward_fused(x, deform=False)
        return self._forward_ref(x)


class AANetFeature(nn.Module):
    """resnet.py:104-194: [B,128,H/3,W/3], [B,256,H/6,W/6], [B,512,H/12,W/12]."""

    def __init__(self, in_channels=32, zero_init_residual=True, groups=1, width_per_group=64,
                 feature_mdconv=True, norm_layer=None):
        super(AANetFeature, self).__init__()
        norm_layer = norm_layer or nn.BatchNorm2d
        self._norm_layer = norm_layer
        self.inplanes = in_channels
        self.dilation = 1
        self.groups = groups
        self.base_width = width_per_group
        blocks = (3, 4, 6)  # ResNet-40
        self.conv1 = FusedSequential(nn.Conv2d(3, self.inplanes, kernel_size=7, stride=3,
                                               padding=3, bias=False),
                                     nn.BatchNorm2d(self.inplanes), nn.ReLU(inplace=True))
        self.layer1 = self._make_layer(Bottleneck, in_channels, blocks[0])
        self.layer2 = self._make_layer(Bottleneck, in_channels * 2, blocks[1], stride=2)
        self.layer3 = self._make_layer(DeformBottleneck if feature_mdconv else Bottleneck,
                                       in_channels * 4, blocks[2], stride=2)

        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        # zero-init the last BN of each residual branch (resnet.py:152-160); DeformBottleneck is
        # not a Bottleneck subclass in the reference, so its bn3 keeps weight 1
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.constant_(m.bn3.weight, 0)
                elif isinstance(m, BasicBlock):
                    nn.init.constant_(m.bn2.weight, 0)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        """resnet.py:162-187."""
        norm_layer = self._norm_layer
        downsample = None
        previous_dilation = self.dilation
        if dilate:
            self.dilation *= stride
            stride = 1
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = FusedSequential(conv1x1(self.inplanes, planes * block.expansion, stride),
                                         norm_layer(planes * block.expansion))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width,
                        previous_dilation, norm_layer)]
        self.inplanes = planes * block.expansion
        layers += [block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                         dilation=self.dilation, norm_layer=norm_layer) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    @fp32_convs
    def forward(self, x):
        x = self.conv1(x)
        layer1 = self.layer1(x)
        layer2 = self.layer2(layer1)
        return [layer1, layer2, self.layer3(layer2)]
