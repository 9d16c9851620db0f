"""Disparity refinement (nets/refinement.py): StereoNet, StereoDRNet (AANet)
and Hourglass (AANet+, with full-resolution HIP DCNs) refinement modules.

The warp is the HIP disp_warp kernel; in eval mode without autograd every plain conv (+BN
+LeakyReLU) runs on the HIP engine, and the last conv adds the upsampled disparity and applies
the ReLU in its epilogue (`relu(disp + final_conv(x))` is one kernel).  Module trees are the
reference's (checkpoint-compatible).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops
from ._fuse import FusedSequential, conv_bn_act, folded, use_fused
from .deform import DeformConv2d
from .feature import BasicBlock, BasicConv, Conv2x, _hourglass2
from .warp import disp_warp
from .._precision import fp32_convs


def conv2d(in_channels, out_channels, kernel_size=3, stride=1, dilation=1, groups=1):
    """refinement.py:10-15: conv + BN + LeakyReLU(0.2)."""
    return FusedSequential(nn.Conv2d(in_channels, out_channels, kernel_size=kernel_size,
                                     stride=stride, padding=dilation, dilation=dilation,
                                     bias=False, groups=groups),
                           nn.BatchNorm2d(out_channels), nn.LeakyReLU(0.2, inplace=True))


def _upsampled_disp(low_disp, img, always_resize=False):
    """[B,h,w] disparity -> [B,1,H,W] at the image size, scaled by W/w (refinement.py:41-44,
    84-90): bilinear, align_corners=False; returned unchanged when already at that size."""
    assert low_disp.dim() == 3
    low = low_disp.unsqueeze(1)
    scale = img.size(-1) / low.size(-1)
    if scale == 1.0 and not always_resize:
        return low
    return F.interpolate(low, size=img.shape[-2:], mode='bilinear', align_corners=False) * scale


def _residual_out(module, feat, disp):
    """relu(disp + final_conv(feat)) squeezed to [B, H, W]."""
    if use_fused(module, feat):
        return conv_bn_act(feat, module.final_conv, None, "relu",
                           residual=disp.contiguous()).squeeze(1)
    return F.relu(disp + module.final_conv(feat), inplace=True).squeeze(1)


class _DilatedStack(nn.Sequential):
    """The six dilated BasicBlocks (refinement.py:30-35 / 74-79; nn.Sequential keys).  In eval
    mode without autograd the chain runs channels-last: one NCHW -> NHWC copy in, then every
    conv reads and writes NHWC (the dilation-1/2 convs take the halo-tile engine path, 1.3-1.5x
    faster than NCHW staging at 32 ch x 384x1248), residuals NHWC; the output stays NHWC for
    final_conv, which reads it in place."""

    def forward(self, x):
        blocks = list(self)
        if not (use_fused(self, x) and all(isinstance(b, BasicBlock) and b.downsample is None and
                                           isinstance(b.bn1, nn.BatchNorm2d) for b in blocks)):
            return super().forward(x)
        h = x.contiguous(memory_format=torch.channels_last)
        for b in blocks:
            act = "leaky" if isinstance(b.relu, nn.LeakyReLU) else "relu"
            out = conv_bn_act(h, b.conv1, b.bn1, act, out_nhwc=True)
            h = conv_bn_act(out, b.conv2, b.bn2, act, residual=h, out_nhwc=True)
        return h


def _dilated_stack():
    return _DilatedStack(*[BasicBlock(32, 32, stride=1, dilation=d) for d in (1, 2, 4, 8, 1, 1)])


class StereoNetRefinement(nn.Module):
    """refinement.py:18-54: image-guided residual on the upsampled disparity."""

    def __init__(self):
        super(StereoNetRefinement, self).__init__()
        self.conv = conv2d(4, 32)
        self.dilation_list = [1, 2, 4, 8, 1, 1]
        self.dilated_blocks = _dilated_stack()
        self.final_conv = nn.Conv2d(32, 1, 3, 1, 1)

    @fp32_convs
    def forward(self, low_disp, left_img, right_img=None):
        disp = _upsampled_disp(low_disp, left_img, always_resize=True)
        out = self.dilated_blocks(self.conv(torch.cat((disp, left_img), dim=1)))
        return _residual_out(self, out, disp)


class _WarpErrorStem(nn.Module):
    """Shared input stage of StereoDRNet / Hourglass refinement (refinement.py:92-99, 148-155):
    warp the right image by the disparity, [error, left] -> 16 ch, disparity -> 16 ch."""

    # whether the eval stem emits its 32 channels channels-last in one kernel (StereoDRNet: the
    # dilated stack reads NHWC, the concat and the NHWC copy go away, AANet 24.0 -> 23.4 ms;
    # Hourglass: conv_start's offset conv on the halo tile and its DCN on the NHWC window form,
    # 1,136 + 1,134 -> 789 + 928 us at full resolution, tools/refine_dcn_layout_bench.py)
    _stem_nhwc = False

    def _stem(self, low_disp, left_img, right_img):
        disp = _upsampled_disp(low_disp, left_img)
        warped_right = disp_warp(right_img, disp)[0]
        if self._stem_fused(left_img):  # one kernel, channels-last out (aanet_refine_stem_f32)
            w1, b1, _ = folded(self.conv1[0], self.conv1[1])
            w2, b2, _ = folded(self.conv2[0], self.conv2[1])
            return disp, ops.refine_stem(warped_right, left_img, disp.contiguous(), w1, b1, w2, b2)
        concat1 = torch.cat((warped_right - left_img, left_img), dim=1)
        return disp, torch.cat((self.conv1(concat1), self.conv2(disp)), dim=1)

    def _stem_fused(self, x):
        """Eval fast path of the stem: both convs the reference's 3x3 pad-1 conv + BN +
        LeakyReLU(0.2) (6 -> 16, 1 -> 16) on 3-channel images."""
        if not (use_fused(self, x) and x.shape[1] == 3 and self._stem_nhwc):
            return False
        for seq, cin in ((self.conv1, 6), (self.conv2, 1)):
            c = seq[0]
            if not (isinstance(c, nn.Conv2d) and tuple(c.weight.shape) == (16, cin, 3, 3) and
                    c.stride == (1, 1) and c.padding == (1, 1) and c.dilation == (1, 1) and
                    c.groups == 1 and isinstance(seq[1], nn.BatchNorm2d) and
                    isinstance(seq[2], nn.LeakyReLU) and seq[2].negative_slope == 0.2 and
                    getattr(seq, "aanet_fuse", True)):
                return False
        return True


class StereoDRNetRefinement(_WarpErrorStem):
    """refinement.py:57-108 (AANet)."""
    _stem_nhwc = True

    def __init__(self):
        super(StereoDRNetRefinement, self).__init__()
        self.conv1 = conv2d(6, 16)
        self.conv2 = conv2d(1, 16)
        self.dilation_list = [1, 2, 4, 8, 1, 1]
        self.dilated_blocks = _dilated_stack()
        self.final_conv = nn.Conv2d(32, 1, 3, 1, 1)

    @fp32_convs
    def forward(self, low_disp, left_img, right_img):
        disp, x = self._stem(low_disp, left_img, right_img)
        return _residual_out(self, self.dilated_blocks(x), disp)


class HourglassRefinement(_WarpErrorStem):
    """refinement.py:111-202 (AANet+).  Height and width must be divisible by 16."""
    _stem_nhwc = True

    def __init__(self):
        super(HourglassRefinement, self).__init__()
        self.conv1 = conv2d(6, 16)
        self.conv2 = conv2d(1, 16)
        self.conv_start = DeformConv2d(32, 32)
        self.conv1a = BasicConv(32, 48, kernel_size=3, stride=2, padding=1)
        self.conv2a = BasicConv(48, 64, kernel_size=3, stride=2, padding=1)
        self.conv3a = DeformConv2d(64, 96, kernel_size=3, stride=2)
        self.conv4a = DeformConv2d(96, 128, kernel_size=3, stride=2)
        chans = (32, 48, 64, 96, 128)
        for sfx in "ab":
            for i in range(4, 0, -1):
                setattr(self, f"deconv{i}{sfx}", Conv2x(chans[i], chans[i - 1], deconv=True))
        self.conv1b = Conv2x(32, 48)
        self.conv2b = Conv2x(48, 64)
        self.conv3b = Conv2x(64, 96, mdconv=True)
        self.conv4b = Conv2x(96, 128, mdconv=True)
        self.final_conv = nn.Conv2d(32, 1, 3, 1, 1)

    @fp32_convs
    def forward(self, low_disp, left_img, right_img):
        disp, x = self._stem(low_disp, left_img, right_img)
        # the last block's output channels-last: final_conv (32 -> 1) reads it NHWC
        if not use_fused(self.conv_start, x):
            x = x.contiguous()  # the stem's channels-last output goes to a reference-order DCN
        feat = _hourglass2(self, self.conv_start(x), last_nhwc=use_fused(self, x))
        return _residual_out(self, feat, disp)
