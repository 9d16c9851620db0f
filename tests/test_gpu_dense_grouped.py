"""A 2-group conv with 16-channel groups (the scale-1 offset_conv, nets/deform.py:63-65: 32 -> 54,
3x3, dilation 2) runs in eval as one ungrouped block-diagonal conv on the split-bf16 engine
(nets/_fuse.py dense_grouped_ok): against fp64, held to the grouped exact-f32 engine's error, and
the weight cache follows parameter updates."""
import pytest
import torch
import torch.nn as nn
import torch.nn.functional as F

from aanet_amd.nets._fuse import conv_bn_act, dense_grouped_ok
from aanet_amd.nets.options import set_options

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("N,H,W,nhwc", [(2, 64, 208, True), (1, 17, 23, True), (1, 9, 12, False)])
def test_dense_grouped_offset_conv_vs_fp64(N, H, W, nhwc):
    torch.manual_seed(5)
    conv = nn.Conv2d(32, 54, 3, padding=2, dilation=2, groups=2, bias=True).to(DEV).eval()
    with torch.no_grad():
        conv.weight.normal_(0, 0.1)
        conv.bias.normal_(0, 0.5)
    x = torch.randn(N, 32, H, W, device=DEV).relu_()
    xin = x.contiguous(memory_format=torch.channels_last) if nhwc else x
    assert dense_grouped_ok(conv, xin)
    y64 = F.conv2d(x.double().cpu(), conv.weight.double().cpu(), conv.bias.double().cpu(),
                   padding=2, dilation=2, groups=2)
    scale = F.conv2d(x.double().cpu().abs(), conv.weight.double().cpu().abs(), padding=2,
                     dilation=2, groups=2) + 1.0
    with torch.no_grad():
        got = conv_bn_act(xin, conv)
        set_options(conv, dense_grouped=False)
        assert not dense_grouped_ok(conv, xin)
        grouped = conv_bn_act(xin, conv)  # the grouped engine (exact-f32 16-channel form)
        set_options(conv, dense_grouped=True)
    err = ((got.double().cpu() - y64).abs() / scale).max().item()
    err_g = ((grouped.double().cpu() - y64).abs() / scale).max().item()
    assert err <= max(4 * err_g, 2e-7), (err, err_g)
    # the block-diagonal weight follows an in-place parameter update (cache keyed on _version)
    with torch.no_grad():
        conv.weight.mul_(-1.0)
        got2 = conv_bn_act(xin, conv)
    y64b = F.conv2d(x.double().cpu(), conv.weight.double().cpu(), conv.bias.double().cpu(),
                    padding=2, dilation=2, groups=2)
    assert ((got2.double().cpu() - y64b).abs() / scale).max().item() <= max(4 * err_g, 2e-7)
