"""GPU parity of the plain-conv engine (aanet_conv2d_fused_f32) and the CSA resize-sum kernel
(aanet_csa_sum_f32) against torch CPU ops (the ops the reference runs for these layers:
nn.Conv2d / BatchNorm2d / LeakyReLU / F.interpolate(bilinear, align_corners=False)).
Tolerance: |err| <= 2e-5 * (1 + max|ref|) (fp32, different summation order)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"

CONV_CASES = [
    # N, C, H, W, Co, k, stride, pad, dil, groups   (the ISA/CSA layer family + edge cases)
    (2, 64, 16, 52, 64, 1, 1, 0, 1, 1),      # conv1 / conv3 / final_conv
    (2, 64, 16, 52, 64, 3, 1, 1, 1, 1),      # SimpleBottleneck conv2
    (2, 64, 16, 52, 54, 3, 1, 2, 2, 2),      # offset_conv (grouped, dilated, Cog = 27)
    (2, 64, 16, 52, 32, 3, 2, 1, 1, 1),      # CSA strided 3x3
    (2, 32, 8, 26, 64, 1, 1, 0, 1, 1),       # CSA 1x1 up-channel
    (1, 16, 5, 13, 16, 3, 2, 1, 1, 1),
    (1, 5, 7, 9, 3, 3, 1, 1, 1, 1),          # tiny, odd channels
    (1, 96, 9, 33, 80, 3, 1, 1, 1, 1),       # Co > 64 (two co tiles)
]


@pytest.mark.parametrize("case", CONV_CASES)
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "bn_leaky_res"])
@pytest.mark.parametrize("packed", [False, True])
def test_conv2d_fused_vs_torch_cpu(case, epi, packed):
    N, C, H, W, Co, k, s, p, d, g = case
    gen = torch.Generator().manual_seed(hash(case) % 1000)
    x = torch.randn(N, C, H, W, generator=gen)
    w = torch.randn(Co, C // g, k, k, generator=gen) / (C // g * k * k) ** 0.5
    b = torch.randn(Co, generator=gen)
    sc = torch.rand(Co, generator=gen) + 0.5
    sh = torch.randn(Co, generator=gen)
    ref = F.conv2d(x, w, None if epi == "plain" else b, s, p, d, g)
    res = None
    if epi == "bn_leaky_res":
        res = torch.randn(ref.shape, generator=gen)
        ref = F.leaky_relu(ref * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1) + res, 0.2)
    elif epi == "bias_relu":
        ref = F.relu(ref)
    act = {"plain": None, "bias_relu": "relu", "bn_leaky_res": "leaky"}[epi]
    wd = w.to(DEV)
    got = ops.conv2d_fused(x.to(DEV), wd, None if epi == "plain" else b.to(DEV), s, p, d, g,
                           act, None if res is None else res.to(DEV),
                           sc.to(DEV) if epi == "bn_leaky_res" else None,
                           sh.to(DEV) if epi == "bn_leaky_res" else None,
                           packed_weight=ops.pack_weight(wd) if packed else None).cpu()
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * (1 + ref.abs().max().item()), err


@pytest.mark.parametrize("sizes", [[(24, 48), (12, 24), (6, 12)], [(12, 24), (24, 48), (6, 12)],
                                   [(6, 12), (12, 24), (24, 48)], [(128, 416), (64, 208), (32, 104)],
                                   [(7, 13), (4, 7)], [(5, 9)]])
@pytest.mark.parametrize("act", [None, "leaky"])
def test_csa_sum_vs_torch_interpolate(sizes, act):
    gen = torch.Generator().manual_seed(len(sizes))
    N, C = 2, 8
    ins = [torch.randn(N, C, h, w, generator=gen) for h, w in sizes]
    H, W = sizes[0]
    ref = ins[0]
    for t in ins[1:]:
        if t.shape[2:] != ins[0].shape[2:]:
            t = F.interpolate(t, size=(H, W), mode="bilinear", align_corners=False)
        ref = ref + t
    if act == "leaky":
        ref = F.leaky_relu(ref, 0.2)
    got = ops.csa_sum([t.to(DEV) for t in ins], act=act).cpu()
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * (1 + ref.abs().max().item()), err
