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
@pytest.mark.parametrize("packed", [False, True, "split"])
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
                           packed_weight=_packed(wd, g, packed)).cpu()
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * (1 + ref.abs().max().item()), err


# the few-channel shapes of aanet_amd/csrc/small_conv.hip (direct VALU conv): AANet's first
# feature conv (3 -> 32, 7x7 / 3), GA-Net's conv_start (3 -> 32, 3x3), the refinement stems
# (6 / 1 -> 16) and final_conv (32 -> 1); ragged tiles (H % 8, W % 32)
DIRECT_CASES = [
    (2, 3, 40, 70, 32, 7, 3, 3, 1, 1),
    (2, 3, 17, 45, 32, 3, 1, 1, 1, 1),
    (2, 3, 17, 45, 20, 3, 1, 1, 1, 1),
    (2, 6, 17, 45, 16, 3, 1, 1, 1, 1),
    (2, 1, 17, 45, 16, 3, 1, 1, 1, 1),
    (2, 32, 17, 45, 1, 3, 1, 1, 1, 1),
]


@pytest.mark.parametrize("case", DIRECT_CASES)
@pytest.mark.parametrize("epi", ["plain", "bias_relu", "bn_leaky_res"])
@pytest.mark.parametrize("packed", [False, True])
@pytest.mark.parametrize("nhwc", [False, True])
def test_conv2d_direct_shapes_vs_torch(case, epi, packed, nhwc):
    """Few-channel convs on the direct kernel vs torch fp64 (exact f32 FMAs: 1e-5 relative)."""
    N, C, H, W, Co, k, s, p, d, g = case
    if nhwc and C % 4:
        pytest.skip("channels-last input needs C % 4 == 0")
    gen = torch.Generator().manual_seed(7 + C + Co)
    x = torch.randn(N, C, H, W, generator=gen)
    w = torch.randn(Co, C, k, k, generator=gen) / (C * k * k) ** 0.5
    b, sc, sh = torch.randn(Co, generator=gen), torch.rand(Co, generator=gen) + 0.5, torch.randn(Co, generator=gen)
    ref = F.conv2d(x.double(), w.double(), None if epi == "plain" else b.double(), s, p, d, g)
    res = None
    if epi == "bn_leaky_res":
        res = torch.randn(ref.shape, generator=gen)
        ref = F.leaky_relu(ref * sc.double().view(1, -1, 1, 1) + sh.double().view(1, -1, 1, 1) + res.double(), 0.2)
    elif epi == "bias_relu":
        ref = F.relu(ref)
    act = {"plain": None, "bias_relu": "relu", "bn_leaky_res": "leaky"}[epi]
    wd, xd = w.to(DEV), x.to(DEV)
    if nhwc:
        xd = xd.contiguous(memory_format=torch.channels_last)
    got = ops.conv2d_fused(xd, wd, None if epi == "plain" else b.to(DEV), s, p, d, g, act,
                           None if res is None else res.to(DEV),
                           sc.to(DEV) if epi == "bn_leaky_res" else None,
                           sh.to(DEV) if epi == "bn_leaky_res" else None,
                           packed_weight=ops.pack_weight(wd) if (packed or nhwc) else None).cpu().double()
    err = (got - ref).abs().max().item()
    assert err <= 1e-5 * (1 + ref.abs().max().item()), err


def _packed(wd, groups, packed):
    """None (reference layout), pack_weight (exact f32 engine) or the split-bf16 buffer (falls
    back to pack_weight where the shape has no split form)."""
    if not packed:
        return None
    if packed == "split":
        ws = ops.pack_weight_split(wd, groups)
        return ws if ws is not None else ops.pack_weight(wd)
    return ops.pack_weight(wd)


@pytest.mark.parametrize("sizes", [[(24, 48), (12, 24), (6, 12)], [(8, 20), (4, 10), (2, 5)], [(4, 8), (1, 2)], [(12, 24), (24, 48), (6, 12)],
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


@pytest.mark.parametrize("C,H,W", [(64, 16, 52), (32, 9, 26), (16, 5, 13), (48, 7, 30)])
def test_conv2d_pw_tail_vs_torch_cpu(C, H, W):
    """conv3x3 + BN + ReLU -> 1x1 conv + BN + identity + ReLU (SimpleBottleneck tail) in one kernel."""
    gen = torch.Generator().manual_seed(C)
    N = 2
    x = torch.randn(N, C, H, W, generator=gen)
    w2 = torch.randn(C, C, 3, 3, generator=gen) / (3 * C ** 0.5)
    b2 = torch.randn(C, generator=gen)
    w3 = torch.randn(C, C, 1, 1, generator=gen) / C ** 0.5
    b3 = torch.randn(C, generator=gen)
    ident = torch.randn(N, C, H, W, generator=gen)
    ref = F.relu(F.conv2d(F.relu(F.conv2d(x, w2, b2, 1, 1)), w3, b3) + ident)
    d = lambda t: t.to(DEV)  # noqa: E731
    got = ops.conv2d_pw(d(x), d(w2), ops.pack_weight(d(w2)), d(b2), None, None, "relu",
                        ops.pack_weight(d(w3)), d(b3), d(ident), "relu", 1, 1, 1).cpu()
    err = (got - ref).abs().max().item()
    assert err <= 3e-5 * (1 + ref.abs().max().item()), err


@pytest.mark.parametrize("C,H,W", [(64, 16, 52), (32, 9, 26), (16, 5, 13)])
def test_mdcn_pw_tail_vs_oracle(C, H, W):
    """DeformSimpleBottleneck tail: DCN (+BN2+ReLU, mask = 2*sigmoid) -> conv3 + BN3 + identity + ReLU."""
    import numpy as np
    from oracle import oracle
    rng = np.random.default_rng(C)
    N, dg = 2, 2
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    om = rng.standard_normal((N, dg * 27, H, W)).astype(np.float32)
    w2 = (rng.standard_normal((C, C, 3, 3)) / (3 * C ** 0.5)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, C).astype(np.float32)
    sh = rng.standard_normal(C).astype(np.float32)
    w3 = (rng.standard_normal((C, C, 1, 1)) / C ** 0.5).astype(np.float32)
    b3 = rng.standard_normal(C).astype(np.float32)
    ident = rng.standard_normal((N, C, H, W)).astype(np.float32)
    mask = (2.0 / (1.0 + np.exp(-om[:, dg * 18:].astype(np.float64)))).astype(np.float32)
    t = oracle.mdcn_forward(x, om[:, :dg * 18], mask, w2, None, 1, 2, 2, 1, dg)
    t = np.maximum(t * sc[None, :, None, None] + sh[None, :, None, None], 0)
    ref = F.relu(F.conv2d(torch.from_numpy(t), torch.from_numpy(w3), torch.from_numpy(b3)) +
                 torch.from_numpy(ident)).numpy()
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    w2d, w3d = d(w2), d(w3)
    got = ops.mdcn_pw(d(x), d(om), w2d, ops.pack_weight(w2d), None, d(sc), d(sh), "relu",
                      ops.pack_weight(w3d), d(b3), d(ident), "relu", 1, 2, 2, dg, 2.0).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-4 * (1 + np.abs(ref).max())


# ---------------------------------------------------------------- NHWC (channels_last) paths
NHWC_CASES = [
    # N, C, H, W, Co, k, stride, pad, dil, groups   (32-channel groups, as NHWC requires)
    (2, 64, 16, 52, 64, 1, 1, 0, 1, 1),      # bottleneck conv1 (NCHW in -> NHWC out)
    (2, 64, 16, 52, 64, 3, 1, 1, 1, 1),      # SimpleBottleneck conv2 (NHWC in)
    (2, 64, 16, 52, 54, 3, 1, 2, 2, 2),      # offset_conv on the NHWC conv1 output
    (1, 64, 9, 27, 32, 3, 2, 1, 1, 1),       # strided, odd sizes, 64-px tiles
    (1, 128, 5, 11, 40, 3, 1, 1, 1, 4),      # 4 groups of 32, Co not a tile multiple
    (2, 32, 9, 26, 54, 3, 1, 2, 2, 2),       # scale-1 offset_conv: 16-channel groups (CFG 1)
    (1, 64, 7, 20, 80, 3, 1, 1, 1, 4),       # 16-channel groups, Cog 20
]


@pytest.mark.parametrize("case", NHWC_CASES)
@pytest.mark.parametrize("layout", [1, 2, 3])
def test_conv2d_fused_nhwc_vs_torch_cpu(case, layout):
    """AANET_LAYOUT_IN_NHWC / OUT_NHWC: same values as the NCHW path (channels_last tensors)."""
    N, C, H, W, Co, k, s, p, d, g = case
    gen = torch.Generator().manual_seed(7 + layout)
    x = torch.randn(N, C, H, W, generator=gen)
    w = torch.randn(Co, C // g, k, k, generator=gen) / (C // g * k * k) ** 0.5
    b = torch.randn(Co, generator=gen)
    res = torch.randn(N, Co, (H + 2 * p - d * (k - 1) - 1) // s + 1,
                      (W + 2 * p - d * (k - 1) - 1) // s + 1, generator=gen)
    ref = F.relu(F.conv2d(x, w, b, s, p, d, g) + res)
    xd = x.to(DEV)
    if layout & 1:
        xd = xd.contiguous(memory_format=torch.channels_last)
    rd = res.to(DEV)
    if layout & 2 and (Co // g) % 4:
        pytest.skip("NHWC output needs (Co / groups) % 4 == 0")
    if layout & 2:
        rd = rd.contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV)
    got = ops.conv2d_fused(xd, wd, b.to(DEV), s, p, d, g, "relu", rd,
                           packed_weight=ops.pack_weight(wd), out_nhwc=bool(layout & 2))
    if layout & 2:
        assert got.is_contiguous(memory_format=torch.channels_last)
    got = got.cpu().contiguous()
    err = (got - ref).abs().max().item()
    assert err <= 2e-5 * (1 + ref.abs().max().item()), err


def test_conv2d_nhwc_requires_full_chunks():
    from aanet_amd._lib import AanetError
    x = torch.randn(1, 16, 8, 8, device=DEV).contiguous(memory_format=torch.channels_last)
    w = torch.randn(16, 16, 3, 3, device=DEV)
    with pytest.raises(AanetError):  # 16-channel chunks need >= 32-wide output tiles
        ops.conv2d_fused(x, w, None, 1, 1, 1, 1, packed_weight=ops.pack_weight(w))
    x = torch.randn(1, 24, 8, 8, device=DEV).contiguous(memory_format=torch.channels_last)
    w = torch.randn(32, 24, 3, 3, device=DEV)
    with pytest.raises(AanetError):  # 24 channels: no full-chunk configuration
        ops.conv2d_fused(x, w, None, 1, 1, 1, 1, packed_weight=ops.pack_weight(w))


@pytest.mark.parametrize("C,H,W", [(64, 16, 52), (64, 9, 26)])
def test_conv2d_pw_tail_nhwc_input(C, H, W):
    gen = torch.Generator().manual_seed(C + H)
    N = 2
    x = torch.randn(N, C, H, W, generator=gen)
    w2 = torch.randn(C, C, 3, 3, generator=gen) / (3 * C ** 0.5)
    b2 = torch.randn(C, generator=gen)
    w3 = torch.randn(C, C, 1, 1, generator=gen) / C ** 0.5
    b3 = torch.randn(C, generator=gen)
    ident = torch.randn(N, C, H, W, generator=gen)
    ref = F.relu(F.conv2d(F.relu(F.conv2d(x, w2, b2, 1, 1)), w3, b3) + ident)
    d = lambda t: t.to(DEV)  # noqa: E731
    xd = d(x).contiguous(memory_format=torch.channels_last)
    got = ops.conv2d_pw(xd, d(w2), ops.pack_weight(d(w2)), d(b2), None, None, "relu",
                        ops.pack_weight(d(w3)), d(b3), d(ident), "relu", 1, 1, 1).cpu()
    err = (got - ref).abs().max().item()
    assert err <= 3e-5 * (1 + ref.abs().max().item()), err


@pytest.mark.parametrize("C,H,W,off_scale,dg", [(64, 16, 52, 1.0, 2), (64, 9, 26, 3.0, 2),
                                                (32, 7, 19, 1.0, 1), (32, 9, 26, 1.5, 2),
                                                (64, 6, 17, 2.0, 4)])
def test_mdcn_pw_tail_nhwc_input_vs_oracle(C, H, W, off_scale, dg):
    """DCN with NHWC corner loads (+BN2+ReLU, mask = 2*sigmoid) -> conv3 + identity + ReLU.
    dg with 16-channel groups: chunks span two groups, one sampling state each (CFG 2)."""
    from oracle import oracle
    rng = np.random.default_rng(C + W)
    N = 2
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    om = rng.standard_normal((N, dg * 27, H, W)).astype(np.float32)
    om[:, :dg * 18] *= off_scale
    w2 = (rng.standard_normal((C, C, 3, 3)) / (3 * C ** 0.5)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, C).astype(np.float32)
    sh = rng.standard_normal(C).astype(np.float32)
    w3 = (rng.standard_normal((C, C, 1, 1)) / C ** 0.5).astype(np.float32)
    b3 = rng.standard_normal(C).astype(np.float32)
    ident = rng.standard_normal((N, C, H, W)).astype(np.float32)
    mask = (2.0 / (1.0 + np.exp(-om[:, dg * 18:].astype(np.float64)))).astype(np.float32)
    t = oracle.mdcn_forward(x, om[:, :dg * 18], mask, w2, None, 1, 2, 2, 1, dg)
    t = np.maximum(t * sc[None, :, None, None] + sh[None, :, None, None], 0)
    ref = F.relu(F.conv2d(torch.from_numpy(t), torch.from_numpy(w3), torch.from_numpy(b3)) +
                 torch.from_numpy(ident)).numpy()
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    w2d, w3d = d(w2), d(w3)
    xd = d(x).contiguous(memory_format=torch.channels_last)
    got = ops.mdcn_pw(xd, d(om), w2d, ops.pack_weight(w2d), None, d(sc), d(sh), "relu",
                      ops.pack_weight(w3d), d(b3), d(ident), "relu", 1, 2, 2, dg, 2.0).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-4 * (1 + np.abs(ref).max())
    # and the same kernel family on NCHW input agrees to rounding
    got2 = ops.mdcn_pw(d(x), d(om), w2d, ops.pack_weight(w2d), None, d(sc), d(sh), "relu",
                       ops.pack_weight(w3d), d(b3), d(ident), "relu", 1, 2, 2, dg, 2.0).cpu().numpy()
    assert np.abs(got - got2).max() <= 2e-5 * (1 + np.abs(ref).max())


def test_mdcn_forward_fused_nhwc_input_vs_oracle():
    from oracle import oracle
    rng = np.random.default_rng(5)
    N, C, H, W, dg = 2, 64, 12, 40, 2
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    om = rng.standard_normal((N, dg * 27, H, W)).astype(np.float32) * 1.5
    w = (rng.standard_normal((C, C, 3, 3)) / (3 * C ** 0.5)).astype(np.float32)
    mask = (2.0 / (1.0 + np.exp(-om[:, dg * 18:].astype(np.float64)))).astype(np.float32)
    ref = oracle.mdcn_forward(x, om[:, :dg * 18], mask, w, None, 1, 2, 2, 1, dg)
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    wd = d(w)
    got = ops.mdcn_forward_fused(d(x).contiguous(memory_format=torch.channels_last), d(om), wd,
                                 None, None, None, None, 1, 2, 2, dg, 2.0,
                                 packed_weight=ops.pack_weight(wd)).cpu().numpy()
    assert np.abs(got - ref).max() <= 2e-5 * (1 + np.abs(ref).max())


@pytest.mark.parametrize("nhwc", [False, True])
@pytest.mark.parametrize("H,W,ups", [(16, 52, [(8, 26), (4, 13)]), (12, 40, [(6, 20)]),
                                     (8, 24, [(2, 6), (4, 12)])])
def test_tail_csa_epilogue_matches_separate_sum(nhwc, H, W, ups):
    """aanet_csa_epilogue_t: the tail kernel's cross-scale sum equals csa_sum over its output."""
    gen = torch.Generator().manual_seed(H * W)
    N, C = 2, 64
    d = lambda t: t.to(DEV)  # noqa: E731
    x = d(torch.randn(N, C, H, W, generator=gen))
    w2 = d(torch.randn(C, C, 3, 3, generator=gen) / (3 * C ** 0.5))
    b2 = d(torch.randn(C, generator=gen))
    w3 = d(torch.randn(C, C, 1, 1, generator=gen) / C ** 0.5)
    b3 = d(torch.randn(C, generator=gen))
    ident = d(torch.randn(N, C, H, W, generator=gen))
    terms = [d(torch.randn(N, C, h, w, generator=gen)) for h, w in ups]
    xin = x.contiguous(memory_format=torch.channels_last) if nhwc else x
    args = (w2, ops.pack_weight(w2), b2, None, None, "relu", ops.pack_weight(w3), b3, ident, "relu",
            1, 1, 1)
    out, csa = ops.conv2d_pw(xin, *args, csa_up=terms)
    ref_out = ops.conv2d_pw(xin, *args)
    ref_csa = ops.csa_sum([ref_out] + terms, act="leaky")
    assert torch.equal(out, ref_out)
    err = (csa - ref_csa).abs().max().item()
    assert err <= 1e-5 * (1 + ref_csa.abs().max().item()), err
    # and against torch's own interpolate
    t = ref_out.cpu()
    for u in terms:
        t = t + F.interpolate(u.cpu(), size=(H, W), mode="bilinear", align_corners=False)
    err = (csa.cpu() - F.leaky_relu(t, 0.2)).abs().max().item()
    assert err <= 2e-5 * (1 + t.abs().max().item()), err


def test_mdcn_tail_csa_epilogue_matches_separate_sum():
    gen = torch.Generator().manual_seed(3)
    N, C, H, W, dg = 2, 64, 16, 52, 2
    d = lambda t: t.to(DEV)  # noqa: E731
    x = d(torch.randn(N, C, H, W, generator=gen)).contiguous(memory_format=torch.channels_last)
    om = d(torch.randn(N, dg * 27, H, W, generator=gen))
    w2 = d(torch.randn(C, C, 3, 3, generator=gen) / (3 * C ** 0.5))
    sc, sh = d(torch.rand(C, generator=gen) + 0.5), d(torch.randn(C, generator=gen))
    w3 = d(torch.randn(C, C, 1, 1, generator=gen) / C ** 0.5)
    b3 = d(torch.randn(C, generator=gen))
    ident = d(torch.randn(N, C, H, W, generator=gen))
    terms = [d(torch.randn(N, C, H // 2, W // 2, generator=gen)),
             d(torch.randn(N, C, H // 4, W // 4, generator=gen))]
    args = (om, w2, ops.pack_weight(w2), None, sc, sh, "relu", ops.pack_weight(w3), b3, ident,
            "relu", 1, 2, 2, dg, 2.0)
    out, csa = ops.mdcn_pw(x, *args, csa_up=terms)
    ref_out = ops.mdcn_pw(x, *args)
    assert torch.equal(out, ref_out)
    ref_csa = ops.csa_sum([ref_out] + terms, act="leaky")
    err = (csa - ref_csa).abs().max().item()
    assert err <= 1e-5 * (1 + ref_csa.abs().max().item()), err


def test_tail_csa_epilogue_rejects_non_integer_ratio():
    N, C, H, W = 1, 32, 8, 24
    x = torch.randn(N, C, H, W, device=DEV)
    w2 = torch.randn(C, C, 3, 3, device=DEV)
    w3 = torch.randn(C, C, 1, 1, device=DEV)
    with pytest.raises(Exception):
        ops.conv2d_pw(x, w2, ops.pack_weight(w2), None, None, None, "relu", ops.pack_weight(w3),
                      None, None, "relu", 1, 1, 1, csa_up=[torch.randn(N, C, 3, 9, device=DEV)])


# ------------------------------------------- dilation > 2: phase-strided halo tiles (HALO 4)
PHASE_CASES = [
    # N, C, H, W, Co, dil   (3x3, stride 1, pad = dil; the refinement's dilated BasicBlocks)
    (2, 32, 40, 104, 32, 4),     # StereoDRNet dilation 4 (nets/refinement.py:60-106)
    (1, 32, 48, 160, 32, 8),     # dilation 8
    (1, 32, 19, 37, 32, 3),      # ragged phases: H, W not multiples of the dilation
    (1, 64, 21, 70, 64, 4),      # 64 channels (two K chunks), 64-channel tile
    (1, 32, 5, 9, 32, 8),        # image smaller than one dilation step in both directions
]


@pytest.mark.parametrize("case", PHASE_CASES)
@pytest.mark.parametrize("residual", [False, True])
def test_conv2d_dilated_phase_halo_vs_torch(case, residual):
    """Split-bf16 3x3 convs of dilation > 2, NHWC in and out (the form the refinement's dilated
    blocks run): the D x D phase-strided halo tiles against torch CPU in fp64, at fp32 accuracy."""
    N, C, H, W, Co, d = case
    gen = torch.Generator().manual_seed(31 + d + C)
    x = torch.randn(N, C, H, W, generator=gen, dtype=torch.float64)
    w = torch.randn(Co, C, 3, 3, generator=gen, dtype=torch.float64) / (C * 9) ** 0.5
    b = torch.randn(Co, generator=gen, dtype=torch.float64)
    res = torch.randn(N, Co, H, W, generator=gen, dtype=torch.float64) if residual else None
    ref = F.conv2d(x, w, b, 1, d, d) + (res if residual else 0)
    ref = F.relu(ref)
    xd = x.float().to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.float().to(DEV)
    wp = ops.pack_weight_split(wd)
    assert wp is not None
    rd = res.float().to(DEV).contiguous(memory_format=torch.channels_last) if residual else None
    got = ops.conv2d_fused(xd, wd, b.float().to(DEV), 1, d, d, 1, "relu", rd, packed_weight=wp,
                           out_nhwc=True)
    assert got.is_contiguous(memory_format=torch.channels_last)
    err = (got.cpu().double() - ref).abs().max().item()
    assert err <= 2e-5 * (1 + ref.abs().max().item()), err


@pytest.mark.parametrize("H,W", [(96, 312), (13, 37)])
def test_refine_stem_matches_separate_convs(H, W):
    """aanet_refine_stem_f32 (the StereoDRNet / Hourglass refinement stem, nets/refinement.py:
    92-99: conv1 on [warped - left, left] and conv2 on the disparity, concatenated) against the
    same convs run one by one on the HIP direct kernel + torch.cat: identical values (same
    per-channel arithmetic), channels-last; and within fp32 of torch CPU."""
    from aanet_amd.nets.refinement import StereoDRNetRefinement
    torch.manual_seed(5)
    m = StereoDRNetRefinement()
    with torch.no_grad():
        for seq in (m.conv1, m.conv2):
            seq[1].running_mean.normal_(0, 0.1)
            seq[1].running_var.uniform_(0.5, 1.5)
    m = m.to(DEV).eval()
    g = torch.Generator(device=DEV).manual_seed(6)
    warped = torch.randn(2, 3, H, W, device=DEV, generator=g)
    left = torch.randn(2, 3, H, W, device=DEV, generator=g)
    disp = torch.rand(2, 1, H, W, device=DEV, generator=g) * 40
    from aanet_amd.nets._fuse import folded
    with torch.no_grad():
        w1, b1, _ = folded(m.conv1[0], m.conv1[1])
        w2, b2, _ = folded(m.conv2[0], m.conv2[1])
        got = ops.refine_stem(warped, left, disp, w1, b1, w2, b2)
        ref = torch.cat((m.conv1(torch.cat((warped - left, left), 1)), m.conv2(disp)), 1)
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, ref)
    cpu = torch.cat((F.leaky_relu(F.conv2d(torch.cat((warped - left, left), 1).cpu().double(),
                                           w1.cpu().double(), b1.cpu().double(), padding=1), 0.2),
                     F.leaky_relu(F.conv2d(disp.cpu().double(), w2.cpu().double(),
                                           b2.cpu().double(), padding=1), 0.2)), 1)
    assert (got.cpu().double() - cpu).abs().max().item() <= 1e-5 * (1 + cpu.abs().max().item())


@pytest.mark.parametrize("C,Co,H,W", [(32, 128, 24, 52), (64, 256, 16, 26), (64, 512, 8, 13),
                                      (32, 192, 5, 7)])
@pytest.mark.parametrize("out_nhwc", [False, True])
def test_pointwise_wide_outputs_vs_torch(C, Co, H, W, out_nhwc):
    """1x1 convs with Co = 128 .. 512 (the ResNet bottlenecks' expansions, nets/resnet.py) on the
    streaming pointwise kernel, one 64-channel tile per grid row: against torch CPU in fp64 with
    bias, residual and activation, NCHW and channels-last output."""
    g = torch.Generator().manual_seed(C + Co + H)
    x = torch.randn(2, C, H, W, generator=g, dtype=torch.float64)
    w = torch.randn(Co, C, 1, 1, generator=g, dtype=torch.float64) / C ** 0.5
    b = torch.randn(Co, generator=g, dtype=torch.float64)
    res = torch.randn(2, Co, H, W, generator=g, dtype=torch.float64)
    ref = F.relu(F.conv2d(x, w, b) + res)
    wd = w.float().to(DEV)
    wp = ops.pack_weight_split(wd)
    assert wp is not None
    rd = res.float().to(DEV)
    if out_nhwc:
        rd = rd.contiguous(memory_format=torch.channels_last)
    got = ops.conv2d_fused(x.float().to(DEV), wd, b.float().to(DEV), act="relu", residual=rd,
                           packed_weight=wp, out_nhwc=out_nhwc)
    err = (got.cpu().double() - ref).abs().max().item()
    assert err <= 2e-5 * (1 + ref.abs().max().item()), err
