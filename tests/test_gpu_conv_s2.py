"""GPU tests of the stride-2 exchange-conv kernel (aanet_amd/csrc/conv_s2.hip,
aanet_conv3x3s2_f32): 3x3 stride-2 pad-1 convs with their output channels split over two
outputs, against an fp64 reference and held to the exact-f32 conv engine's error on the same
conv (as tests/test_gpu_pointwise.py holds the 1x1 kernel); odd sizes (zero padding at every
border), one and two outputs, C = 32 / 64, and the C2 scale-0 merged 64 -> 32 + 64 launch."""
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # N, C, H, W, co, co_a, act_a, act_b
    (2, 64, 24, 52, 96, 32, None, "leaky"),   # scale-0 heads: branch 1 (64->32) + branch 2 (64->64)
    (1, 64, 17, 23, 96, 32, None, "leaky"),   # odd H, W (last output row/column half padded)
    (2, 64, 9, 40, 16, 16, None, None),       # second conv of the branch-2 chain (64 -> 16)
    (3, 32, 13, 30, 16, 16, None, None),      # scale 1 -> 2 (32 -> 16)
    (1, 32, 5, 7, 48, 16, "relu", "leaky"),   # 3 co blocks, partial tiles
    (1, 64, 6, 10, 64, 0, None, "leaky"),     # every channel to the second output
    (1, 64, 128, 416, 96, 32, None, "leaky"),  # C2 scale 0, one image
    (2, 96, 11, 26, 16, 16, None, None),      # three chunks (the merged branch-2 contraction)
    (1, 128, 7, 18, 32, 16, "leaky", None),   # four chunks: the runtime-loop instantiation
]

ACTS = {None: lambda t: t, "relu": lambda t: t.clamp_min(0),
        "leaky": lambda t: torch.where(t > 0, t, 0.2 * t)}


class exact_f32:
    def __enter__(self):
        self.prev = _lib.set_exact_f32(True)

    def __exit__(self, *a):
        _lib.set_exact_f32(self.prev)


@pytest.mark.parametrize("case", CASES, ids=[f"c{c[1]}co{c[4]}a{c[5]}h{c[2]}w{c[3]}" for c in CASES])
def test_conv3x3_s2_vs_fp64(case):
    N, C, H, W, co, co_a, act_a, act_b = case
    g = torch.Generator().manual_seed(7)
    x = torch.randn(N, C, H, W, generator=g) * 2
    w = torch.randn(co, C, 3, 3, generator=g) / (3 * C ** 0.5)
    b = torch.randn(co, generator=g)
    y = F.conv2d(x.double(), w.double(), b.double(), stride=2, padding=1)
    scale = F.conv2d(x.double().abs(), w.double().abs(), stride=2, padding=1) + 1.0
    xd, wd, bd = x.to(DEV), w.to(DEV), b.to(DEV)
    ws = ops.pack_conv3x3s2(wd)
    got_a, got_b = ops.conv3x3_s2(xd, ws, bd, co, co_a, act_a, act_b)
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    with exact_f32():  # the engine's exact-f32 contraction of the same conv, as the error bar
        ref_e = ops.conv2d_fused(xd, wd, bd, 2, 1, 1, 1, None, packed_weight=ops.pack_weight(wd))
    err_e = ((ref_e.cpu().double() - y).abs() / scale).max().item()
    for got, lo, hi, act in ((got_a, 0, co_a, act_a), (got_b, co_a, co, act_b)):
        if hi == lo:
            assert got is None
            continue
        assert got.shape == (N, hi - lo, Ho, Wo) and got.is_contiguous()
        ref = ACTS[act](y[:, lo:hi])
        err = ((got.cpu().double() - ref).abs() / scale[:, lo:hi]).max().item()
        assert err <= max(4 * err_e, 2e-7), (err, err_e)
    # run to run: no atomics, fixed order
    again = ops.conv3x3_s2(xd, ws, bd, co, co_a, act_a, act_b)
    for a1, a2 in zip((got_a, got_b), again):
        assert (a1 is None and a2 is None) or torch.equal(a1, a2)


TERM_CASES = [
    # N, C, C2, H, W, co, co_a, identity, up (h, w) or None, act_a, act_b
    (2, 64, 0, 24, 52, 96, 32, True, (6, 13), "leaky", "leaky"),  # branch 1 sum in the heads launch
    (2, 64, 32, 24, 52, 16, 16, True, None, "leaky", None),        # branch 2: both down terms + x2
    (1, 64, 0, 17, 23, 48, 16, True, (4, 5), "leaky", None),       # odd sizes, non-integer ratio
    (1, 32, 64, 9, 14, 16, 16, False, (3, 4), None, None),         # x2 first chunk boundary, up only
    (1, 64, 0, 128, 416, 96, 32, True, (32, 104), "leaky", "leaky"),  # C2 scale 0, one image
    (1, 64, 32, 64, 208, 16, 16, True, None, "leaky", None),       # C2 scale 1 -> 2, one image
]


@pytest.mark.parametrize("case", TERM_CASES, ids=[f"c{c[1]}+{c[2]}co{c[5]}h{c[3]}w{c[4]}" for c in TERM_CASES])
def test_conv3x3_s2_csa_terms_vs_fp64(case):
    """aanet_conv3x3s2_terms_f32: out_a = act(conv(x ++ x2) + bias + identity + resize(up)) in
    the reference's term order (aggregation.py:388-400), against fp64 with the same error bar as
    the plain form plus the fp32 rounding of the added terms."""
    N, C, C2, H, W, co, co_a, with_id, up_hw, act_a, act_b = case
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, C, H, W, generator=g) * 2
    x2 = torch.randn(N, C2, H, W, generator=g) * 2 if C2 else None
    CT = C + C2
    w = torch.randn(co, CT, 3, 3, generator=g) / (3 * CT ** 0.5)
    b = torch.randn(co, generator=g)
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    ident = torch.randn(N, co_a, Ho, Wo, generator=g) if with_id else None
    up = torch.randn(N, co_a, *up_hw, generator=g) if up_hw else None
    xin = x if x2 is None else torch.cat([x, x2], 1)
    y = F.conv2d(xin.double(), w.double(), b.double(), stride=2, padding=1)
    scale = F.conv2d(xin.double().abs(), w.double().abs(), stride=2, padding=1) + 1.0
    ya = y[:, :co_a].clone()
    if ident is not None:
        ya = ya + ident.double()
    if up is not None:
        ya = ya + F.interpolate(up.double(), size=(Ho, Wo), mode="bilinear", align_corners=False)
    dev = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    wd = w.to(DEV)
    ws = ops.pack_conv3x3s2(wd)
    got_a, got_b = ops.conv3x3_s2(dev(x), ws, dev(b), co, co_a, act_a, act_b, x2=dev(x2),
                                  identity=dev(ident), up=dev(up))
    with exact_f32():
        ref_e = ops.conv2d_fused(dev(xin), wd, dev(b), 2, 1, 1, 1, None,
                                 packed_weight=ops.pack_weight(wd))
    err_e = ((ref_e.cpu().double() - y).abs() / scale).max().item()
    tol = max(4 * err_e, 2e-7)
    ref_a = ACTS[act_a](ya)
    err = ((got_a.cpu().double() - ref_a).abs() / (scale[:, :co_a] + ya.abs())).max().item()
    assert err <= tol, (err, err_e)
    if co_a < co:
        ref_b = ACTS[act_b](y[:, co_a:])
        err = ((got_b.cpu().double() - ref_b).abs() / scale[:, co_a:]).max().item()
        assert err <= tol, (err, err_e)
    else:
        assert got_b is None
    again = ops.conv3x3_s2(dev(x), ws, dev(b), co, co_a, act_a, act_b, x2=dev(x2),
                           identity=dev(ident), up=dev(up))
    assert torch.equal(again[0], got_a)


def test_conv3x3_s2_rejects_unsupported_shapes():
    x = torch.zeros(1, 48, 8, 8, device=DEV)  # c % 32 != 0
    ws = torch.zeros(64, device=DEV, dtype=torch.int16)
    with pytest.raises(_lib.AanetError):
        ops.conv3x3_s2(x, ws, None, 16, 16)
    assert ops.pack_conv3x3s2(torch.zeros(112, 64, 3, 3, device=DEV)) is None  # co > 96
    assert ops.pack_conv3x3s2(torch.zeros(24, 64, 3, 3, device=DEV)) is None   # co % 16
