"""GPU tests of the streaming 1x1 convolution (aanet_amd/csrc/pointwise.hip), which
aanet_conv2d_fused_f32 takes for split-bf16 1x1 convs with 32/64 input channels: against an fp64
reference, held to the exact-f32 engine's error (as tests/test_gpu_split.py holds the engine),
over both layouts on each side, bias / folded-BN / residual / activation epilogues, output widths
1..64 and pixel counts that are not a multiple of the 16-pixel block (blocks spanning images).
NCHW input with 2 or 4 output-channel blocks takes the split-once kernel (pw_conv_nchw_s_kernel),
with 1 block the per-wave-split one: both are covered."""
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import _lib, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # N, C, H, W, Co, in_nhwc, out_nhwc, bias, post, residual, act
    (2, 64, 24, 52, 64, False, True, True, False, False, "relu"),   # conv1 (csa0 NCHW -> NHWC)
    (2, 64, 24, 52, 64, True, True, True, False, False, "relu"),
    (2, 64, 24, 52, 64, False, False, True, False, False, None),    # final_conv (bias)
    (1, 32, 17, 23, 64, False, False, False, True, False, None),    # exchange term 32 -> 64, BN
    (3, 32, 7, 9, 32, True, False, True, True, True, "leaky"),      # ragged P = 63, residual
    (2, 64, 5, 11, 16, False, True, False, False, True, "relu"),    # Co = 16, NHWC residual
    (1, 64, 9, 13, 54, True, False, True, False, False, None),      # Co = 54 (partial block)
    (2, 32, 3, 5, 1, False, False, True, False, False, None),       # Co = 1
    (1, 64, 128, 416, 64, False, True, True, False, False, "relu"),  # C2 scale-0 conv1, one image
    (2, 64, 13, 27, 24, False, False, True, True, False, "leaky"),  # NCHW, 2 co blocks (split once)
    (1, 32, 11, 30, 32, False, True, True, False, True, "relu"),     # NCHW, 32 ch, 2 co blocks
]


class exact_f32:
    def __enter__(self):
        self.prev = _lib.set_exact_f32(True)

    def __exit__(self, *a):
        _lib.set_exact_f32(self.prev)


@pytest.mark.parametrize("case", CASES, ids=[f"c{c[1]}co{c[4]}i{int(c[5])}o{int(c[6])}p{c[2]*c[3]}"
                                             for c in CASES])
def test_pointwise_conv_vs_fp64(case):
    N, C, H, W, Co, inh, onh, has_b, post, has_res, act = case
    g = torch.Generator().manual_seed(11)
    x = torch.randn(N, C, H, W, generator=g) * 2
    w = torch.randn(Co, C, 1, 1, generator=g) / C ** 0.5
    b = torch.randn(Co, generator=g) if has_b else None
    ps = torch.rand(Co, generator=g) + 0.5 if post else None
    ph = torch.randn(Co, generator=g) if post else None
    res = torch.randn(N, Co, H, W, generator=g) if has_res else None
    y = F.conv2d(x.double(), w.double(), None if b is None else b.double())
    if post:
        y = y * ps.double().view(1, -1, 1, 1) + ph.double().view(1, -1, 1, 1)
    if has_res:
        y = y + res.double()
    if act == "relu":
        y = y.clamp_min(0)
    elif act == "leaky":
        y = torch.where(y > 0, y, 0.2 * y)
    scale = F.conv2d(x.double().abs(), w.double().abs()) + 1.0
    xd = x.to(DEV)
    if inh:
        xd = xd.contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV)
    pw = ops.pack_weight_split(wd)
    dv = lambda t: None if t is None else t.to(DEV)  # noqa: E731
    rd = dv(res)
    if rd is not None and onh:
        rd = rd.contiguous(memory_format=torch.channels_last)
    args = dict(bias=dv(b), act=act, residual=rd, post_scale=dv(ps), post_shift=dv(ph),
                packed_weight=pw, out_nhwc=onh)
    got = ops.conv2d_fused(xd, wd, **args)
    with exact_f32():
        ref_e = ops.conv2d_fused(xd, wd, **args)
    assert got.shape == (N, Co, H, W) and got.is_contiguous(
        memory_format=torch.channels_last if onh else torch.contiguous_format)
    err = ((got.cpu().double() - y).abs() / scale).max().item()
    err_e = ((ref_e.cpu().double() - y).abs() / scale).max().item()
    assert err <= max(4 * err_e, 2e-7), (err, err_e)
    # run to run: no atomics, fixed order
    assert torch.equal(got, ops.conv2d_fused(xd, wd, **args))
