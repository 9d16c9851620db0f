"""The conv engine's split-bf16 contraction (include/aanet_mi355x.h AANET_CONV_EXACT_F32 /
AANET_CONV_WEIGHTS_SPLIT; aanet_amd/csrc/mdcn.hip split3).  Every fp32 operand is carried as
three bf16 pieces and six piece products are accumulated in fp32; the claim is fp32 accuracy.
These tests hold it to that: against an fp64 reference (torch double conv2d / the oracle's fp64
DCN) the split path's error may not exceed the exact f32 MFMA engine's by more than a small
factor, and its pieces must reconstruct the weights exactly."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import _lib, ops
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


class exact_f32:
    def __enter__(self):
        self.prev = _lib.set_exact_f32(True)

    def __exit__(self, *a):
        _lib.set_exact_f32(self.prev)


def _errs(got, ref64, scale64):
    e = (got.double() - ref64).abs()
    return e.max().item(), e.mean().item(), (e / (scale64 + 1e-30)).max().item()


@pytest.mark.parametrize("case", [
    # N, C, H, W, Co, k, stride, pad, dil, groups, nhwc
    (2, 64, 24, 52, 64, 3, 1, 1, 1, 1, True),     # SimpleBottleneck conv2 (NHWC staging)
    (2, 64, 24, 52, 64, 3, 1, 1, 1, 1, False),    # same, NCHW staging
    (2, 64, 24, 52, 54, 3, 1, 2, 2, 2, True),     # offset_conv: grouped, dilated, Cog = 27
    (2, 64, 24, 52, 64, 1, 1, 0, 1, 1, False),    # conv1 / conv3
    (2, 64, 24, 52, 32, 3, 2, 1, 1, 1, False),    # CSA strided 3x3
    (2, 64, 25, 36, 64, 3, 2, 1, 1, 1, False),    # stride 2, 64-ch tile, ragged rows / columns
    (1, 32, 16, 40, 32, 3, 2, 1, 1, 1, False),    # stride 2, one input chunk
    (1, 128, 12, 40, 96, 3, 1, 1, 1, 1, False),   # Co > 64: two output tiles
    # halo-tile form (NHWC 3x3 stride 1): odd chunk counts, ragged tiles, Wo % 4 != 0, dil 2
    (1, 96, 13, 30, 64, 3, 1, 1, 1, 1, True),     # 3 channel chunks, element epilogue
    (1, 64, 9, 20, 40, 3, 1, 2, 2, 1, True),      # dilation 2, Co = 40 of a 64 tile
    (2, 32, 8, 16, 32, 3, 1, 1, 1, 1, True),      # one chunk, 32-channel tile, exact tile fit
    # group width 16 (mod 32): zero-padded last chunk (the hourglasses' 48-channel convs)
    (2, 48, 24, 52, 64, 3, 1, 1, 1, 1, False),    # 3x3 stride 1
    (2, 48, 25, 36, 64, 3, 2, 1, 1, 1, False),    # conv2a: stride 2, ragged
    (1, 48, 13, 30, 128, 2, 1, 1, 1, 1, False),   # deconv1 phase conv: 2x2 pad 1, two co tiles
    (1, 80, 9, 20, 32, 3, 1, 1, 1, 1, False),     # three chunks, the last half empty
])
def test_split_conv_accuracy_vs_fp64(case):
    N, C, H, W, Co, k, s, p, d, g, nhwc = case
    gen = torch.Generator().manual_seed(7)
    x = torch.randn(N, C, H, W, generator=gen) * 3
    w = torch.randn(Co, C // g, k, k, generator=gen) / (C // g * k * k) ** 0.5
    ref = F.conv2d(x.double(), w.double(), None, s, p, d, g)
    scale = F.conv2d(x.double().abs(), w.double().abs(), None, s, p, d, g)
    xd, wd = x.to(DEV), w.to(DEV)
    if nhwc:
        xd = xd.contiguous(memory_format=torch.channels_last)
    wsplit = ops.pack_weight_split(wd, g)
    assert wsplit is not None and wsplit._aanet_split
    got_s = ops.conv2d_fused(xd, wd, None, s, p, d, g, packed_weight=wsplit).cpu()
    with exact_f32():
        got_e = ops.conv2d_fused(xd, wd, None, s, p, d, g, packed_weight=wsplit).cpu()
    es, ee = _errs(got_s, ref, scale), _errs(got_e, ref, scale)
    assert not torch.equal(got_s, got_e), "split and exact paths are not distinct launches"
    # fp32-accurate: max and mean error within 1.5x / 1.25x of the exact f32 fma chain's, and
    # below 2^-21 of sum |x||w| (the chain's own error is ~2^-22 at K <= 1152)
    assert es[0] <= 1.5 * ee[0] + 1e-7, (es, ee)
    assert es[1] <= 1.25 * ee[1] + 1e-9, (es, ee)
    assert es[2] <= 2.0 ** -21, (es, ee)


def test_split_dcn_accuracy_vs_fp64_oracle():
    rng = np.random.default_rng(3)
    N, C, H, W, Co, dg = 1, 64, 20, 44, 64, 2
    x = (rng.standard_normal((N, C, H, W)) * 2).astype(np.float32)
    off = (rng.standard_normal((N, 2 * dg * 9, H, W)) * 1.5).astype(np.float32)
    mlog = rng.standard_normal((N, dg * 9, H, W)).astype(np.float32)
    w = (rng.standard_normal((Co, C, 3, 3)) / 24).astype(np.float32)
    mask = (2.0 / (1.0 + np.exp(-mlog.astype(np.float64)))).astype(np.float32)
    ref = torch.from_numpy(oracle.mdcn_forward(x, off, mask, w, None, 1, 2, 2, 1, dg, dtype=np.float64))
    scale = torch.from_numpy(oracle.mdcn_forward(np.abs(x), off, mask, np.abs(w), None, 1, 2, 2, 1, dg,
                                                 dtype=np.float64))
    om = torch.from_numpy(np.concatenate([off, mlog], 1)).to(DEV)
    xd = torch.from_numpy(x).to(DEV).contiguous(memory_format=torch.channels_last)
    wd = torch.from_numpy(w).to(DEV)
    wsplit = ops.pack_weight_split(wd)
    got_s = ops.mdcn_forward_fused(xd, om, wd, None, None, None, None, 1, 2, 2, dg, 2.0,
                                   packed_weight=wsplit).cpu()
    with exact_f32():
        got_e = ops.mdcn_forward_fused(xd, om, wd, None, None, None, None, 1, 2, 2, dg, 2.0,
                                       packed_weight=wsplit).cpu()
    es, ee = _errs(got_s, ref, scale), _errs(got_e, ref, scale)
    # the sampled values themselves carry fp32 rounding (bilinear blend), shared by both paths
    assert es[0] <= 1.5 * ee[0] + 1e-7, (es, ee)
    assert es[1] <= 1.25 * ee[1] + 1e-9, (es, ee)


@pytest.mark.parametrize("dcn", [False, True])
def test_split_tail_kernels_match_exact(dcn):
    """Bottleneck tail kernels (conv2/DCN + conv3 pointwise GEMM + CSA epilogue) on the split
    path against the exact engine: fp32-level agreement."""
    gen = torch.Generator(device=DEV).manual_seed(11)
    N, C, H, W = 2, 64, 16, 52
    x = torch.randn(N, C, H, W, device=DEV, generator=gen).contiguous(memory_format=torch.channels_last)
    w3 = torch.randn(C, C, 3, 3, device=DEV, generator=gen) * 0.04
    w1 = torch.randn(C, C, 1, 1, device=DEV, generator=gen) * 0.1
    b = torch.randn(C, device=DEV, generator=gen)
    res = torch.randn(N, C, H, W, device=DEV, generator=gen)
    ups = [torch.randn(N, C, H // r, W // r, device=DEV, generator=gen) for r in (2, 4)]
    p3, p1 = ops.pack_weight_split(w3), ops.pack_weight_split(w1)
    om = torch.randn(N, 54, H, W, device=DEV, generator=gen)

    def run():
        if dcn:
            return ops.mdcn_pw(x, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2, 2,
                               csa_up=ups)
        return ops.conv2d_pw(x, w3, p3, b, None, None, "relu", p1, b, res, "relu", 1, 1, 1, csa_up=ups)

    s_out, s_csa = run()
    with exact_f32():
        e_out, e_csa = run()
    for a, e in ((s_out, e_out), (s_csa, e_csa)):
        assert (a - e).abs().max().item() <= 2e-5 * (1 + e.abs().max().item())


def test_split_pack_reconstructs_weights_exactly():
    """Head of the buffer = pack_weight (bit-exact); pieces h + m + l == w exactly."""
    gen = torch.Generator(device=DEV).manual_seed(5)
    Co, Cg, k, g = 54, 32, 3, 2
    w = torch.randn(Co, Cg, k, k, device=DEV, generator=gen) * 0.3
    ws = ops.pack_weight_split(w, g)
    assert torch.equal(ws, ops.pack_weight(w))
    buf = ws._aanet_buf.cpu().numpy().view(np.uint8)
    off = ((Co * Cg * k * k * 4 + 255) // 256) * 256
    frag = buf[off:].view(np.uint16).reshape(-1, 3, 64, 8)  # (g, t, k, cc, blk) x piece x lane x 8
    f32 = lambda u: (u.astype(np.uint32) << 16).view(np.float32).astype(np.float64)  # noqa: E731
    total = f32(frag[:, 0]) + f32(frag[:, 1]) + f32(frag[:, 2])
    Cog, T, NCC, K = Co // g, 1, Cg // 32, k * k
    wn = w.cpu().numpy().astype(np.float64)
    total = total.reshape(g, T, K, NCC, 4, 64, 8)
    for gi in range(g):
        for kk in range(K):
            for blk in range(4):
                for lane in range(64):
                    row = 16 * blk + (lane & 15)
                    for j in range(8):
                        c = 8 * (lane >> 4) + j
                        want = wn[gi * Cog + row, c, kk // k, kk % k] if row < Cog else 0.0
                        assert total[gi, 0, kk, 0, blk, lane, j] == want


def test_split_unsupported_shapes_fall_back():
    """cg % 32 != 0: no split buffer (None); the fused path then runs the exact engine."""
    w = torch.randn(16, 16, 3, 3, device=DEV)
    assert ops.pack_weight_split(w) is None
    x = torch.randn(1, 16, 8, 8, device=DEV)
    got = ops.conv2d_fused(x, w, None, 1, 1, 1, 1, packed_weight=ops.pack_weight(w)).cpu()
    ref = F.conv2d(x.cpu(), w.cpu(), None, 1, 1)
    assert (got - ref).abs().max().item() <= 2e-5 * (1 + ref.abs().max().item())


def test_halo_conv_nhwc_output_vs_torch():
    """Halo-tile 3x3 with a channels-last output (AANET_LAYOUT_OUT_NHWC) and a residual."""
    gen = torch.Generator().manual_seed(9)
    x = torch.randn(2, 64, 11, 36, generator=gen)
    w = torch.randn(64, 64, 3, 3, generator=gen) / 24
    b = torch.randn(64, generator=gen)
    res = torch.randn(2, 64, 11, 36, generator=gen)
    ref = F.relu(F.conv2d(x, w, b, 1, 1) + res)
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    rd = res.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV)
    got = ops.conv2d_fused(xd, wd, b.to(DEV), 1, 1, 1, 1, "relu", rd,
                           packed_weight=ops.pack_weight_split(wd), out_nhwc=True)
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert (got.cpu() - ref).abs().max().item() <= 2e-5 * (1 + ref.abs().max().item())


def test_stride2_nhwc_output_vs_torch():
    """Stride-2 engine conv (NCHW input, im2col form) with a channels-last output, bias, BN affine
    and LeakyReLU: the CSA down-sampling exchange conv of aggregation.py:364-372."""
    gen = torch.Generator().manual_seed(10)
    x = torch.randn(2, 64, 21, 44, generator=gen)
    w = torch.randn(64, 64, 3, 3, generator=gen) / 24
    b = torch.randn(64, generator=gen)
    sc, sh = torch.rand(64, generator=gen) + 0.5, torch.randn(64, generator=gen)
    y = (F.conv2d(x, w, b, 2, 1) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
    ref = torch.where(y > 0, y, 0.2 * y)
    xd, wd = x.to(DEV), w.to(DEV)
    got = ops.conv2d_fused(xd, wd, b.to(DEV), 2, 1, 1, 1, "leaky", post_scale=sc.to(DEV),
                           post_shift=sh.to(DEV), packed_weight=ops.pack_weight_split(wd), out_nhwc=True)
    assert got.shape == ref.shape and got.is_contiguous(memory_format=torch.channels_last)
    assert (got.cpu() - ref).abs().max().item() <= 2e-5 * (1 + ref.abs().max().item())


def test_fused_paths_bit_reproducible():
    """Identical launches give identical bits on every fused path the hot path uses, at the C2
    scale-0 shape (B=8, contention on every CU) with fractional DCN offsets."""
    gen = torch.Generator(device=DEV).manual_seed(0)
    B, C, H, W = 8, 64, 128, 416
    x = torch.randn(B, C, H, W, device=DEV, generator=gen)
    xn = x.contiguous(memory_format=torch.channels_last)
    res = torch.randn(B, C, H, W, device=DEV, generator=gen)
    w1 = torch.randn(C, C, 1, 1, device=DEV, generator=gen) * 0.1
    w3 = torch.randn(C, C, 3, 3, device=DEV, generator=gen) * 0.04
    wo = torch.randn(54, 32, 3, 3, device=DEV, generator=gen) * 0.01
    bo = torch.randn(54, device=DEV, generator=gen)
    b = torch.randn(C, device=DEV, generator=gen)
    p1, p3, po = ops.pack_weight_split(w1), ops.pack_weight_split(w3), ops.pack_weight_split(wo, 2)
    om = ops.conv2d_fused(xn, wo, bo, 1, 2, 2, 2, packed_weight=po)
    ups = [torch.randn(B, C, H // r, W // r, device=DEV, generator=gen) for r in (2, 4)]
    cases = {
        "halo 3x3": lambda: ops.conv2d_fused(xn, w3, b, 1, 1, 1, 1, "relu", packed_weight=p3),
        "halo offset conv": lambda: ops.conv2d_fused(xn, wo, bo, 1, 2, 2, 2, packed_weight=po),
        "halo stride 2": lambda: ops.conv2d_fused(x, w3, b, 2, 1, 1, 1, "leaky", packed_weight=p3,
                                                  out_nhwc=True),
        "conv1 nhwc out": lambda: ops.conv2d_fused(x, w1, b, act="relu", packed_weight=p1, out_nhwc=True),
        "dcn nhwc": lambda: ops.mdcn_forward_fused(xn, om, w3, None, b, b, "relu", 1, 2, 2, 2, 2.0,
                                                   packed_weight=p3),
        "dcn tail nhwc + csa": lambda: ops.mdcn_pw(xn, om, w3, p3, None, b, b, "relu", p1, b, res, "relu",
                                                   1, 2, 2, 2, csa_up=ups)[1],
        "conv tail nhwc + csa": lambda: ops.conv2d_pw(xn, w3, p3, b, None, None, "relu", p1, b, res, "relu",
                                                      1, 1, 1, csa_up=ups)[1],
    }
    for name, fn in cases.items():
        ref = fn().clone()
        for _ in range(4):
            assert torch.equal(fn(), ref), name


def test_split_dcn_tail_c2_scale_reproducible_and_exact():
    """The NHWC deformable tail kernel on the split path at the C2 scale-0 shape (B=8, every CU
    busy, fractional offsets), launched 10 times: bit-identical every time and within fp32
    rounding of the exact engine.  Its packed-fp32 corner blend (v_pk_fma_f32 with a broadcast
    weight) once moved whole pixels staged by lanes 48-63 (tools/repro_packed_fp32_hazard.py); the blend is
    scalar v_fma_f32 now."""
    gen = torch.Generator(device=DEV).manual_seed(3)
    B, C, H, W = 8, 64, 128, 416
    x = torch.randn(B, C, H, W, device=DEV, generator=gen)
    xn = x.contiguous(memory_format=torch.channels_last)
    w1 = torch.randn(C, C, 1, 1, device=DEV, generator=gen) * 0.1
    w3 = torch.randn(C, C, 3, 3, device=DEV, generator=gen) * 0.04
    wo = torch.randn(54, 32, 3, 3, device=DEV, generator=gen) * 0.01
    bo = torch.randn(54, device=DEV, generator=gen)
    b = torch.randn(C, device=DEV, generator=gen)
    p1, p3, po = ops.pack_weight_split(w1), ops.pack_weight_split(w3), ops.pack_weight_split(wo, 2)
    om = ops.conv2d_fused(x, wo, bo, 1, 2, 2, 2, packed_weight=po)
    fn = lambda: ops.mdcn_pw(xn, om, w3, p3, None, b, b, "relu", p1, b, None, None, 1, 2, 2, 2)  # noqa: E731
    ref = fn().clone()
    for _ in range(10):
        assert torch.equal(fn(), ref)
    with exact_f32():
        ex = fn()
    assert (ref - ex).abs().max().item() <= 2e-5 * (1 + ex.abs().max().item())
