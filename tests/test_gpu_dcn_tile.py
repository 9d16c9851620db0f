"""The LDS-window deformable bottleneck tail (aanet_amd/csrc/dcn_tile.hip), which aanet_mdcn_pw_f32
takes for the aggregation's scale-0 DeformSimpleBottleneck (64 channels, two 32-channel
deformable groups) and scale-1 one (32 channels, two 16-channel groups), 3x3, dilation 2, NHWC
conv1 output, split weights.  Checked against the CPU
oracle (restated kernel.cu:467-767 + torch-CPU conv3) and against the generic engine it replaces
(AANET_CONV_GENERIC_DCN), including samples that leave the window (global-gather fallback),
ragged tiles and the CSA epilogue."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _case(N, H, W, off_scale, seed, bias=False, C=64):
    rng = np.random.default_rng(seed)
    dg = 2
    x = np.maximum(rng.standard_normal((N, C, H, W)), 0).astype(np.float32)
    om = rng.standard_normal((N, dg * 27, H, W)).astype(np.float32)
    om[:, :dg * 18] *= off_scale
    w2 = (rng.standard_normal((C, C, 3, 3)) / (3 * C ** 0.5)).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, C).astype(np.float32)
    sh = rng.standard_normal(C).astype(np.float32)
    w3 = (rng.standard_normal((C, C, 1, 1)) / C ** 0.5).astype(np.float32)
    b3 = rng.standard_normal(C).astype(np.float32)
    b2 = rng.standard_normal(C).astype(np.float32) if bias else None
    ident = rng.standard_normal((N, C, H, W)).astype(np.float32)
    return x, om, w2, b2, sc, sh, w3, b3, ident


def _oracle(x, om, w2, b2, sc, sh, w3, b3, ident):
    from oracle import oracle
    dg = 2
    mask = (2.0 / (1.0 + np.exp(-om[:, dg * 18:].astype(np.float64)))).astype(np.float32)
    t = oracle.mdcn_forward(x, om[:, :dg * 18], mask, w2, b2, 1, 2, 2, 1, dg)
    t = np.maximum(t * sc[None, :, None, None] + sh[None, :, None, None], 0)
    return F.relu(F.conv2d(torch.from_numpy(t), torch.from_numpy(w3), torch.from_numpy(b3)) +
                  torch.from_numpy(ident)).numpy()


def _run(x, om, w2, b2, sc, sh, w3, b3, ident, generic=False, csa_up=None):
    d = lambda a: None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    w2d, w3d = d(w2), d(w3)
    p2, p3 = ops.pack_weight_split(w2d), ops.pack_weight_split(w3d)
    assert p2 is not None and p3 is not None
    xd = d(x).contiguous(memory_format=torch.channels_last)
    return ops.mdcn_pw(xd, d(om), w2d, p2, d(b2), d(sc), d(sh), "relu", p3, d(b3), d(ident), "relu",
                       1, 2, 2, 2, 2.0, csa_up=csa_up, generic_dcn=generic)


@pytest.mark.parametrize("C", [64, 32])
@pytest.mark.parametrize("N,H,W,off_scale,bias", [
    (2, 16, 48, 1.0, False),   # whole tiles, offsets mostly inside the window
    (2, 16, 48, 4.0, False),   # most samples leave the window: global-gather fallback
    (1, 13, 36, 1.5, True),    # ragged tiles (13 % 8, 36 % 16), DCN bias
    (1, 8, 4, 0.7, False),     # one tile narrower than the window's column margin
])
def test_dcn_tile_vs_oracle(N, H, W, off_scale, bias, C):
    args = _case(N, H, W, off_scale, seed=H * 100 + W + C, bias=bias, C=C)
    ref = _oracle(*args)
    got = _run(*args).cpu().numpy()
    err = np.abs(got - ref).max()
    assert err <= 1e-4 * (1 + np.abs(ref).max()), err


@pytest.mark.parametrize("off_scale", [0.5, 3.0])
def test_dcn_tile_matches_generic_engine_with_csa(off_scale):
    """Window kernel vs the generic engine on the same split weights at the C2 scale-0 shape
    (B=2), CSA epilogue on: fp32-rounding agreement of both outputs."""
    args = _case(2, 128, 416, off_scale, seed=1)
    gen = torch.Generator(device=DEV).manual_seed(2)
    ups = [torch.randn(2, 64, 128 // r, 416 // r, device=DEV, generator=gen) for r in (2, 4)]
    o_w, c_w = _run(*args, csa_up=ups)
    o_g, c_g = _run(*args, generic=True, csa_up=ups)
    for a, b in ((o_w, o_g), (c_w, c_g)):
        assert (a - b).abs().max().item() <= 2e-5 * (1 + b.abs().max().item())


@pytest.mark.parametrize("off_scale", [0.5, 3.0])
def test_dcn_tile_c32_matches_generic_engine(off_scale):
    """Scale-1 shape (32 channels, two 16-channel groups, C2 64 x 208, B=2): the window kernel
    vs the generic engine on the same split weights, fp32-rounding agreement."""
    args = _case(2, 64, 208, off_scale, seed=3, C=32)
    o_w, o_g = _run(*args), _run(*args, generic=True)
    assert (o_w - o_g).abs().max().item() <= 2e-5 * (1 + o_g.abs().max().item())


@pytest.mark.parametrize("C,H,W", [(64, 128, 416), (32, 64, 208)])
def test_dcn_tile_c2_reproducible(C, H, W):
    """B=8 C2 scale 0 / scale 1, every CU busy: identical bits over repeated launches."""
    args = _case(8, H, W, 1.0, seed=4, C=C)
    ref = _run(*args).clone()
    for _ in range(4):
        assert torch.equal(_run(*args), ref)


@pytest.mark.parametrize("C", [64, 32])
def test_dcn_tile_sampling_edges(C):
    """Offsets placing samples exactly on integer grid points, at -1 / H boundaries and far
    outside the image (zero contribution) in both deformable groups."""
    x, om, w2, b2, sc, sh, w3, b3, ident = _case(1, 16, 32, 0.0, seed=9, C=C)
    rng = np.random.default_rng(10)
    vals = np.array([0.0, 1.0, -1.0, 2.0, -2.0, 0.5, -0.5, 1.999, -2.001, 17.0, -40.0, 3.25],
                    dtype=np.float32)
    om[:, :36] = rng.choice(vals, size=om[:, :36].shape)
    ref = _oracle(x, om, w2, b2, sc, sh, w3, b3, ident)
    got = _run(x, om, w2, b2, sc, sh, w3, b3, ident).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-4 * (1 + np.abs(ref).max())
