"""The few-channel deformable conv (aanet_amd/csrc/dcn_small.hip): 16 channels in two 8-channel
deformable groups, Co = 16, 3x3 -- the aggregation's coarsest-scale DeformSimpleBottleneck
(nets/deform.py:216-236 at scale 2 of the C2 config).  aanet_mdcn_fwd_f32 / aanet_mdcn_fwd_fused_f32
take it for the op-level DCN and aanet_mdcn_pw_f32 for the bottleneck tail (NCHW conv1 output).
Checked against the CPU oracle (restated kernel.cu:467-767 + torch-CPU conv3) and against the
generic engine it replaces (AANET_CONV_GENERIC_DCN), with ragged tiles, samples far outside the
image, integer-grid offsets and the C2 full size."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"
C = 16


def _case(N, H, W, off_scale, seed, bias=False, dg=2):
    rng = np.random.default_rng(seed)
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


def _mask(om, dg=2):
    return (2.0 / (1.0 + np.exp(-om[:, dg * 18:].astype(np.float64)))).astype(np.float32)


def _oracle_tail(x, om, w2, b2, sc, sh, w3, b3, ident, dil=2):
    from oracle import oracle
    t = oracle.mdcn_forward(x, om[:, :36], _mask(om), w2, b2, 1, dil, dil, 1, 2)
    t = np.maximum(t * sc[None, :, None, None] + sh[None, :, None, None], 0)
    return F.relu(F.conv2d(torch.from_numpy(t), torch.from_numpy(w3), torch.from_numpy(b3)) +
                  torch.from_numpy(ident)).numpy()


def _d(a):
    return None if a is None else torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _run_tail(x, om, w2, b2, sc, sh, w3, b3, ident, generic=False, dil=2):
    w2d, w3d = _d(w2), _d(w3)
    assert ops.pack_weight_split(w2d) is None  # 16 channels: no split form, fp32 weights
    return ops.mdcn_pw(_d(x), _d(om), w2d, ops.pack_weight(w2d), _d(b2), _d(sc), _d(sh), "relu",
                       ops.pack_weight(w3d), _d(b3), _d(ident), "relu", 1, dil, dil, 2, 2.0,
                       generic_dcn=generic)


@pytest.mark.parametrize("N,H,W,off_scale,bias,dil", [
    (2, 32, 104, 1.0, False, 2),   # C2 scale-2 rows, offsets of a trained model's size
    (2, 16, 48, 6.0, False, 2),    # most samples far from their tap, many outside the image
    (1, 13, 37, 1.5, True, 2),     # ragged: 481 pixels (7.5 waves), odd width, DCN bias
    (1, 3, 2, 0.7, False, 1),      # fewer pixels than a wave, dilation 1
])
def test_dcn_small_tail_vs_oracle(N, H, W, off_scale, bias, dil):
    args = _case(N, H, W, off_scale, seed=H * 100 + W, bias=bias)
    ref = _oracle_tail(*args, dil=dil)
    got = _run_tail(*args, dil=dil).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-5 * (1 + np.abs(ref).max())


@pytest.mark.parametrize("off_scale", [0.5, 3.0])
def test_dcn_small_tail_matches_generic_engine(off_scale):
    """C2 scale-2 shape at B=8 (32 x 104): the direct kernel vs the implicit-GEMM engine it
    replaces, on the same packed fp32 weights: fp32-rounding agreement."""
    args = _case(8, 32, 104, off_scale, seed=5)
    o_s, o_g = _run_tail(*args), _run_tail(*args, generic=True)
    assert (o_s - o_g).abs().max().item() <= 1e-5 * (1 + o_g.abs().max().item())


@pytest.mark.parametrize("N,H,W,off_scale,bias,dil", [
    (8, 32, 104, 1.0, True, 2),
    (1, 13, 37, 5.0, False, 2),
    (2, 7, 9, 1.0, True, 1),
])
def test_dcn_small_op_forward_vs_oracle(N, H, W, off_scale, bias, dil):
    """ModulatedDeformConvFunction's forward (deform_conv_cuda.cpp:490-569) at 16 channels /
    two groups: aanet_mdcn_fwd_f32 (separate offset and mask tensors, raw weights)."""
    from oracle import oracle
    x, om, w2, b2, *_ = _case(N, H, W, off_scale, seed=N * 1000 + H, bias=bias)
    off, msk = om[:, :36], _mask(om)
    ref = oracle.mdcn_forward(x, off, msk, w2, b2, 1, dil, dil, 1, 2)
    got = ops.mdcn_forward(_d(x), _d(off), _d(msk), _d(w2), _d(b2), 1, dil, dil, 1, 2).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-5 * (1 + np.abs(ref).max())


def test_dcn_small_fused_eval_vs_oracle():
    """DeformConv2d's eval path (nets/deform.py:78-97 + BN + ReLU): aanet_mdcn_fwd_fused_f32 with
    the offset / mask logits read in place from offset_conv's output."""
    from oracle import oracle
    x, om, w2, b2, sc, sh, *_ = _case(2, 32, 104, 1.0, seed=17, bias=True)
    ref = oracle.mdcn_forward(x, om[:, :36], _mask(om), w2, b2, 1, 2, 2, 1, 2)
    ref = np.maximum(ref * sc[None, :, None, None] + sh[None, :, None, None], 0)
    for packed in (False, True):
        w2d = _d(w2)
        got = ops.mdcn_forward_fused(_d(x), _d(om), w2d, _d(b2), _d(sc), _d(sh), "relu", 1, 2, 2, 2,
                                     2.0, packed_weight=ops.pack_weight(w2d) if packed else None)
        assert np.abs(got.cpu().numpy() - ref).max() <= 1e-5 * (1 + np.abs(ref).max()), packed


def test_dcn_small_sampling_edges():
    """Offsets on integer grid points, at the -1 / H boundaries and far outside the image (zero
    contribution: invalid corners are out-of-range buffer loads) in both deformable groups."""
    x, om, w2, b2, sc, sh, w3, b3, ident = _case(1, 16, 32, 0.0, seed=9)
    rng = np.random.default_rng(10)
    vals = np.array([0.0, 1.0, -1.0, 2.0, -2.0, 0.5, -0.5, 1.999, -2.001, 17.0, -40.0, 3.25],
                    dtype=np.float32)
    om[:, :36] = rng.choice(vals, size=om[:, :36].shape)
    ref = _oracle_tail(x, om, w2, b2, sc, sh, w3, b3, ident)
    got = _run_tail(x, om, w2, b2, sc, sh, w3, b3, ident).cpu().numpy()
    assert np.abs(got - ref).max() <= 1e-5 * (1 + np.abs(ref).max())


def test_dcn_small_reproducible_b8():
    """B=8 C2 scale 2: identical bits over repeated launches (no atomics; fixed sum order)."""
    args = _case(8, 32, 104, 1.0, seed=4)
    ref = _run_tail(*args).clone()
    for _ in range(3):
        assert torch.equal(_run_tail(*args), ref)
