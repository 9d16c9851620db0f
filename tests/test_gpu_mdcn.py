"""GPU parity of the modulated deformable conv (HIP, through the C ABI) vs the CPU oracle.

* sampling indices (h_low, w_low, validity) and im2col values: BIT-EXACT (SURVEY §8c pin 6);
* forward: |err| <= 2e-5 * (1 + |ref|) (GEMM summation order differs);
* backward: grad_offset / grad_mask / grad_weight / grad_bias rtol 1e-4 + atol scaled to the
  tensor's magnitude; grad_x uses float atomics like the reference (order-dependent rounding).
"""
import numpy as np
import pytest
import torch

from aanet_amd import _lib, nets, ops
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda"


def g2t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def t2n(t):
    torch.cuda.synchronize()
    return t.detach().cpu().numpy()


def make_case(seed, N, C, H, W, Co, k=3, stride=1, pad=2, dil=2, dg=2, groups=1, off_scale=2.0,
              integer_heavy=False):
    rng = np.random.default_rng(seed)
    Ho = oracle.out_size(H, k, stride, pad, dil)
    Wo = oracle.out_size(W, k, stride, pad, dil)
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    off = (rng.standard_normal((N, dg * 2 * k * k, Ho, Wo)) * off_scale).astype(np.float32)
    if integer_heavy:  # exact integers / halves stress floor() and the strict range checks
        off = np.round(off * 2) / 2
        off[..., ::3] = -1.0 - rng.integers(0, 3, off[..., ::3].shape)
    msk = rng.uniform(0, 2, (N, dg * k * k, Ho, Wo)).astype(np.float32)
    w = (rng.standard_normal((Co, C // groups, k, k)) / np.sqrt(C * k * k)).astype(np.float32)
    b = rng.standard_normal(Co).astype(np.float32)
    return x, off, msk, w, b


CASES = [
    # N, C, H, W, Co, k, stride, pad, dil, dg, groups
    (2, 64, 16, 52, 64, 3, 1, 2, 2, 2, 1),     # aggregation scale-0 shape family
    (2, 32, 9, 26, 32, 3, 1, 2, 2, 2, 1),      # scale 1
    (2, 16, 5, 13, 16, 3, 1, 2, 2, 2, 1),      # scale 2 (cpg = 8)
    (1, 128, 8, 26, 128, 3, 1, 1, 1, 2, 1),    # feature-extractor DCN (C=128, dil 1)
    (1, 128, 16, 52, 128, 3, 2, 1, 1, 2, 1),   # stride 2
    (1, 24, 7, 11, 40, 3, 1, 1, 1, 3, 2),      # groups=2, dg=3, Co not a tile multiple
    (2, 6, 5, 7, 5, 1, 1, 0, 1, 1, 1),         # 1x1 kernel, tiny
    (1, 8, 6, 9, 12, 3, 2, 2, 2, 4, 1),        # dg=4, cpg=2
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("integer_heavy", [False, True])
def test_mdcn_sample_index_and_im2col_bit_exact(case, integer_heavy):
    N, C, H, W, Co, k, s, p, d, dg, groups = case
    x, off, msk, w, b = make_case(1, N, C, H, W, Co, k, s, p, d, dg, groups,
                                  integer_heavy=integer_heavy)
    hl, wl, vd = ops.mdcn_sample_index(g2t(off), H, W, k, k, s, p, d, dg)
    ohl, owl, ovd = oracle.mdcn_sample_index(off, H, W, k, k, s, p, d, dg)
    assert np.array_equal(t2n(hl), ohl) and np.array_equal(t2n(wl), owl)
    assert np.array_equal(t2n(vd), ovd)
    for n in range(N):
        col = ops.mdcn_im2col(g2t(x[n]), g2t(off[n]), g2t(msk[n]), k, k, s, p, d, dg)
        assert np.array_equal(t2n(col), oracle.mdcn_im2col(x[n], off[n], msk[n], k, k, s, p, d, dg))


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("with_bias", [False, True])
def test_mdcn_forward_vs_oracle(case, with_bias):
    N, C, H, W, Co, k, s, p, d, dg, groups = case
    x, off, msk, w, b = make_case(2, N, C, H, W, Co, k, s, p, d, dg, groups)
    bias = b if with_bias else None
    out = ops.mdcn_forward(g2t(x), g2t(off), g2t(msk), g2t(w), g2t(bias) if with_bias else None,
                           s, p, d, groups, dg)
    ref = oracle.mdcn_forward(x, off, msk, w, bias, s, p, d, groups, dg)
    got = t2n(out)
    err = np.abs(got - ref)
    assert err.max() <= 2e-5 * (1 + np.abs(ref).max()), err.max()


def test_mdcn_forward_zero_offset_equals_conv2d():
    """KAT 1 on the GPU: offsets 0, mask 1 => torch conv2d (MIOpen)."""
    x, off, msk, w, b = make_case(3, 2, 64, 20, 40, 64)
    off[:] = 0
    msk[:] = 1
    out = ops.mdcn_forward(g2t(x), g2t(off), g2t(msk), g2t(w), None, 1, 2, 2, 1, 2)
    ref = torch.nn.functional.conv2d(g2t(x), g2t(w), None, 1, 2, 2)
    assert torch.allclose(out, ref, rtol=1e-4, atol=1e-4)


def test_mdcn_fused_eval_path_vs_oracle():
    """Fused path: offset/mask read in place from the offset_conv output, 2*sigmoid, BN, ReLU."""
    rng = np.random.default_rng(4)
    N, C, H, W, dg = 2, 64, 12, 40, 2
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    om = rng.standard_normal((N, dg * 27, H, W)).astype(np.float32)
    w = (rng.standard_normal((C, C, 3, 3)) / 24).astype(np.float32)
    sc = rng.uniform(0.5, 1.5, C).astype(np.float32)
    sh = rng.standard_normal(C).astype(np.float32)
    wt = g2t(w)
    out = ops.mdcn_forward_fused(g2t(x), g2t(om), wt, None, g2t(sc), g2t(sh), 1, 1, 2, 2, dg, 2.0,
                                 packed_weight=ops.pack_weight(wt))
    mask = 2.0 / (1.0 + np.exp(-om[:, dg * 18:].astype(np.float64)))
    ref = oracle.mdcn_forward(x, om[:, :dg * 18], mask.astype(np.float32), w, None, 1, 2, 2, 1, dg)
    ref = np.maximum(ref * sc[None, :, None, None] + sh[None, :, None, None], 0)
    got = t2n(out)
    assert np.abs(got - ref).max() <= 1e-4 * (1 + np.abs(ref).max())


BWD_CASES = [
    (2, 16, 24, 48, 16, 3, 1, 2, 2, 2),   # golden-model layer shapes (max_disp=16)
    (2, 8, 12, 24, 8, 3, 1, 2, 2, 2),
    (2, 4, 6, 12, 4, 3, 1, 2, 2, 2),
    (2, 64, 12, 30, 64, 3, 1, 2, 2, 2),
    (2, 32, 9, 26, 32, 3, 1, 2, 2, 2),
    (1, 16, 5, 13, 16, 3, 1, 2, 2, 2),
    (1, 48, 10, 21, 36, 3, 2, 1, 1, 3),
    (1, 128, 8, 20, 128, 3, 2, 2, 2, 2),   # feature-extractor DCN: Co=128 (> 64 KB LDS tile)
    (1, 64, 7, 18, 96, 3, 2, 2, 2, 2),     # GANet conv3a: 64 -> 96, stride 2
]


@pytest.mark.parametrize("case", BWD_CASES)
@pytest.mark.parametrize("off_scale", [0.7, 2.0])
@pytest.mark.parametrize("deterministic", [False, True])
def test_mdcn_backward_vs_oracle(case, off_scale, deterministic):
    N, C, H, W, Co, k, s, p, d, dg = case
    x, off, msk, w, b = make_case(5, N, C, H, W, Co, k, s, p, d, dg, off_scale=off_scale)
    Ho, Wo = off.shape[2:]
    go = np.random.default_rng(6).standard_normal((N, Co, Ho, Wo)).astype(np.float32)
    xt, ot, mt = g2t(x).requires_grad_(), g2t(off).requires_grad_(), g2t(msk).requires_grad_()
    wt, bt = g2t(w).requires_grad_(), g2t(b).requires_grad_()
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(deterministic)
    try:
        out = ops.modulated_deform_conv(xt, ot, mt, wt, bt, s, p, d, 1, dg)
        out.backward(g2t(go))
    finally:
        torch.use_deterministic_algorithms(prev)
    gx, goff, gm, gw, gb = oracle.mdcn_backward(x, off, msk, w, go, True, s, p, d, 1, dg)
    for name, got, ref in (("grad_input", xt.grad, gx), ("grad_offset", ot.grad, goff),
                           ("grad_mask", mt.grad, gm), ("grad_weight", wt.grad, gw),
                           ("grad_bias", bt.grad, gb)):
        got = t2n(got)
        scale = np.abs(ref).max() + 1e-12
        err = np.abs(got - ref)
        assert err.max() <= 1e-4 * scale + 1e-6, f"{name}: max err {err.max():.3g} (scale {scale:.3g})"


@pytest.mark.parametrize("case", BWD_CASES)
@pytest.mark.parametrize("nchw_scatter", [False, True])
def test_mdcn_backward_entry_points_vs_oracle(case, nchw_scatter):
    """Both float-atomic entry points: aanet_mdcn_bwd_ws_f32 (NHWC workspace scatter + transpose,
    the default) and the workspace-free aanet_mdcn_bwd_f32 (NCHW scatter)."""
    N, C, H, W, Co, k, s, p, d, dg = case
    x, off, msk, w, b = make_case(7, N, C, H, W, Co, k, s, p, d, dg, off_scale=1.3)
    Ho, Wo = off.shape[2:]
    go = np.random.default_rng(8).standard_normal((N, Co, Ho, Wo)).astype(np.float32)
    got = ops.mdcn_backward(g2t(x), g2t(off), g2t(msk), g2t(w), g2t(go), True, s, p, d, 1, dg,
                            deterministic=False, nchw_scatter=nchw_scatter)
    ref = oracle.mdcn_backward(x, off, msk, w, go, True, s, p, d, 1, dg)
    for name, gt, r in zip(("grad_input", "grad_offset", "grad_mask", "grad_weight", "grad_bias"), got, ref):
        err = np.abs(t2n(gt) - r)
        scale = np.abs(r).max() + 1e-12
        assert err.max() <= 1e-4 * scale + 1e-6, f"{name}: max err {err.max():.3g} (scale {scale:.3g})"


def test_deform_conv_cuda_shim_matches_reference_call_sequence():
    """The pybind-compatible module, called exactly as nets/deform_conv/deform_conv.py:140-166
    calls deform_conv_cuda (in-place output, zeroed grads, vestigial bufs)."""
    from aanet_amd import deform_conv_cuda
    x, off, msk, w, b = make_case(8, 2, 32, 9, 26, 32)
    xt, ot, mt, wt, bt = (g2t(a) for a in (x, off, msk, w, b))
    bufs = [xt.new_empty(0), xt.new_empty(0)]
    out = xt.new_empty((2, 32, 9, 26))
    deform_conv_cuda.modulated_deform_conv_cuda_forward(xt, wt, bt, bufs[0], ot, mt, out, bufs[1],
                                                        3, 3, 1, 1, 2, 2, 2, 2, 1, 2, True)
    ref = oracle.mdcn_forward(x, off, msk, w, b, 1, 2, 2, 1, 2)
    assert np.abs(t2n(out) - ref).max() <= 2e-5 * (1 + np.abs(ref).max())
    go = np.random.default_rng(1).standard_normal(ref.shape).astype(np.float32)
    gi, goff, gm = torch.zeros_like(xt), torch.zeros_like(ot), torch.zeros_like(mt)
    gw, gb = torch.ones_like(wt), torch.ones_like(bt)  # accumulate semantics: start at 1
    deform_conv_cuda.modulated_deform_conv_cuda_backward(xt, wt, bt, bufs[0], ot, mt, bufs[1], gi, gw,
                                                         gb, goff, gm, g2t(go), 3, 3, 1, 1, 2, 2, 2,
                                                         2, 1, 2, True)
    rx, roff, rm, rw, rb = oracle.mdcn_backward(x, off, msk, w, go, True, 1, 2, 2, 1, 2)
    for got, r in ((gi, rx), (goff, roff), (gm, rm), (gw, rw + 1), (gb, rb + 1)):
        assert np.abs(t2n(got) - r).max() <= 1e-4 * (np.abs(r).max() + 1)


@pytest.mark.parametrize("C,dg,Co", [(32, 2, 32), (64, 4, 64), (32, 2, 48)])
@pytest.mark.parametrize("packed", [False, True])
def test_mdcn_fused_sixteen_channel_groups_vs_oracle(C, dg, Co, packed):
    """16-channel deformable groups: 32-channel chunks spanning two groups (conv engine CFG 2)."""
    rng = np.random.default_rng(C * dg)
    N, H, W = 2, 9, 26
    x = rng.standard_normal((N, C, H, W)).astype(np.float32)
    om = (rng.standard_normal((N, dg * 27, H, W)) * 1.5).astype(np.float32)
    w = (rng.standard_normal((Co, C, 3, 3)) / (3 * C ** 0.5)).astype(np.float32)
    mask = (2.0 / (1.0 + np.exp(-om[:, dg * 18:].astype(np.float64)))).astype(np.float32)
    ref = oracle.mdcn_forward(x, om[:, :dg * 18], mask, w, None, 1, 2, 2, 1, dg)
    wd = g2t(w)
    got = ops.mdcn_forward_fused(g2t(x), g2t(om), wd, None, None, None, None, 1, 2, 2, dg, 2.0,
                                 packed_weight=ops.pack_weight(wd) if packed else None)
    assert np.abs(t2n(got) - ref).max() <= 2e-5 * (1 + np.abs(ref).max())


def test_torch_ops_match_functional_ops_and_autograd():
    """torch.ops.aanet.* (custom operators) == aanet_amd.ops, gradients included."""
    import aanet_amd  # noqa: F401
    rng = np.random.default_rng(11)
    N, C, H, W, Co, dg = 2, 16, 9, 13, 8, 2
    x = g2t(rng.standard_normal((N, C, H, W)).astype(np.float32)).requires_grad_()
    off = g2t(rng.standard_normal((N, dg * 18, H, W)).astype(np.float32)).requires_grad_()
    msk = g2t(rng.uniform(0, 1, (N, dg * 9, H, W)).astype(np.float32)).requires_grad_()
    w = g2t((rng.standard_normal((Co, C, 3, 3)) * 0.1).astype(np.float32)).requires_grad_()
    b = g2t(rng.standard_normal(Co).astype(np.float32)).requires_grad_()
    y1 = torch.ops.aanet.mdcn_forward(x, off, msk, w, b, 1, 2, 2, 1, dg)
    y2 = ops.modulated_deform_conv(x, off, msk, w, b, 1, 2, 2, 1, dg)
    assert torch.equal(y1, y2)
    gy = torch.randn_like(y1)
    g1 = torch.autograd.grad(y1, (x, off, msk, w, b), gy)
    g2 = torch.autograd.grad(y2, (x, off, msk, w, b), gy)
    for a, c in zip(g1, g2):
        assert torch.allclose(a, c, rtol=1e-5, atol=1e-5 * (1 + c.abs().max().item()))
    L = torch.randn(2, 32, 6, 20, device="cuda", requires_grad=True)
    R = torch.randn(2, 32, 6, 20, device="cuda", requires_grad=True)
    v1 = torch.ops.aanet.corr_volume(L, R, 8)
    v2 = ops.CorrelationVolumeFunction.apply(L, R, 8)
    assert torch.equal(v1, v2)
    d1 = torch.ops.aanet.disp_regress(v1, False)
    d2 = ops.DisparityRegressionFunction.apply(v2, False)
    assert torch.equal(d1, d2)
    gd = torch.randn_like(d1)
    ga = torch.autograd.grad(d1, (L, R), gd)
    gb = torch.autograd.grad(d2, (L, R), gd)
    for a, c in zip(ga, gb):
        assert torch.equal(a, c)


@pytest.mark.parametrize("case", [(2, 64, 16, 52, 64, 3, 1, 2, 2, 2), (1, 32, 9, 26, 32, 3, 2, 1, 1, 2)])
def test_mdcn_backward_deterministic_is_bit_reproducible(case):
    """aanet_mdcn_bwd_det_f32: identical bits on every run (the atomic form need not be)."""
    N, C, H, W, Co, k, s, p, d, dg = case
    x, off, msk, w, b = make_case(9, N, C, H, W, Co, k, s, p, d, dg, off_scale=2.0)
    Ho, Wo = off.shape[2:]
    go = g2t(np.random.default_rng(3).standard_normal((N, Co, Ho, Wo)).astype(np.float32))
    args = (g2t(x), g2t(off), g2t(msk), g2t(w), go, True, s, p, d, 1, dg)
    runs = [ops.mdcn_backward(*args, deterministic=True) for _ in range(3)]
    for r in runs[1:]:
        for a_, b_ in zip(runs[0], r):
            assert torch.equal(a_, b_)
    atomic = ops.mdcn_backward(*args, deterministic=False)
    for a_, b_ in zip(runs[0], atomic):
        scale = b_.abs().max().item() + 1e-12
        assert (a_ - b_).abs().max().item() <= 1e-5 * scale


def test_deterministic_mode_reaches_shim_and_torch_ops():
    """torch.use_deterministic_algorithms(True) selects the deterministic kernels in every entry
    point: the autograd Function, torch.ops.aanet.mdcn_backward and the deform_conv_cuda shim."""
    import aanet_amd  # noqa: F401
    from aanet_amd import deform_conv_cuda
    x, off, msk, w, b = make_case(4, 2, 32, 9, 26, 32, off_scale=1.5)
    xt, ot, mt, wt, bt = (g2t(a) for a in (x, off, msk, w, b))
    go = g2t(np.random.default_rng(2).standard_normal((2, 32, 9, 26)).astype(np.float32))
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        ref = ops.mdcn_backward(xt, ot, mt, wt, go, True, 1, 2, 2, 1, 2, deterministic=True)
        got = torch.ops.aanet.mdcn_backward(xt, ot, mt, wt, go, True, 1, 2, 2, 1, 2)
        for a_, b_ in zip(ref, got):
            assert torch.equal(a_, b_)
        gi, goff, gm = torch.zeros_like(xt), torch.zeros_like(ot), torch.zeros_like(mt)
        gw, gb = torch.zeros_like(wt), torch.zeros_like(bt)
        e = xt.new_empty(0)
        deform_conv_cuda.modulated_deform_conv_cuda_backward(xt, wt, bt, e, ot, mt, e, gi, gw, gb,
                                                             goff, gm, go, 3, 3, 1, 1, 2, 2, 2, 2,
                                                             1, 2, True)
        for a_, b_ in zip(ref, (gi, goff, gm, gw, gb)):
            assert torch.equal(a_, b_)
    finally:
        torch.use_deterministic_algorithms(prev)


@pytest.mark.parametrize("case", BWD_CASES)
@pytest.mark.parametrize("algo", ["window", "global"])
def test_mdcn_backward_window_form_vs_oracle(case, algo):
    """The LDS-window grad_x form (mdcn_bwd_data_win_kernel: stride 1, <= 32 channels per
    deformable group, channel counts that allow channels-last reads; int64 fixed-point window,
    16-channel slices) and the global-atomic form, each in float and fixed-point mode, against
    the oracle, with offsets large enough that some corners fall outside the window.  Shapes the
    window form does not take report AANET_EUNSUPPORTED."""
    N, C, H, W, Co, k, s, p, d, dg = case
    x, off, msk, w, b = make_case(9, N, C, H, W, Co, k, s, p, d, dg, off_scale=2.5)
    Ho, Wo = off.shape[2:]
    go = np.random.default_rng(10).standard_normal((N, Co, Ho, Wo)).astype(np.float32)
    for det in (False, True):
        try:
            got = ops.mdcn_backward(g2t(x), g2t(off), g2t(msk), g2t(w), g2t(go), True, s, p, d, 1,
                                    dg, deterministic=det, algo=algo)
        except _lib.AanetError as e:
            assert algo == "window" and e.status == _lib.EUNSUPPORTED and \
                not ops.window_bwd_ok(C, Co, k, k, s, d, dg), (case, e)
            return
        if algo == "window":
            assert ops.window_bwd_ok(C, Co, k, k, s, d, dg), case
        ref = oracle.mdcn_backward(x, off, msk, w, go, True, s, p, d, 1, dg)
        for name, gt, r in zip(("grad_input", "grad_offset", "grad_mask", "grad_weight", "grad_bias"), got, ref):
            err = np.abs(t2n(gt) - r)
            scale = np.abs(r).max() + 1e-12
            assert err.max() <= 1e-4 * scale + 1e-6, f"{name} det={det}: max err {err.max():.3g}"


@pytest.mark.parametrize("form", ["atomic", "window", "deterministic", "deterministic_global"])
def test_mdcn_backward_c4_agg_s0_vs_oracle(form):
    """SURVEY C4 at the aggregation's scale-0 shape: one image of 64 channels at 128x416,
    dg 2, 3x3, dil 2 (the C2 bottleneck DCN), against the oracle, for the global float-atomic
    (NHWC workspace scatter), window (the default in both modes: int64 fixed-point LDS window)
    and fixed-point deterministic (window and global) forms.  Grids ~100x those of BWD_CASES (deform_conv_cuda_kernel.cu:635-767)."""
    N, C, H, W, Co, k, s, p, d, dg = 1, 64, 128, 416, 64, 3, 1, 2, 2, 2
    x, off, msk, w, b = make_case(11, N, C, H, W, Co, k, s, p, d, dg, off_scale=0.7)
    go = np.random.default_rng(12).standard_normal((N, Co, H, W)).astype(np.float32)
    algo = {"atomic": "global", "window": "window", "deterministic": "auto",
            "deterministic_global": "global"}[form]
    got = ops.mdcn_backward(g2t(x), g2t(off), g2t(msk), g2t(w), g2t(go), True, s, p, d, 1, dg,
                            deterministic=form.startswith("deterministic"), algo=algo)
    ref = oracle.mdcn_backward(x, off, msk, w, go, True, s, p, d, 1, dg)
    for name, gt, r in zip(("grad_input", "grad_offset", "grad_mask", "grad_weight", "grad_bias"), got, ref):
        err = np.abs(t2n(gt) - r)
        scale = np.abs(r).max() + 1e-12
        assert err.max() <= 1e-4 * scale + 1e-6, f"{form} {name}: max err {err.max():.3g} (scale {scale:.3g})"


@pytest.mark.parametrize("shape", ["feat_s1", "feat_s2"])
@pytest.mark.parametrize("det", [False, True])
def test_mdcn_backward_c4_feature_dcn_window_vs_oracle(shape, det):
    """SURVEY C4 at the feature extractor's DCN shapes (nets/resnet.py:133-134: 128 channels, two
    deformable groups of 64, Co = 128, dil 2; stride 1 at 32x104 and stride 2 from 64x208), one
    image at full size: the window form (round 6: 64-channel groups in four 16-channel slices,
    Co = 128 in two 64-channel weight-gradient blocks, the stride-2 window) against the oracle,
    float and fixed-point."""
    N, C, Co, k, p, d, dg = 1, 128, 128, 3, 2, 2, 2
    H, W, s = (32, 104, 1) if shape == "feat_s1" else (64, 208, 2)
    assert ops.window_bwd_ok(C, Co, k, k, s, d, dg)
    x, off, msk, w, b = make_case(13, N, C, H, W, Co, k, s, p, d, dg, off_scale=0.7)
    Ho, Wo = off.shape[2:]
    go = np.random.default_rng(14).standard_normal((N, Co, Ho, Wo)).astype(np.float32)
    got = ops.mdcn_backward(g2t(x), g2t(off), g2t(msk), g2t(w), g2t(go), True, s, p, d, 1, dg,
                            deterministic=det, algo="window")
    ref = oracle.mdcn_backward(x, off, msk, w, go, True, s, p, d, 1, dg)
    for name, gt, r in zip(("grad_input", "grad_offset", "grad_mask", "grad_weight", "grad_bias"), got, ref):
        err = np.abs(t2n(gt) - r)
        scale = np.abs(r).max() + 1e-12
        assert err.max() <= 1e-4 * scale + 1e-6, f"{shape} det={det} {name}: max err {err.max():.3g}"


@pytest.mark.parametrize("det", [False, True])
@pytest.mark.parametrize("bad", [np.inf, np.nan])
def test_mdcn_backward_nonfinite_grad_out_propagates(det, bad):
    """a non-finite grad_out value must give a non-finite grad_input, as the reference's
    float col2im does, in the window (fixed-point) form of both modes -- not finite garbage from
    converting inf/NaN to int64.  The other gradients stay computed in float and carry it too."""
    N, C, H, W, Co, k, s, p, d, dg = 1, 64, 16, 24, 64, 3, 1, 2, 2, 2
    x, off, msk, w, b = make_case(31, N, C, H, W, Co, k, s, p, d, dg, off_scale=0.7)
    go = np.random.default_rng(32).standard_normal((N, Co, H, W)).astype(np.float32)
    go[0, 5, 7, 9] = bad
    assert ops.window_bwd_ok(C, Co, k, k, s, d, dg)
    got = ops.mdcn_backward(g2t(x), g2t(off), g2t(msk), g2t(w), g2t(go), True, s, p, d, 1, dg,
                            deterministic=det, algo="window")
    gx = t2n(got[0])
    assert not np.isfinite(gx).all()
    assert not np.isfinite(t2n(got[3])).all()       # grad_weight
    # a clean grad_out through the same form is finite (the poison comes from the bad value)
    go[0, 5, 7, 9] = 0.0
    clean = ops.mdcn_backward(g2t(x), g2t(off), g2t(msk), g2t(w), g2t(go), True, s, p, d, 1, dg,
                              deterministic=det, algo="window")
    assert all(np.isfinite(t2n(t)).all() for t in clean if t is not None)


def test_mdcn_backward_window_deterministic_bit_reproducible():
    """The window form in fixed-point mode (the default deterministic path at the aggregation
    shapes): its LDS window, the global fallback and the flush all add int64 fixed-point values,
    whose sum does not depend on the order the atomics land in, so two runs give identical bits --
    with offsets large enough that both the window and the fallback paths run, and with clustered
    offsets that pile many pixels onto the same window positions."""
    N, C, H, W, Co, k, s, p, d, dg = 2, 64, 40, 96, 64, 3, 1, 2, 2, 2
    x, off, msk, w, b = make_case(21, N, C, H, W, Co, k, s, p, d, dg, off_scale=1.5)
    go = np.random.default_rng(22).standard_normal((N, Co, H, W)).astype(np.float32)
    # clustered offsets in one corner of the image: many pixels share a table position
    off[:, :, :8, :8] = -np.arange(8, dtype=np.float32)[None, None, None, :] * 0.999
    args = (g2t(x), g2t(off), g2t(msk), g2t(w), g2t(go), True, s, p, d, 1, dg)
    a = ops.mdcn_backward(*args, deterministic=True, algo="window")
    b2 = ops.mdcn_backward(*args, deterministic=True, algo="window")
    for u, v in zip(a, b2):
        assert torch.equal(u, v)
    ref = oracle.mdcn_backward(x, off, msk, w, go, True, s, p, d, 1, dg)
    for name, gt, r in zip(("grad_input", "grad_offset", "grad_mask", "grad_weight", "grad_bias"), a, ref):
        err = np.abs(t2n(gt) - r)
        scale = np.abs(r).max() + 1e-12
        assert err.max() <= 1e-4 * scale + 1e-6, f"{name}: max err {err.max():.3g}"


def test_mdcn_backward_deterministic_chunks_images():
    """The deterministic backward runs over the batch in chunks of images (two at a time for the
    agg_s0 shape: 96 MB of int64 grad_x + channels-last x each), so its workspace stays <= 128 MB
    at any batch.  Each chunk is its own fixed-point problem: the per-image gradients of the last
    chunk are bit-identical to a run over that image alone, the weight / bias gradients are the
    chunk sums added in chunk order, bits repeat run to run, and the result matches the float
    (atomic) form."""
    N, C, H, W, Co, k, s, p, d, dg = 3, 64, 128, 416, 64, 3, 1, 2, 2, 2
    L = _lib.lib()
    ws = L.aanet_mdcn_bwd_det_workspace_size(N, C, H, W, Co, k, k, s, p, d, 1, dg)
    assert ws == L.aanet_mdcn_bwd_det_workspace_size(2, C, H, W, Co, k, k, s, p, d, 1, dg) <= 128 << 20
    x, off, msk, w, b = make_case(41, N, C, H, W, Co, k, s, p, d, dg, off_scale=1.0)
    go = np.random.default_rng(42).standard_normal((N, Co, H, W)).astype(np.float32)
    xt, ot, mt, wt, gt = g2t(x), g2t(off), g2t(msk), g2t(w), g2t(go)

    def run(sl, det=True):
        return ops.mdcn_backward(xt[sl].contiguous(), ot[sl].contiguous(), mt[sl].contiguous(), wt,
                                 gt[sl].contiguous(), True, s, p, d, 1, dg, deterministic=det)

    full, again = run(slice(0, 3)), run(slice(0, 3))
    for u, v in zip(full, again):
        assert torch.equal(u, v)
    head, tail = run(slice(0, 2)), run(slice(2, 3))
    for i in range(3):  # grad_input, grad_offset, grad_mask: per image
        assert torch.equal(full[i][:2], head[i]) and torch.equal(full[i][2:], tail[i])
    assert torch.equal(full[3], head[3] + tail[3])  # grad_weight: chunk sums in chunk order
    atomic = run(slice(0, 3), det=False)
    for name, u, v in zip(("grad_input", "grad_offset", "grad_mask", "grad_weight", "grad_bias"), full, atomic):
        scale = v.abs().max().item() + 1e-12
        assert (u - v).abs().max().item() <= 1e-5 * scale, name


def test_split_weight_cache_follows_the_tensor_not_its_address():
    """ops._split_weight keeps the packed weight on the tensor: a new weight that reuses a freed
    one's device address (the caching allocator hands the block straight back) at version 0 must
    be packed from its own values (round 5: a dict keyed by data_ptr returned the old packing and
    the window forward came out wrong in 1 of ~4 suite runs)."""
    g = torch.Generator(device=DEV).manual_seed(3)
    w1 = torch.randn(64, 64, 3, 3, device=DEV, generator=g)
    p1 = ops._split_weight(w1).clone()
    addr = w1.data_ptr()
    del w1
    w2 = torch.randn(64, 64, 3, 3, device=DEV, generator=g)
    p2 = ops._split_weight(w2)
    assert torch.equal(p2, ops.pack_weight_split(w2))
    if w2.data_ptr() == addr:  # the case the old cache got wrong
        assert not torch.equal(p2, p1)
    w2.mul_(2.0)  # in place: new version, re-packed
    assert torch.equal(ops._split_weight(w2), ops.pack_weight_split(w2))


def test_split_weight_cache_dropped_with_the_fold_caches():
    """Writes through `.data` (and HIP graph replays: Trainer.graph_step) change a weight without
    bumping its _version, so the pack kept on the tensor would go stale; clear_fold_caches (which
    train()/eval() and graph_step call) drops it with the folded-weight caches.  The
    sequence graph_step -> eager forward -> graph_step -> eager forward then runs the second eager
    forward on the current weights: checked here on a DeformConv2d against algo='generic'."""
    from aanet_amd.nets._fuse import clear_fold_caches
    torch.manual_seed(0)
    m = nets.DeformConv2d(64, 64).to(DEV)
    with torch.no_grad():
        m.deform_conv.weight.normal_(0, 0.05)
        m.offset_conv.weight.normal_(0, 0.01)
        m.offset_conv.bias.normal_(0, 0.5)
    m.train()  # the reference op order: ModulatedDeformConv -> ops.mdcn_forward (window kernel)
    x = torch.randn(1, 64, 12, 32, device=DEV)
    w = m.deform_conv.weight
    p1 = ops._split_weight(w).clone()
    w.data.mul_(-0.5)  # no version bump: the kept pack is stale ...
    assert torch.equal(ops._split_weight(w), p1)
    clear_fold_caches(m)  # ... until the caches are dropped
    assert torch.equal(ops._split_weight(w), ops.pack_weight_split(w))
    with torch.no_grad():
        off = m._offset_conv(x)
        out = m(x)
        om = off[:, 36:].sigmoid() * 2
        ref = ops.mdcn_forward(x, off[:, :36].contiguous(), om.contiguous(), w, None, 1, 2, 2, 1, 2,
                               algo="generic")
    assert float((out - ref).abs().max()) <= 2e-5 * max(1.0, float(ref.abs().max()))


WINDOW_FWD = [
    # N, C, H, W, off_scale: ragged tiles (H % 8, W % 16), offsets that leave the window
    (2, 64, 16, 52, 0.7),
    (1, 64, 13, 36, 3.0),
    (2, 32, 9, 28, 0.7),
    (1, 32, 21, 20, 3.0),
    (2, 128, 16, 52, 0.7),  # 64-channel groups (SURVEY C4 feat_s1 shape class): 4 phases, 8 co blocks
    (1, 128, 13, 36, 3.0),
]


@pytest.mark.parametrize("case", WINDOW_FWD)
@pytest.mark.parametrize("nhwc", [False, True])
def test_mdcn_forward_window_vs_oracle(case, nhwc):
    """Op-level DCN forward on the LDS-window kernel (dcn_tile.hip, plain epilogue; NCHW x as
    ModulatedDeformConvFunction passes it, or channels-last x through the fused entry) against
    the oracle, the generic engine and itself (bit-reproducible).  deform_conv_cuda.cpp:490-569."""
    N, C, H, W, osc = case
    x, off, msk, w, b = make_case(41, N, C, H, W, C, off_scale=osc)
    assert ops.window_fwd_ok(C, C, 3, 3, 1, 2, 2, 1, 2, W)
    ref = oracle.mdcn_forward(x, off, msk, w, b, 1, 2, 2, 1, 2)
    xt, wt = g2t(x), g2t(w)
    if nhwc:
        xt = xt.contiguous(memory_format=torch.channels_last)
        om = torch.cat([g2t(off), g2t(msk)], 1)
        fn = lambda: ops.mdcn_forward_fused(xt, om, wt, g2t(b), None, None, None, 1, 2, 2, 2,  # noqa: E731
                                            packed_weight=ops.pack_weight_split(wt))
        # mask values, not logits: the fused entry's mask_logits flag is set by mdcn_forward_fused,
        # so compare with the logits' image instead
        ref = oracle.mdcn_forward(x, off, (2.0 / (1.0 + np.exp(-msk.astype(np.float64)))).astype(np.float32),
                                  w, b, 1, 2, 2, 1, 2)
    else:
        fn = lambda: ops.mdcn_forward(xt, g2t(off), g2t(msk), wt, g2t(b), 1, 2, 2, 1, 2)  # noqa: E731
    got = fn()
    err = np.abs(t2n(got) - ref)
    assert err.max() <= 2e-5 * (1 + np.abs(ref).max()), err.max()
    assert torch.equal(fn(), got)
    if not nhwc:
        gen = ops.mdcn_forward(xt, g2t(off), g2t(msk), wt, g2t(b), 1, 2, 2, 1, 2, algo="generic")
        assert (gen - got).abs().max().item() <= 2e-5 * (1 + gen.abs().max().item())
