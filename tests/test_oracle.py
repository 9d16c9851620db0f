"""Pin the CPU oracle (test infrastructure) before trusting it as the checker.

* cost volumes / regression / pyramid / aggregation: against golden vectors produced by the
  reference's own nets/cost.py, nets/estimation.py, nets/aggregation.py (tests/golden/).
* modulated DCN: known-answer tests from the CUDA kernel semantics (SURVEY.md §8c pins 1-5),
  because the reference DCN is CUDA-only and cannot run here.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import aggregation as oagg
from oracle import oracle
from tests.golden_io import golden, golden_names, state_dict_of


# ----------------------------------------------------------------- golden-vector pins ---
@pytest.mark.parametrize("name", golden_names("corr_"))
def test_corr_volume_matches_reference(name):
    g = golden(name)
    out = oracle.corr_volume(g["left"], g["right"], int(g["max_disp"]))
    np.testing.assert_allclose(out, g["out"], rtol=1e-6, atol=1e-6)
    D = int(g["max_disp"])
    for d in range(D):  # zero fill for x < d (cost.py:41)
        assert np.all(out[:, d, :, :d] == 0)


@pytest.mark.parametrize("name", golden_names("concat_") + golden_names("diff_"))
def test_concat_diff_volume_bit_exact(name):
    g = golden(name)
    fn = oracle.concat_volume if name.startswith("concat") else oracle.diff_volume
    out = fn(g["left"], g["right"], int(g["max_disp"]))
    assert np.array_equal(out, g["out"])


def test_pyramid_matches_reference():
    g = golden("pyramid")
    outs = oracle.cost_volume_pyramid([g[f"left{s}"] for s in range(3)],
                                      [g[f"right{s}"] for s in range(3)], int(g["max_disp"]))
    for s in range(3):
        assert outs[s].shape[1] == int(g["max_disp"]) >> s
        np.testing.assert_allclose(outs[s], g[f"out{s}"], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name", golden_names("regress_"))
def test_regression_matches_reference(name):
    g = golden(name)
    out = oracle.disp_regress(g["cost"], bool(g["match_similarity"]))
    np.testing.assert_allclose(out, g["out"], rtol=1e-5, atol=2e-5)


def test_regression_backward_finite_difference():
    rng = np.random.default_rng(0)
    cost = rng.standard_normal((1, 6, 2, 3))
    gd = rng.standard_normal((1, 2, 3))
    for sim in (True, False):
        an = oracle.disp_regress_bwd(cost, gd, sim, dtype=np.float64)
        num = np.zeros_like(cost)
        eps = 1e-6
        for idx in np.ndindex(cost.shape):
            cp, cm = cost.copy(), cost.copy()
            cp[idx] += eps
            cm[idx] -= eps
            fp = (oracle.disp_regress(cp, sim, np.float64) * gd).sum()
            fm = (oracle.disp_regress(cm, sim, np.float64) * gd).sum()
            num[idx] = (fp - fm) / (2 * eps)
        np.testing.assert_allclose(an, num, rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("tag", ["inter", "final"])
def test_aggregation_oracle_matches_reference(tag):
    g = golden(f"aggregation_{tag}")
    sd = state_dict_of(g)
    inter = tag == "inter"
    aggs = oagg.adaptive_aggregation([g[f"volume{s}"] for s in range(3)], sd,
                                     intermediate_supervision=inter)
    assert len(aggs) == (3 if inter else 1)
    for i, a in enumerate(aggs):
        np.testing.assert_allclose(a.detach().numpy(), g[f"agg{i}"], rtol=1e-5, atol=1e-5)
    disps = oagg.hot_path([g[f"feat_left{s}"] for s in range(3)],
                          [g[f"feat_right{s}"] for s in range(3)], sd, 16,
                          intermediate_supervision=inter)
    for i, d in enumerate(disps):
        np.testing.assert_allclose(d, g[f"disp{i}"], atol=1e-4)


# --------------------------------------------------------- DCN known-answer tests -------
def _dcn_inputs(rng, N=2, C=8, H=9, W=11, Co=6, dg=2, dtype=np.float32):
    x = rng.standard_normal((N, C, H, W)).astype(dtype)
    w = rng.standard_normal((Co, C, 3, 3)).astype(dtype) * 0.2
    return x, w


@pytest.mark.parametrize("stride,pad,dil", [(1, 2, 2), (1, 1, 1), (2, 1, 1), (2, 2, 2)])
def test_dcn_zero_offset_is_conv2d(stride, pad, dil):
    """KAT 1: offsets 0, mask 1 => F.conv2d (SURVEY §8c pin 1)."""
    rng = np.random.default_rng(1)
    x, w = _dcn_inputs(rng)
    N, C, H, W = x.shape
    Ho, Wo = oracle.out_size(H, 3, stride, pad, dil), oracle.out_size(W, 3, stride, pad, dil)
    off = np.zeros((N, 2 * 2 * 9, Ho, Wo), np.float32)
    msk = np.ones((N, 2 * 9, Ho, Wo), np.float32)
    b = rng.standard_normal(w.shape[0]).astype(np.float32)
    out = oracle.mdcn_forward(x, off, msk, w, b, stride, pad, dil, 1, 2)
    ref = F.conv2d(torch.from_numpy(x), torch.from_numpy(w), torch.from_numpy(b), stride, pad, dil)
    np.testing.assert_allclose(out, ref.numpy(), rtol=1e-5, atol=1e-5)


def test_dcn_integer_offset_is_shifted_conv():
    """KAT 2: integer offsets (dy, dx) on every tap => conv of the shifted, zero-filled input."""
    rng = np.random.default_rng(2)
    x, w = _dcn_inputs(rng, dg=1)
    N, C, H, W = x.shape
    dy, dx = 1, -2
    off = np.zeros((N, 18, H, W), np.float32)
    off[:, 0::2] = dy
    off[:, 1::2] = dx
    msk = np.ones((N, 9, H, W), np.float32)
    out = oracle.mdcn_forward(x, off, msk, w, None, 1, 1, 1, 1, 1)
    # out[y, x] = sum_ij w_ij * x0[y + dy + i - 1, x + dx + j - 1] with x0 = zero-extended x:
    # a valid conv over x padded by 3, read at (y + dy + 2, x + dx + 2).
    full = F.conv2d(F.pad(torch.from_numpy(x), (3, 3, 3, 3)), torch.from_numpy(w)).numpy()
    ref = full[:, :, dy + 2: dy + 2 + H, dx + 2: dx + 2 + W]
    np.testing.assert_allclose(out, ref, rtol=1e-5, atol=1e-5)


def test_dcn_half_offset_is_two_tap_average():
    """KAT 3: offset_w = 0.5 => average of the two horizontal neighbours (inside the image)."""
    x = np.arange(1 * 1 * 4 * 6, dtype=np.float32).reshape(1, 1, 4, 6)
    off = np.zeros((1, 2, 4, 6), np.float32)
    off[:, 1] = 0.5
    msk = np.ones((1, 1, 4, 6), np.float32)
    col = oracle.mdcn_im2col(x[0], off[0], msk[0], 1, 1, 1, 0, 1, 1).reshape(4, 6)
    expect = np.zeros((4, 6), np.float32)
    expect[:, :5] = 0.5 * (x[0, 0, :, :5] + x[0, 0, :, 1:])
    expect[:, 5] = 0.5 * x[0, 0, :, 5]  # right neighbour out of range -> 0
    assert np.array_equal(col, expect)


def test_dcn_boundary_partial_taps_and_strict_range():
    """KAT 4: coords in (-1,0) and (H-1,H) give partial taps; exactly -1 or H give 0 (kernel.cu:618)."""
    x = np.full((1, 1, 3, 3), 2.0, np.float32)
    msk = np.ones((1, 1, 3, 3), np.float32)

    def sample(oh, ow):
        off = np.zeros((1, 2, 3, 3), np.float32)
        off[0, 0], off[0, 1] = oh, ow
        return oracle.mdcn_im2col(x[0], off[0], msk[0], 1, 1, 1, 0, 1, 1).reshape(3, 3)

    s = sample(-0.25, 0.0)  # pixel (0,0): h=-0.25 -> only the h_high row contributes 0.75*2
    assert s[0, 0] == np.float32(1.5)
    s = sample(-1.0, 0.0)  # h == -1 -> outside the strict range -> 0
    assert s[0, 0] == 0.0
    s = sample(1.0, 0.0)  # pixel (2,*): h == 3 == H -> 0
    assert np.all(s[2] == 0.0) and np.all(s[:2] == 2.0)
    s = sample(0.5, 0.0)  # pixel (2,*): h = 2.5 in (H-1, H) -> 0.5*2
    assert np.all(s[2] == np.float32(1.0))


def test_dcn_sample_index_floor_semantics():
    off = np.array([-0.5, 0.0, 0.999999, -1e-7], np.float32).reshape(1, 2, 1, 2)
    hl, wl, vd = oracle.mdcn_sample_index(off, 1, 2, 1, 1, 1, 0, 1, 1)
    # h = 0 + off_h ; w = wo + off_w
    assert hl.reshape(-1).tolist() == [-1, 0]
    assert wl.reshape(-1).tolist() == [0, 0]


def test_dcn_backward_matches_finite_difference_f64():
    """KAT 5: float64 gradient check of the restated backward (fwd/bwd consistency)."""
    rng = np.random.default_rng(3)
    N, C, H, W, Co, dg = 1, 4, 5, 6, 3, 2
    x = rng.standard_normal((N, C, H, W))
    w = rng.standard_normal((Co, C, 3, 3)) * 0.3
    off = rng.uniform(-1.7, 1.7, (N, dg * 18, H, W))
    # keep sampling points away from integer grid lines where bilinear is not differentiable
    frac = off - np.floor(off)
    off = np.where(np.abs(frac - 0.5) > 0.45, off + 0.2, off)
    msk = rng.uniform(0.1, 1.9, (N, dg * 9, H, W))
    go = rng.standard_normal((N, Co, H, W))
    args = dict(stride=1, padding=2, dilation=2, groups=1, deformable_groups=dg, dtype=np.float64)
    gx, goff, gm, gw, gb = oracle.mdcn_backward(x, off, msk, w, go, with_bias=True, **args)

    def f(x_, off_, m_, w_):
        return (oracle.mdcn_forward(x_, off_, m_, w_, None, **args) * go).sum()

    eps = 1e-6
    for arr, grad in ((x, gx), (off, goff), (msk, gm), (w, gw)):
        flat = arr.reshape(-1)
        for idx in rng.choice(flat.size, 25, replace=False):
            old = flat[idx]
            flat[idx] = old + eps
            fp = f(x, off, msk, w)
            flat[idx] = old - eps
            fm = f(x, off, msk, w)
            flat[idx] = old
            np.testing.assert_allclose(grad.reshape(-1)[idx], (fp - fm) / (2 * eps), rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(gb, go.sum(axis=(0, 2, 3)), rtol=1e-12)


def test_cost_volume_backward_matches_torch_autograd_of_reference_formula():
    """Pin the cost-volume backward restatement against torch autograd of cost.py:22-48's ops."""
    rng = np.random.default_rng(4)
    B, C, H, W, D = 2, 3, 4, 9, 5
    Lf, Rf = rng.standard_normal((B, C, H, W)), rng.standard_normal((B, C, H, W))
    L = torch.tensor(Lf, requires_grad=True)
    R = torch.tensor(Rf, requires_grad=True)
    corr = L.new_zeros(B, D, H, W)
    for i in range(D):
        corr[:, i, :, i:] = (L[:, :, :, i:] * R[:, :, :, :W - i]).mean(dim=1)
    g = torch.tensor(rng.standard_normal((B, D, H, W)))
    gl, gr = torch.autograd.grad(corr, (L, R), g)
    ol, or_ = oracle.corr_volume_bwd(Lf, Rf, g.numpy(), dtype=np.float64)
    np.testing.assert_allclose(ol, gl.numpy(), rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(or_, gr.numpy(), rtol=1e-12, atol=1e-12)
    for concat in (True, False):
        L.grad = R.grad = None
        OC = 2 * C if concat else C
        vol = L.new_zeros(B, OC, D, H, W)
        for i in range(D):
            if concat:
                vol[:, :, i, :, i:] = torch.cat((L[:, :, :, i:], R[:, :, :, :W - i]), dim=1)
            else:
                vol[:, :, i, :, i:] = L[:, :, :, i:] - R[:, :, :, :W - i]
        g = torch.tensor(rng.standard_normal((B, OC, D, H, W)))
        gl, gr = torch.autograd.grad(vol, (L, R), g)
        ol, or_ = oracle.shift_volume_bwd(g.numpy(), C, concat, dtype=np.float64)
        np.testing.assert_allclose(ol, gl.numpy(), rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(or_, gr.numpy(), rtol=1e-12, atol=1e-12)


# ------------------------------------------------------------------ disparity warp --------
@pytest.mark.parametrize("tag", ["a", "b"])
def test_disp_warp_vs_reference_golden(tag):
    """oracle.disp_warp against nets/warp.py:41-64 run by the reference (make_model_golden.py)."""
    g = golden(f"warp_{tag}")
    warped, valid = oracle.disp_warp(g["img"], g["disp"])
    assert np.abs(warped - g["warped"]).max() <= 1e-6
    assert np.array_equal(valid, g["valid"])


def test_disp_warp_bwd_vs_torch_autograd_f64():
    import torch
    import torch.nn.functional as F
    g = golden("warp_a")
    img = torch.from_numpy(g["img"]).double()
    disp = torch.from_numpy(g["disp"]).double().requires_grad_()
    B, C, H, W = img.shape
    xs = torch.arange(W, dtype=torch.float64).view(1, 1, W).expand(B, H, W)
    ys = torch.arange(H, dtype=torch.float64).view(1, H, 1).expand(B, H, W)
    gx = 2 * ((xs - disp[:, 0]) / (W - 1)) - 1
    gy = 2 * (ys / (H - 1)) - 1
    out = F.grid_sample(img, torch.stack((gx, gy), -1), mode="bilinear", padding_mode="border",
                        align_corners=True)
    go = torch.randn(out.shape, generator=torch.Generator().manual_seed(3), dtype=torch.float64)
    (out * go).sum().backward()
    ref = oracle.disp_warp_bwd(g["img"], g["disp"], go.numpy())
    assert np.abs(ref - disp.grad.numpy()).max() <= 1e-9


@pytest.mark.parametrize("tag", ["hotpath_d64", "hotpath_c1"])
def test_production_config_oracle_matches_reference(tag):
    """The oracle at the production widths (max_disp 64: C2's; 24: C1's) against the reference
    graph's own output (tests/golden/make_production_golden.py)."""
    from tests.golden_io import production_case
    g, sd, _, left, right = production_case(tag)
    L = [t.numpy() for t in left]
    R = [t.numpy() for t in right]
    max_disp = int(g["max_disp"])
    vols = oagg.oracle.cost_volume_pyramid(L, R, max_disp)
    agg0 = oagg.adaptive_aggregation(vols, sd, intermediate_supervision=False)[0].detach().numpy()
    a0 = agg0.ravel()
    scale = np.abs(g["agg0_sample"]).max()
    np.testing.assert_allclose(a0[g["agg0_idx"]], g["agg0_sample"], atol=1e-5 * scale, rtol=0)
    assert abs(a0.astype(np.float64).sum() - g["agg0_sum"]) <= 1e-5 * g["agg0_abs_sum"]
    disp = oagg.oracle.disp_regress(agg0)
    err = np.abs(disp - g["disp0"]).max()
    assert err <= 1e-4, f"{tag}: oracle vs reference {err:.3g} px"
