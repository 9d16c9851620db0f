"""Post stage of the tail kernels (aanet_post_stage_t): the next pointwise conv of the path run in
the scale-0 tail kernel's epilogue on its CSA output -- the next AAModule's bottleneck conv1 +
BN1 + ReLU (channels-last), or final_conv + the soft-argmin (nets/aggregation.py:443-447,
nets/estimation.py:13-30).  Checked against the same stages run as separate kernels on the
tail's own CSA output, and the module path against the post-free schedules
(set_options(post_fusion="none" / "final"), nets/options.py)."""
import pytest
import torch

from aanet_amd import nets, ops
from aanet_amd.nets._fuse import conv_bn_act, folded
from tests.golden_io import fill_synthetic, synthetic_pyramid

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _tail_inputs(B=2, H=24, W=64, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    C = 64
    x = torch.randn(B, C, H, W, device=DEV, generator=g).relu_().contiguous(memory_format=torch.channels_last)
    res = torch.randn(B, C, H, W, device=DEV, generator=g)
    w3 = torch.randn(C, C, 3, 3, device=DEV, generator=g) * 0.04
    w1 = torch.randn(C, C, 1, 1, device=DEV, generator=g) * 0.1
    b = torch.randn(C, device=DEV, generator=g)
    om = torch.randn(B, 54, H, W, device=DEV, generator=g) * 0.7
    ups = [torch.randn(B, C, H // r, W // r, device=DEV, generator=g) for r in (2, 4)]
    wn = torch.randn(C, C, 1, 1, device=DEV, generator=g) * 0.1
    bn_ = torch.randn(C, device=DEV, generator=g)
    return x, res, w3, w1, b, om, ups, wn, bn_


@pytest.mark.parametrize("kind", ["conv1", "regress"])
def test_dcn_tail_post_stage_matches_separate_kernels(kind):
    x, res, w3, w1, b, om, ups, wn, bn_ = _tail_inputs()
    p3, p1, pn = ops.pack_weight_split(w3), ops.pack_weight_split(w1), ops.pack_weight_split(wn)
    if kind == "conv1":
        post = {"packed": pn, "bias": bn_, "act": "relu", "nhwc": True}
    else:
        post = {"packed": pn, "bias": bn_, "act": None, "disp": True}
    out, csa, pres = ops.mdcn_pw(x, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2, 2,
                                 csa_up=ups, post=post)
    assert pres is not None, "the window DCN tail must take the post stage at this shape"
    out0, csa0 = ops.mdcn_pw(x, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2, 2,
                             csa_up=ups)
    assert torch.equal(out, out0) and torch.equal(csa, csa0)  # the post stage changes nothing else
    t = ops.conv2d_fused(csa0, wn, bn_, packed_weight=pn,
                         act="relu" if kind == "conv1" else None)
    if kind == "conv1":
        got = pres["out"]
        assert got.is_contiguous(memory_format=torch.channels_last)
        err = (got - t).abs().max().item()
        assert err <= 2e-5 * max(1.0, t.abs().max().item()), err
    else:
        ref = ops.disp_regress(t)
        err = (pres["disp"] - ref).abs().max().item()
        assert err <= 1e-4, err
        # skip_outputs: the same disparities, the tail's own outputs left unwritten
        post_s = dict(post, skip_outputs=True)
        _, _, pres_s = ops.mdcn_pw(x, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2,
                                   2, csa_up=ups, post=post_s)
        assert torch.equal(pres_s["disp"], pres["disp"])


def test_plain_tail_post_stage_matches_separate_kernel():
    """The plain 3x3 halo tail (SimpleBottleneck, nets/deform.py:171-184) with the conv1 post
    stage; the regression form is not implemented there: the op repeats the call without it and
    reports None (the caller then runs the stage itself)."""
    x, res, w3, w1, b, om, ups, wn, bn_ = _tail_inputs(seed=3)
    w2 = torch.randn(64, 64, 3, 3, device=DEV, generator=torch.Generator(device=DEV).manual_seed(4)) * 0.04
    p2, p1, pn = ops.pack_weight_split(w2), ops.pack_weight_split(w1), ops.pack_weight_split(wn)
    out, csa, pres = ops.conv2d_pw(x, w2, p2, b, None, None, "relu", p1, b, res, "relu", 1, 1, 1,
                                   csa_up=ups,
                                   post={"packed": pn, "bias": bn_, "act": "relu", "nhwc": True})
    assert pres is not None, "the halo tail must take the conv1 post stage at this shape"
    out0, csa0 = ops.conv2d_pw(x, w2, p2, b, None, None, "relu", p1, b, res, "relu", 1, 1, 1,
                               csa_up=ups)
    assert torch.equal(out, out0) and torch.equal(csa, csa0)
    t = ops.conv2d_fused(csa0, wn, bn_, packed_weight=pn, act="relu")
    err = (pres["out"] - t).abs().max().item()
    assert err <= 2e-5 * max(1.0, t.abs().max().item()), err
    r = ops.conv2d_pw(x, w2, p2, b, None, None, "relu", p1, b, res, "relu", 1, 1, 1, csa_up=ups,
                      post={"packed": pn, "bias": bn_, "act": None, "disp": True})
    assert r[2] is None and torch.equal(r[0], out0) and torch.equal(r[1], csa0)


@pytest.mark.parametrize("mode", ["none", "final"])
def test_hot_path_post_fusion_matches_unfused(mode):
    """C2-width hot path (D=64) on a small pyramid: disparities with the post stages (conv1 folds,
    tail regression) vs without them (post_fusion="none") or with the last one only ("final")."""
    torch.manual_seed(0)
    m = nets.AANetHotPath(64, no_intermediate_supervision=True, num_deform_blocks=3)
    fill_synthetic(m.aggregation, 7)
    m = m.to(DEV).eval()
    left, right = synthetic_pyramid(2, 128, 48, 96, 7)
    left, right = [t.to(DEV) for t in left], [t.to(DEV) for t in right]
    with torch.no_grad():
        d_post = m(left, right)[0]
        m.set_options(post_fusion=mode)
        d_ref = m(left, right)[0]
    err = (d_post - d_ref).abs().max().item()
    assert err <= 2e-4, err
