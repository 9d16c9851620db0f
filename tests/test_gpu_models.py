"""GPU parity of the full models and the refinement warp against the
reference's own outputs (tests/golden/make_model_golden.py: nets/aanet.py run on CPU with the
oracle DCN, name-keyed synthetic weights, seeded image pairs).  Eval mode runs with the HIP
engine fusions on and off."""
import json

import numpy as np
import pytest
import torch

from aanet_amd import nets, ops, train
from oracle import oracle
from tests.golden_io import fill_synthetic, fixture_scales, golden, golden_names, synthetic_pair

pytestmark = pytest.mark.gpu
DEV = "cuda"
MODEL_FIXTURES = golden_names("model_")


# ------------------------------------------------------------------ disparity warp --------
@pytest.mark.parametrize("tag", ["a", "b"])
def test_disp_warp_vs_reference_golden(tag):
    g = golden(f"warp_{tag}")
    img, disp = torch.from_numpy(g["img"]).to(DEV), torch.from_numpy(g["disp"]).to(DEV)
    warped, valid = nets.disp_warp(img, disp)
    assert np.abs(warped.cpu().numpy() - g["warped"]).max() <= 1e-5
    assert np.array_equal(valid.cpu().numpy(), g["valid"])


@pytest.mark.parametrize("tag", ["a", "b"])
def test_disp_warp_backward_vs_oracle(tag):
    g = golden(f"warp_{tag}")
    img = torch.from_numpy(g["img"]).to(DEV).requires_grad_()
    disp = torch.from_numpy(g["disp"]).to(DEV).requires_grad_()
    warped, _ = nets.disp_warp(img, disp)
    go = torch.randn(warped.shape, generator=torch.Generator().manual_seed(5)).to(DEV)
    (warped * go).sum().backward()
    ref_d = oracle.disp_warp_bwd(g["img"], g["disp"], go.cpu().numpy())
    assert np.abs(disp.grad.cpu().numpy() - ref_d).max() <= 1e-4 * max(1.0, np.abs(ref_d).max())
    # image gradient: the transpose of the bilinear sampling, checked through linearity --
    # <grad_img, img> equals <grad_out, warped> because warped is linear in img
    lhs = float((img.grad.double() * img.detach().double()).sum())
    rhs = float((go.double() * warped.detach().double()).sum())
    assert lhs == pytest.approx(rhs, rel=1e-5, abs=1e-4)


def test_disp_warp_rejects_bad_shapes():
    img = torch.zeros(1, 3, 4, 5, device=DEV)
    with pytest.raises(ValueError):
        ops.disp_warp(img, torch.zeros(1, 3, 4, 5, device=DEV))


# ------------------------------------------------------------------ full models -----------
def build(tag, fuse=True):
    g = golden(tag)
    m = nets.AANet(int(g["max_disp"]), 1, **json.loads(str(g["config"])))
    fill_synthetic(m, int(g["seed"]), fixture_scales(g))
    m = m.to(DEV).eval()
    for mod in m.modules():
        mod.aanet_fuse = fuse
    B, H, W = (int(v) for v in g["shape"])
    left, right = synthetic_pair(B, H, W, int(g["seed"]))
    return g, m, left.to(DEV), right.to(DEV)


# the hot-path (adaptive aggregation) models: held to the 1e-3 px bar against the reference's
# fp32 output itself.  PSMNet-AA joins them on its conditioned fixture (make_model_golden.py
# SCALES_OF: the plain fill put its soft-argmin in a hard-argmax near-tie regime where the
# reference's own fp32 run was 0.2-0.7 px off its fp64 run)
STRICT = {"model_aanet", "model_aanet_inter", "model_aanetplus", "model_psmnet_aa"}
FLIP = 0.05  # px: a near-tie soft-argmin flip
# near-tie fixtures: the reference's own fp32 run flips hundreds of pixels against its fp64 run,
# and that count is one draw of a heavy-tailed distribution (its own level-1 flips range 0-151
# over 27 runs whose images differ by one rounding unit, profiles/r06_raw_stages.txt E).  They
# are checked stage by stage against data the fixture holds (make_model_golden.near_tie_data):
# the feature pyramid against fp64, the refinement alone, and the pyramid against the envelope
# of the reference's own pipeline with twice its own feature error (_check_near_tie).
NEAR_TIE = {"model_psmnet_aa_raw"}


def _stats(e):
    return float(e.mean()), float(np.percentile(e, 99)), float(e.max())


@pytest.mark.parametrize("fuse", [True, False])
@pytest.mark.parametrize("tag", MODEL_FIXTURES)
def test_full_model_vs_reference_golden(tag, fuse):
    """Every level of the disparity pyramid against the reference run on the same weights and
    images.  Each fixture also holds the reference's float64 run; per level our fp32 result must
    be no further from it than the reference's own fp32 result, up to
      * flips (|d - d64| > 0.05 px): at most 2x the reference's count + 4;
      * mean over the pixels that neither run flips: at most 2x the reference's;
      * p99 within 2x, max within 4x;
    and the adaptive-aggregation models (STRICT) additionally max |d - d32| <= 1e-3 px against
    the reference's fp32 output.  model_psmnet_aa_raw is PSMNet-AA without the fixture
    conditioning: the reference's own fp32 run flips 3 / 29 / 697 pixels (up to 0.2 / 0.3 /
    0.7 px) against its fp64 run there: that fixture is checked stage by stage instead
    (_check_near_tie), on both paths."""
    g, m, left, right = build(tag, fuse)
    # the plain convs of the reference-order run (those that are not ours) go through PyTorch's
    # native fp32 convolution (im2col + fp32 GEMM), not MIOpen: which MIOpen solver runs a conv
    # differs from box to box even with deterministic=True, benchmark=False, and some of its
    # gfx950 fp32 solvers round like TF32 -- PSMNet-AA level 1 went from 39 flips to 103-118
    # (bound 62) on boxes that picked them, and with MIOPEN_DEBUG_CONV_WINOGRAD=0 every time
    # (tools/diag_psmnet_flips.sh); TF32 proper gave 137.  A third-party algorithm choice is
    # not what this test measures, so it is taken out of the run.
    feats = []
    hook = m.fpn.register_forward_hook(lambda mod, i, o: feats.append([t.cpu() for t in o])) \
        if tag in NEAR_TIE else None
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False, allow_tf32=False):
        pyr = m(left, right)
    if hook is not None:
        hook.remove()
        return _check_near_tie(g, m, left, right, pyr, feats, fuse)
    n = len([k for k in g if k.startswith("disp") and not k.startswith("disp64")])
    assert len(pyr) == n
    report = []
    for i, d in enumerate(pyr):
        ref32, ref64 = g[f"disp{i}"], g[f"disp64_{i}"]
        assert tuple(d.shape) == ref32.shape
        ours = d.cpu().numpy().astype(np.float64)
        e32 = _stats(np.abs(ours - ref32))
        e64 = _stats(np.abs(ours - ref64))
        sens = _stats(np.abs(ref32.astype(np.float64) - ref64))
        report.append((i, e32, e64, sens))

        err64 = np.abs(ours - ref64)
        errref = np.abs(ref32.astype(np.float64) - ref64)
        flips, flips_ref = int((err64 > FLIP).sum()), int((errref > FLIP).sum())
        assert flips <= 2 * flips_ref + 4, (i, "flips", flips, "reference's own", flips_ref)
        calm = (err64 <= FLIP) & (errref <= FLIP)
        m_calm, m_calm_ref = float(err64[calm].mean()), float(errref[calm].mean())
        assert m_calm <= 2 * m_calm_ref + 1e-6, (i, "mean over non-flipped px", m_calm, m_calm_ref)
        # p99 within 2x the reference's own fp32 distance; the max (a single near-tie flip, a
        # noisy one-sample statistic) within 4x
        for got, bound, k, slack in zip(e64[1:], sens[1:], (2, 4), (1e-4, 1e-3)):
            assert got <= k * bound + slack, (i, "vs fp64", e64, "ref fp32 vs fp64", sens)
        if tag in STRICT:
            assert e32[2] <= 1e-3, (i, e32)
    print(tag, "fused" if fuse else "ref-order", ["L%d vs32 mean/p99/max %.1e/%.1e/%.1e | "
          "vs64 %.1e/%.1e/%.1e | ref32-vs-64 %.1e/%.1e/%.1e" % ((i,) + a + b + c)
          for i, a, b, c in report])


def _flip_stats(d, ref):
    e = np.abs(np.asarray(d, np.float64) - ref)
    return int((e > FLIP).sum()), float(np.percentile(e, 99)), float(e.max())


def _check_near_tie(g, m, left, right, pyr, feats, fuse):
    """A near-tie fixture (model_psmnet_aa_raw), stage by stage (profiles/r06_raw_stages.txt):
      1. the feature pyramid, both images: normwise error against the reference's fp64 features
         within 2x the reference's own fp32 error (+1e-7: the fp64 features are stored as float32);
      2. the refinement alone, fed the fp64 level-0 disparity: flips <= 2x the reference's + 4,
         p99 within 2x and max within 4x of the reference's own fp32 refinement of that input;
      3. every pyramid level within the envelope of the reference's own fp32 pipeline when its
         features carry twice its own error (48 seeded runs, make_model_golden.near_tie_data):
         flips, p99 and max |d - d64| no larger than the largest of those runs (p99 / max with
         the 1e-4 / 1e-3 px slack of the other fixtures' bounds).
    Step 3 is where the single-draw bound of the other fixtures does not hold: every level-1/2
    flip sits within 64 px of a level-0 flip, and the refinement alone flips nothing (step 2), so
    the counts are the level-0 near-ties (fp64 top-2 logit gaps down to 0.48 on logits of
    +-1.5e4) amplified; with 1.9x the reference's feature error -- the GPU fp32 conv accumulation,
    ours and torch's alike -- the reference's own pipeline gives 2-8 / 3-888 / 15-6052 flips."""
    tag = "fused" if fuse else "ref-order"
    assert len(feats) == 2
    e_ref = g["feat_err32"]
    for img in range(2):
        for s, t in enumerate(feats[img]):
            ref = g[f"feat64_{img}_{s}"].astype(np.float64)
            e = float(np.linalg.norm(t.numpy().astype(np.float64) - ref) / np.linalg.norm(ref))
            assert e <= 2 * e_ref[img * 3 + s] + 1e-7, (tag, "features", img, s, e, e_ref[img * 3 + s])
    d0 = torch.from_numpy(g["disp64_0"].astype(np.float32)).to(DEV)
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False, allow_tf32=False):
        cond = m.disparity_refinement(left, right, d0)
    for i, (c, (f_ref, p99_ref, max_ref)) in enumerate(zip(cond, g["cond32_stats"])):
        f, p99, mx = _flip_stats(c.cpu().numpy(), g[f"disp64_{i + 1}"])
        assert f <= 2 * f_ref + 4 and p99 <= 2 * p99_ref + 1e-6 and mx <= 4 * max_ref + 1e-5, \
            (tag, "refinement alone", i + 1, (f, p99, mx), tuple(g["cond32_stats"][i]))
    env = g["envelope"].max(0)
    report = []
    for i, d in enumerate(pyr):
        got = _flip_stats(d.cpu().numpy(), g[f"disp64_{i}"])
        # (p99 / max with the slack of the single-draw bounds above: 1e-4 / 1e-3 px)
        lim = tuple(float(v) + sl for v, sl in zip(env[3 * i:3 * i + 3], (0, 1e-4, 1e-3)))
        report.append((i, got, lim))
        assert all(a <= b for a, b in zip(got, lim)), (tag, "level", i, got, "envelope", lim)
    print("near-tie", tag, "per level (flips, p99, max) vs envelope:", report)


def test_aanetplus_c3_full_size_properties():
    """BASELINE configs[2] at its own image size: AANet+ (GANetFeature + FeaturePyrmaid +
    hourglass refinement, max_disp 192; scripts/aanet+_train.sh:12-15) on one 576x960 pair.
    The 32/64/128-channel feature pyramid at 192x320 / 96x160 / 48x80 feeds the hot path; the
    outputs must have the reference's shapes, be finite, the regressed level must lie in
    [0, D-1] = [0, 63] and the refined levels (ReLU'd, nets/refinement.py) be >= 0."""
    g = golden("model_aanetplus")
    m = nets.AANet(192, 1, **json.loads(str(g["config"])))
    fill_synthetic(m, int(g["seed"]))
    m = m.to(DEV).eval()
    left, right = synthetic_pair(1, 576, 960, int(g["seed"]))
    with torch.no_grad():
        feats = m.feature_extraction(left.to(DEV))
        assert [tuple(f.shape) for f in feats] == [(1, 32, 192, 320), (1, 64, 96, 160),
                                                   (1, 128, 48, 80)]
        pyr = m(left.to(DEV), right.to(DEV))
    assert [tuple(d.shape) for d in pyr] == [(1, 192, 320), (1, 288, 480), (1, 576, 960)]
    for d in pyr:
        assert torch.isfinite(d).all()
        assert float(d.min()) >= 0.0
    assert float(pyr[0].max()) <= 63.0
    print("AANet+ 576x960: disparity ranges", [(float(d.min()), float(d.max())) for d in pyr])


def test_full_model_training_step():
    """AANet with intermediate supervision in train mode: the 5-level pyramid, the reference
    loss weights, backward through every HIP kernel (DCN in the feature extractor and the
    aggregation, warp in the refinement), finite non-zero gradients everywhere."""
    g, m, left, right = build("model_aanet_inter")
    m.train()
    pyr = m(left, right)
    assert len(pyr) == 5
    gt = torch.rand(left.shape[0], *left.shape[2:], device=DEV) * 40 + 1
    total, per = train.disparity_loss(pyr, gt, gt > 0)
    total.backward()
    assert torch.isfinite(total)
    groups = {"feature_extractor": 0.0, "fpn": 0.0, "aggregation": 0.0, "refinement": 0.0}
    for name, p in m.named_parameters():
        assert p.grad is not None, name
        assert torch.isfinite(p.grad).all(), name
        top = name.split(".")[0]
        if top in groups:
            groups[top] += float(p.grad.abs().sum())
    assert all(v > 0 for v in groups.values()), groups
