"""CPU tests of the full-model plumbing: every model configuration of
the reference's fixtures builds here with the reference's exact state-dict keys, shapes, weight
sharing and (name-keyed synthetic) weights; checkpoints round-trip through the reference's
file format, including its `module.` prefix behaviour.  Forward passes need the GPU
(tests/test_gpu_models.py)."""
import json
import os

import numpy as np
import pytest
import torch

from aanet_amd import checkpoint, nets
from tests.golden_io import fill_synthetic, fixture_scales, golden, golden_names, synthetic_pair

MODEL_FIXTURES = golden_names("model_")


def build(tag):
    g = golden(tag)
    m = nets.AANet(int(g["max_disp"]), 1, **json.loads(str(g["config"])))
    names = fill_synthetic(m, int(g["seed"]), fixture_scales(g))
    return g, m, names


def test_fixture_set():
    assert {"model_aanet", "model_aanetplus", "model_psmnet_hg", "model_gcnet_3d",
            "model_stereonet_3d"} <= set(MODEL_FIXTURES)


@pytest.mark.parametrize("tag", MODEL_FIXTURES)
def test_state_dict_matches_reference(tag):
    g, m, names = build(tag)
    ref = dict(zip(g["names"].tolist(), g["shapes"].tolist()))
    ours = {n: ",".join(map(str, s)) for n, s in names}
    assert set(ours) == set(ref), (set(ref) - set(ours), set(ours) - set(ref))
    assert all(ours[k] == ref[k] for k in ref)
    # same weights, incl. the reference's shared blocks (last write wins in state-dict order)
    cs = sum(float(v.double().abs().sum()) for v in m.state_dict().values())
    assert cs == pytest.approx(float(g["checksum"]), rel=1e-12)
    B, H, W = (int(v) for v in g["shape"])
    left, right = synthetic_pair(B, H, W, int(g["seed"]))
    assert float(left.double().sum() + right.double().abs().sum()) == \
        pytest.approx(float(g["img_checksum"]), rel=1e-12)


def test_psmnet_basic_shares_conv1_like_reference():
    m = nets.PSMNetBasicAggregation(16)
    assert m.dres1[0] is m.dres0[2] is m.classify[0] is m.dres4[2]


def test_checkpoint_round_trip_and_module_prefix(tmp_path):
    _, m, _ = build("model_gcnet_aa")
    opt = torch.optim.Adam(m.parameters(), lr=1e-3)
    checkpoint.save_checkpoint(str(tmp_path), opt, m, epoch=7, num_iter=70, epe=1.5, best_epe=1.2,
                               best_epoch=5)
    assert sorted(os.listdir(tmp_path)) == ["aanet_epoch_007.pth", "optimizer_epoch_007.pth"]
    fresh = nets.AANet(48, 1, **json.loads(str(golden("model_gcnet_aa")["config"])))
    meta = checkpoint.load_pretrained_net(fresh, str(tmp_path / "aanet_epoch_007.pth"),
                                          return_epoch_iter=True, verbose=False)
    assert meta == (7, 70, 1.2, 5)
    for (k, a), b in zip(m.state_dict().items(), fresh.state_dict().values()):
        assert torch.equal(a, b), k
    # DDP-saved keys carry `module.`: the reference loader (no stripping) loads nothing with
    # no_strict and fails strict loads; strip_module_prefix fixes the keys
    ddp_path = tmp_path / "ddp.pth"
    torch.save({"state_dict": {"module." + k: v for k, v in m.state_dict().items()}}, ddp_path)
    fresh2 = nets.AANet(48, 1, **json.loads(str(golden("model_gcnet_aa")["config"])))
    missing, unexpected = checkpoint.load_pretrained_net(fresh2, str(ddp_path), no_strict=True,
                                                         verbose=False)
    # (BatchNorm back-fills a missing num_batches_tracked without reporting it)
    assert set(missing) == {k for k in m.state_dict() if not k.endswith("num_batches_tracked")}
    assert len(unexpected) == len(m.state_dict())
    with pytest.raises(RuntimeError):
        checkpoint.load_pretrained_net(fresh2, str(ddp_path), verbose=False)
    missing, unexpected = checkpoint.load_pretrained_net(fresh2, str(ddp_path),
                                                         strip_module_prefix=True, verbose=False)
    assert not missing and not unexpected
    assert torch.equal(fresh2.state_dict()["fpn.out1.0.weight"], m.state_dict()["fpn.out1.0.weight"])
    with pytest.raises(RuntimeError):
        checkpoint.resume_latest_ckpt(str(tmp_path / "none"), fresh2, "aanet")


def test_refinement_and_aggregator_constructors():
    """Every refinement / aggregation / feature type named by AANet's constructor builds."""
    for ref in ("stereonet", "stereodrnet", "hourglass", None, "None"):
        nets.AANet(48, refinement_type=ref)
    for agg, sim in (("psmnet_basic", "concat"), ("psmnet_hourglass", "concat"),
                     ("gcnet", "concat"), ("stereonet", "difference")):
        nets.AANet(48, feature_type="psmnet", feature_similarity=sim, aggregation_type=agg,
                   refinement_type=None)
    with pytest.raises(NotImplementedError):
        nets.AANet(48, feature_type="vgg")
    with pytest.raises(NotImplementedError):
        nets.AANet(48, aggregation_type="sgm")
    with pytest.raises(NotImplementedError):
        nets.AANet(48, refinement_type="crf")
