"""GPU parity of the drop-in modules (aanet_amd.nets) against the reference's golden outputs.

The golden fixtures were produced by the REFERENCE's nets/cost.py + nets/aggregation.py +
nets/estimation.py graph (tests/golden/make_golden.py), with parameters loaded here by
state-dict key.  Tolerances: aggregation outputs 1e-4 abs; disparities 1e-3 px max abs (the
north-star bar), checked at 2e-4 here.
"""
import numpy as np
import pytest
import torch

from aanet_amd import nets
from oracle import aggregation as oagg
from tests.golden_io import golden, state_dict_of

pytestmark = pytest.mark.gpu
DEV = "cuda"


def g2t(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def build(tag, fuse=True):
    g = golden(f"aggregation_{tag}")
    inter = tag == "inter"
    m = nets.AANetHotPath(16, no_intermediate_supervision=not inter, num_deform_blocks=3)
    sd = {"aggregation." + k: torch.from_numpy(v) for k, v in state_dict_of(g).items()}
    missing, unexpected = m.load_state_dict(sd, strict=False)
    assert not unexpected and not missing, (missing, unexpected)
    m = m.to(DEV).eval()
    for mod in m.modules():
        mod.aanet_fuse = fuse
    return g, m


@pytest.mark.parametrize("tag", ["inter", "final"])
@pytest.mark.parametrize("fuse", [True, False])
def test_adaptive_aggregation_vs_reference_golden(tag, fuse):
    g, m = build(tag, fuse)
    vols = [g2t(g[f"volume{s}"]) for s in range(3)]
    caller_list = list(vols)
    with torch.no_grad():
        outs = m.aggregation(caller_list)
    # aggregation.py:382 mutates the caller's list in place (x[i] = dconv(x[i]))
    assert all(a is not b for a, b in zip(caller_list, vols))
    assert len(outs) == (3 if tag == "inter" else 1)
    for i, o in enumerate(outs):
        ref = g[f"agg{i}"]
        err = np.abs(o.cpu().numpy() - ref).max()
        assert err <= 1e-4, f"agg{i}: {err:.3g}"


@pytest.mark.parametrize("tag", ["inter", "final"])
def test_hot_path_disparity_vs_reference_golden(tag):
    g, m = build(tag)
    with torch.no_grad():
        disps = m([g2t(g[f"feat_left{s}"]) for s in range(3)],
                  [g2t(g[f"feat_right{s}"]) for s in range(3)])
    n = 3 if tag == "inter" else 1
    assert len(disps) == n
    for i in range(n):
        err = np.abs(disps[i].cpu().numpy() - g[f"disp{i}"]).max()
        assert err <= 2e-4, f"disp{i}: max abs {err:.3g} px"


def test_training_step_gradients_vs_oracle():
    """Train-mode forward+backward of the whole path (BN batch stats, HIP DCN backward) against
    the CPU oracle graph with torch autograd + the C oracle DCN backward."""
    g = golden("aggregation_inter")
    sd_np = state_dict_of(g)
    m = nets.AANetHotPath(16, no_intermediate_supervision=False, num_deform_blocks=3)
    m.load_state_dict({"aggregation." + k: torch.from_numpy(v) for k, v in sd_np.items()})
    m = m.to(DEV).train()
    fl = [g2t(g[f"feat_left{s}"]).requires_grad_() for s in range(3)]
    fr = [g2t(g[f"feat_right{s}"]).requires_grad_() for s in range(3)]
    disps = m(fl, fr)
    loss = sum((d * (i + 1)).mean() for i, d in enumerate(disps))
    loss.backward()

    # oracle: same math on CPU (torch autograd for stock ops, oracle C for DCN + cost + regression)
    params = {k: torch.from_numpy(v.copy()).requires_grad_(v.dtype == np.float32 and "running" not in k
                                                            and "num_batches" not in k)
              for k, v in sd_np.items()}
    vols = [torch.tensor(g[f"volume{s}"]) for s in range(3)]
    for v in vols:
        v.requires_grad_()
    oagg.TRAINING = True
    try:
        aggs = oagg.adaptive_aggregation(vols, params, intermediate_supervision=True)
    finally:
        oagg.TRAINING = False
    # regression as torch ops (estimation.py:19-28) for autograd
    ref_loss = 0
    for i in range(3):
        a = aggs[2 - i]
        p = torch.softmax(a, 1)
        d = (p * torch.arange(a.shape[1], dtype=a.dtype).view(1, -1, 1, 1)).sum(1)
        ref_loss = ref_loss + (d * (i + 1)).mean()
    ref_loss.backward()
    assert abs(float(loss) - float(ref_loss)) <= 1e-4 * max(1.0, abs(float(ref_loss)))
    named = dict(m.aggregation.named_parameters())
    checked = 0
    for k, p in params.items():
        if p.grad is None:
            continue
        got = named[k].grad.cpu().numpy()
        ref = p.grad.numpy()
        scale = np.abs(ref).max() + 1e-8
        err = np.abs(got - ref).max()
        assert err <= 2e-3 * scale + 1e-6, f"{k}: err {err:.3g} scale {scale:.3g}"
        checked += 1
    assert checked > 100
    # cost-volume gradient w.r.t. the features: compare through the volume gradient
    for s in range(3):
        assert fl[s].grad is not None and torch.isfinite(fl[s].grad).all()
