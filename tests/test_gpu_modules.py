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


def _grads_vs_oracle(sd_np, train_bn):
    """Forward+backward of the whole path on the GPU (HIP DCN / cost / regression backward) and
    of the oracle graph on the CPU (torch autograd for stock ops + the C oracle DCN backward).
    Returns (our loss, oracle loss, [(name, ours, oracle)])."""
    g = golden("aggregation_inter")
    m = nets.AANetHotPath(16, no_intermediate_supervision=False, num_deform_blocks=3)
    m.load_state_dict({"aggregation." + k: torch.from_numpy(v) for k, v in sd_np.items()})
    m = m.to(DEV)
    m.train(train_bn)
    fl = [g2t(g[f"feat_left{s}"]).requires_grad_() for s in range(3)]
    fr = [g2t(g[f"feat_right{s}"]).requires_grad_() for s in range(3)]
    disps = m(fl, fr)
    loss = sum((d * (i + 1)).mean() for i, d in enumerate(disps))
    loss.backward()

    params = {k: torch.from_numpy(v.copy()).requires_grad_("running" not in k and "num_batches" not in k)
              for k, v in sd_np.items()}
    with torch.no_grad():
        vols = [torch.from_numpy(v) for v in
                oagg.oracle.cost_volume_pyramid([g[f"feat_left{s}"] for s in range(3)],
                                                [g[f"feat_right{s}"] for s in range(3)], 16)]
    oagg.TRAINING = train_bn
    try:
        aggs = oagg.adaptive_aggregation(vols, params, intermediate_supervision=True)
    finally:
        oagg.TRAINING = False
    ref_loss = 0
    for i in range(3):  # estimation.py:19-28 as torch ops, reverse scale order (aanet.py:161)
        a = aggs[2 - i]
        p = torch.softmax(a, 1)
        d = (p * torch.arange(a.shape[1], dtype=a.dtype).view(1, -1, 1, 1)).sum(1)
        ref_loss = ref_loss + (d * (i + 1)).mean()
    ref_loss.backward()
    named = dict(m.aggregation.named_parameters())
    pairs = [(k, named[k].grad.cpu().numpy(), p.grad.numpy()) for k, p in params.items()
             if p.grad is not None]
    return float(loss.detach()), float(ref_loss.detach()), pairs


def test_training_gradients_vs_oracle_strict():
    """Eval-mode BN (linear) and offsets that are exact fractional constants (offset_conv weight 0,
    random bias): CPU and GPU forwards then take identical floor() branches, so every gradient
    must agree to rounding.  Checks the autograd wiring of all HIP backward kernels."""
    sd = dict(state_dict_of(golden("aggregation_inter")))
    rng = np.random.default_rng(9)
    for k in list(sd):
        if k.endswith("offset_conv.weight"):
            sd[k] = np.zeros_like(sd[k])
        if k.endswith("offset_conv.bias"):
            b = rng.uniform(0.1, 0.9, sd[k].shape) * rng.choice([-1, 1], sd[k].shape)
            sd[k] = b.astype(np.float32)
    loss, ref_loss, pairs = _grads_vs_oracle(sd, train_bn=False)
    assert abs(loss - ref_loss) <= 1e-5 * max(1.0, abs(ref_loss))
    bad = []
    for k, got, ref in pairs:
        scale = np.abs(ref).max() + 1e-8
        err = np.abs(got - ref).max()
        if err > 1e-3 * scale + 1e-6:
            bad.append(f"{k}: err {err:.3g} scale {scale:.3g}")
    assert len(pairs) > 100
    assert not bad, f"{len(bad)}/{len(pairs)} params off:\n" + "\n".join(bad[:40])


def test_training_gradients_vs_oracle_train_bn_random_offsets():
    """Train-mode BN (batch statistics) with learned-like random offsets.  The bilinear sampler's
    derivative jumps where a sample crosses an integer grid line, and CPU/GPU offsets differ in
    the last bits, so a handful of samples may take different branches: the gradients are
    compared by direction (cosine similarity) rather than element-wise."""
    sd = state_dict_of(golden("aggregation_inter"))
    loss, ref_loss, pairs = _grads_vs_oracle(sd, train_bn=True)
    assert abs(loss - ref_loss) <= 1e-4 * max(1.0, abs(ref_loss))
    allg = np.concatenate([g.ravel() for _, g, _ in pairs])
    allr = np.concatenate([r.ravel() for _, _, r in pairs])
    cos = float(allg @ allr / (np.linalg.norm(allg) * np.linalg.norm(allr)))
    assert cos > 0.999, cos
    for k, got, ref in pairs:
        n = np.linalg.norm(ref)
        if n > 1e-6:
            assert float(got.ravel() @ ref.ravel()) / (np.linalg.norm(got) * n) > 0.99, k
