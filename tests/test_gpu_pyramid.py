"""One-launch correlation pyramid (aanet_corr_pyramid_f32, nets/cost.py:58-76): every scale is
bit-identical to its single-volume launch (same tile code), on the C2 and C1 pyramids, ragged
widths and the separate-launch fallback (width % 4 != 0); CostVolumePyramid's autograd matches
per-scale CostVolume."""
import pytest
import torch

from aanet_amd import ops
from aanet_amd.nets import CostVolume, CostVolumePyramid

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _pyr(B, C, H, W, ns, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    left = [torch.randn(B, C, H >> s, W >> s, device=DEV, generator=g) for s in range(ns)]
    right = [torch.randn(B, C, H >> s, W >> s, device=DEV, generator=g) for s in range(ns)]
    return left, right


@pytest.mark.parametrize("B,C,H,W,D,ns", [
    (2, 128, 128, 416, 64, 3),   # C2 pyramid (B=2)
    (1, 128, 96, 192, 24, 3),    # C1 pyramid: D = 24 / 12 / 6
    (2, 32, 20, 72, 40, 2),      # ragged x tiles, D not a multiple of 16
    (1, 16, 9, 36, 70, 1),       # D > 64: several disparity chunks
    (1, 8, 12, 50, 16, 2),       # width % 4 != 0 at scale 1: separate launches
])
def test_pyramid_equals_single_volumes(B, C, H, W, D, ns):
    left, right = _pyr(B, C, H, W, ns, seed=W + D)
    outs = ops.corr_pyramid(left, right, D)
    for s in range(ns):
        ref = ops.corr_volume(left[s], right[s], D >> s)
        assert outs[s].shape == ref.shape
        assert torch.equal(outs[s], ref), s


def test_cost_volume_pyramid_autograd_matches_per_scale():
    left, right = _pyr(2, 32, 24, 64, 3, seed=3)
    lp = [t.clone().requires_grad_() for t in left]
    rp = [t.clone().requires_grad_() for t in right]
    vols = CostVolumePyramid(32)(lp, rp)
    g = torch.Generator(device=DEV).manual_seed(4)
    gos = [torch.randn(v.shape, device=DEV, generator=g) for v in vols]
    sum((v * go).sum() for v, go in zip(vols, gos)).backward()
    for s in range(3):
        ls, rs = left[s].clone().requires_grad_(), right[s].clone().requires_grad_()
        v = CostVolume(32 >> s)(ls, rs)
        assert torch.equal(v.detach(), vols[s].detach())
        (v * gos[s]).sum().backward()
        assert torch.allclose(ls.grad, lp[s].grad, rtol=1e-6, atol=1e-6)
        assert torch.allclose(rs.grad, rp[s].grad, rtol=1e-6, atol=1e-6)
