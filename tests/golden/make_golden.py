"""Generate golden vectors for the hot path from the REFERENCE's own Python code.

Run in the build container only (needs /root/reference; never on the GPU box):
    python tests/golden/make_golden.py

What it imports from the reference, by file path (so nets/__init__.py, which needs the
CUDA-only deform_conv_cuda extension, is never executed -- SURVEY.md §8c):
  * nets/cost.py        CostVolume, CostVolumePyramid           (cost.py:5-76)
  * nets/estimation.py  DisparityEstimation                     (estimation.py:6-30)
  * nets/deform.py + nets/aggregation.py  AdaptiveAggregation    (aggregation.py:313-464)
    with ``nets.deform_conv`` replaced by a stand-in whose ModulatedDeformConv runs the
    oracle's C restatement of the CUDA kernel (the reference DCN cannot run here).  The DCN
    numerics inside the aggregation fixtures are therefore the oracle's; the surrounding graph
    (ISA/CSA wiring, BN, interpolation, LeakyReLU, final conv) is the reference's.

Every fixture is DATA ONLY (inputs, parameters, expected outputs) in .npz form.
"""
import importlib.util
import math
import os
import sys
import types

import numpy as np
import torch
import torch.nn as nn

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("AANET_REFERENCE", "/root/reference")
sys.path.insert(0, REPO)
from oracle import oracle  # noqa: E402


def _load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


class _StandInModulatedDeformConv(nn.Module):
    """Same constructor/parameters as deform_conv.py:304-351; forward runs the oracle."""

    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1,
                 groups=1, deformable_groups=1, bias=True):
        super().__init__()
        self.in_channels, self.out_channels = in_channels, out_channels
        self.kernel_size = (kernel_size, kernel_size) if isinstance(kernel_size, int) else tuple(kernel_size)
        self.stride, self.padding, self.dilation = stride, padding, dilation
        self.groups, self.deformable_groups = groups, deformable_groups
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels // groups, *self.kernel_size))
        self.bias = nn.Parameter(torch.zeros(out_channels)) if bias else None
        stdv = 1.0 / math.sqrt(in_channels * self.kernel_size[0] * self.kernel_size[1])
        self.weight.data.uniform_(-stdv, stdv)

    def forward(self, x, offset, mask):
        dtype = np.float64 if x.dtype == torch.float64 else np.float32  # fp64: sensitivity runs
        out = oracle.mdcn_forward(x.detach().numpy(), offset.detach().numpy(), mask.detach().numpy(),
                                  self.weight.detach().numpy(),
                                  None if self.bias is None else self.bias.detach().numpy(),
                                  self.stride, self.padding, self.dilation, self.groups,
                                  self.deformable_groups, dtype=dtype)
        return torch.from_numpy(out)


def load_reference():
    cost = _load("ref_cost", os.path.join(REF, "nets", "cost.py"))
    est = _load("ref_estimation", os.path.join(REF, "nets", "estimation.py"))
    # Stand-in package so that `from nets.deform import ...` resolves to the reference file
    # while nets/__init__.py (which imports the CUDA extension) is never run.
    pkg = types.ModuleType("nets")
    pkg.__path__ = [os.path.join(REF, "nets")]
    sys.modules["nets"] = pkg
    dc = types.ModuleType("nets.deform_conv")
    dc.ModulatedDeformConv = _StandInModulatedDeformConv
    dc.DeformConv = None  # unmodulated DCN is dead code for AANet
    sys.modules["nets.deform_conv"] = dc
    _load("nets.deform", os.path.join(REF, "nets", "deform.py"))
    agg = _load("nets.aggregation", os.path.join(REF, "nets", "aggregation.py"))
    return cost, est, agg


def save(name, **arrays):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **{k: np.asarray(v) for k, v in arrays.items()})
    print(f"wrote {name}.npz ({os.path.getsize(path)} B)")


def structured_pair(g, B, C, H, W, maxd):
    """Random texture; right = left shifted by a per-row disparity field (peaked softmax)."""
    right = torch.randn(B, C, H, W + maxd, generator=g)
    disp = torch.randint(0, maxd, (B, H), generator=g)
    left = torch.empty(B, C, H, W)
    for b in range(B):
        for y in range(H):
            d = int(disp[b, y])
            left[b, :, y, :] = right[b, :, y, maxd - d: maxd - d + W]
    return left, right[..., maxd:].contiguous()


def randomize_bn_and_offsets(model, g):
    for name, m in model.named_modules():
        if isinstance(m, nn.BatchNorm2d):
            m.running_mean.copy_(0.1 * torch.randn(m.num_features, generator=g))
            m.running_var.copy_(0.5 + torch.rand(m.num_features, generator=g))
            m.weight.data.copy_(1.0 + 0.1 * torch.randn(m.num_features, generator=g))
            m.bias.data.copy_(0.1 * torch.randn(m.num_features, generator=g))
        if name.endswith("offset_conv"):
            # offset_conv is zero-initialised in the reference (deform.py:75-76), which would
            # make the DCN a plain conv; SURVEY §8c asks for nonzero offsets in parity tests.
            m.weight.data.copy_(0.3 * torch.randn(m.weight.shape, generator=g))
            m.bias.data.copy_(0.5 * torch.randn(m.bias.shape, generator=g))


def main():
    cost, est, agg = load_reference()
    g = torch.Generator().manual_seed(20261015)

    # ---- correlation volumes (cost.py:40-48)
    corr_cases = {
        "randn_small": (2, 8, 12, 40, 16),
        "randn_c128": (1, 128, 8, 48, 24),
        "d_gt_w": (1, 16, 6, 10, 16),
        "odd": (3, 5, 7, 33, 9),
    }
    for tag, (B, C, H, W, D) in corr_cases.items():
        l, r = torch.randn(B, C, H, W, generator=g), torch.randn(B, C, H, W, generator=g)
        out = cost.CostVolume(D, "correlation")(l, r)
        save(f"corr_{tag}", left=l, right=r, max_disp=D, out=out)
    l, r = structured_pair(g, 2, 32, 16, 64, 24)
    save("corr_structured", left=l, right=r, max_disp=24, out=cost.CostVolume(24)(l, r))
    l = torch.randn(1, 64, 8, 40, generator=g).abs()
    r = torch.randn(1, 64, 8, 40, generator=g).abs()
    save("corr_relu", left=l, right=r, max_disp=20, out=cost.CostVolume(20)(l, r))

    # ---- concat / difference volumes (cost.py:22-38)
    for tag, (B, C, H, W, D) in {"a": (2, 4, 6, 20, 8), "b": (1, 3, 5, 7, 9)}.items():
        l, r = torch.randn(B, C, H, W, generator=g), torch.randn(B, C, H, W, generator=g)
        save(f"concat_{tag}", left=l, right=r, max_disp=D, out=cost.CostVolume(D, "concat")(l, r))
        save(f"diff_{tag}", left=l, right=r, max_disp=D, out=cost.CostVolume(D, "difference")(l, r))

    # ---- pyramid (cost.py:58-76)
    pl = [torch.randn(2, 8, 16 >> s, 48 >> s, generator=g) for s in range(3)]
    pr = [torch.randn(2, 8, 16 >> s, 48 >> s, generator=g) for s in range(3)]
    outs = cost.CostVolumePyramid(16)(pl, pr)
    save("pyramid", **{f"left{s}": pl[s] for s in range(3)}, **{f"right{s}": pr[s] for s in range(3)},
         **{f"out{s}": outs[s] for s in range(3)}, max_disp=16)

    # ---- disparity regression (estimation.py:13-30)
    reg_cases = {
        "sim": (torch.randn(2, 16, 8, 20, generator=g) * 3, 16, True),
        "cost": (torch.randn(2, 16, 8, 20, generator=g) * 3, 16, False),
        "d_ne_maxdisp": (torch.randn(1, 12, 5, 9, generator=g), 24, True),
        "peaked": (torch.randn(1, 64, 4, 33, generator=g) * 40, 64, True),
        "flat": (torch.zeros(1, 10, 3, 7), 10, True),
        "d192": (torch.randn(1, 192, 3, 17, generator=g) * 2, 192, False),
    }
    for tag, (c, maxd, sim) in reg_cases.items():
        save(f"regress_{tag}", cost=c, max_disp=maxd, match_similarity=int(sim),
             out=est.DisparityEstimation(maxd, sim)(c))

    # ---- AdaptiveAggregation + full hot path (aggregation.py:406-464, aanet.py:146-167)
    torch.manual_seed(7)
    for inter in (True, False):
        model = agg.AdaptiveAggregation(max_disp=16, num_scales=3, num_fusions=6, num_stage_blocks=1,
                                        num_deform_blocks=3, intermediate_supervision=inter,
                                        deformable_groups=2, mdconv_dilation=2)
        randomize_bn_and_offsets(model, g)
        model.eval()
        fl = [torch.randn(2, 16, 24 >> s, 48 >> s, generator=g) for s in range(3)]
        fr = [torch.randn(2, 16, 24 >> s, 48 >> s, generator=g) for s in range(3)]
        with torch.no_grad():
            vols = cost.CostVolumePyramid(16)(fl, fr)
            vol_in = [v.clone() for v in vols]
            aggs = model(vols)
            estimation = est.DisparityEstimation(16, True)
            disps = [estimation(aggs[len(aggs) - 1 - i]) for i in range(len(aggs))]
        sd = {("param." + k): v.numpy() for k, v in model.state_dict().items()}
        tag = "inter" if inter else "final"
        save(f"aggregation_{tag}", **sd,
             **{f"feat_left{s}": fl[s] for s in range(3)}, **{f"feat_right{s}": fr[s] for s in range(3)},
             **{f"volume{s}": vol_in[s] for s in range(3)},
             **{f"agg{i}": a for i, a in enumerate(aggs)},
             **{f"disp{i}": d for i, d in enumerate(disps)})
        print(f"  aggregation_{tag}: agg0 std {aggs[0].std():.3f}, max|.| {aggs[0].abs().max():.3f}")


if __name__ == "__main__":
    main()
