"""Production-configuration golden vectors of the hot path from the REFERENCE's own code.

Run in the build container only (needs /root/reference; never on the GPU box):
    python tests/golden/make_production_golden.py

The round-1 hot-path fixtures (make_golden.py) run AdaptiveAggregation at max_disp=16, where
every scale is narrower than 32 channels, so the GPU tests against them exercise the exact-f32
NCHW engine only.  These fixtures pin the configurations the bench and the users actually run:

  hotpath_d64  max_disp=64 (the C2 width: train.py --max_disp 192 // 3), features
               [2,128,32,96] pyramid -> scale widths 64/32/16: the split-bf16 contraction, the
               NHWC bottleneck tails and the CSA epilogue (exact 2x/4x terms, W % 4 == 0)
  hotpath_c1   max_disp=24 (BASELINE configs[0]: 288x576, --max_disp 72 // 3), features
               [1,128,96,192] pyramid -> widths 24/12/6
  hotpath_c3   max_disp=64, AANet+ feature widths (BASELINE configs[2]: GANetFeature +
               FeaturePyrmaid, nets/feature.py:150,379-419): [1,32,48,80] / [1,64,24,40] /
               [1,128,12,20] -- the C3 pyramid's channel counts at a reduced H x W

The reference graph is nets/cost.py CostVolumePyramid -> nets/aggregation.py
AdaptiveAggregation(num_deform_blocks=3, intermediate_supervision=False) ->
nets/estimation.py DisparityEstimation in reverse scale order (nets/aanet.py:146-167), imported
by file path exactly as make_golden.py does (the DCN inside is the oracle's C restatement, the
reference DCN being CUDA-only).  Weights are the name-keyed deterministic fill of
tests/golden_io.synthetic_value (offset_conv non-zero), features tests/golden_io.synthetic_pyramid:
the fixture holds DATA ONLY -- the output disparities, the same graph's float64 output (the
reference's own fp32 rounding distance) and checksums of the weights and inputs.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from make_golden import load_reference, save  # noqa: E402
from tests.golden_io import fill_synthetic, synthetic_pyramid  # noqa: E402

CASES = {
    # tag: (max_disp, B, C, H, W, seed[, per-scale channels])
    "hotpath_d64": (64, 2, 128, 32, 96, 64),
    "hotpath_c1": (24, 1, 128, 96, 192, 24),
    "hotpath_c3": (64, 1, 32, 48, 80, 3, (32, 64, 128)),
}


def run(cost, est, agg, max_disp, left, right, model):
    vols = cost.CostVolumePyramid(max_disp)(left, right)
    aggs = model(vols)
    estimation = est.DisparityEstimation(max_disp, True)
    return [estimation(aggs[len(aggs) - 1 - i]) for i in range(len(aggs))], aggs[0]


def main():
    cost, est, agg = load_reference()
    for tag, case in CASES.items():
        max_disp, B, C, H, W, seed = case[:6]
        channels = case[6] if len(case) > 6 else None
        torch.manual_seed(seed)
        model = agg.AdaptiveAggregation(max_disp=max_disp, num_scales=3, num_fusions=6,
                                        num_stage_blocks=1, num_deform_blocks=3,
                                        intermediate_supervision=False, deformable_groups=2,
                                        mdconv_dilation=2)
        names = fill_synthetic(model, seed)
        model.eval()
        left, right = synthetic_pyramid(B, C, H, W, seed, channels=channels)
        with torch.no_grad():
            disp, agg0 = run(cost, est, agg, max_disp, left, right, model)
            disp64, _ = run(cost, est, agg, max_disp, [t.double() for t in left],
                            [t.double() for t in right], model.double())
        # the aggregated cost itself (before the soft-argmin flattens it), sampled on a fixed
        # stride so the fixture stays small, plus whole-tensor sums
        a0 = agg0.numpy().ravel()
        idx = np.arange(0, a0.size, 61, dtype=np.int64)
        sd_sum = np.float64(sum(float(v.double().abs().sum()) for v in model.state_dict().values()))
        feat_sum = np.float64(sum(float(t.double().abs().sum()) for t in left + right))
        save(tag, max_disp=max_disp, shape=np.array([B, C, H, W]), seed=seed,
             names=np.array([n for n, _ in names]), checksum=sd_sum, feat_checksum=feat_sum,
             agg0_shape=np.array(agg0.shape), agg0_idx=idx, agg0_sample=a0[idx],
             agg0_sum=np.float64(a0.astype(np.float64).sum()),
             agg0_abs_sum=np.float64(np.abs(a0.astype(np.float64)).sum()),
             **{f"disp{i}": d for i, d in enumerate(disp)},
             **({"channels": np.array(channels)} if channels is not None else {}),
             **{f"disp64_{i}": d for i, d in enumerate(disp64)})
        d, d64 = disp[0].double().numpy(), disp64[0].numpy()
        print(f"  {tag}: disp {tuple(disp[0].shape)} mean {d.mean():.3f} std {d.std():.3f}; "
              f"reference fp32 vs fp64: max {np.abs(d - d64).max():.3g} mean {np.abs(d - d64).mean():.3g}")


if __name__ == "__main__":
    main()
