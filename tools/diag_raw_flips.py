"""Per-level near-tie flip counts of one full-model fixture (default model_psmnet_aa_raw), fused
and reference-order, against the reference's fp32 and fp64 outputs (the quantities of
tests/test_gpu_models.py).  GPU diagnosis: run under different AANET_* settings and compare.
Usage: python tools/diag_raw_flips.py [tag]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import _lib  # noqa: E402
from tests.test_gpu_models import FLIP, build  # noqa: E402

tag = sys.argv[1] if len(sys.argv) > 1 else "model_psmnet_aa_raw"
for fuse in (True, False):
    g, m, left, right = build(tag, fuse)
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False, allow_tf32=False):
        pyr = m(left, right)
    row = []
    for i, d in enumerate(pyr):
        ours = d.cpu().numpy().astype(np.float64)
        e64 = np.abs(ours - g[f"disp64_{i}"])
        eref = np.abs(g[f"disp{i}"].astype(np.float64) - g[f"disp64_{i}"])
        e32 = np.abs(ours - g[f"disp{i}"])
        row.append(f"L{i} flips {int((e64 > FLIP).sum())} (ref {int((eref > FLIP).sum())}) "
                   f"max|d-d32| {e32.max():.2e} mean {e32.mean():.2e}")
    print(tag, "fused" if fuse else "ref-order", "exact" if _lib.exact_f32_enabled() else "split", " | ".join(row),
          flush=True)
