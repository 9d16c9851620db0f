"""Compare the GPU stage dump of tools/diag_psmnet_stages.py (gpurun_out/psm_stages.npz) with the
REFERENCE's own PSMNet-AA stages in fp32 and fp64 (build container only: imports
/root/reference by path, as tests/golden/make_model_golden.py does), on the round-3
(unconditioned) fill.  Prints, per stage, the normwise and max error against fp64 of the
reference's fp32 run and of our fused / reference-order runs, then the level-0 pixels where any
run is > 0.05 px off fp64, with the fp64 top-2 logit gap there.

    python tools/diag_psmnet_compare.py [gpurun_out/psm_stages.npz]
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

from make_golden import load_reference  # noqa: E402
from tests.golden_io import fill_synthetic, golden, synthetic_pair  # noqa: E402


def reference_stages():
    load_reference()
    aanet = importlib.import_module("nets.aanet")
    g = golden("model_psmnet_aa")
    m = aanet.AANet(int(g["max_disp"]), 1, **json.loads(str(g["config"])))
    fill_synthetic(m, int(g["seed"]))
    m.eval()
    B, H, W = (int(v) for v in g["shape"])
    left, right = synthetic_pair(B, H, W, int(g["seed"]))
    res = {}
    for tag, dt in (("r32", torch.float32), ("r64", torch.float64)):
        cap = {}
        hs = [m.fpn.register_forward_hook(lambda mod, i, o: cap.setdefault("feat", []).append(o)),
              # (cloned: the aggregation replaces the list's entries in place, aggregation.py:382)
              m.cost_volume.register_forward_hook(lambda mod, i, o: cap.__setitem__("cost", [t.clone() for t in o])),
              m.aggregation.register_forward_hook(lambda mod, i, o: cap.__setitem__("agg", o[0]))]
        m.to(dt)
        with torch.no_grad():
            pyr = m(left.to(dt), right.to(dt))
        for h in hs:
            h.remove()
        res[f"{tag}_agg"] = cap["agg"].numpy()
        res[f"{tag}_disp0"] = pyr[0].numpy()
        for s in range(3):
            res[f"{tag}_featL{s}"] = cap["feat"][0][s].numpy()
            res[f"{tag}_featR{s}"] = cap["feat"][1][s].numpy()
            res[f"{tag}_cost{s}"] = cap["cost"][s].numpy()
    return res


def main():
    ours = dict(np.load(sys.argv[1] if len(sys.argv) > 1 else
                        os.path.join(REPO, "gpurun_out", "psm_stages.npz")))
    ref = reference_stages()
    stages = ["featL0", "featL1", "featL2", "cost0", "cost1", "cost2", "agg", "disp0"]
    print(f"{'stage':8s} " + " | ".join(f"{t:>22s}" for t in ("ref fp32", "ours fused", "ours ref-order")))
    for st in stages:
        e64 = ref[f"r64_{st}"]
        cols = []
        for src, key in ((ref, f"r32_{st}"), (ours, f"fused_{st}"), (ours, f"ref_{st}")):
            d = src[key].astype(np.float64) - e64
            cols.append(f"{np.linalg.norm(d) / np.linalg.norm(e64):.1e} / {np.abs(d).max():.1e}")
        print(f"{st:8s} " + " | ".join(f"{c:>22s}" for c in cols) + f"   (max|x| {np.abs(e64).max():.2g})")
    d64 = ref["r64_disp0"][0]
    top2 = np.sort(ref["r64_agg"][0], axis=0)[-2:]
    gap = top2[1] - top2[0]
    errs = {k: np.abs(v[0].astype(np.float64) - d64) for k, v in
            (("ref32", ref["r32_disp0"]), ("fused", ours["fused_disp0"]), ("reforder", ours["ref_disp0"]))}
    bad = np.argwhere(np.maximum.reduce(list(errs.values())) > 0.05)
    print("level-0 pixels > 0.05 px off fp64 (y, x): fp64 disp, top-2 logit gap, |err| ref32 / fused / ref-order")
    for y, x in bad:
        print(f"  ({y:2d},{x:2d}) d64 {d64[y, x]:6.3f} gap {gap[y, x]:8.3f}  " +
              " / ".join(f"{errs[k][y, x]:.3f}" for k in ("ref32", "fused", "reforder")))
    for k in ("r32", "fused", "ref"):
        src = ref if k == "r32" else ours
        e = np.abs(src[f"{k}_agg"][0].astype(np.float64) - ref["r64_agg"][0])
        d, y, x = np.unravel_index(np.argmax(e), e.shape)
        col0 = e[:, :, 0].max()
        print(f"  {k:6s} agg: max err {e.max():.1f} at (d {d}, y {y}, x {x}); max over column x=0 "
              f"{col0:.1f}, over x>=2 {e[:, :, 2:].max():.1f}")
    for y, x in bad:
        print(f"  logits at ({y},{x}): fp64 " + " ".join(f"{v:.1f}" for v in ref["r64_agg"][0][:, y, x]))
        print(f"              ref-order " + " ".join(f"{v:.1f}" for v in ours["ref_agg"][0][:, y, x]))
    print(f"fp64 top-2 logit gap: min {gap.min():.3f}, 0.1 % quantile {np.quantile(gap, 1e-3):.3f}, "
          f"median {np.median(gap):.1f}; logit span median "
          f"{np.median(ref['r64_agg'][0].max(0) - ref['r64_agg'][0].min(0)):.0f}")


if __name__ == "__main__":
    main()
