"""Stage dump of PSMNet-AA on the GPU for the round-3 parity failure.

Runs the model_psmnet_aa configuration with the round-3 (UNconditioned) name-keyed fill, on the
fused and the reference-order eval paths, and saves per stage -- left/right features per scale,
the cost-volume pyramid, the aggregation output (soft-argmin logits) and the level-0 disparity --
to gpurun_out/psm_stages.npz.  tools/diag_psmnet_compare.py (build container) compares them with
the reference's own fp32 and fp64 stages to show where the error enters.

    python tools/diag_psmnet_stages.py
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from aanet_amd import nets  # noqa: E402
from tests.golden_io import fill_synthetic, golden, synthetic_pair  # noqa: E402


def run(fuse):
    g = golden("model_psmnet_aa")
    m = nets.AANet(int(g["max_disp"]), 1, **json.loads(str(g["config"])))
    fill_synthetic(m, int(g["seed"]))  # round-3 fill: no conditioning scales
    m = m.to("cuda").eval()
    for mod in m.modules():
        mod.aanet_fuse = fuse
    cap = {}
    fe, run_agg = m.feature_extraction, m.aggregation._run

    def feat(img):
        out = fe(img)
        cap.setdefault("feat", []).append([t.detach().cpu().numpy() for t in out])
        return out

    def agg(cv, regress=False):
        cap["cost"] = [t.detach().cpu().numpy() for t in cv]
        out, disp = run_agg(cv, regress=False)
        cap["agg"] = out[0].detach().cpu().numpy()
        return out, None

    m.feature_extraction, m.aggregation._run = feat, agg
    B, H, W = (int(v) for v in g["shape"])
    left, right = synthetic_pair(B, H, W, int(g["seed"]))
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False, allow_tf32=False):
        pyr = m(left.cuda(), right.cuda())
    tag = "fused" if fuse else "ref"
    res = {f"{tag}_agg": cap["agg"], f"{tag}_disp0": pyr[0].cpu().numpy()}
    for s in range(3):
        res[f"{tag}_featL{s}"] = cap["feat"][0][s]
        res[f"{tag}_featR{s}"] = cap["feat"][1][s]
        res[f"{tag}_cost{s}"] = cap["cost"][s]
    return res


def main():
    out = {}
    for fuse in (True, False):
        out.update(run(fuse))
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    path = os.path.join(REPO, "gpurun_out", "psm_stages.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
