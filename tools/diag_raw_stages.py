"""Stage dump of model_psmnet_aa_raw on the GPU (VERDICT r5 "next" item 1: why the reference-order
path flips 784 / 5647 pixels at levels 1 / 2 against the reference's own 29 / 697).

For the fused and the reference-order eval paths it saves, to gpurun_out/raw_stages.npz:
  * the output of every module down to depth 4 whose forward runs (forward hooks; the fused path
    bypasses most sub-module forwards, the reference-order path runs them all),
  * the disparity pyramid,
  * the refinement run ALONE on the reference's own fp64 level-0 disparity (the fixture's
    `disp64_0`): `<tag>_cond1` / `<tag>_cond2`, which isolates the refinement's own error from
    the level-0 flips it inherits.
tools/diag_raw_compare.py (build container, imports the reference) prints the stage table.

    python tools/diag_raw_stages.py
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from aanet_amd import nets  # noqa: E402
from tests.golden_io import fill_synthetic, fixture_scales, golden, synthetic_pair  # noqa: E402

TAG = sys.argv[1] if len(sys.argv) > 1 else "model_psmnet_aa_raw"


def _flat(o, out, key):
    if isinstance(o, torch.Tensor):
        out[key] = o.detach().float().cpu().numpy()
    elif isinstance(o, (list, tuple)):
        for i, t in enumerate(o):
            _flat(t, out, f"{key}#{i}")


# the fusions where the reference-order path's error first leaves 2x the reference's own
# (profiles/r06_raw_stages.txt): every sub-module, and the inputs of the DCN ops
DEEP = ("aggregation.fusions.3.", "aggregation.fusions.4.")
# AANET_DIAG_FEATURES=1: the feature extractor's stages instead (firstconv, layer1..4, branches,
# lastconv), to find where the first 2x of the reference's own error enters
FEATURES = os.environ.get("AANET_DIAG_FEATURES") == "1"


def keep(name):
    """The stages worth a table row (and a dump that fits gpurun_out): the top-level stages, the
    aggregation's fusion modules and their branches / fuse layers, the refinement modules."""
    if FEATURES:
        return name.startswith("feature_extractor") and name.count(".") <= 1
    if name.startswith(DEEP):
        return True
    if not name or name.count(".") > 3:
        return False
    top = name.split(".")[0]
    if top in ("feature_extractor", "fpn", "cost_volume", "disparity_estimation"):
        return "." not in name
    if top == "refinement":
        return name.count(".") <= 1
    return top == "aggregation"


def run(fuse):
    g = golden(TAG)
    m = nets.AANet(int(g["max_disp"]), 1, **json.loads(str(g["config"])))
    fill_synthetic(m, int(g["seed"]), fixture_scales(g))
    m = m.to("cuda").eval()
    for mod in m.modules():
        mod.aanet_fuse = fuse
    tag = "fused" if fuse else "ref"
    res, seen = {}, {}
    hooks = []
    for name, mod in m.named_modules():
        if not keep(name):
            continue

        def hook(mod, i, o, name=name):
            k = seen.get(name, 0)  # the feature extractor runs twice (left, right)
            seen[name] = k + 1
            _flat(o, res, f"{tag}|{name}|{k}")
            if name.endswith("deform_conv"):
                _flat(i, res, f"{tag}|{name}.in|{k}")
        hooks.append(mod.register_forward_hook(hook))
    B, H, W = (int(v) for v in g["shape"])
    left, right = synthetic_pair(B, H, W, int(g["seed"]))
    left, right = left.cuda(), right.cuda()
    with torch.no_grad(), torch.backends.cudnn.flags(enabled=False, allow_tf32=False):
        pyr = m(left, right)
        for h in hooks:
            h.remove()
        for i, d in enumerate(pyr):
            res[f"{tag}_disp{i}"] = d.cpu().numpy()
        # the refinement alone, fed the reference's fp64 level-0 disparity
        d0 = torch.from_numpy(g["disp64_0"].astype(np.float32)).cuda()
        for i, d in enumerate(m.disparity_refinement(left, right, d0)):
            res[f"{tag}_cond{i + 1}"] = d.cpu().numpy()
    return res


def main():
    out = {}
    for fuse in (True, False):
        out.update(run(fuse))
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    path = os.path.join(REPO, "gpurun_out", "raw_stages.npz")
    np.savez_compressed(path, **out)
    print("wrote", path, len(out), "arrays", sum(v.nbytes for v in out.values()) >> 20, "MiB")


if __name__ == "__main__":
    main()
