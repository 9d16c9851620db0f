"""Per-level near-tie flip report of the full-model goldens.

For each fixture and both eval paths (fused HIP engine / reference op order on MIOpen) prints,
per disparity level: mean / p99 / max of |ours - fp64| and of the reference's own |fp32 - fp64|,
and the count of "flipped" pixels (|error| > 0.05 px) for each.  Run it once as is and once with
MIOPEN_DEBUG_CONV_WINOGRAD=0 (read by MIOpen at start-up) to see whether MIOpen's fp32 Winograd
convolutions are what moves the reference-order path.

    python tools/flip_report.py [--tf32 0|1] [--cudnn 0|1] [tag ...]

--tf32 sets torch.backends.cudnn.allow_tf32 inside the run (torch's cudnn.flags() context
defaults it to True); --cudnn 0 sends the reference-order convs to PyTorch's native kernels
instead of MIOpen.
"""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from aanet_amd import nets  # noqa: E402
from tests.golden_io import fill_synthetic, fixture_scales, golden, golden_names, synthetic_pair  # noqa: E402

FLIP = 0.05


def stats(e):
    return f"{e.mean():.2e}/{np.percentile(e, 99):.2e}/{e.max():.2e} flips {int((e > FLIP).sum())}"


def main():
    args = sys.argv[1:]
    opts = {"--tf32": 1, "--cudnn": 1}
    while args and args[0] in opts:
        opts[args[0]] = int(args[1])
        args = args[2:]
    tags = args or golden_names("model_")
    env = (f"wino={os.environ.get('MIOPEN_DEBUG_CONV_WINOGRAD', 'default')} "
           f"tf32={opts['--tf32']} cudnn={opts['--cudnn']}")
    for tag in tags:
        g = golden(tag)
        for fuse in (True, False):
            m = nets.AANet(int(g["max_disp"]), 1, **json.loads(str(g["config"])))
            fill_synthetic(m, int(g["seed"]), fixture_scales(g))
            m = m.to("cuda").eval()
            for mod in m.modules():
                mod.aanet_fuse = fuse
            B, H, W = (int(v) for v in g["shape"])
            left, right = synthetic_pair(B, H, W, int(g["seed"]))
            with torch.no_grad(), torch.backends.cudnn.flags(enabled=bool(opts["--cudnn"]),
                                                             benchmark=False, deterministic=True,
                                                             allow_tf32=bool(opts["--tf32"])):
                pyr = m(left.cuda(), right.cuda())
            for i, d in enumerate(pyr):
                ours = d.cpu().numpy().astype(np.float64)
                r32, r64 = g[f"disp{i}"].astype(np.float64), g[f"disp64_{i}"]
                print(f"{tag} {env} {'fused' if fuse else 'ref-order'} L{i} "
                      f"ours-vs-64 {stats(np.abs(ours - r64))} | ref32-vs-64 {stats(np.abs(r32 - r64))}"
                      f" | ours-vs-32 {stats(np.abs(ours - r32))} | n {ours.size}", flush=True)


if __name__ == "__main__":
    main()
