"""How much of model_psmnet_aa_raw's near-tie flip count is a rounding lottery (build container
only: runs the REFERENCE's own nets/aanet.py on CPU, as tests/golden/make_model_golden.py does).

The reference's fp32 forward is re-run with its inputs perturbed by one rounding unit --
every pixel of both images multiplied by (1 + u * 2^-24), u uniform in {-1, 0, 1}, i.e. a
rounding error of the size fp32 itself makes when it stores the images -- for several seeds, and
with 1 / 4 / 8 intra-op threads (the CPU conv's blocking and summation order).  Each run's
pyramid is compared with the fixture's fp64 output: the spread of the per-level flip counts
(|d - d64| > 0.05 px) is the reference's OWN run-to-run variation under perturbations no larger
than its own rounding.

    python tools/diag_raw_lottery.py [n_seeds] > profiles/r06_raw_lottery.txt
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
from tests.golden_io import fill_synthetic, fixture_scales, golden, synthetic_pair  # noqa: E402

TAG = "model_psmnet_aa_raw"
FLIP = 0.05


def main():
    n_seeds = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    load_reference()
    aanet = importlib.import_module("nets.aanet")
    g = golden(TAG)
    m = aanet.AANet(int(g["max_disp"]), 1, **json.loads(str(g["config"])))
    fill_synthetic(m, int(g["seed"]), fixture_scales(g))
    m.eval()
    B, H, W = (int(v) for v in g["shape"])
    left, right = synthetic_pair(B, H, W, int(g["seed"]))
    d64 = [g[f"disp64_{i}"] for i in range(3)]

    def flips(pyr):
        """per-level flip counts, then the level-0 max |d - d64| (px)"""
        e = [np.abs(d.numpy().astype(np.float64) - r) for d, r in zip(pyr, d64)]
        return [int((x > FLIP).sum()) for x in e] + [round(float(e[0].max()), 3)]

    print(f"# {TAG}: the reference's own fp32 run, flips per level (|d - d64| > {FLIP} px) against "
          "the fixture's fp64 output")
    rows = []
    with torch.no_grad():
        for threads in (8, 4, 1):
            torch.set_num_threads(threads)
            f = flips(m(left, right))
            rows.append(f)
            print(f"unperturbed, {threads} threads: L0/L1/L2 flips, L0 max px {f}")
        torch.set_num_threads(8)
        for s in range(n_seeds):
            gen = torch.Generator().manual_seed(s)
            u = [torch.randint(-1, 2, t.shape, generator=gen).float() for t in (left, right)]
            lp, rp = (t * (1 + uu * 2.0 ** -24) for t, uu in zip((left, right), u))
            f = flips(m(lp, rp))
            rows.append(f)
            print(f"images x (1 + u 2^-24), seed {s:2d}: L0/L1/L2 flips, L0 max px {f}", flush=True)
    a = np.array(rows)
    if len(sys.argv) > 2:  # save the distribution (tests/golden fixture builder)
        np.save(sys.argv[2], a)
    print(f"over {len(rows)} runs: min {a.min(0).tolist()}, median {np.median(a, 0).tolist()}, "
          f"max {a.max(0).tolist()}")


if __name__ == "__main__":
    main()
