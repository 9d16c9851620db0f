"""Localise run-to-run differences of the concurrent-scale schedule: for each option set, the
batch-8 step 5 times (eager) against the one-stream result of the same options."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
model = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev, "randn")


def run():
    with torch.no_grad():
        out = model(left, right)[0].clone()
    torch.cuda.synchronize()
    return out


OPTS = [{}, {"s2_sums": False}, {"post_fusion": "none"}, {"dense_grouped": False},
        {"s2_sums": False, "post_fusion": "none", "dense_grouped": False}]
for opts in (OPTS[:1] if os.environ.get("PROBE_DEFAULT_ONLY") else OPTS):
    base = {"s2_sums": True, "post_fusion": "all", "dense_grouped": True}
    base.update(opts)
    model.set_options(concurrent_scales=False, **base)
    ref = run()
    ref2 = run()
    model.set_options(concurrent_scales=True, **base)
    res = [run() for _ in range(5)]
    print(opts, "one-stream repeat equal:", torch.equal(ref, ref2), "concurrent vs one-stream:",
          [torch.equal(r, ref) for r in res], "max diff", max((r - ref).abs().max().item() for r in res),
          flush=True)
