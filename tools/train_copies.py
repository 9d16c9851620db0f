"""Which Python call sites launch the training step's copies and fills?  Builds the bench.py
--train step (eager), profiles one step with torch.profiler (shapes + stacks) and prints the
aten::copy_ / fill_ / zero_ / add_ calls grouped by their innermost aanet_amd (or torch.nn) frame
and input shapes.  Usage: python tools/train_copies.py"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from aanet_amd import train as atrain  # noqa: E402

dev = torch.device("cuda:0")
model = bench.build_model(dev, intermediate_supervision=True).train()
trainer = atrain.Trainer(model, lr=1e-3)
left, right = bench.make_features(4, 0, dev, "randn", bench.TRAIN_IMG)
gt = torch.rand((4,) + bench.TRAIN_IMG, device=dev) * (bench.MAXD_IMG - 1)
mask = (gt > 0) & (gt < bench.MAXD_IMG)
for _ in range(3):
    trainer.step(left, right, gt, mask)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402
with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    trainer.step(left, right, gt, mask)
    torch.cuda.synchronize()
WANT = ("aten::copy_", "aten::fill_", "aten::zero_", "aten::add_", "aten::add")
groups = collections.Counter()
for ev in prof.events():
    if ev.name not in WANT:
        continue
    stack = [s for s in (ev.stack or []) if "aanet_amd" in s or "torch/nn" in s or "torch/autograd" in s]
    site = stack[0] if stack else (ev.stack[0] if ev.stack else "?")
    groups[(ev.name, site[-90:], str(ev.input_shapes)[:80])] += 1
for (name, site, shapes), n in groups.most_common(40):
    print(f"{n:4d} {name:13s} {site} {shapes}")
