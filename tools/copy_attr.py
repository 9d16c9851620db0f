"""Attribute the device copies (`__amd_rocclr_copyBuffer` in rocprof) of the C2 inference step:
runs eager bench steps under torch.profiler and prints, per Python call site, how many
hipMemcpy*/aten copy calls one step makes.  python tools/copy_attr.py"""
import collections
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
model = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev)


def step():
    with torch.no_grad():
        return model(left, right)[0]


for _ in range(3):
    step()
torch.cuda.synchronize()
STEPS = 2
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True,
             record_shapes=True) as prof:
    for _ in range(STEPS):
        step()
    torch.cuda.synchronize()

sites = collections.Counter()
names = collections.Counter()
for ev in prof.events():
    n = ev.name
    if not any(k in n.lower() for k in ("memcpy", "copy_", "memset", "copybuffer", "fillbuffer")):
        continue
    names[n] += 1
    st = [f for f in (ev.stack or []) if "aanet_amd" in f or "bench" in f]
    sites[(n, st[0] if st else "?", tuple(ev.input_shapes[:2]) if ev.input_shapes else ())] += 1
print("per step:")
for n, c in names.most_common():
    print(f"  {c / STEPS:6.1f}  {n}")
print("call sites (per step):")
for (n, s, shp), c in sites.most_common(60):
    print(f"  {c / STEPS:6.1f}  {n:28s} {s}  {shp}")
