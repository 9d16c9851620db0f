"""Is the concurrent-scale schedule's result independent of how the side streams are assigned?
Batch-8 step: one stream (concurrent_scales=False) vs the default two side streams vs both coarse
scales on ONE side stream, eager, several runs each; prints which runs differ and where."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from aanet_amd.nets import aggregation as agg  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
model = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev, "randn")


def run():
    with torch.no_grad():
        out = model(left, right)[0].clone()
    torch.cuda.synchronize()
    return out


model.set_options(concurrent_scales=False)
ref = run()
model.set_options(concurrent_scales=True)
default = [run() for _ in range(3)]
print("default side streams vs one stream:", [torch.equal(d, ref) for d in default])
s = torch.cuda.Stream()
saved = list(agg._SIDE_STREAMS.get(dev, []))
agg._SIDE_STREAMS[dev] = [s, s]
shared = [run() for _ in range(3)]
print("one shared side stream vs one stream:", [torch.equal(d, ref) for d in shared])
for d in shared:
    if not torch.equal(d, ref):
        diff = (d - ref).abs()
        print("  max |diff|", diff.max().item(), "pixels differing", int((diff > 0).sum()), "of", diff.numel())
        break
agg._SIDE_STREAMS[dev] = saved
