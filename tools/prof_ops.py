"""torch.profiler op table of one eager bench step (which aten ops launch what): usage
python tools/prof_ops.py [--train].  Prints the top ops by device time and the ops whose
children are device memcpys."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda")
train = "--train" in sys.argv
if train:
    from aanet_amd import train as atrain
    model = bench.build_model(dev, intermediate_supervision=True).train()
    left, right = bench.make_features(4, 0, dev, "randn", bench.TRAIN_IMG)
    tr = atrain.Trainer(model, lr=1e-3)
    gt = torch.rand((4,) + bench.TRAIN_IMG, device=dev) * 100

    def step():
        tr.step(left, right, gt)
else:
    model = bench.build_model(dev)
    left, right = bench.make_features(8, 0, dev)

    def step():
        with torch.no_grad():
            model(left, right)

for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages().table(sort_by="device_time_total", row_limit=40, max_name_column_width=60))
evs = prof.events()
memcpy_parents = {}
for e in evs:
    for k in e.kernels if hasattr(e, "kernels") else []:
        if "copy" in k.name.lower() or "memcpy" in k.name.lower():
            memcpy_parents[e.name] = memcpy_parents.get(e.name, 0) + 1
print("ops launching copies:", sorted(memcpy_parents.items(), key=lambda kv: -kv[1])[:20])
