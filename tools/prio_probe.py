"""Does a high-priority stream for the scale-0 chain help the concurrent-scale schedule?  Times the
bench step (eager and HIP-graph replay) issued from the default stream vs from a priority -1
stream (the side streams of the coarse scales stay at the default priority).
Usage: python tools/prio_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
model = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev, "randn")
print("priority range", torch.cuda.Stream.priority_range())


def step():
    with torch.no_grad():
        return model(left, right)[0]


def timeit(fn, n=20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


res = {}
for name, prio in (("default", None), ("high", -1)):
    s = torch.cuda.current_stream() if prio is None else torch.cuda.Stream(priority=prio)
    with torch.cuda.stream(s):
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            step()
        torch.cuda.synchronize()
        te = min(timeit(step) for _ in range(3))
        tg = min(timeit(g.replay) for _ in range(3))
    res[name] = (te, tg)
    print(f"{name:8s} eager {te:.4f} ms  graph {tg:.4f} ms", flush=True)
