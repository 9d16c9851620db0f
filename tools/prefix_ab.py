"""Same-process A/B of the prefix_stream option (AdaptiveAggregation): HIP-graph replay and eager
step time of the bench model, alternating rounds, best of each."""
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


graphs = {}
for opt in (False, True):
    model.set_options(prefix_stream=opt)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        step()
    torch.cuda.synchronize()
    graphs[opt] = g
best = {(o, k): float("inf") for o in (False, True) for k in ("graph", "eager")}
for _ in range(5):
    for opt in (False, True):
        best[(opt, "graph")] = min(best[(opt, "graph")], timeit(graphs[opt].replay))
        model.set_options(prefix_stream=opt)
        best[(opt, "eager")] = min(best[(opt, "eager")], timeit(step))
for opt in (False, True):
    print(f"prefix_stream={opt}: graph {best[(opt, 'graph')]:.4f} ms  eager {best[(opt, 'eager')]:.4f} ms")
