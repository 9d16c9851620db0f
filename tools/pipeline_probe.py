"""Probe: the bench step as two concurrent half-batch pipelines (each on its own stream and its
own side streams) vs one batch-8 pipeline.  Per-pair results must be identical (every kernel
works per image).  Usage: python tools/pipeline_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from aanet_amd.nets import aggregation as agg  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
model = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev, "randn")
main = torch.cuda.current_stream()
sl = lambda feats, k: [f[4 * k:4 * k + 4].contiguous() for f in feats] if isinstance(feats, (list, tuple)) else feats[4 * k:4 * k + 4].contiguous()  # noqa: E731
halves = [(sl(left, k), sl(right, k)) for k in range(2)]


def one():
    with torch.no_grad():
        return model(left, right)[0]


def make_split(nside):
    pipes = []
    for k in range(2):
        s = torch.cuda.Stream()
        side = [torch.cuda.Stream() for _ in range(nside)]
        side = (side * 2)[:2]
        pipes.append((s, side))

    def split():
        outs = []
        cur = torch.cuda.current_stream()
        for k, (s, side) in enumerate(pipes):
            s.wait_stream(cur)
            agg._SIDE_STREAMS[dev] = list(side)
            with torch.cuda.stream(s), torch.no_grad():
                outs.append(model(halves[k][0], halves[k][1])[0])
        for s, _ in pipes:
            cur.wait_stream(s)
        return torch.cat(outs)
    return split


def timeit(fn, n=20):
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e3


def graph_of(fn):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        out = fn()
    torch.cuda.synchronize()
    return g, out


ref = one().clone()
saved = list(agg._SIDE_STREAMS.get(dev, []))
for nside in (2, 1):
    sp = make_split(nside)
    got = sp()
    torch.cuda.synchronize()
    print(f"split (side streams per pipeline {nside}): identical to the batch-8 result: {torch.equal(got, ref)}")
    te = min(timeit(sp) for _ in range(3))
    print(f"  eager {te:.4f} ms", flush=True)
    if os.environ.get("PROBE_GRAPH"):
        g, out = graph_of(sp)
        tg = min(timeit(g.replay) for _ in range(3))
        g.replay()
        torch.cuda.synchronize()
        print(f"  graph {tg:.4f} ms  graph identical: {torch.equal(out, ref)}", flush=True)
agg._SIDE_STREAMS[dev] = saved
te = min(timeit(one) for _ in range(3))
g, out = graph_of(one)
tg = min(timeit(g.replay) for _ in range(3))
print(f"batch-8 one pipeline: eager {te:.4f} ms  graph {tg:.4f} ms", flush=True)
