"""Batch pipelining with one HIP graph per chunk (round 6 probe).  ROCm's graph executor ran the
chunks of ONE captured graph one after the other even when captured round robin on separate
streams (profiles/r06_chains_timeline.txt).  Here chunk c of the C2 batch is captured into its
own graph and the k graphs are replayed on k streams each step: does the GPU then overlap one
chunk's small serial kernels with another chunk's large ones?  Prints ms per 8-pair step for
k = 1, 2, 4 and checks the outputs against the one-graph step bit for bit.

    python tools/multigraph_probe.py"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    model = bench.build_model(dev)
    B = 8
    left, right = bench.make_features(B, 0, dev, "randn")
    with torch.no_grad():
        ref = model(left, right)[0].clone()
    res = {}
    for k in (1, 2, 4):
        bounds = [B * c // k for c in range(k + 1)]
        graphs, outs = [], []
        for c in range(k):
            lc = [t[bounds[c]:bounds[c + 1]].contiguous() for t in left]
            rc = [t[bounds[c]:bounds[c + 1]].contiguous() for t in right]
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s), torch.no_grad():
                for _ in range(2):
                    model(lc, rc)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g), torch.no_grad():
                o = model(lc, rc)[0]
            graphs.append((g, lc, rc))
            outs.append(o)
        streams = [torch.cuda.Stream() for _ in range(k)]
        cur = torch.cuda.current_stream()

        def step():
            for (g, _, _), st in zip(graphs, streams):
                st.wait_stream(cur)
                with torch.cuda.stream(st):
                    g.replay()
            for st in streams:
                cur.wait_stream(st)

        best = float("inf")
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                step()
            torch.cuda.synchronize()
            best = min(best, (time.perf_counter() - t0) / 10)
        same = torch.equal(torch.cat(outs), ref)
        res[k] = best * 1e3
        print(f"k={k}: {best * 1e3:.3f} ms per 8-pair step, bit-identical to one graph: {same}",
              flush=True)
        del graphs, outs
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
