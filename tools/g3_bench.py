"""Microbenchmark of the deformable offset_conv at the C2 scale-0 shape (B=8, 64 -> 54, two groups,
dilation 2, channels-last input): the grouped direct kernel (conv_g3.hip) against the conv
engine's halo form.  python tools/g3_bench.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import ops  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(8, 64, 128, 416, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    w = torch.randn(54, 32, 3, 3, device=dev, generator=g) * 0.05
    b = torch.randn(54, device=dev, generator=g)
    ws = ops.pack_conv3x3_grouped(w, 2)
    pw = ops.pack_weight_split(w, 2)  # the engine's split-bf16 halo form, as in the step
    res = {"direct_g3": timed(lambda: ops.conv3x3_grouped_nhwc(x, ws, b, 54, 2, 2)),
           "engine_halo": timed(lambda: ops.conv2d_fused(x, w, b, 1, 2, 2, 2, None, packed_weight=pw))}
    flops = 2.0 * 8 * 128 * 416 * 54 * 32 * 9
    res["split_ceiling_us"] = flops * 6 / 2.5e15 * 1e6
    print(json.dumps({k: round(v, 2) for k, v in res.items()}))


if __name__ == "__main__":
    main()
