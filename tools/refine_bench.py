"""Refinement-shape convs (32 ch at full 384x1248 resolution, B=8, 3x3, dilation 1/2/4/8):
NCHW input vs channels-last input, NCHW vs NHWC output (A/B for an NHWC refinement chain)."""
import sys

import torch

sys.path.insert(0, ".")
from aanet_amd import ops  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(8, 32, 384, 1248, device=dev, generator=g)
xn = x.contiguous(memory_format=torch.channels_last)
w = torch.randn(32, 32, 3, 3, device=dev, generator=g) * 0.05
b = torch.randn(32, device=dev, generator=g)
pw = ops.pack_weight_split(w)
flops = 2 * 8 * 384 * 1248 * 32 * 32 * 9


def t(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for d in (1, 2, 4, 8):
    r = {}
    r["nchw->nchw"] = t(lambda: ops.conv2d_fused(x, w, b, 1, d, d, 1, "leaky", packed_weight=pw))
    r["nchw->nhwc"] = t(lambda: ops.conv2d_fused(x, w, b, 1, d, d, 1, "leaky", packed_weight=pw, out_nhwc=True))
    r["nhwc->nchw"] = t(lambda: ops.conv2d_fused(xn, w, b, 1, d, d, 1, "leaky", packed_weight=pw))
    r["nhwc->nhwc"] = t(lambda: ops.conv2d_fused(xn, w, b, 1, d, d, 1, "leaky", packed_weight=pw, out_nhwc=True))
    print(f"dil {d}: " + "  ".join(f"{k} {v:6.1f} us ({flops / v / 1e6:5.1f} TF/s)" for k, v in r.items()), flush=True)
