"""C5 concat / difference volume alone (features [4, 32, 96, 312], D = 48): HIP-event
time per launch and the fraction of 8 TB/s on the algorithmic bytes (two feature reads + the
volume write).  Usage: python tools/shift_bench.py [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import _lib  # noqa: E402
from aanet_amd._lib import call, ptr, stream_of  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
B, C, H, W, D = 4, 32, 96, 312, 48
g = torch.Generator(device="cuda").manual_seed(0)
L = torch.randn(B, C, H, W, device="cuda", generator=g)
R = torch.randn(B, C, H, W, device="cuda", generator=g)
for name, oc in (("aanet_concat_volume_f32", 2 * C), ("aanet_diff_volume_f32", C)):
    out = torch.empty(B, oc, D, H, W, device="cuda")
    fn = lambda: call(name, ptr(L), ptr(R), ptr(out), B, C, H, W, D, stream_of(L))  # noqa: E731
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / iters
    byts = 2.0 * B * C * H * W * 4 + out.numel() * 4.0
    print(f"{os.path.basename(_lib.LIB_PATH)} {name}: {us:7.1f} us  {byts / us / 1e6:6.2f} TB/s  "
          f"{byts / us / 1e6 / 8.0:.3f} of 8 TB/s", flush=True)
