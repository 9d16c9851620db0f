"""Memory-bound passes of the hourglass Conv2x blocks at the AANet+ sizes, B=8: the deconv
assembly in NCHW and channels-last form (aanet_deconv2x_assemble[_nhwc]_f32), the channels-last
concat (aanet_concat_nhwc_f32), torch.cat, and a device copy of the same output bytes as the
bandwidth reference.  Median of 20 HIP-event timings after warm-up."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import _lib, ops  # noqa: E402
from aanet_amd._lib import call, ptr, stream_of  # noqa: E402

dev = "cuda"
B = 8


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(n):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e))
    ts.sort()
    return ts[len(ts) // 2] * 1e3


for co, h, w in [(32, 192, 624), (48, 96, 312), (64, 48, 156), (32, 96, 312)]:
    ph = torch.randn(B, 4 * co, h + 1, w + 1, device=dev)
    rem = torch.randn(B, co, 2 * h, 2 * w, device=dev)
    o1 = torch.empty(B, 2 * co, 2 * h, 2 * w, device=dev)
    o2 = torch.empty_like(o1, memory_format=torch.channels_last)
    f1 = lambda: call("aanet_deconv2x_assemble_f32", ptr(ph), ptr(rem), ptr(o1), B, co, co, h, w, stream_of(ph))  # noqa
    f2 = lambda: call("aanet_deconv2x_assemble_nhwc_f32", ptr(ph), ptr(rem), ptr(o2), B, co, co, h, w, stream_of(ph))  # noqa
    a = torch.randn(B, co, 2 * h, 2 * w, device=dev)
    f3 = lambda: ops.concat_nhwc(a, rem)  # noqa
    f4 = lambda: torch.cat((a, rem), 1)  # noqa
    f5 = lambda: o1.copy_(o2)  # noqa: channels-last -> NCHW copy of the output bytes
    gb = o1.numel() * 4 * 2 / 1e9  # output written once + ~the same read
    t = [timeit(f) for f in (f1, f2, f3, f4, f5)]
    print(f"co {co:3d} out {2*h}x{2*w}: assemble nchw {t[0]:7.1f}  nhwc {t[1]:7.1f}  concat_nhwc {t[2]:7.1f}  "
          f"torch.cat {t[3]:7.1f}  copy {t[4]:7.1f} us  ({gb / t[0] * 1e3:.1f} / {gb / t[1] * 1e3:.1f} TB/s)")
