"""A/B of the hourglass transposed convs (Conv2x(deconv=True) conv1 + BN + ReLU + concat) at the
AANet+ sizes, B=8: MIOpen (torch conv_transpose2d, fp32-pinned) + BN + ReLU + torch.cat vs the
HIP phase form (ops.deconv2x: engine 2x2 phase conv + assembly).  Median of 20 after warm-up."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import ops  # noqa: E402
from aanet_amd._precision import fp32_scope  # noqa: E402

dev = "cuda"
B = 8
# (ci, co, h, w) at the refinement's full resolution (384 x 1248 input) and half resolution
SHAPES = [(128, 96, 24, 78), (96, 64, 48, 156), (64, 48, 96, 312), (48, 32, 192, 624),
          (128, 96, 12, 39), (96, 64, 24, 78), (64, 48, 48, 156), (48, 32, 96, 312)]


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


tot_m = tot_h = 0.0
for ci, co, h, w in SHAPES:
    x = torch.randn(B, ci, h, w, device=dev)
    rem = torch.randn(B, co, 2 * h, 2 * w, device=dev)
    wt = torch.randn(ci, co, 4, 4, device=dev) / (ci * 4) ** 0.5
    sc, sh = torch.rand(co, device=dev) + 0.5, torch.randn(co, device=dev)
    wd = ops.deconv2x_phase_weight(wt, sc)
    wp = ops.pack_weight_split(wd)
    wp = ops.pack_weight(wd) if wp is None else wp
    b4 = sh.repeat_interleave(4)

    def miopen():
        with fp32_scope():
            y = F.conv_transpose2d(x, wt, stride=2, padding=1)
        y = F.relu(y * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1))
        return torch.cat((y, rem), 1)

    def hip():
        return ops.deconv2x(x, wd, b4, "relu", packed_weight=wp, rem=rem)

    err = (miopen() - hip()).abs().max().item()
    tm, th = timeit(miopen), timeit(hip)
    tot_m += tm
    tot_h += th
    gf = 2.0 * B * h * w * ci * co * 16 / 1e9
    print(f"ci {ci:3d} co {co:3d} in {h:3d}x{w:3d}: miopen {tm:8.1f} us  hip {th:8.1f} us  "
          f"({gf / th * 1e3:6.1f} TF/s)  max|diff| {err:.2e}", flush=True)
print(f"total: miopen {tot_m:.1f} us  hip {tot_h:.1f} us")
