"""A/B timing of the scale-0 deformable bottleneck tail (DCN + conv3 + CSA, C2 shape, B=8): the
LDS-window kernel (dcn_tile.hip) vs the generic engine, over offset statistics.  Offsets =
per-channel bias N(0, s^2) + spatial noise N(0, 0.2^2) (bench.py's model: offset_conv bias std
0.5 -> s = 0.5).  Usage: python tools/dcn_tile_bench.py [iters] [s,s,...]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import ops  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
scales = [float(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0.0, 0.5, 1.0, 2.0]
dev = "cuda"
B, C, H, W = 8, 64, 128, 416
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B, C, H, W, device=dev, generator=g).relu_().contiguous(memory_format=torch.channels_last)
res = torch.randn(B, C, H, W, device=dev, generator=g)
w1 = torch.randn(C, C, 1, 1, device=dev, generator=g) * 0.1
w3 = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.04
b = torch.randn(C, device=dev, generator=g)
p1, p3 = ops.pack_weight_split(w1), ops.pack_weight_split(w3)
ups = [torch.randn(B, C, H // r, W // r, device=dev, generator=g) for r in (2, 4)]
noise = torch.randn(B, 54, H, W, device=dev, generator=g) * 0.2
bias = torch.randn(54, device=dev, generator=g)


def timeit(fn):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


for sc in scales:
    om = noise + (bias * sc).view(1, 54, 1, 1)
    om[:, 36:] = noise[:, 36:] * 5  # mask logits
    fw = lambda: ops.mdcn_pw(x, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2, 2,  # noqa: E731
                             csa_up=ups)
    fg = lambda: ops.mdcn_pw(x, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2, 2,  # noqa: E731
                             csa_up=ups, generic_dcn=True)
    out_w, out_g = fw()[1], fg()[1]
    err = (out_w - out_g).abs().max().item()
    offs = om[:, :36]
    outside = ((offs < -2) | (offs >= 2)).float().mean().item()
    print(f"offset bias std {sc:4.1f}: window {timeit(fw):7.1f} us  generic {timeit(fg):7.1f} us  "
          f"(|window - generic| {err:.1e}; offsets outside [-2,2): {100 * outside:.1f} %)", flush=True)
