"""Kernel-level determinism under concurrency: the offset conv (conv_g3), the DCN tail (dcn_tile)
and the stride-2 heads (conv_s2) on fixed inputs, each run alone once (reference) and then
N times while another stream runs unrelated work; counts the runs whose output bits differ."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import ops  # noqa: E402

dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
B, C, H, W = 8, 64, 128, 416
N = int(os.environ.get("N", "20"))
x = torch.randn(B, C, H, W, device=dev, generator=g).relu_().contiguous(memory_format=torch.channels_last)
xn = x.contiguous()
w = torch.randn(54, 32, 3, 3, device=dev, generator=g) * 0.05
b = torch.randn(54, device=dev, generator=g)
wsp = ops.pack_conv3x3_grouped(w, 2)
res = torch.randn(B, C, H, W, device=dev, generator=g)
w1 = torch.randn(C, C, 1, 1, device=dev, generator=g) * 0.1
w3 = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.04
bb = torch.randn(C, device=dev, generator=g)
p1, p3 = ops.pack_weight_split(w1), ops.pack_weight_split(w3)
ups = [torch.randn(B, C, H // r, W // r, device=dev, generator=g) for r in (2, 4)]
noise = torch.randn(B, 54, H, W, device=dev, generator=g) * 0.2
om = noise + (torch.randn(54, device=dev, generator=g) * 0.5).view(1, 54, 1, 1)
big = torch.randn(4096, 4096, device=dev, generator=g)
ws2 = ops.pack_conv3x3s2(torch.randn(96, C, 3, 3, device=dev, generator=g) * 0.04)
b2 = torch.randn(96, device=dev, generator=g)
side = torch.cuda.Stream()

cases = {
    "offset_conv (conv_g3)": lambda: ops.conv3x3_grouped_nhwc(x, wsp, b, 54, 2, 2),
    "DCN tail (dcn_tile)": lambda: ops.mdcn_pw(x, om, w3, p3, None, bb, bb, "relu", p1, bb, res, "relu",
                                               1, 2, 2, 2, csa_up=ups)[1],
    "stride-2 heads (conv_s2)": lambda: torch.cat([t.flatten() for t in ops.conv3x3_s2(xn, ws2, b2, 96, 32, "leaky", "leaky")]),
}


def noise_work():
    with torch.cuda.stream(side):
        for _ in range(3):
            torch.mm(big, big)
        ops.conv3x3_grouped_nhwc(x, wsp, b, 54, 2, 2)


for name, fn in cases.items():
    ref = fn().clone()
    torch.cuda.synchronize()
    alone = sum(not torch.equal(fn(), ref) for _ in range(5))
    torch.cuda.synchronize()
    bad, maxd = 0, 0.0
    for _ in range(N):
        side.wait_stream(torch.cuda.current_stream())
        noise_work()
        out = fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        if not torch.equal(out, ref):
            bad += 1
            maxd = max(maxd, (out - ref).abs().max().item())
    print(f"{name}: alone differing {alone}/5, beside other work differing {bad}/{N} (max |diff| {maxd:.3g})", flush=True)
