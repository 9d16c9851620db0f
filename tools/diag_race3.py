"""Race localisation: the NHWC split DCN tail kernel with an identity pointwise tail (output =
relu(DCN)), so a corrupted im2col row shows as whole pixels and a corrupted tail operand as
4-channel groups."""
import os
import sys
from collections import Counter

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import ops  # noqa: E402

dev = "cuda"
B, C, H, W = 8, 64, 128, 416
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B, C, H, W, device=dev, generator=g)
xn = x.contiguous(memory_format=torch.channels_last)
w3 = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.04
wo = torch.randn(54, 32, 3, 3, device=dev, generator=g) * 0.01
bo = torch.randn(54, device=dev, generator=g)
b = torch.randn(C, device=dev, generator=g)
p3, po = ops.pack_weight_split(w3), ops.pack_weight_split(wo, 2)
om = ops.conv2d_fused(x, wo, bo, 1, 2, 2, 2, packed_weight=po)
eye = torch.eye(C, device=dev).view(C, C, 1, 1)
pe = ops.pack_weight_split(eye)
zero = torch.zeros(C, device=dev)
for name, om_ in (("fractional", om), ("integer", om.round()), ("zero", torch.zeros_like(om))):
    fn = lambda: ops.mdcn_pw(xn, om_, w3, p3, None, b, b, None, pe, zero, None, None, 1, 2, 2, 2)  # noqa
    ref = fn().clone()
    diff = torch.zeros_like(ref, dtype=torch.bool)
    for _ in range(10):
        diff |= fn() != ref
    idx = diff.nonzero().cpu()
    n, co, y, xx = idx.unbind(1) if idx.numel() else (torch.zeros(0, dtype=torch.long),) * 4
    p = y * W + xx
    print(name, "differing", idx.shape[0], flush=True)
    if idx.numel():
        print("  co per pixel", Counter(Counter((n * 1000000 + p).tolist()).values()).most_common(6))
        print("  co groups of 4", sorted(Counter((co // 4).tolist()).items()))
        print("  px%16", sorted(Counter((p % 16).tolist()).items()))
        print("  px in tile", Counter((p % 128).tolist()).most_common(12))
