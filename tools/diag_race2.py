"""Where do run-to-run differences of the split NHWC DCN tail kernel fall (tile pixel / channel /
image histogram)?"""
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
res = torch.randn(B, C, H, W, device=dev, generator=g)
w1 = torch.randn(C, C, 1, 1, device=dev, generator=g) * 0.1
w3 = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.04
wo = torch.randn(54, 32, 3, 3, device=dev, generator=g) * 0.01
bo = torch.randn(54, device=dev, generator=g)
b = torch.randn(C, device=dev, generator=g)
p1, p3, po = ops.pack_weight_split(w1), ops.pack_weight_split(w3), ops.pack_weight_split(wo, 2)
om = ops.conv2d_fused(x, wo, bo, 1, 2, 2, 2, packed_weight=po)
fn = lambda: ops.mdcn_pw(xn, om, w3, p3, None, b, b, "relu", p1, b, None, None, 1, 2, 2, 2)  # noqa: E731
ref = fn().clone()
diff = torch.zeros_like(ref, dtype=torch.bool)
for _ in range(8):
    diff |= fn() != ref
idx = diff.nonzero().cpu()
print("differing", idx.shape[0])
n, co, y, xx = idx.unbind(1)
p = y * W + xx
print("image", Counter(n.tolist()).most_common(8))
print("co", sorted(Counter(co.tolist()).items())[:64])
print("px in tile", Counter((p % 128).tolist()).most_common(20))
print("px block (16)", sorted(Counter(((p % 128) // 16).tolist()).items()))
print("tiles", len(set((n * 10000 + p // 128).tolist())), "of", B * H * W // 128)
d = (fn() - ref).abs()
print("per-differing-pixel: how many co differ", Counter(Counter((n * 1000000 + p).tolist()).values()).most_common(10))
