"""Diagnostic: run-to-run bit reproducibility of each conv-engine op family on the split path at
C2 scale-0 shapes (B=8): a data race shows up as differing outputs between identical launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import _lib, ops  # noqa: E402

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
ups = [torch.randn(B, C, H // r, W // r, device=dev, generator=g) for r in (2, 4)]
om0 = torch.zeros_like(om)
eye = torch.eye(C, device=dev).view(C, C, 1, 1)
pe = ops.pack_weight_split(eye)
zero = torch.zeros(C, device=dev)
cases = {
    "dcn_pw nhwc": lambda: ops.mdcn_pw(xn, om, w3, p3, None, b, b, "relu", p1, b, None, None, 1, 2, 2, 2),
    "dcn_pw nhwc + csa": lambda: ops.mdcn_pw(xn, om, w3, p3, None, b, b, "relu", p1, b, res, "relu",
                                             1, 2, 2, 2, csa_up=ups)[1],
    "dcn_pw nchw": lambda: ops.mdcn_pw(x, om, w3, p3, None, b, b, "relu", p1, b, None, None, 1, 2, 2, 2),
}
refs = {}
for exact in (True, False):
    _lib.set_exact_f32(exact)
    for name, fn in cases.items():
        ref = fn().clone()
        bad = 0
        mx = 0.0
        for _ in range(12):
            o = fn()
            bad = max(bad, int((o != ref).sum()))
            mx = max(mx, float((o - ref).abs().max()))
        if exact:
            refs[name] = ref
        dx = float((ref - refs[name]).abs().max()) if name in refs else float("nan")
        print(f"{'exact' if exact else 'split'} {name:28s} differing {bad:9d}  max {mx:.3e}  vs exact {dx:.3e}",
              flush=True)
