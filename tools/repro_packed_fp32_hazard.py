"""Minimal repro of the packed-fp32 hazard ("The split DCN-tail reproducibility bug").

The NHWC split DCN tail (DCN + identity pointwise tail) at C2 scale 0, launched 10 times on the
same inputs: every launch must be bit-identical.  With the library built WITHOUT the
`-packed-fp32-ops` guard of aanet_amd/csrc/Makefile, fractional offsets give whole-pixel
differences in pixels 8w+6 / 8w+7 of each 64-pixel group (lanes 48-63 of a wave read a
broadcast operand before the v_mov that writes it has landed):

    make -C aanet_amd/csrc NOPK= LIB=/tmp/libaanet_pk.so
    AANET_MI355X_LIB=/tmp/libaanet_pk.so python tools/repro_packed_fp32_hazard.py   # differs
    python tools/repro_packed_fp32_hazard.py                                        # 0 differing

Integer and zero offsets stay clean either way (every corner weight is 0 or 1, so a stale
weight is invisible).  tests/test_gpu_split.py holds the shipped library to the same property.
"""
import os
import sys

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
pe = ops.pack_weight_split(torch.eye(C, device=dev).view(C, C, 1, 1))
zero = torch.zeros(C, device=dev)
bad = 0
for name, om_ in (("fractional", om), ("integer", om.round()), ("zero", torch.zeros_like(om))):
    fn = lambda: ops.mdcn_pw(xn, om_, w3, p3, None, b, b, None, pe, zero, None, None, 1, 2, 2, 2)  # noqa: E731
    ref = fn().clone()
    diff = torch.zeros_like(ref, dtype=torch.bool)
    for _ in range(10):
        diff |= fn() != ref
    n = int(diff.sum())
    bad += n
    print(f"{name} offsets: {n} differing outputs over 10 launches", flush=True)
sys.exit(1 if bad else 0)
