"""Per-scale correlation volume timings vs the one-launch pyramid (C2, B=8): python tools/corr_scales.py"""
import torch, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import ops
dev = "cuda"
B = 8
feats = [(128, 128 >> s, 416 >> s, 64 >> s) for s in range(3)]
L = [torch.randn(B, c, h, w, device=dev) for c, h, w, d in feats]
R = [torch.randn(B, c, h, w, device=dev) for c, h, w, d in feats]
def t(fn, it=50):
    fn(); torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3
tot = 0
for i, (c, h, w, d) in enumerate(feats):
    us = t(lambda: ops.corr_volume(L[i], R[i], d))
    by = 4 * (2 * B * c * h * w + B * d * h * w)
    tot += by
    print(f"scale {i}: {us:7.1f} us  {by/us/1e6:6.0f} GB/s  ({by/1e6:.1f} MB)")
us = t(lambda: ops.corr_pyramid(L, R, 64))
print(f"pyramid: {us:7.1f} us  {tot/us/1e6:6.0f} GB/s  ({tot/1e6:.1f} MB)")
