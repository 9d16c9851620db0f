"""Census of the engine convs of one full-model forward (bench.FULL_MODELS; fused eval path):
input shape, weight shape, stride / padding / dilation, input layout and time of every
ops.conv2d_fused / ops.deconv2x / ops.mdcn_forward_fused call (synchronised HIP events around the
call, after a warm-up forward), grouped by signature.  Usage: python tools/model_conv_census.py
[aanet|aanetplus]"""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from aanet_amd import ops  # noqa: E402
from aanet_amd.nets import AANet  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "aanetplus"
stats = defaultdict(list)
timing = [False]
for fname in ("conv2d_fused", "deconv2x", "mdcn_forward_fused", "conv3x3_s2", "concat_nhwc"):
    f = getattr(ops, fname)

    def wrap(*a, _f=f, _n=fname, **k):
        if not timing[0]:
            return _f(*a, **k)
        x = a[0]
        w = tuple(a[1].shape) if torch.is_tensor(a[1]) else a[1]
        if _n == "mdcn_forward_fused":
            w = tuple(a[2].shape)
        geo = tuple(a[3:6]) if _n == "conv2d_fused" else ""
        nhwc = x.dim() == 4 and not x.is_contiguous()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        out = _f(*a, **k)
        e.record()
        torch.cuda.synchronize()
        stats[(_n, tuple(x.shape), w, geo, "nhwc" if nhwc else "nchw")].append(s.elapsed_time(e))
        return out

    setattr(ops, fname, wrap)

B, H, W = 8, bench.H_IMG, bench.W_IMG
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = AANet(bench.MAXD_IMG, **bench.FULL_MODELS[name]).to(dev).eval()
left = torch.randn(B, 3, H, W, device=dev)
right = torch.randn(B, 3, H, W, device=dev)
with torch.no_grad():
    model(left, right)
    timing[0] = True
    model(left, right)
tot = 0.0
rows = []
for key, ts in stats.items():
    rows.append((sum(ts), len(ts), key))
    tot += sum(ts)
for t, n, key in sorted(rows, reverse=True):
    print(f"{t * 1e3:9.1f} us  x{n:2d}  {key}")
print(f"total {tot:.3f} ms (synchronised per call)")
