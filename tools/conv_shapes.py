"""Census of the engine calls of one hot-path forward, with each call's time (synchronised HIP
events around the call, after a warm-up forward): where the non-bottleneck convs spend."""
import sys
from collections import defaultdict

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from aanet_amd import ops  # noqa: E402

stats = defaultdict(list)
timing = [False]
for name in ("conv2d_fused", "conv2d_pw", "mdcn_pw", "mdcn_forward_fused", "csa_sum"):
    f = getattr(ops, name)

    def wrap(*a, _f=f, _n=name, **k):
        if not timing[0]:
            return _f(*a, **k)
        x = a[0]
        shp = [tuple(t.shape) for t in x] if isinstance(x, list) else tuple(x.shape)
        w = None
        if _n in ("conv2d_fused", "conv2d_pw"):
            w = tuple(a[1].shape)
        elif _n in ("mdcn_pw", "mdcn_forward_fused"):
            w = tuple(a[2].shape)
        geo = (a[3], a[4]) if _n == "conv2d_fused" and len(a) > 4 else ""
        nhwc = (not isinstance(x, list)) and x.dim() == 4 and not x.is_contiguous()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        out = _f(*a, **k)
        e.record()
        torch.cuda.synchronize()
        stats[(_n, str(shp), str(w), str(geo), "nhwc" if nhwc else "nchw",
               "out_nhwc" if k.get("out_nhwc") else "")].append(s.elapsed_time(e) * 1e3)
        return out
    setattr(ops, name, wrap)
dev = torch.device("cuda", 0)
m = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev)
with torch.no_grad():
    m(left, right)
    timing[0] = True
    m(left, right)
tot = 0.0
for k, v in sorted(stats.items(), key=lambda kv: -sum(kv[1])):
    tot += sum(v)
    print(f"{sum(v):8.1f} us  {len(v)}x {sum(v) / len(v):7.1f}  {k}")
print(f"total {tot:.1f} us")
