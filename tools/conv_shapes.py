"""List the engine calls of one hot-path forward (shape census for tuning)."""
import sys
from collections import Counter

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from aanet_amd import ops  # noqa: E402

calls = Counter()
for name in ("conv2d_fused", "conv2d_pw", "mdcn_pw", "mdcn_forward_fused", "csa_sum"):
    f = getattr(ops, name)

    def wrap(*a, _f=f, _n=name, **k):
        x = a[0]
        shp = [tuple(t.shape) for t in x] if isinstance(x, list) else tuple(x.shape)
        w = tuple(a[1].shape) if len(a) > 1 and hasattr(a[1], "shape") and _n != "mdcn_pw" else \
            (tuple(a[2].shape) if _n in ("mdcn_pw", "mdcn_forward_fused") else None)
        nhwc = (not isinstance(x, list)) and x.dim() == 4 and x.is_contiguous(memory_format=torch.channels_last) \
            and not x.is_contiguous()
        calls[(_n, str(shp), str(w), str(a[2:5] if _n == "conv2d_fused" else ""), nhwc)] += 1
        return _f(*a, **k)
    setattr(ops, name, wrap)
dev = torch.device("cuda", 0)
m = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev)
with torch.no_grad():
    m(left, right)
for k, v in sorted(calls.items(), key=lambda kv: -kv[1]):
    print(v, k)
