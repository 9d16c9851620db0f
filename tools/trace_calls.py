"""Log every HIP op call (name, input/weight shapes, conv geometry) of one eager bench forward,
with its device time: python tools/trace_calls.py.  Finds which module a conv kernel of the
rocprof summary belongs to."""
import functools
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from aanet_amd import ops  # noqa: E402

log = []


def wrap(name):
    f = getattr(ops, name)

    @functools.wraps(f)
    def g(*args, **kw):
        shapes = [tuple(a.shape) + (("cl",) if a.dim() == 4 and a.is_contiguous(memory_format=torch.channels_last)
                                    and not a.is_contiguous() else ())
                  for a in args[:2] if torch.is_tensor(a)]
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = f(*args, **kw)
        e.record()
        geo = [a for a in args if isinstance(a, (int, str))][:6]
        log.append((name, shapes, geo, sorted(k for k, v in kw.items() if v is not None), s, e))
        return out
    return g


for n in ("conv2d_fused", "conv2d_pw", "mdcn_pw", "mdcn_forward_fused", "csa_sum", "corr_pyramid",
          "disp_regress"):
    setattr(ops, n, wrap(n))
dev = torch.device("cuda")
model = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev)
with torch.no_grad():
    for it in range(2):
        log.clear()
        model(left, right)
torch.cuda.synchronize()
tot = 0.0
for name, shapes, geo, kws, s, e in log:
    t = s.elapsed_time(e) * 1e3
    tot += t
    print(f"{t:8.1f} us  {name:18s} {shapes} {geo} {kws}")
print(f"total {tot:.1f} us over {len(log)} calls")
