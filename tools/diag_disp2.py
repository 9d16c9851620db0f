"""Diagnostic: which module family's split contraction moves the hot-path disparity away from the
CPU oracle.  Each variant runs exact f32 on one module family (forward pre/post hooks toggle
_lib.set_exact_f32) and the split contraction elsewhere."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from aanet_amd import _lib  # noqa: E402
from aanet_amd.nets.deform import DeformSimpleBottleneck, SimpleBottleneck  # noqa: E402
from oracle import aggregation as oagg  # noqa: E402

dev = torch.device("cuda", 0)
model = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev)
sd = {k: v.detach().cpu().numpy() for k, v in model.aggregation.state_dict().items()}
ref = oagg.hot_path([t[:1].cpu().numpy() for t in left], [t[:1].cpu().numpy() for t in right], sd,
                    bench.MAXD, intermediate_supervision=False)[0][0].astype(np.float64)


def run(pred, default_exact=False):
    hooks = []
    for name, m in model.named_modules():
        if pred(name, m):
            hooks.append(m.register_forward_pre_hook(lambda *a: _lib.set_exact_f32(not default_exact) and None))
            hooks.append(m.register_forward_hook(lambda *a: _lib.set_exact_f32(default_exact) and None))
    _lib.set_exact_f32(default_exact)
    with torch.no_grad():
        d = model(left, right)[0][0].cpu().numpy().astype(np.float64)
    for h in hooks:
        h.remove()
    e = np.abs(d - ref)
    return e.max(), (e > 1e-4).sum()


variants = {
    "all split": lambda n, m: False,
    "DCN blocks exact": lambda n, m: isinstance(m, DeformSimpleBottleneck),
    "plain blocks exact": lambda n, m: isinstance(m, SimpleBottleneck),
    "fuse layers exact": lambda n, m: ".fuse_layers." in n and n.count(".") == 4,
    "final conv exact": lambda n, m: "final_conv" in n,
    "DCN offset conv exact": lambda n, m: n.endswith("offset_conv"),
}
with torch.no_grad():
    _lib.set_exact_f32(False)
    outs = [model(left, right)[0].clone() for _ in range(4)]
    print("split run-to-run max diff:", max(float((o - outs[0]).abs().max()) for o in outs),
          [int((o != outs[0]).sum()) for o in outs])
    _lib.set_exact_f32(True)
    outs = [model(left, right)[0].clone() for _ in range(4)]
    print("exact run-to-run max diff:", max(float((o - outs[0]).abs().max()) for o in outs))
for k, f in variants.items():
    mx, cnt = run(f)
    print(f"{k:24s} max {mx:.3e}  n>1e-4 {cnt}")
only = {
    "only DCN blocks split": lambda n, m: isinstance(m, DeformSimpleBottleneck),
    "only plain blocks split": lambda n, m: isinstance(m, SimpleBottleneck),
    "only offset convs split": lambda n, m: n.endswith("offset_conv"),
}
for k, f in only.items():
    mx, cnt = run(f, default_exact=True)
    print(f"{k:24s} max {mx:.3e}  n>1e-4 {cnt}")
