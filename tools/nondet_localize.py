"""Localise the first fusion whose outputs differ between the concurrent-scale schedule and the
one-stream schedule (eager, batch 8): every fusion's output list is cloned on the main stream
after it waits for the side streams (this adds a join per fusion)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from aanet_amd.nets import aggregation as agg  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
model = bench.build_model(dev)
left, right = bench.make_features(8, 0, dev, "randn")
rec = []
JOIN = os.environ.get("NOJOIN") is None


def wrap(f):
    orig = f.forward

    def fwd(*a, **k):
        out = orig(*a, **k)
        main = torch.cuda.current_stream()
        if JOIN:
            for s in agg._SIDE_STREAMS.get(dev, []):
                main.wait_stream(s)
        outs = [t.clone() if t is not None else None for t in out]
        post = k.get("post")
        res = post.get("result") if post is not None else None
        if res is not None and res.get("out") is not None:
            outs.append(res["out"].clone())  # the post stage's output (next fusion's conv1)
        rec.append(outs)
        return out
    f.forward = fwd


for f in model.aggregation.fusions:
    wrap(f)

from aanet_amd import ops  # noqa: E402
_mdcn_pw = ops.mdcn_pw
tail_rec = []


def mdcn_pw_rec(x1, om, *a, csa_up=None, **k):
    # inputs as the tail kernel reads them (cloned on the launch stream, after the join)
    ins = [x1.clone(), om.clone()] + [t.clone() for t in (csa_up or [])]
    r = _mdcn_pw(x1, om, *a, csa_up=csa_up, **k)
    outs = [t.clone() for t in (r if isinstance(r, (tuple, list)) else [r]) if torch.is_tensor(t)]
    tail_rec.append((ins, outs))
    return r


ops.mdcn_pw = mdcn_pw_rec
from aanet_amd.nets import deform as _deform  # noqa: E402
if hasattr(_deform, "ops"):
    _deform.ops.mdcn_pw = mdcn_pw_rec


def run():
    rec.clear()
    tail_rec.clear()
    with torch.no_grad():
        out = model(left, right)[0].clone()
    torch.cuda.synchronize()
    return out, [list(r) for r in rec], list(tail_rec)


model.set_options(concurrent_scales=False)
ref, rref, tref = run()
model.set_options(concurrent_scales=True)
for it in range(4):
    out, r, tr = run()
    for n, ((ia, oa), (ib, ob)) in enumerate(zip(tr, tref)):
        di = [torch.equal(x, y) for x, y in zip(ia, ib)]
        do = [torch.equal(x, y) for x, y in zip(oa, ob)]
        if not all(di) or not all(do):
            print(f"  run {it} DCN tail {n}: inputs equal {di} (x1, offset_mask, up...), outputs equal {do}")
    first = None
    for i, (a, b) in enumerate(zip(r, rref)):
        for j, (x, y) in enumerate(zip(a, b)):
            if x is not None and not torch.equal(x, y):
                first = (i, j, (x - y).abs().max().item(), int((x != y).sum()))
                break
        if first:
            break
    print(f"run {it}: output equal {torch.equal(out, ref)}; first differing fusion/branch "
          f"(branch 3 = post-stage conv1 output) {first}", flush=True)
