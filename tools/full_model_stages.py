"""Per-stage time and roofline fraction of a full model (bench.py --model).

Stages follow the reference's forward (nets/aanet.py:140-229): the feature extractor (left +
right), the FPN / pyramid, the cost volume, the aggregation (+ regression), the refinement.
Times: HIP events around each stage on the launch stream, eager, fused eval path, median of
--iters runs after a warm-up.  Work: algorithmic FLOPs from forward hooks on every Conv2d /
ConvTranspose2d / Conv3d / DeformConv2d in a reference-order pass (the fused path skips the module
forwards; the FLOPs are the same), 2 * MACs; bytes: every conv's input + output once (a lower
bound on HBM traffic).  Each stage is priced against the roof its intensity puts it under:
FLOP/byte above the ridge (416.7 TF/s split-bf16 / 8 TB/s = 52) -> MFMA (416.7 TF/s fp32-equiv),
below -> HBM (8 TB/s).  Usage: python tools/full_model_stages.py [aanet|aanetplus|psmnet_aa|psmnet_hg] [--iters N]
"""
import json
import os
import sys

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from aanet_amd.nets import AANet  # noqa: E402
from aanet_amd.nets.aggregation import AdaptiveAggregation  # noqa: E402
from aanet_amd.nets.deform import DeformConv2d  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith("-") else "aanet"
iters = int(sys.argv[sys.argv.index("--iters") + 1]) if "--iters" in sys.argv else 5
B, H, W = 8, bench.H_IMG, bench.W_IMG
SPLIT_TF, HBM_GBS = 2500.0 / 6, 8000.0
dev = torch.device("cuda", 0)

torch.manual_seed(0)
model = AANet(bench.MAXD_IMG, **bench.FULL_MODELS[name])
g = torch.Generator().manual_seed(1)
with torch.no_grad():
    for mname, mod in model.named_modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.copy_(0.05 * torch.randn(mod.num_features, generator=g))
            mod.running_var.copy_(0.8 + 0.4 * torch.rand(mod.num_features, generator=g))
        if mname.endswith("offset_conv"):
            mod.weight.normal_(0.0, 0.01, generator=g)
            mod.bias.normal_(0.0, 0.5, generator=g)
model = model.to(dev).eval()
gen = torch.Generator(device=dev).manual_seed(4321)
left = torch.randn((B, 3, H, W), device=dev, generator=gen)
right = torch.randn((B, 3, H, W), device=dev, generator=gen)


def stages(m):
    """The forward of nets/aanet.py split into named stages: [(name, fn)] sharing state."""
    st = {}

    def feat():
        st["lf"] = m.feature_extractor(left)
        st["rf"] = m.feature_extractor(right)

    def fpn():
        if m.feature_pyramid_network or m.feature_pyramid:
            st["lf"], st["rf"] = m.fpn(st["lf"]), m.fpn(st["rf"])

    def cost():
        st["cv"] = m.cost_volume_construction(st["lf"], st["rf"])

    def agg():
        if not isinstance(m.aggregation, AdaptiveAggregation):  # 3-D aggregators (C5)
            st["disp"] = m.disparity_computation(m.aggregation(st["cv"]))
            return
        regress = (not m.aggregation.intermediate_supervision and not m.training and
                   m.disparity_estimation.match_similarity)
        a, d = m.aggregation._run(st["cv"], regress=regress)
        st["disp"] = [d] if d is not None else m.disparity_computation(a)

    def refine():
        st["out"] = m.disparity_refinement(left, right, st["disp"][-1])

    return [("feature extractor", feat), ("fpn / pyramid", fpn), ("cost volume", cost),
            ("aggregation + regression", agg), ("refinement", refine)]


# ---- work per stage: hooks on a reference-order pass
work = {}
cur = [None]


def hook(mod, inp, out):
    x = inp[0]
    o = out[0] if isinstance(out, (tuple, list)) else out
    if isinstance(mod, DeformConv2d):
        w = mod.deform_conv.weight
        macs = o.numel() * w.shape[1] * w.shape[2] * w.shape[3]
    elif isinstance(mod, nn.modules.conv._ConvTransposeNd):
        k = 1
        for v in mod.kernel_size:
            k *= v
        macs = x.numel() * (mod.out_channels // mod.groups) * k
    else:
        k = 1
        for v in mod.kernel_size:
            k *= v
        macs = o.numel() * (mod.in_channels // mod.groups) * k
    f, b = work.get(cur[0], (0.0, 0.0))
    work[cur[0]] = (f + 2.0 * macs, b + 4.0 * (x.numel() + o.numel()))


handles = []
for mod in model.modules():
    if isinstance(mod, (nn.modules.conv._ConvNd, DeformConv2d)):
        handles.append(mod.register_forward_hook(hook))
for mod in model.modules():
    mod.aanet_fuse = False
with torch.no_grad():
    for sname, fn in stages(model):
        cur[0] = sname
        fn()
for h in handles:
    h.remove()
for mod in model.modules():
    mod.aanet_fuse = True
torch.cuda.synchronize()

# ---- time per stage (fused eval path)
stream = torch.cuda.current_stream()
times = {s: [] for s, _ in stages(model)}
with torch.no_grad():
    for it in range(iters + 2):
        for sname, fn in stages(model):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            fn()
            e1.record(stream)
            e1.synchronize()
            if it >= 2:
                times[sname].append(e0.elapsed_time(e1))
total = 0.0
rows = []
for sname, _ in stages(model):
    ms = sorted(times[sname])[len(times[sname]) // 2]
    total += ms
    f, b = work.get(sname, (0.0, 0.0))
    inten = f / b if b else 0.0
    if f and inten >= SPLIT_TF * 1e12 / (HBM_GBS * 1e9):
        bound, ach, peak, unit = "mfma", f / ms / 1e9, SPLIT_TF, "TF/s"
    else:
        bound, ach, peak, unit = "hbm", b / ms / 1e6, HBM_GBS, "GB/s"
    rows.append(dict(stage=sname, ms=ms, gflop=f / 1e9, mb=b / 1e6, intensity=inten, bound=bound,
                     achieved=ach, peak=peak, unit=unit, frac=ach / peak if peak else 0.0))
print(f"# tools/full_model_stages.py {name}: B={B}, {H}x{W}, eval, fused path, eager stage timing "
      f"(median of {iters}); work from conv hooks (2*MACs; conv in+out bytes as the HBM lower bound)")
print(f"{'stage':28s} {'ms':>8s} {'share':>6s} {'GFLOP':>9s} {'MB':>9s} {'FLOP/B':>7s} bound  achieved        frac")
for r in rows:
    print(f"{r['stage']:28s} {r['ms']:8.3f} {r['ms'] / total:6.1%} {r['gflop']:9.1f} {r['mb']:9.1f} "
          f"{r['intensity']:7.1f} {r['bound']:5s} {r['achieved']:8.1f} {r['unit']:5s} {r['frac']:6.3f}")
print(f"{'total (stages, eager)':28s} {total:8.3f}")
print(json.dumps({"model": name, "stages": rows, "total_ms": total}))
