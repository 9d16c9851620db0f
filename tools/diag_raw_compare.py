"""Stage table for model_psmnet_aa_raw (build container only: imports /root/reference by path, as
tests/golden/make_model_golden.py does).  Compares the GPU dump of tools/diag_raw_stages.py
(gpurun_out/raw_stages.npz) with the REFERENCE's own fp32 and fp64 runs of the same model,
hooked at the same module names:

  * per stage: normwise / max error against the reference's fp64 output, for the reference's
    fp32 run, our fused run and our reference-order run, and the ratio of ours to the
    reference's own normwise error;
  * per pyramid level: flips (|d - d64| > 0.05 px) end to end;
  * the refinement alone, fed the fp64 level-0 disparity (fixture `disp64_0`): flips of the
    reference's fp32 refinement and of ours against the fp64 refinement of the same input;
  * where the end-to-end level-1/2 flips sit relative to the level-0 flips (cascade).

    python tools/diag_raw_compare.py [gpurun_out/raw_stages.npz] > profiles/r06_raw_stages.txt
"""
import importlib
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))

from make_golden import load_reference  # noqa: E402
from tests.golden_io import fill_synthetic, fixture_scales, golden, synthetic_pair  # noqa: E402
from tools.diag_raw_stages import keep  # noqa: E402

TAG = "model_psmnet_aa_raw"
FLIP = 0.05


def _flat(o, out, key):
    if isinstance(o, torch.Tensor):
        out[key] = o.detach().double().numpy().copy()
    elif isinstance(o, (list, tuple)):
        for i, t in enumerate(o):
            _flat(t, out, f"{key}#{i}")


def reference_stages():
    load_reference()
    aanet = importlib.import_module("nets.aanet")
    g = golden(TAG)
    m = aanet.AANet(int(g["max_disp"]), 1, **json.loads(str(g["config"])))
    fill_synthetic(m, int(g["seed"]), fixture_scales(g))
    m.eval()
    B, H, W = (int(v) for v in g["shape"])
    left, right = synthetic_pair(B, H, W, int(g["seed"]))
    res = {}
    for tag, dt in (("r32", torch.float32), ("r64", torch.float64)):
        seen, hooks = {}, []
        for name, mod in m.named_modules():
            if not keep(name):
                continue

            def hook(mod, i, o, name=name, tag=tag):
                k = seen.get(name, 0)
                seen[name] = k + 1
                # cloned: the aggregation replaces list entries in place (aggregation.py:382)
                _flat(o, res, f"{tag}|{name}|{k}")
                if name.endswith("deform_conv"):
                    _flat(i, res, f"{tag}|{name}.in|{k}")
            hooks.append(mod.register_forward_hook(hook))
        m.to(dt)
        with torch.no_grad():
            pyr = m(left.to(dt), right.to(dt))
            for h in hooks:
                h.remove()
            for i, d in enumerate(pyr):
                res[f"{tag}_disp{i}"] = d.double().numpy()
            d0 = torch.from_numpy(g["disp64_0"]).to(dt)
            for i, d in enumerate(m.disparity_refinement(left.to(dt), right.to(dt), d0)):
                res[f"{tag}_cond{i + 1}"] = d.double().numpy()
    return res


def nw(a, ref):
    return np.linalg.norm(a - ref) / max(np.linalg.norm(ref), 1e-300)


def main():
    ours = dict(np.load(sys.argv[1] if len(sys.argv) > 1 else
                        os.path.join(REPO, "gpurun_out", "raw_stages.npz")))
    ref = reference_stages()
    print(f"# {TAG}: stage errors against the reference's own fp64 run (normwise / max abs); "
          "'x ref' = our normwise error / the reference fp32 run's")
    print(f"{'stage':48s} {'ref fp32':>18s} | {'ours fused':>18s} {'x ref':>6s} | "
          f"{'ours ref-order':>18s} {'x ref':>6s}")
    keys = [k[4:] for k in ref if k.startswith("r64|")]
    for k in keys:
        e64 = ref["r64|" + k]
        r32 = ref.get("r32|" + k)
        if r32 is None or r32.shape != e64.shape:
            continue
        base = nw(r32, e64)
        cols = [f"{base:.1e} / {np.abs(r32 - e64).max():.1e}"]
        for src in ("fused", "ref"):
            o = ours.get(f"{src}|{k}")
            if o is None or o.shape != e64.shape:
                cols.append(f"{'-':>18s} {'':>6s}")
                continue
            e = nw(o.astype(np.float64), e64)
            cols.append(f"{e:.1e} / {np.abs(o - e64).max():.1e} {e / max(base, 1e-300):6.2f}")
        print(f"{k:48s} {cols[0]:>18s} | {cols[1]:>25s} | {cols[2]:>25s}")

    g = golden(TAG)
    dcn = sorted({k.split("|")[1][:-3] for k in ours if k.startswith("ref|") and k.endswith(".in|0#0")})
    if dcn:
        from oracle import oracle
        from tests.golden_io import synthetic_value
        print("\n# each DCN op alone: our reference-order output against the fp64 DCN of OUR OWN "
              "inputs (the op's own error), the oracle's fp32 DCN on the same inputs beside it, and "
              "the fp64 DCN with only one input taken from our run (which input's error the "
              "stage error above comes from)")
        for st in dcn:
            ins = [ours[f"ref|{st}.in|0#{i}"].astype(np.float64) for i in range(3)]
            ins64 = [ref[f"r64|{st}.in|0#{i}"] for i in range(3)]
            C = ins[0].shape[1]
            w = synthetic_value(st + ".weight", (C, C, 3, 3), int(g["seed"])).numpy()

            def f(x, o, m, dt=np.float64):
                return oracle.mdcn_forward(x.astype(dt), o.astype(dt), m.astype(dt), w.astype(dt),
                                           None, 1, 2, 2, 1, 2, dtype=dt)
            own = f(*ins)
            o32 = f(*ins, dt=np.float32)
            base = f(*ins64)
            one = []
            for i in range(3):
                a = list(ins64)
                a[i] = ins[i]
                one.append(nw(f(*a), base))
            print(f"  {st}: ours {nw(ours[f'ref|{st}|0'], own):.1e}, oracle fp32 {nw(o32, own):.1e}"
                  f" | only x {one[0]:.1e}, only offset {one[1]:.1e}, only mask {one[2]:.1e} "
                  f"(all: {nw(ours[f'ref|{st}|0'], base):.1e}); |offset| max "
                  f"{np.abs(ins64[1]).max():.0f} px, |x| max {np.abs(ins64[0]).max():.0f}")
    print("\n# end to end, per level: flips (|d - d64| > 0.05 px) and normwise error vs fp64")
    for i in range(3):
        d64 = g[f"disp64_{i}"]
        row = [f"L{i}"]
        for name, d in (("ref fp32", ref[f"r32_disp{i}"]), ("fused", ours[f"fused_disp{i}"]),
                        ("ref-order", ours[f"ref_disp{i}"])):
            e = np.abs(d.astype(np.float64) - d64)
            row.append(f"{name} {int((e > FLIP).sum()):5d} flips, max {e.max():.2e}, "
                       f"nw {nw(d.astype(np.float64), d64):.1e}")
        print("  " + " | ".join(row))

    print("\n# the refinement alone, fed the fp64 level-0 disparity: flips vs the fp64 refinement "
          "of the same input (its own error, no inherited level-0 flips)")
    for i in (1, 2):
        c64 = ref[f"r64_cond{i}"]
        assert np.abs(c64 - g[f"disp64_{i}"]).max() < 1e-9  # = the fixture's fp64 chain
        row = [f"L{i}"]
        for name, d in (("ref fp32", ref[f"r32_cond{i}"]), ("fused", ours[f"fused_cond{i}"]),
                        ("ref-order", ours[f"ref_cond{i}"])):
            e = np.abs(d.astype(np.float64) - c64)
            row.append(f"{name} {int((e > FLIP).sum()):5d} flips, max {e.max():.2e}, "
                       f"nw {nw(d.astype(np.float64), c64):.1e}")
        print("  " + " | ".join(row))

    print("\n# cascade: level-0 flips and the level-1/2 flips within r px of their upsampled position")
    for name, key in (("ref fp32", None), ("fused", "fused"), ("ref-order", "ref")):
        d0 = ref["r32_disp0"] if key is None else ours[f"{key}_disp0"]
        e0 = np.abs(d0.astype(np.float64) - g["disp64_0"])[0]
        f0 = np.argwhere(e0 > FLIP)
        desc = ", ".join(f"({y},{x}) {e0[y, x]:.2f}px" for y, x in f0)
        print(f"  {name}: level-0 flips {desc}")
        for i in (1, 2):
            di = ref[f"r32_disp{i}"] if key is None else ours[f"{key}_disp{i}"]
            ei = np.abs(di.astype(np.float64) - g[f"disp64_{i}"])[0]
            fi = np.argwhere(ei > FLIP)
            s = 2 ** i
            for r in (16, 32, 64):
                near = 0
                for y, x in fi:
                    if len(f0) and (np.max(np.abs(f0 * s + s // 2 - np.array([y, x])), axis=1) <= r).any():
                        near += 1
                print(f"    L{i}: {len(fi)} flips, {near} within {r} px of an upsampled level-0 flip")


if __name__ == "__main__":
    main()
