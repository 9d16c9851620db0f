"""Microbenchmark of the stride-2 exchange convs (conv_s2.hip) at the C2 (B=8, 384x1248) shapes:
the scale-0 heads launch (64 -> 32 + 64) plain and with branch 1's CSA terms, the merged branch-2
launch (64 + 32 -> 16 with x2 + identity) and the plain narrow convs.  A/B against another build
of the library: AANET_MI355X_LIB=/path/to/lib.so python tools/s2_bench.py (terms cases are
skipped when that library lacks aanet_conv3x3s2_terms_f32)."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
from aanet_amd import _lib, ops  # noqa: E402


def timed(fn, iters=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3


def main():
    only = sys.argv[1] if len(sys.argv) > 1 else None
    dev = "cuda"
    B = 8
    g = torch.Generator(device=dev).manual_seed(0)
    x0 = torch.randn(B, 64, 128, 416, device=dev, generator=g)
    x1 = torch.randn(B, 32, 64, 208, device=dev, generator=g)
    hb = torch.randn(B, 64, 64, 208, device=dev, generator=g)
    x2 = torch.randn(B, 16, 32, 104, device=dev, generator=g)
    t12 = torch.randn(B, 32, 32, 104, device=dev, generator=g)
    w96 = torch.randn(96, 64, 3, 3, device=dev, generator=g) * 0.05
    w16 = torch.randn(16, 64, 3, 3, device=dev, generator=g) * 0.05
    w16b = torch.randn(16, 32, 3, 3, device=dev, generator=g) * 0.05
    w16m = torch.cat([w16, w16b], 1)
    b96, b16 = torch.randn(96, device=dev), torch.randn(16, device=dev)
    p96, p16, p16b, p16m = (ops.pack_conv3x3s2(w) for w in (w96, w16, w16b, w16m))
    has_terms = hasattr(_lib.lib(), "aanet_conv3x3s2_terms_f32")
    res = {"lib": _lib.LIB_PATH}
    if only == "heads":  # profiling: the heads launch alone
        res["heads_64to96"] = timed(lambda: ops.conv3x3_s2(x0, p96, b96, 96, 32, None, "leaky"), 20)
        print(json.dumps(res))
        return
    res["heads_64to96"] = timed(lambda: ops.conv3x3_s2(x0, p96, b96, 96, 32, None, "leaky"))
    res["s1to2_32to16"] = timed(lambda: ops.conv3x3_s2(x1, p16b, b16, 16, 16))
    res["hb_64to16"] = timed(lambda: ops.conv3x3_s2(hb, p16, b16, 16, 16))
    if has_terms:
        res["heads_terms"] = timed(lambda: ops.conv3x3_s2(x0, p96, b96, 96, 32, "leaky", "leaky",
                                                          identity=x1, up=t12))
        res["branch2_merged"] = timed(lambda: ops.conv3x3_s2(hb, p16m, b16, 16, 16, "leaky",
                                                             x2=x1, identity=x2))
    # roofline of the heads launch: split-bf16 ceiling (6 bf16 MFMA products per fp32 MAC)
    flops = 2.0 * B * 64 * 208 * 96 * 64 * 9
    res["heads_split_ceiling_us"] = flops * 6 / 2.5e15 * 1e6
    print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
