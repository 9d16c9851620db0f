"""Microbenchmark of the scale-0 layers of one AAModule (C2 shapes, B=8), each launched alone
(for rocprofv3 passes and A/B timing).  Usage: python tools/conv_microbench.py [iters] [names]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aanet_amd import ops  # noqa: E402

iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
names = sys.argv[2].split(",") if len(sys.argv) > 2 else None
dev = "cuda"
B, C, H, W = 8, 64, 128, 416
g = torch.Generator(device=dev).manual_seed(0)
x = torch.randn(B, C, H, W, device=dev, generator=g)
res = torch.randn(B, C, H, W, device=dev, generator=g)
w1 = torch.randn(C, C, 1, 1, device=dev, generator=g) * 0.1
w3 = torch.randn(C, C, 3, 3, device=dev, generator=g) * 0.04
wo = torch.randn(54, 32, 3, 3, device=dev, generator=g) * 0.01
bo = torch.randn(54, device=dev, generator=g)
b = torch.randn(C, device=dev, generator=g)
p1, p3, po = ops.pack_weight_split(w1), ops.pack_weight_split(w3), ops.pack_weight_split(wo, 2)
if os.environ.get("AANET_PACK_F32") == "1":  # plain f32 packed weights (exact engine only)
    p1, p3, po = ops.pack_weight(w1), ops.pack_weight(w3), ops.pack_weight(wo)
om = ops.conv2d_fused(x, wo, bo, 1, 2, 2, 2, packed_weight=po)
p3h = ops.pack_weight_split(w3[:32].contiguous())
xn = x.contiguous(memory_format=torch.channels_last)
up1, up2 = res[:, :, :64, :208].contiguous(), res[:, :, :32, :104].contiguous()
up1f, up2f = up1, up2  # the CSA exchange terms of branch 0 (64 ch at 1/2 and 1/4 of the size)
fl = torch.randn(B, 128, H, W, device=dev, generator=g)
fr = torch.randn(B, 128, H, W, device=dev, generator=g)
vol64 = torch.randn(B, 64, H, W, device=dev, generator=g)
f5l = torch.randn(4, 32, 96, 312, device=dev, generator=g)
f5r = torch.randn(4, 32, 96, 312, device=dev, generator=g)
x1 = torch.randn(B, 64, H // 2, W // 2, device=dev, generator=g)    # scale 1, 64 ch (branch-2 chain)
x1b = torch.randn(B, 32, H // 2, W // 2, device=dev, generator=g)   # scale 1, 32 ch (block output)
w96 = torch.randn(96, C, 3, 3, device=dev, generator=g) * 0.04
b96 = torch.randn(96, device=dev, generator=g)
w16, w16b = w3[:16].contiguous(), w3[:16, :32].contiguous()
ws96, ws16, ws16b = ops.pack_conv3x3s2(w96), ops.pack_conv3x3s2(w16), ops.pack_conv3x3s2(w16b)
p16, p16b = ops.pack_weight_split(w16), ops.pack_weight_split(w16b)
b16 = b[:16].contiguous()
cases = {
    # CSA down convs: the merged scale-0 heads (64 -> 32 + 64) and the narrow 64/32 -> 16 convs
    "s2_heads96": (lambda: ops.conv3x3_s2(x, ws96, b96, 96, 32, None, "leaky"),
                   2 * B * (H // 2) * (W // 2) * 96 * C * 9),
    "s2_64to16": (lambda: ops.conv3x3_s2(x1, ws16, b16, 16, 16), 2 * B * (H // 4) * (W // 4) * 16 * 64 * 9),
    "s2_64to16_engine": (lambda: ops.conv2d_fused(x1, w16, b16, 2, 1, 1, 1, packed_weight=p16),
                         2 * B * (H // 4) * (W // 4) * 16 * 64 * 9),
    "s2_32to16": (lambda: ops.conv3x3_s2(x1b, ws16b, b16, 16, 16), 2 * B * (H // 4) * (W // 4) * 16 * 32 * 9),
    "s2_32to16_engine": (lambda: ops.conv2d_fused(x1b, w16b, b16, 2, 1, 1, 1, packed_weight=p16b),
                         2 * B * (H // 4) * (W // 4) * 16 * 32 * 9),
    "conv1x1": (lambda: ops.conv2d_fused(x, w1, b, act="relu", packed_weight=p1), 2 * B * H * W * C * C),
    "conv1x1_res": (lambda: ops.conv2d_fused(x, w1, b, act="relu", residual=res, packed_weight=p1),
                    2 * B * H * W * C * C),
    "conv3x3": (lambda: ops.conv2d_fused(x, w3, b, 1, 1, 1, 1, "relu", packed_weight=p3),
                2 * B * H * W * C * C * 9),
    "offset_conv": (lambda: ops.conv2d_fused(x, wo, bo, 1, 2, 2, 2, packed_weight=po),
                    2 * B * H * W * 54 * 32 * 9),
    "dcn_pw": (lambda: ops.mdcn_pw(x, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2, 2),
               2 * B * H * W * C * C * 10),
    "conv3x3_pw": (lambda: ops.conv2d_pw(x, w3, p3, b, None, None, "relu", p1, b, res, "relu", 1, 1, 1),
                   2 * B * H * W * C * C * 10),
    "dcn": (lambda: ops.mdcn_forward_fused(x, om, w3, None, b, b, "relu", 1, 2, 2, 2, 2.0,
                                           packed_weight=p3), 2 * B * H * W * C * C * 9),
    "conv1x1_onhwc": (lambda: ops.conv2d_fused(x, w1, b, act="relu", packed_weight=p1, out_nhwc=True),
                      2 * B * H * W * C * C),
    "conv3x3_nhwc": (lambda: ops.conv2d_fused(xn, w3, b, 1, 1, 1, 1, "relu", packed_weight=p3),
                     2 * B * H * W * C * C * 9),
    "offset_nhwc": (lambda: ops.conv2d_fused(xn, wo, bo, 1, 2, 2, 2, packed_weight=po),
                    2 * B * H * W * 54 * 32 * 9),
    "dcn_nhwc": (lambda: ops.mdcn_forward_fused(xn, om, w3, None, b, b, "relu", 1, 2, 2, 2, 2.0,
                                                packed_weight=p3), 2 * B * H * W * C * C * 9),
    "dcn_pw_nhwc": (lambda: ops.mdcn_pw(xn, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2, 2),
                    2 * B * H * W * C * C * 10),
    "conv3x3_pw_nhwc": (lambda: ops.conv2d_pw(xn, w3, p3, b, None, None, "relu", p1, b, res, "relu", 1, 1, 1),
                        2 * B * H * W * C * C * 10),
    "csa_sum": (lambda: ops.csa_sum([x, up1, up2]), 0),
    "dcn_pw_nhwc_csa": (lambda: ops.mdcn_pw(xn, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2, 2, 2,
                                            csa_up=[up1f, up2f]), 2 * B * H * W * C * C * 10),
    "dcn_pw_nhwc_csa_generic": (lambda: ops.mdcn_pw(xn, om, w3, p3, None, b, b, "relu", p1, b, res, "relu", 1, 2,
                                                    2, 2, csa_up=[up1f, up2f], generic_dcn=True),
                                2 * B * H * W * C * C * 10),
    "conv3x3_pw_nhwc_csa": (lambda: ops.conv2d_pw(xn, w3, p3, b, None, None, "relu", p1, b, res, "relu", 1, 1, 1,
                                                  csa_up=[up1f, up2f]), 2 * B * H * W * C * C * 10),
    # the fusion layers' scale 0 -> 1 exchange convs (3x3 stride 2, NCHW input)
    "conv3x3_s2_64": (lambda: ops.conv2d_fused(x, w3, b, 2, 1, 1, 1, "leaky", packed_weight=p3),
                      2 * B * (H // 2) * (W // 2) * C * C * 9),
    "conv3x3_s2_32": (lambda: ops.conv2d_fused(x, w3[:32].contiguous(), b[:32].contiguous(), 2, 1, 1, 1,
                                               packed_weight=p3h), 2 * B * (H // 2) * (W // 2) * 32 * C * 9),
    "conv3x3_s2_64_nhwc": (lambda: ops.conv2d_fused(xn, w3, b, 2, 1, 1, 1, "leaky", packed_weight=p3,
                                                    out_nhwc=True), 2 * B * (H // 2) * (W // 2) * C * C * 9),
    "conv3x3_s2_32_nhwc": (lambda: ops.conv2d_fused(xn, w3[:32].contiguous(), b[:32].contiguous(), 2, 1, 1, 1,
                                                    packed_weight=p3h, out_nhwc=True),
                           2 * B * (H // 2) * (W // 2) * 32 * C * 9),
    "conv1x1_in_nhwc": (lambda: ops.conv2d_fused(xn, w1, b, act="relu", packed_weight=p1, out_nhwc=True),
                        2 * B * H * W * C * C),
    "corr": (lambda: ops.corr_volume(fl, fr, 64), 0),
    "regress": (lambda: ops.disp_regress(vol64), 0),
    # C5 (PSMNet 4-D volume, 384x1248 -> 1/4: [B,32,96,312], D=192/4=48), B=4
    "concat": (lambda: ops.shift_volume(f5l, f5r, 48, True), 0),
    "diff": (lambda: ops.shift_volume(f5l, f5r, 48, False), 0),
}
for name, (fn, flops) in cases.items():
    if names and name not in names:
        continue
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / iters
    gbs = {"corr": 4 * (2 * B * 128 * H * W + B * 64 * H * W), "regress": 4 * (B * 64 * H * W + B * H * W),
           "csa_sum": 4 * (2 * B * C * H * W + B * C * H * W * 5 // 16),
           "concat": 4 * (2 * 4 * 32 * 96 * 312 + 4 * 64 * 48 * 96 * 312),
           "diff": 4 * (2 * 4 * 32 * 96 * 312 + 4 * 32 * 48 * 96 * 312)}.get(name)
    rate = f"{gbs / ms / 1e6:6.0f} GB/s" if gbs else f"{flops / ms / 1e9:6.1f} TF/s"
    print(f"{name:12s} {ms * 1e3:8.1f} us  {rate}")
