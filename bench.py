#!/usr/bin/env python3
"""bench.py -- AANet cost-volume hot path on MI355X: stereo-pairs/s @384x1248, D=64, fp32.

One step = the north-star path over one batch of B=8 synthetic stereo pairs per GPU, inputs
resident in HBM: CostVolumePyramid (correlation, D=64/32/16) -> AdaptiveAggregation
(6 fusions, 3 deformable, eval, no intermediate supervision) -> DisparityEstimation.
Features are the 1/3, 1/6, 1/12 pyramids of a 384x1248 pair: [8,128,128,416], [8,128,64,208],
[8,128,32,104] (BASELINE.json configs[1]).  Random-init weights of that architecture
(offset_conv nonzero), synthetic N(0,1) features: there is no network for data/checkpoints.

Launch: `python bench.py [--gpus N --steps K --warmup W]`.  For N>1 it either runs under
torch.distributed.run (RANK/WORLD_SIZE set) or starts the N rank processes itself
(launch_ranks; one process per GPU, RCCL).  Pairs are sharded across ranks with no data-path collective
(weak scaling); one all_gather of a per-rank metrics record at the end.  Rank 0 prints ONE
JSON line.  `roofline` is measured live (HIP events on the launch stream) for the dominant
HIP kernel; `cpu_baseline` times the CPU oracle (port of the reference path) on one pair.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "stereo-pairs/s @384x1248 D=64 fp32, 1/2/4/8 MI355X; EPE vs ref"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec
STORE_CEILING_GBS = 6490.0  # measured store-only ceiling (profiles/r06_write_ceiling.txt: hipMemsetAsync)
FP32_MFMA_PEAK_TF = 157.3  # MI355X_MICROARCH.md: v_mfma_f32_16x16x4_f32 = f32 vector rate
BF16_DENSE_PEAK_TF = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (no sparsity)
L2_GATHER_GBPS = 17800.0     # MI355X_MICROARCH.md "Indexed rows": L2-served gather, 16.8-18.8 TB/s
# The conv engine's split-bf16 contraction (include/aanet_mi355x.h AANET_CONV_EXACT_F32) runs an
# fp32 MAC as six bf16 piece products on the matrix cores: its ceiling in fp32-equivalent FLOP/s
# is the dense bf16 peak / 6.  The exact f32 engine (--exact-f32) is bounded by FP32_MFMA_PEAK_TF.
SPLIT_PEAK_TF = BF16_DENSE_PEAK_TF / 6
H_IMG, W_IMG, MAXD_IMG = 384, 1248, 192
MAXD = MAXD_IMG // 3       # cost-volume disparities at 1/3 resolution (nets/aanet.py:56-59)
FEAT_C = 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=8, help="stereo pairs per GPU")
    ap.add_argument("--no-graph", action="store_true", help="time eager launches, not a HIP graph")
    ap.add_argument("--graph", action="store_true",
                    help="time the HIP-graph replay even when eager launches probe faster")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--kernel-iters", type=int, default=50)
    ap.add_argument("--features", default="randn", choices=sorted(FEATURE_KINDS),
                    help="synthetic feature variant (SURVEY.md §8d)")
    ap.add_argument("--train", action="store_true",
                    help="time the training step (fwd+bwd+Adam, SyncBN+DDP for N>1) instead")
    ap.add_argument("--train-batch", type=int, default=4, help="training pairs per GPU")
    ap.add_argument("--engine-convs", choices=("auto", "on", "off"), default="auto",
                    help="--train: plain convs on the HIP engine (auto: with --deterministic)")
    ap.add_argument("--deterministic", action="store_true",
                    help="--train with torch.use_deterministic_algorithms (det DCN backward)")
    ap.add_argument("--img", default=None,
                    help="--model: image HxW (default 384x1248, KITTI; BASELINE C3 is 576x960)")
    ap.add_argument("--model", default=None, choices=sorted(FULL_MODELS),
                    help="time the full model (features + hot path + refinement) instead")
    ap.add_argument("--exact-f32", action="store_true",
                    help="conv engine on exact f32 MFMA instead of the split-bf16 contraction")
    ap.add_argument("--dcn-sweep", action="store_true",
                    help="C4: deform_conv2d forward + backward microbench over the aggregation / "
                         "feature-extractor DCN shapes (secondary lines, not the headline)")
    ap.add_argument("--dcn-shapes", default=None, help="--dcn-sweep: comma-separated subset of DCN_SHAPES")
    ap.add_argument("--plumbing", action="store_true",
                    help="launcher/record/gather plumbing only: gloo on CPU, a stand-in CPU step "
                         "(tests/test_distributed.py); never a metric")
    ap.add_argument("--only", default=None,
                    help="profiling mode: run only one kernel family (corr|mdcn|regress|step)")
    ap.add_argument("--option", action="append", default=[], metavar="NAME=VALUE",
                    help="eval schedule option of the model (aanet_amd/nets/options.py), e.g. "
                         "side_heads=false; repeatable (A/B runs; recorded in config.options)")
    return ap.parse_args()


def parse_options(items):
    """--option NAME=VALUE list -> set_options kwargs (true/false -> bool)."""
    out = {}
    for it in items:
        k, _, v = it.partition("=")
        out[k] = {"true": True, "false": False}.get(v.lower(), int(v) if v.isdigit() else v)
    return out


def build_model(device, intermediate_supervision=False):
    from aanet_amd.nets import AANetHotPath
    torch.manual_seed(0)  # identical weights on every rank
    m = AANetHotPath(MAXD, feature_similarity="correlation", num_scales=3, num_fusions=6,
                     deformable_groups=2, mdconv_dilation=2,
                     no_intermediate_supervision=not intermediate_supervision,
                     num_stage_blocks=1, num_deform_blocks=3)
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for name, mod in m.named_modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.copy_(0.05 * torch.randn(mod.num_features, generator=g))
                mod.running_var.copy_(0.8 + 0.4 * torch.rand(mod.num_features, generator=g))
            if name.endswith("offset_conv"):
                mod.weight.normal_(0.0, 0.01, generator=g)   # nonzero, std 0.01
                mod.bias.normal_(0.0, 0.5, generator=g)
    return m.to(device).eval()


FEATURE_KINDS = {
    "randn": "N(0,1) feature pyramids",
    "relu": "post-ReLU |N(0,1)| feature pyramids",
    "structured": "random texture, right = left shifted by a known per-row disparity in [0,63] "
                  "at 1/3 scale (2x2-average-pooled for 1/6, 1/12), so the softmax is peaked",
}


def make_features(batch, rank, device, kind="randn", img=(H_IMG, W_IMG)):
    """SURVEY.md §8(d) primary timed unit: seeded (1234 + rank) on-device feature pyramids."""
    gen = torch.Generator(device=device).manual_seed(1234 + rank)
    shapes = [(batch, FEAT_C, (img[0] // 3) >> s, (img[1] // 3) >> s) for s in range(3)]
    if kind in ("randn", "relu"):
        left = [torch.randn(s, device=device, generator=gen) for s in shapes]
        right = [torch.randn(s, device=device, generator=gen) for s in shapes]
        if kind == "relu":
            left, right = [t.abs_() for t in left], [t.abs_() for t in right]
        return left, right
    if kind != "structured":
        raise SystemExit(f"unknown --features {kind}")
    B, C, H, W = shapes[0]
    tex = torch.randn((B, C, H, W + MAXD), device=device, generator=gen)
    d = torch.randint(0, MAXD, (B, 1, H, 1), device=device, generator=gen)
    x = torch.arange(W, device=device).view(1, 1, 1, W)
    left0 = tex[..., MAXD:].contiguous()                       # L(x) = T(x + MAXD)
    idx = (x + MAXD - d).expand(B, C, H, W)                    # R(x) = T(x + MAXD - d) = L(x - d)
    right0 = torch.gather(tex, 3, idx).contiguous()
    left, right = [left0], [right0]
    for _ in range(2):
        left.append(torch.nn.functional.avg_pool2d(left[-1], 2).contiguous())
        right.append(torch.nn.functional.avg_pool2d(right[-1], 2).contiguous())
    return left, right


def time_events(fn, iters, stream, warm_ms=30.0):
    """Average launch duration of fn's kernel(s) over `iters` back-to-back launches on `stream`,
    after at least `warm_ms` of untimed launches of the same fn: an idle GPU clocks down, and a
    20-launch window right after host-side work read the correlation pyramid 35 % slow (bench
    r03: 172 us vs 127 us steady; tools/corr_lab2.hip rounds 0 vs 1-3)."""
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    while (time.perf_counter() - t0) * 1e3 < warm_ms:
        for _ in range(4):
            fn()
        torch.cuda.synchronize()
    start.record(stream)
    for _ in range(iters):
        fn()
    end.record(stream)
    torch.cuda.synchronize()
    return start.elapsed_time(end) / iters  # ms


def time_graph(fn, iters, stream, reps=3):
    """Per-launch device time of fn with the host out of the loop: `iters` calls captured in one
    HIP graph, replayed `reps` times between HIP events (for launches shorter than their Python
    call, which time_events would measure instead).  fn must not allocate per call."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=stream):
        for _ in range(iters):
            fn()
    start, end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    torch.cuda.synchronize()
    start.record(stream)
    for _ in range(reps):
        g.replay()
    end.record(stream)
    torch.cuda.synchronize()
    return start.elapsed_time(end) / (iters * reps)


def kernel_rooflines(model, left, right, batch, iters):
    """Per-kernel average duration (HIP events on the launch stream) and roofline fractions."""
    from aanet_amd import ops
    from aanet_amd.nets._fuse import bn_affine, conv_bn_act, folded
    stream = torch.cuda.current_stream()
    res = {}
    # correlation, scale 0 (one launch): algorithmic bytes = read L,R once + write volume
    B, C, H, W = left[0].shape
    corr_bytes = 4 * (2 * B * C * H * W + B * MAXD * H * W)
    ms = time_events(lambda: ops.corr_volume(left[0], right[0], MAXD), iters, stream)
    res["corr_volume_s0"] = dict(bound="hbm", ms=ms, algo=corr_bytes, unit="GB/s",
                                 achieved=corr_bytes / ms / 1e6, peak=HBM_PEAK_GBS)
    # the whole correlation pyramid in one launch (CostVolumePyramid, nets/cost.py:58-76)
    pyr_bytes = sum(4 * (2 * B * C * (H >> s) * (W >> s) + B * (MAXD >> s) * (H >> s) * (W >> s))
                    for s in range(len(left)))
    ms = time_events(lambda: ops.corr_pyramid(left, right, MAXD), iters, stream)
    res["corr_pyramid"] = dict(bound="hbm", ms=ms, algo=pyr_bytes, unit="GB/s",
                               achieved=pyr_bytes / ms / 1e6, peak=HBM_PEAK_GBS)
    # regression, scale 0
    vol = ops.corr_volume(left[0], right[0], MAXD)
    reg_bytes = 4 * (B * MAXD * H * W + B * H * W)
    ms = time_events(lambda: ops.disp_regress(vol), iters, stream)
    res["disp_regress_s0"] = dict(bound="hbm", ms=ms, algo=reg_bytes, unit="GB/s",
                                  achieved=reg_bytes / ms / 1e6, peak=HBM_PEAK_GBS)
    # the bottleneck conv1 (1x1 + BN + ReLU, NCHW in -> channels-last out; pointwise.hip), scale 0:
    # algorithmic bytes = read the 64-channel input once + write the 64-channel output once
    blk1 = model.aggregation.fusions[5].branches[0][0]
    with torch.no_grad():
        w1, b1, p1 = folded(blk1.conv1, blk1.bn1)
        ms = time_events(lambda: ops.conv2d_fused(vol, w1, b1, act="relu", packed_weight=p1,
                                                  out_nhwc=True), iters, stream)
    pw_bytes = 4 * B * H * W * (w1.shape[1] + w1.shape[0])
    res["conv1x1_s0"] = dict(bound="hbm", ms=ms, algo=pw_bytes, unit="GB/s",
                             achieved=pw_bytes / ms / 1e6, peak=HBM_PEAK_GBS)
    # modulated DCN as the hot path runs it (DeformSimpleBottleneck of the last fusion, scale 0):
    # NHWC conv1 output in, DCN + BN2 + ReLU -> conv3 + BN3 + identity + ReLU -> block output and
    # the scale-0 cross-scale sum, in one kernel
    blk = model.aggregation.fusions[5].branches[0][0]
    with torch.no_grad():
        x1 = conv_bn_act(vol, blk.conv1, blk.bn1, "relu", out_nhwc=True)
        c2 = blk.conv2
        dc = c2.deform_conv
        om = conv_bn_act(x1, c2.offset_conv)
        ps, psh = bn_affine(blk.bn2)
        wp = folded(dc, None)[2]
        w3, b3, p3 = folded(blk.conv3, blk.bn3)
        # the CSA epilogue's coarser exchange terms (2x and 4x smaller), as in the module
        ups = [torch.randn(B, w3.shape[0], H // r, W // r, device=vol.device) for r in (2, 4)]
        fn = lambda: ops.mdcn_pw(x1, om, dc.weight, wp, dc.bias, ps, psh, "relu", p3, b3, vol,  # noqa: E731
                                 "relu", 1, dc.padding, dc.dilation, c2.deformable_groups, 2.0,
                                 csa_up=ups)
        ms = time_events(fn, iters, stream)
    Co, Ci = dc.weight.shape[:2]
    Co2 = w3.shape[0]
    flops = 2.0 * B * H * W * (Co * Ci * 9 + Co2 * Co)
    # the contraction runs on the engine's selected form (split-bf16 unless --exact-f32); its
    # tighter bound is the corner gather: 9 taps x Ci channels x 4 corners x 4 B per output
    # pixel, mostly L1/L2 hits, against the L2-served gather rate of MI355X_MICROARCH.md
    gather = 4.0 * 4 * 9 * Ci * B * H * W
    res["mdcn_pw_s0"] = dict(bound="mfma", ms=ms, algo=flops, unit="TFLOP/s",
                             achieved=flops / ms / 1e9, peak=conv_peak(),
                             gather={"bytes_per_launch": gather, "achieved_GBps": gather / ms / 1e6,
                                     "peak_GBps": L2_GATHER_GBPS,
                                     "frac": gather / ms / 1e6 / L2_GATHER_GBPS})
    # the plain-3x3 ISA bottleneck tail (SimpleBottleneck of fusion 0, scale 0): halo-tile conv2
    # + BN2 + ReLU -> conv3 + BN3 + identity + ReLU, with the scale-0 CSA sum
    blk0 = model.aggregation.fusions[0].branches[0][0]
    with torch.no_grad():
        x1 = conv_bn_act(vol, blk0.conv1, blk0.bn1, "relu", out_nhwc=True)
        w2, b2, p2 = folded(blk0.conv2, blk0.bn2)
        w3, b3, p3 = folded(blk0.conv3, blk0.bn3)
        fn = lambda: ops.conv2d_pw(x1, w2, p2, b2, None, None, "relu", p3, b3, vol, "relu",  # noqa: E731
                                   1, 1, 1, csa_up=ups)
        ms = time_events(fn, iters, stream)
    flops = 2.0 * B * H * W * (w2.shape[0] * w2.shape[1] * 9 + w3.shape[0] * w3.shape[1])
    res["conv3x3_pw_s0"] = dict(bound="mfma", ms=ms, algo=flops, unit="TFLOP/s",
                                achieved=flops / ms / 1e9, peak=conv_peak())
    # the offset_conv of the scale-0 deformable block (3x3, dilation 2, 2 groups, 64 -> 54, on the
    # channels-last conv1 output), on the path the step takes (nets/_fuse.offset_conv_eval)
    from aanet_amd.nets._fuse import offset_conv_eval
    oc = blk.conv2.offset_conv
    with torch.no_grad():
        x1 = conv_bn_act(vol, blk.conv1, blk.bn1, "relu", out_nhwc=True)
        ms = time_events(lambda: offset_conv_eval(x1, oc), iters, stream)
    flops = 2.0 * B * H * W * oc.out_channels * (oc.in_channels // oc.groups) * 9
    res["offset_conv_s0"] = dict(bound="mfma", ms=ms, algo=flops, unit="TFLOP/s",
                                 achieved=flops / ms / 1e9, peak=conv_peak())
    # the scale-0 heads launch of the CSA exchange (conv_s2.hip: the 64 -> 32 branch-1 conv with
    # branch 1's CSA sum in its epilogue + the 64 -> 64 first conv of the branch-2 chain, 3x3
    # stride 2), as AdaptiveAggregationModule._heads_sum1 runs it (fusion 4: the last one has a
    # single output branch)
    agg = model.aggregation.fusions[4]
    if agg._s2_sums_ok([vol, torch.empty(B, 32, (H + 1) // 2, (W + 1) // 2, device=vol.device),
                        torch.empty(B, 16, (H + 3) // 4, (W + 3) // 4, device=vol.device)]):
        x1s = torch.randn(B, 32, (H + 1) // 2, (W + 1) // 2, device=vol.device)
        t12 = torch.randn(B, 32, (H + 3) // 4, (W + 3) // 4, device=vol.device)
        with torch.no_grad():
            ms = time_events(lambda: agg._heads_sum1(vol, x1s, t12), iters, stream)
        flops = 2.0 * B * ((H + 1) // 2) * ((W + 1) // 2) * 96 * 64 * 9
        res["s2_heads_s0"] = dict(bound="mfma", ms=ms, algo=flops, unit="TFLOP/s",
                                  achieved=flops / ms / 1e9, peak=conv_peak())
    # BASELINE configs[4] (PSMNet-AA / GwcNet-AA, nets/cost.py:31-38): the concat volume of one
    # 384x1248 pair's PSMNet features [B,32,96,312] at D = 192/4 = 48, HBM write-bound:
    # algorithmic bytes = read 2 x 32 x 96 x 312 x 4 + write 64 x 48 x 96 x 312 x 4 = 375.7 MB
    # per pair; timed at B = 4 pairs (1.5 GB written per launch)
    Bc, Cc, Hc, Wc, Dc = 4, 32, H_IMG // 4, W_IMG // 4, MAXD_IMG // 4
    gc = torch.Generator(device=left[0].device).manual_seed(5)
    lc = torch.randn(Bc, Cc, Hc, Wc, device=left[0].device, generator=gc)
    rc = torch.randn(Bc, Cc, Hc, Wc, device=left[0].device, generator=gc)
    cc_bytes = 4 * (2 * Bc * Cc * Hc * Wc + Bc * 2 * Cc * Dc * Hc * Wc)
    ms = time_events(lambda: ops.shift_volume(lc, rc, Dc, True), iters, stream)
    res["concat_volume_c5"] = dict(bound="hbm", ms=ms, algo=cc_bytes, unit="GB/s",
                                   achieved=cc_bytes / ms / 1e6, peak=HBM_PEAK_GBS,
                                   pairs=Bc, bytes_per_pair=cc_bytes / Bc, in_step=False)
    # 92% of its bytes are stores: priced also against the store ceiling measured on this part
    # (tools/write_ceiling.hip, profiles/r06_write_ceiling.txt: hipMemsetAsync 6.49 TB/s, the best
    # kernel store pattern 6.19 TB/s), which is what a write-bound kernel can reach
    res["concat_volume_c5"]["store_ceiling_GBps"] = STORE_CEILING_GBS
    res["concat_volume_c5"]["frac_of_store_ceiling"] = cc_bytes / ms / 1e6 / STORE_CEILING_GBS
    del lc, rc
    for v in res.values():
        v["frac"] = v["achieved"] / v["peak"]
    return res


def conv_contraction():
    from aanet_amd import _lib
    if _lib.conv_flags():
        return "exact f32 MFMA (v_mfma_f32_16x16x4_f32)"
    return ("fp32 operands split into three exact bf16 pieces, six v_mfma_f32_16x16x32_bf16 "
            "products, fp32 accumulation (fp32-accurate; tests/test_gpu_split.py)")


def peak_basis(dom):
    if dom["unit"] != "TFLOP/s":
        return "HBM 8.0 TB/s spec"
    if dom["peak"] == FP32_MFMA_PEAK_TF:
        return "f32 MFMA 157.3 TF/s"
    return ("split-bf16 contraction: dense bf16 MFMA 2.5 PF/s / 6 products = 416.7 TF/s "
            "fp32-equivalent (the native f32 MFMA peak is 157.3)")


def conv_peak():
    from aanet_amd import _lib
    return FP32_MFMA_PEAK_TF if _lib.conv_flags() else SPLIT_PEAK_TF


CPU_SAMPLE_S = 12.0  # seconds of CPU work in the cpu_baseline sample


def _oracle_inputs(model, left, right, count=None):
    sd = {k: v.detach().cpu().numpy() for k, v in model.aggregation.state_dict().items()}
    B = left[0].shape[0] if count is None else min(count, left[0].shape[0])
    pairs = [([t[i:i + 1].cpu().numpy() for t in left], [t[i:i + 1].cpu().numpy() for t in right])
             for i in range(B)]
    return sd, pairs


def _oracle_disp(sd, pair):
    from oracle import aggregation as oagg  # checker only
    return oagg.hot_path(pair[0], pair[1], sd, MAXD, intermediate_supervision=False)[0]


def parity_vs_oracle(model, left, right, gpu_disp):
    """SURVEY.md §8(e) per-rank parity payload: this rank's GPU disparity of its pair 0 against
    the CPU oracle (restated reference path) on the same input -> (sum|dd|, max|dd|, n_px,
    oracle seconds)."""
    sd, pairs = _oracle_inputs(model, left, right, count=1)
    t0 = time.perf_counter()
    ref = _oracle_disp(sd, pairs[0])
    dt = time.perf_counter() - t0
    ours = gpu_disp[:1].cpu().numpy()
    diff = np.abs(ours.astype(np.float64) - ref.astype(np.float64))
    return float(diff.sum()), float(diff.max()), float(diff.size), dt


def host_cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(model, left, right):
    """Time the CPU oracle (restated reference path) on a bounded sample of the batch's pairs
    (pairs 0, 1, ... cyclically until >= CPU_SAMPLE_S seconds of CPU work, at least 2 pairs).

    Threads: every core of os.sched_getaffinity(0), capped at this process's CPU
    share when the launcher sets one (OMP_NUM_THREADS; 16 per GPU on the one-GPU boxes, whose
    affinity mask lists the whole 8-GPU host's 256 cores: threads past the share only
    oversubscribe it).  `cores` is the thread count actually used; `affinity_cores` the mask."""
    affinity = len(os.sched_getaffinity(0))
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(affinity, share) if share > 0 else affinity
    prev_threads = torch.get_num_threads()
    torch.set_num_threads(threads)
    sd, pairs = _oracle_inputs(model, left, right)
    n = 0
    t0 = time.perf_counter()
    while n < 2 or time.perf_counter() - t0 < CPU_SAMPLE_S:
        _oracle_disp(sd, pairs[n % len(pairs)])
        n += 1
    dt = time.perf_counter() - t0
    torch.set_num_threads(prev_threads)
    return dict(value=n / dt, unit="stereo-pairs/s", cores=threads, kind="port",
                cpu_model=host_cpu_model(), affinity_cores=affinity,
                threads_basis=("OMP_NUM_THREADS (this process's CPU share)" if share > 0 and share < affinity
                               else "os.sched_getaffinity(0)"),
                sample=f"{n} pairs of the C2 workload (features 128x128x416 pyramid, D=64), "
                       f"{dt:.1f} s on {threads} threads: oracle/ C restatement (cost volume, DCN, "
                       "regression) + torch-CPU convs", seconds=dt)


def _time_calls(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n


def timed_run(step, args, world):
    """W warmup steps, optional HIP-graph capture of one step, then exactly K timed steps between
    barrier + synchronize pairs.  -> (last output, elapsed seconds, graph or None).

    The graph replay is not always the faster schedule: ROCm's graph executor maps the captured
    multi-stream DAG onto its own queues, and on the eval aggregation it lost most of the
    concurrent-scale overlap (3.91-3.93 ms vs 3.76 ms eager on the same box,
    the round-2 schedule A/B, in git history as tools/ab_schedules.sh).  So after capture untimed replays and eager steps are probed (5 alternating
    rounds of 5, best of each)
    and the faster one is timed (--graph / --no-graph force one); args.schedule records it."""
    for _ in range(args.warmup):
        out = step()
    torch.cuda.synchronize()
    graph = None
    if not args.no_graph:
        try:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    out = step()
            torch.cuda.current_stream().wait_stream(s)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                out = step()
            torch.cuda.synchronize()
        except Exception as e:  # capture unsupported by some library op: time eager launches
            print(f"hip graph capture failed ({e}); timing eager launches", file=sys.stderr)
            graph = None
            torch.cuda.synchronize()
    run = graph.replay if graph is not None else step
    args.schedule = {"timed": "hip_graph" if graph is not None else "eager"}
    if graph is not None and not getattr(args, "graph", False):
        # alternating rounds, best of each: one short probe per schedule is noisier than the
        # few-percent difference it decides
        tg = te = float("inf")
        for _ in range(5):
            tg = min(tg, _time_calls(graph.replay, 5))
            te = min(te, _time_calls(step, 5))
        args.schedule = {"graph_probe_ms": round(tg * 1e3, 4), "eager_probe_ms": round(te * 1e3, 4)}
        if te < tg:
            run, graph = step, None
        args.schedule["timed"] = "hip_graph" if graph is not None else "eager"
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = run()
        if r is not None:  # eager step output (a graph replay returns None: out is its buffer)
            out = r
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    return out, time.perf_counter() - t0, graph


def _free_port():
    import socket
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(n, argv):
    """`bench.py --gpus N` without an external launcher: start N rank processes of this script
    (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on 127.0.0.1), one per GPU, the
    way torch.distributed.run would (reference: train.py:113-123 under torch.distributed.launch).
    The parent never touches the GPU.  Rank 0 prints the JSON line (inherited stdout).  If one
    rank fails, the others are terminated (exact PIDs) so no rank waits in a collective forever.
    -> exit code (the first non-zero child code, else 0)."""
    import subprocess
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:  # a dead rank leaves the others blocked in a collective
                    q.terminate()
        time.sleep(0.05)
    return rc


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
    if args.plumbing:
        plumbing_main(args, rank, world)
        return
    device = torch.device("cuda", local_rank)
    torch.cuda.set_device(device)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    if args.exact_f32:
        from aanet_amd import _lib
        _lib.set_exact_f32(True)

    if args.train:
        train_main(args, device, rank, world)
        return
    if args.model:
        model_main(args, device, rank, world)
        return
    if args.dcn_sweep:
        dcn_sweep_main(args, device, rank)
        return
    model = build_model(device)
    opts = parse_options(args.option)
    if opts:
        model.set_options(**opts)
    left, right = make_features(args.batch, rank, device, args.features)

    def step():
        with torch.no_grad():
            return model(left, right)[0]

    if args.only:
        profile_only(args, model, left, right, step)
        return

    out, elapsed, graph = timed_run(step, args, world)
    disp = out  # graph output buffer (or last eager output)

    # per-rank parity payload (this rank's pair 0 vs the CPU oracle), outside the timed region
    sum_err, max_err, n_px, _ = parity_vs_oracle(model, left, right, disp)
    from aanet_amd import dist as adist
    record = adist.make_record(device, pairs=args.batch * args.steps, elapsed_s=elapsed,
                               sum_abs_err=sum_err, max_abs_err=max_err, n_px=n_px,
                               disp_min=float(disp.min()), disp_max=float(disp.max()))
    records = adist.gather_records(record)  # the one collective (metrics only)
    summary = adist.summarize(records)
    total_pairs, t_max = summary["pairs"], summary["elapsed_max_s"]

    if rank == 0:
        roof = kernel_rooflines(model, left, right, args.batch, args.kernel_iters)
        # the dominant kernel of the timed C2 step (the C5 concat line is a separate config)
        dom_name = max((k for k in roof if roof[k].get("in_step", True)), key=lambda k: roof[k]["ms"])
        dom = roof[dom_name]
        traffic = load_traffic(dom_name)
        line = {
            "metric": METRIC,
            "value": total_pairs / t_max,
            "unit": "stereo-pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * t_max / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "contraction": conv_contraction(),
            "data": f"synthetic ({FEATURE_KINDS[args.features]} on device, seeded per rank; "
                    "random-init weights)",
            "config": {
                "workload": "C2: KITTI 384x1248 stereo pairs, features 128ch at 1/3,1/6,1/12, "
                            "correlation volume D=64/32/16 -> AdaptiveAggregation (6 fusions, 3 "
                            "deformable, eval) -> soft-argmin",
                "batch_per_gpu": args.batch,
                "global_batch": args.batch * world,
                "parallelism": f"dp{world} (pairs sharded, no data-path collective)",
                "hip_graph": graph is not None, "schedule": getattr(args, "schedule", None),
                **({"options": parse_options(args.option)} if args.option else {}),
            },
            "roofline": {"kernel": dom_name, "bound": dom["bound"], "achieved": dom["achieved"],
                         "peak": dom["peak"], "unit": dom["unit"], "frac": dom["frac"],
                         "traffic": traffic, "ms_per_launch": dom["ms"],
                         "algorithmic_per_launch": dom["algo"],
                         "peak_basis": peak_basis(dom),
                         **({"gather": dom["gather"]} if "gather" in dom else {})},
            "kernels": {k: {kk: v[kk] for kk in ("bound", "ms", "achieved", "unit", "frac", "gather",
                                                 "pairs", "bytes_per_pair", "store_ceiling_GBps",
                                                 "frac_of_store_ceiling")
                            if kk in v}
                        for k, v in roof.items()},
            # EPE vs ref: mean / max |dd| of every rank's pair 0 against the CPU oracle
            "epe_vs_ref": summary["epe"],
            "max_abs_disp_err_vs_ref": summary["max_abs_err"],
            "parity_pairs": len(records),
            "per_rank": [{"pairs": r[0], "elapsed_s": r[1], "max_abs_err": r[3]}
                         for r in records.tolist()],
        }
        if not args.no_cpu_baseline and world == 1:  # the CPU baseline is an N=1 figure only
            line["cpu_baseline"] = cpu_baseline(model, left, right)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def plumbing_main(args, rank, world):
    """--plumbing: the multi-rank launch, per-rank record, all_gather and max-over-ranks clock of
    the real bench, on CPU with gloo and a stand-in step (a CPU matmul per pair), so the N>1
    path is covered where there is no GPU (tests/test_distributed.py).  Not a measurement."""
    if world > 1:
        dist.init_process_group("gloo")
    if os.environ.get("AANET_PLUMBING_FAIL_RANK") == str(rank):  # launcher failure test
        raise SystemExit(3)
    from aanet_amd import dist as adist
    g = torch.Generator().manual_seed(1234 + rank)
    a = torch.randn(64, 64, generator=g)
    t0 = time.perf_counter()
    for _ in range(args.warmup + args.steps):
        for _ in range(args.batch):
            a = torch.tanh(a @ a)
    elapsed = time.perf_counter() - t0 + 0.01 * rank  # distinct per rank: the max must win
    rec = adist.make_record("cpu", pairs=args.batch * args.steps, elapsed_s=elapsed,
                            sum_abs_err=0.0, max_abs_err=1e-6 * (rank + 1), n_px=1.0)
    records = adist.gather_records(rec)
    summary = adist.summarize(records)
    if rank == 0:
        print(json.dumps({"metric": "plumbing (not a measurement)", "n_gpus": world,
                          "value": summary["pairs"] / summary["elapsed_max_s"],
                          "pairs": summary["pairs"], "elapsed_max_s": summary["elapsed_max_s"],
                          "max_abs_disp_err_vs_ref": summary["max_abs_err"],
                          "per_rank": [{"pairs": r[0], "elapsed_s": r[1]} for r in records.tolist()]}),
              flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


# (name, C, H, W, stride) -- the AdaptiveAggregation DCN at its three scales
# (C2 sizes) and AANetFeature layer3's DeformBottleneck DCNs (128 ch at 1/12, stride 1 and 2).
# All deformable_groups=2, 3x3, dilation 2, padding 2, no bias (nets/deform.py:17-45).
DCN_SHAPES = [("agg_s0", 64, 128, 416, 1), ("agg_s1", 32, 64, 208, 1), ("agg_s2", 16, 32, 104, 1),
              ("feat_s1", 128, 32, 104, 1), ("feat_s2", 128, 64, 208, 2)]


def dcn_sweep_main(args, device, rank):
    """C4 microbench: the modulated DCN op (ops.mdcn_forward = the reference's
    modulated_deform_conv_cuda_forward: the LDS-window kernel for the aggregation's scale-0/1
    shapes, the direct kernel (dcn_small.hip) for scale 2, `fwd_generic_us` the generic
    implicit-GEMM engine; aanet_mdcn_bwd_f32 / _det_f32 =
    ..._backward) per shape,
    B=--batch, offsets N(0, 0.5^2) (fractional, some out of the image), mask U(0, 1).
    Forward times are per-launch device times from HIP-graph replays (`fwd_eager_call_us`: the
    eager per-call time, host launch overhead included); backward times are eager.
    Flops: forward 2*B*Ho*Wo*Co*C*9 (the MFMA contraction; bilinear lerps excluded); backward
    counts dgrad + wgrad contractions (2x the forward).  One JSON line per shape on rank 0, then
    the num_scales 1 / 3 aggregation totals."""
    from aanet_amd import ops
    B, dg, k, dil, pad = args.batch, 2, 3, 2, 2
    gen = torch.Generator(device=device).manual_seed(1234 + rank)
    stream = torch.cuda.current_stream()
    iters = max(args.kernel_iters, 5)
    tot = {}
    pick = args.dcn_shapes.split(",") if args.dcn_shapes else None
    for name, C, H, W, stride in DCN_SHAPES:
        if pick and name not in pick:
            continue
        Ho, Wo = (H + 2 * pad - dil * (k - 1) - 1) // stride + 1, (W + 2 * pad - dil * (k - 1) - 1) // stride + 1
        x = torch.randn((B, C, H, W), device=device, generator=gen)
        off = 0.5 * torch.randn((B, 2 * dg * k * k, Ho, Wo), device=device, generator=gen)
        mask = torch.rand((B, dg * k * k, Ho, Wo), device=device, generator=gen)
        w = 0.05 * torch.randn((C, C, k, k), device=device, generator=gen)
        out = torch.empty((B, C, Ho, Wo), device=device)
        go = torch.randn((B, C, Ho, Wo), device=device, generator=gen)
        fwd = lambda: ops.mdcn_forward(x, off, mask, w, None, stride, pad, dil, 1, dg, out=out)  # noqa: E731
        fwd_gen = lambda: ops.mdcn_forward(x, off, mask, w, None, stride, pad, dil, 1, dg, out=out,  # noqa: E731
                                           algo="generic")
        bwd = lambda: ops.mdcn_backward(x, off, mask, w, go, False, stride, pad, dil, 1, dg,  # noqa: E731
                                        deterministic=False)
        bwd_det = lambda: ops.mdcn_backward(x, off, mask, w, go, False, stride, pad, dil, 1, dg,  # noqa: E731
                                            deterministic=True)
        bwd_glob = lambda: ops.mdcn_backward(x, off, mask, w, go, False, stride, pad, dil, 1, dg,  # noqa: E731
                                             deterministic=False, algo="global")
        flops = 2.0 * B * Ho * Wo * C * C * k * k
        ms_b, ms_d, ms_g = (time_events(f, iters, stream) for f in (bwd, bwd_det, bwd_glob))
        # forwards write into `out`: timed as graph replays (device time; the 16-channel scale's
        # launch is shorter than its Python call), with the eager per-call time beside them
        ms_fh = time_events(fwd, iters, stream)
        side = torch.cuda.Stream(device)
        side.wait_stream(stream)
        with torch.cuda.stream(side):
            ms_f, ms_fg = (time_graph(f, iters, side) for f in (fwd, fwd_gen))
        stream.wait_stream(side)
        line = {"bench": "dcn_sweep (C4)", "shape": name, "input": [B, C, H, W], "stride": stride,
                "deformable_groups": dg, "dilation": dil, "fwd_us": ms_f * 1e3,
                "fwd_window": ops.window_fwd_ok(C, C, k, k, stride, pad, dil, 1, dg, W),
                "fwd_direct": ops.direct_fwd_ok(C, C, k, k, stride, pad, dil, 1, dg),
                "fwd_generic_us": ms_fg * 1e3, "fwd_eager_call_us": ms_fh * 1e3,
                "bwd_us": ms_b * 1e3,
                "bwd_det_us": ms_d * 1e3, "bwd_global_atomic_us": ms_g * 1e3,
                "fwd_tflops": flops / ms_f / 1e9, "bwd_tflops": 2 * flops / ms_b / 1e9,
                "fwd_frac_f32_mfma": flops / ms_f / 1e9 / FP32_MFMA_PEAK_TF,
                "bwd_frac_f32_mfma": 2 * flops / ms_b / 1e9 / FP32_MFMA_PEAK_TF,
                "data": "synthetic", "dtype": "f32"}
        tot[name] = (ms_f, ms_b)
        if rank == 0:
            print(json.dumps(line), flush=True)
    if rank == 0:
        for ns, names in ((1, ["agg_s0"]), (3, ["agg_s0", "agg_s1", "agg_s2"])):
            if any(n not in tot for n in names):
                continue
            f = sum(tot[n][0] for n in names)
            b = sum(tot[n][1] for n in names)
            print(json.dumps({"bench": "dcn_sweep (C4)", "num_scales": ns, "fwd_us": f * 1e3,
                              "fwd_bwd_us": (f + b) * 1e3, "per_module": "one DCN per scale"}),
                  flush=True)


FULL_MODELS = {
    # scripts/aanet_inference.sh / aanet+_inference.sh (KITTI): constructor kwargs
    "aanet": dict(feature_type="aanet", feature_pyramid_network=True, refinement_type="stereodrnet",
                  no_intermediate_supervision=True),
    "aanetplus": dict(feature_type="ganet", feature_pyramid=True, refinement_type="hourglass",
                      no_intermediate_supervision=True),
    # BASELINE configs[4] (C5): the 4-D concat cost volume (nets/cost.py:22-38) at 384x1248,
    # D=192 (48 at the 1/4 feature scale): PSMNet features + the PSMNet hourglass 3-D aggregator,
    # and PSMNet-AA (the same features, adaptive aggregation on the correlation pyramid)
    "psmnet_hg": dict(feature_type="psmnet", feature_similarity="concat",
                      aggregation_type="psmnet_hourglass", refinement_type=None),
    "psmnet_aa": dict(feature_type="psmnet", feature_pyramid=True, no_intermediate_supervision=True),
}


def model_main(args, device, rank, world):
    """--model: the whole network of the reference's KITTI inference scripts on synthetic
    384x1248 image pairs (ImageNet-normalised noise), eval, random-init weights of that
    architecture (offset convs non-zero).  Secondary line: not the headline metric."""
    from aanet_amd.nets import AANet
    torch.manual_seed(0)
    model = AANet(MAXD_IMG, **FULL_MODELS[args.model])
    g = torch.Generator().manual_seed(1)
    with torch.no_grad():
        for name, mod in model.named_modules():
            if isinstance(mod, torch.nn.BatchNorm2d):
                mod.running_mean.copy_(0.05 * torch.randn(mod.num_features, generator=g))
                mod.running_var.copy_(0.8 + 0.4 * torch.rand(mod.num_features, generator=g))
            if name.endswith("offset_conv"):
                mod.weight.normal_(0.0, 0.01, generator=g)
                mod.bias.normal_(0.0, 0.5, generator=g)
    model = model.to(device).eval()
    gen = torch.Generator(device=device).manual_seed(4321 + rank)
    ih, iw = (int(v) for v in args.img.lower().split("x")) if args.img else (H_IMG, W_IMG)
    left = torch.randn((args.batch, 3, ih, iw), device=device, generator=gen)
    right = torch.randn((args.batch, 3, ih, iw), device=device, generator=gen)

    def step():
        with torch.no_grad():
            return model(left, right)[-1]

    out, elapsed, graph = timed_run(step, args, world)
    from aanet_amd import dist as adist
    rec = adist.make_record(device, pairs=args.batch * args.steps, elapsed_s=elapsed,
                            disp_min=float(out.min()), disp_max=float(out.max()))
    summary = adist.summarize(adist.gather_records(rec))
    if rank == 0:
        print(json.dumps({
            "metric": f"full-model stereo-pairs/s @{ih}x{iw} ({args.model}, KITTI config) fp32",
            "value": summary["pairs"] / summary["elapsed_max_s"], "unit": "stereo-pairs/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": 1000.0 * summary["elapsed_max_s"] / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (N(0,1) image pairs, random-init weights)",
            "config": {"workload": f"{args.model}: {FULL_MODELS[args.model]}, max_disp 192",
                       "batch_per_gpu": args.batch, "global_batch": args.batch * world,
                       "parallelism": f"dp{world} (pairs sharded, no data-path collective)",
                       "hip_graph": graph is not None, "schedule": getattr(args, "schedule", None)},
            "disp_range": [summary["disp_min"], summary["disp_max"]]}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


TRAIN_IMG = (288, 576)   # scripts/aanet_train.sh (Scene Flow): --img_height 288 --img_width 576
TRAIN_METRIC = "training stereo-pairs/s @288x576 D=64 fp32 (hot path fwd+bwd+Adam)"


def train_main(args, device, rank, world):
    """--train: the training step of the path (aanet_amd/train.py) -- forward in train mode
    (batch-statistics BN, intermediate supervision: 3 disparities), pyramid smooth-L1 against a
    full-resolution synthetic ground truth, HIP backward kernels, Adam with the offset_conv
    0.1x group; SyncBN + DDP over RCCL when N>1 (the gradient all-reduce is the one data-path
    collective).  Secondary line: not the headline metric."""
    from aanet_amd import train as atrain
    if args.deterministic:
        torch.use_deterministic_algorithms(True, warn_only=True)
        # the NaN fill of every torch.empty is a debugging aid, not part of determinism (the
        # kernels overwrite their outputs; tests keep it on): ~2.5k fill launches per step
        torch.utils.deterministic.fill_uninitialized_memory = False
    model = build_model(device, intermediate_supervision=True).train()
    model = atrain.wrap_data_parallel(model, device)
    use_graph = world == 1 and not args.no_graph
    engine = {"auto": None, "on": True, "off": False}[args.engine_convs]
    trainer = atrain.Trainer(model, lr=1e-3, engine_convs=engine, capturable=use_graph)
    left, right = make_features(args.train_batch, rank, device, args.features, TRAIN_IMG)
    gen = torch.Generator(device=device).manual_seed(99 + rank)
    gt = torch.rand((args.train_batch,) + TRAIN_IMG, device=device, generator=gen) * (MAXD_IMG - 1)
    mask = (gt > 0) & (gt < MAXD_IMG)
    step = lambda: trainer.step(left, right, gt, mask)  # noqa: E731
    if use_graph:  # one HIP graph per step (the eager step is launch-bound: ~2.9k launches)
        try:
            trainer.graph_step(left, right, gt, mask)
            step = lambda: trainer.graph_step(left, right, gt, mask)  # noqa: E731
        except Exception as e:  # noqa: BLE001
            print(f"training graph capture failed ({e}); timing eager steps", file=sys.stderr)
            use_graph = False
            trainer = atrain.Trainer(model, lr=1e-3, engine_convs=engine)
            step = lambda: trainer.step(left, right, gt, mask)  # noqa: E731
    for _ in range(args.warmup):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    from aanet_amd import dist as adist
    rec = adist.make_record(device, pairs=args.train_batch * args.steps, elapsed_s=elapsed)
    summary = adist.summarize(adist.gather_records(rec))
    if rank == 0:
        print(json.dumps({
            "metric": TRAIN_METRIC,
            "value": summary["pairs"] / summary["elapsed_max_s"],
            "unit": "stereo-pairs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": 1000.0 * summary["elapsed_max_s"] / args.steps,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (N(0,1) feature pyramids, uniform ground truth; random-init "
                    "weights)",
            "config": {"workload": "Scene Flow training crop 288x576: features 128ch at "
                                   "1/3,1/6,1/12, D=64/32/16, AdaptiveAggregation train mode "
                                   "with intermediate supervision, pyramid smooth-L1, Adam",
                       "batch_per_gpu": args.train_batch,
                       "global_batch": args.train_batch * world,
                       "parallelism": f"dp{world} (SyncBN + DDP all-reduce)" if world > 1
                       else "dp1", "deterministic": bool(args.deterministic),
                       "hip_graph": use_graph,
                       "engine_convs": args.engine_convs},
            "final_loss": float(loss)}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def load_traffic(kernel):
    """HBM bytes per launch from the committed rocprofv3 PMC pass (profiles/pmc_*.json)."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get(kernel)


def profile_only(args, model, left, right, step):
    """Profiling helper: run one kernel family args.steps times (for rocprofv3 passes)."""
    from aanet_amd import ops
    if args.only == "step":
        fn = step
    elif args.only == "corr":
        fn = lambda: ops.corr_volume(left[0], right[0], MAXD)  # noqa: E731
    elif args.only == "pyramid":
        fn = lambda: ops.corr_pyramid(left, right, MAXD)  # noqa: E731
    elif args.only == "regress":
        vol = ops.corr_volume(left[0], right[0], MAXD)
        fn = lambda: ops.disp_regress(vol)  # noqa: E731
    elif args.only == "mdcn":
        roof_iters = args.steps
        kernel_rooflines(model, left, right, args.batch, roof_iters)
        torch.cuda.synchronize()
        return
    else:
        raise SystemExit(f"unknown --only {args.only}")
    for _ in range(args.warmup + args.steps):
        fn()
    torch.cuda.synchronize()
    print(json.dumps({"only": args.only, "steps": args.steps}))


if __name__ == "__main__":
    main()
