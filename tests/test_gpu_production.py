"""GPU parity of the hot path in the configurations that production (and bench.py) runs.

The round-1 end-to-end goldens run AdaptiveAggregation at max_disp=16, where no scale is 32
channels wide, so they exercise the exact-f32 NCHW engine only.  Here:

* hotpath_d64 -- the reference graph's own output at max_disp=64 (the C2 width), features
  [2,128,32,96]: scale widths 64/32/16, i.e. the split-bf16 contraction, the NHWC bottleneck
  tails (DCN + conv3 and 3x3 + conv3) and the CSA epilogue -- the kernels bench.py times;
* hotpath_c1 -- BASELINE configs[0] (288x576, D=24): features [1,128,96,192];
* C2 pair 0 at full size ([1,128,128,416] pyramid, D=64) against the CPU oracle (which the
  d64 fixture pins to the reference at the same widths);
* hotpath_c3 -- BASELINE configs[2] (AANet+: GANetFeature + FeaturePyrmaid) feature widths
  32/64/128 at a reduced size, the reference graph's own output; and C3 pair 0 at its full
  size ([1,32,192,320] / [1,64,96,160] / [1,128,48,80], D=64) against the CPU oracle;
* the eval-cache, CSA-epilogue-precondition and grouped-DCN regressions of ADVICE round 1.

Tolerances: disparity 5e-4 px max abs (half the north-star bar of 1e-3) and 5e-5 px mean abs;
aggregated cost 1e-4 x its scale.  The max is set by near-tie pixels of the soft-argmin, where
the fp32 summation order alone moves it: the same kernels with the CSA sums of branches 1 / 2 in
aanet_csa_sum_f32 kernels or in the stride-2 kernels' epilogues (set_options(s2_sums=False / True): the same
terms in another fp32 order) measured C3 1.2e-4 / 1.6e-4 px and C3 pair 0 vs oracle 1.8e-4 /
2.1e-4 px, d64 2.3e-4 px with the epilogue sums, every mean unchanged.
"""
import numpy as np
import pytest
import torch

from aanet_amd import nets, ops
from aanet_amd.nets._fuse import folded
from aanet_amd.nets.aggregation import csa_epilogue_ok
from oracle import aggregation as oagg
from tests.golden_io import fill_synthetic, production_case, synthetic_pyramid

pytestmark = pytest.mark.gpu
DEV = "cuda"
DISP_TOL = 5e-4
DISP_MEAN_TOL = 5e-5


def _model(tag, fuse=True):
    g, sd, m, left, right = production_case(tag)
    m = m.to(DEV).eval()
    for mod in m.modules():
        mod.aanet_fuse = fuse
    return g, sd, m, [t.to(DEV) for t in left], [t.to(DEV) for t in right]


def _production_kernels_engaged(m):
    """The d64 configuration must run the split-bf16 weight buffers at every scale-0/1 conv of
    the bottlenecks, with NHWC-capable widths and an accepted CSA epilogue."""
    blk = m.aggregation.fusions[5].branches[0][0]        # DeformSimpleBottleneck, scale 0
    assert getattr(folded(blk.conv2.deform_conv, None)[2], "_aanet_split", False)
    assert getattr(folded(blk.conv3, blk.bn3)[2], "_aanet_split", False)
    blk0 = m.aggregation.fusions[0].branches[0][0]       # SimpleBottleneck, scale 0
    assert getattr(folded(blk0.conv2, blk0.bn2)[2], "_aanet_split", False)
    assert blk0.conv1.weight.shape[0] % 32 == 0 and blk.conv1.weight.shape[0] % 32 == 0


@pytest.mark.parametrize("fuse", [True, False])
def test_hotpath_d64_vs_reference(fuse):
    g, _, m, left, right = _model("hotpath_d64", fuse)
    with torch.no_grad():
        vols = m.cost_volume(left, right)
        assert csa_epilogue_ok(vols[0], [vols[1], vols[2]])
        agg0 = m.aggregation(list(vols))[0]
        disps = m(left, right)
    if fuse:
        _production_kernels_engaged(m)
    a0 = agg0.cpu().numpy().ravel()
    scale = np.abs(g["agg0_sample"]).max()
    aerr = np.abs(a0[g["agg0_idx"]] - g["agg0_sample"]).max()
    assert aerr <= 1e-4 * scale, f"aggregated cost: {aerr:.3g} (scale {scale:.3g})"
    assert len(disps) == 1
    d = disps[0].cpu().numpy()
    err = np.abs(d - g["disp0"])
    print(f"hotpath_d64 fuse={fuse}: max|dd| {err.max():.3g} px, mean {err.mean():.3g}, "
          f"reference fp32 vs fp64 max {np.abs(g['disp0'] - g['disp64_0']).max():.3g}")
    assert err.max() <= DISP_TOL, f"max |dd| {err.max():.3g} px"
    assert err.mean() <= DISP_MEAN_TOL, f"mean |dd| {err.mean():.3g} px"


def test_hotpath_c1_vs_reference():
    """BASELINE configs[0]: 288x576 pair, D=24 (max_disp 72), B=1 -- on the MI355X."""
    g, _, m, left, right = _model("hotpath_c1")
    with torch.no_grad():
        disps = m(left, right)
    d = disps[0].cpu().numpy()
    assert d.shape == g["disp0"].shape == (1, 96, 192)
    err = np.abs(d - g["disp0"])
    print(f"hotpath_c1: max|dd| {err.max():.3g} px, mean {err.mean():.3g}")
    assert err.max() <= DISP_TOL, f"max |dd| {err.max():.3g} px"
    assert err.mean() <= DISP_MEAN_TOL, f"mean |dd| {err.mean():.3g} px"


def test_c2_pair0_full_size_vs_oracle():
    """C2 at full size: one 384x1248 pair ([1,128,128,416] / [64,208] / [32,104] pyramid, D=64),
    the bench configuration's kernels, against the CPU oracle on the same input."""
    torch.manual_seed(0)
    m = nets.AANetHotPath(64, no_intermediate_supervision=True, num_deform_blocks=3)
    fill_synthetic(m.aggregation, 2)
    sd = {k: v.numpy().copy() for k, v in m.aggregation.state_dict().items()}
    m = m.to(DEV).eval()
    left, right = synthetic_pyramid(1, 128, 128, 416, 2)
    with torch.no_grad():
        d = m([t.to(DEV) for t in left], [t.to(DEV) for t in right])[0].cpu().numpy()
    ref = oagg.hot_path([t.numpy() for t in left], [t.numpy() for t in right], sd, 64,
                        intermediate_supervision=False)[0]
    err = np.abs(d.astype(np.float64) - ref)
    print(f"C2 pair 0 vs oracle: max|dd| {err.max():.3g} px, mean {err.mean():.3g}")
    assert d.shape == (1, 128, 416)
    assert err.max() <= DISP_TOL, f"max |dd| {err.max():.3g} px"
    assert err.mean() <= DISP_MEAN_TOL, f"mean |dd| {err.mean():.3g} px"


def test_hotpath_c3_vs_reference():
    """BASELINE configs[2] (AANet+): per-scale feature widths 32/64/128 (nets/feature.py:379-419)
    -> the register-ring correlation tile at C = 32 and 64, then the D=64 aggregation."""
    g, _, m, left, right = _model("hotpath_c3")
    assert [t.shape[1] for t in left] == [32, 64, 128]
    with torch.no_grad():
        disps = m(left, right)
    d = disps[0].cpu().numpy()
    assert d.shape == g["disp0"].shape == (1, 48, 80)
    err = np.abs(d - g["disp0"])
    print(f"hotpath_c3: max|dd| {err.max():.3g} px, mean {err.mean():.3g}, reference fp32 vs "
          f"fp64 max {np.abs(g['disp0'] - g['disp64_0']).max():.3g}")
    assert err.max() <= DISP_TOL, f"max |dd| {err.max():.3g} px"
    assert err.mean() <= DISP_MEAN_TOL, f"mean |dd| {err.mean():.3g} px"


def test_c3_pair0_full_size_vs_oracle():
    """C3 at its own shapes: one 576x960 AANet+ pair -- features [1,32,192,320] /
    [1,64,96,160] / [1,128,48,80] (scripts/aanet+_train.sh:12-15, max_disp 192 -> D=64) --
    through the bench kernels, against the CPU oracle on the same input."""
    torch.manual_seed(0)
    m = nets.AANetHotPath(64, no_intermediate_supervision=True, num_deform_blocks=3)
    fill_synthetic(m.aggregation, 5)
    sd = {k: v.numpy().copy() for k, v in m.aggregation.state_dict().items()}
    m = m.to(DEV).eval()
    left, right = synthetic_pyramid(1, 32, 192, 320, 5, channels=(32, 64, 128))
    with torch.no_grad():
        d = m([t.to(DEV) for t in left], [t.to(DEV) for t in right])[0].cpu().numpy()
    ref = oagg.hot_path([t.numpy() for t in left], [t.numpy() for t in right], sd, 64,
                        intermediate_supervision=False)[0]
    err = np.abs(d.astype(np.float64) - ref)
    print(f"C3 pair 0 vs oracle: max|dd| {err.max():.3g} px, mean {err.mean():.3g}")
    assert d.shape == (1, 192, 320)
    assert err.max() <= DISP_TOL, f"max |dd| {err.max():.3g} px"
    assert err.mean() <= DISP_MEAN_TOL, f"mean |dd| {err.mean():.3g} px"


def test_eval_after_train_mode_forward_refolds_bn():
    """eval forward -> train-mode forward (BN running statistics updated in place, no _version
    bump) -> eval forward must fold the NEW statistics (stale folded-BN cache)."""
    g, _, m, left, right = _model("hotpath_d64")
    with torch.no_grad():
        m(left, right)                      # populates the folded-weight caches
        m.train()
        m(left, right)                      # batch-statistics BN: running stats move
        m.eval()
        fused = m(left, right)[0]
        for mod in m.modules():
            mod.aanet_fuse = False
        unfused = m(left, right)[0]         # reference op order, BN modules as they are now
    err = (fused - unfused).abs().max().item()
    assert err <= DISP_TOL, err


def test_eval_bn_cache_sees_direct_running_stat_writes_in_train_mode():
    """A train-mode BN forward WITHOUT a train()/eval() switch in between (the module left in
    training state but its BN layers in eval): num_batches_tracked moves the cache key."""
    bn = torch.nn.BatchNorm2d(8).to(DEV)
    from aanet_amd.nets._fuse import bn_affine
    bn.eval()
    s0, _ = bn_affine(bn)
    s0 = s0.clone()
    bn.train()
    with torch.no_grad():
        bn(torch.randn(4, 8, 5, 5, device=DEV) * 3)
    bn.training = False                     # flip the flag without going through .eval()
    s1, _ = bn_affine(bn)
    assert not torch.equal(s0, s1)


def test_csa_epilogue_precondition_falls_back_on_odd_width():
    """Scale-0 width 42 (not a multiple of 4): the tail kernel's CSA epilogue cannot take branch
    0, so it is summed by the general resize kernel instead of raising."""
    torch.manual_seed(1)
    m = nets.AANetHotPath(64, no_intermediate_supervision=True, num_deform_blocks=3)
    fill_synthetic(m.aggregation, 3)
    sd = {k: v.numpy().copy() for k, v in m.aggregation.state_dict().items()}
    m = m.to(DEV).eval()
    left, right = synthetic_pyramid(1, 32, 16, 42, 3)
    with torch.no_grad():
        vols = m.cost_volume([t.to(DEV) for t in left], [t.to(DEV) for t in right])
        assert not csa_epilogue_ok(vols[0], [vols[1], vols[2]])
        d = m([t.to(DEV) for t in left], [t.to(DEV) for t in right])[0].cpu().numpy()
    ref = oagg.hot_path([t.numpy() for t in left], [t.numpy() for t in right], sd, 64,
                        intermediate_supervision=False)[0]
    assert np.abs(d - ref).max() <= DISP_TOL


def test_grouped_deform_conv_fused_matches_autograd_path():
    """DeformConv2d(groups=2) in eval: the fused kernel must contract per group (the
    fused entry point was called with groups=1)."""
    torch.manual_seed(4)
    dc = nets.DeformConv2d(64, 64, groups=2, deformable_groups=2).to(DEV)
    with torch.no_grad():
        dc.offset_conv.weight.normal_(0, 0.05)
        dc.offset_conv.bias.normal_(0, 0.5)
    dc.eval()
    x = torch.randn(2, 64, 12, 20, device=DEV)
    with torch.no_grad():
        fused = dc(x)
    ref = dc(x.clone().requires_grad_()).detach()   # autograd path (ModulatedDeformConvFunction)
    assert (fused - ref).abs().max().item() <= 2e-4 * (1 + ref.abs().max().item())


def test_two_stream_schedule_graph_replay_and_single_stream_match():
    """The eval aggregation's concurrent-scale schedule (each coarse scale on its own side stream,
    every cross-stream edge through the capturing stream) captured in a HIP graph, as bench.py
    runs it: replays give the eager result bit for bit, at every pyramid level, and so does the
    one-stream schedule (set_options(concurrent_scales=False): the kernels and their inputs are
    the same, only their issue order differs)."""
    from aanet_amd.nets.options import get_option
    g, sd, m, left, right = _model("hotpath_d64")
    with torch.no_grad():
        eager = [t.clone() for t in m(left, right)]
        m.set_options(concurrent_scales=False)
        assert not get_option(m.aggregation, "concurrent_scales")
        single = [t.clone() for t in m(left, right)]
        m.set_options(concurrent_scales=True)
        assert get_option(m.aggregation, "concurrent_scales")
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static = m(left, right)
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            for a, b, c in zip(eager, static, single):
                assert torch.equal(a, b) and torch.equal(a, c)


def test_prep_stream_option_bit_identical():
    """prep_stream (a deformable scale-0 block's conv1 + offset conv on their own side stream,
    beside the previous module's stride-2 heads) only moves kernels between streams: the same
    bits as prep_stream=False, eagerly and under HIP graph replay (run to run, three times)."""
    g, sd, m, left, right = _model("hotpath_d64")
    with torch.no_grad():
        m.set_options(prep_stream=False)
        ref = [t.clone() for t in m(left, right)]
        m.set_options(prep_stream=True)
        try:
            _prep_runs(m, left, right, ref)
        finally:
            m.set_options(prep_stream=False)


def _prep_runs(m, left, right, ref):
    with torch.no_grad():
        for _ in range(3):
            assert all(torch.equal(a, b) for a, b in zip(ref, m(left, right)))
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static = m(left, right)
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            assert all(torch.equal(a, b) for a, b in zip(ref, static))


def test_pipeline_option_matches_default_eager_and_graph():
    """The cross-module pipelined schedule (set_options(pipeline=True): each scale-0 block on a
    side stream beside the previous module's heads and the coarse blocks, branch 0's sum as its
    own kernel) computes the same terms: within fp32 summation order of the default schedule and
    the reference fixture, bit-reproducible run to run, and the HIP-graph replay equal to the
    eager result bit for bit."""
    g, sd, m, left, right = _model("hotpath_d64")
    with torch.no_grad():
        ref = m(left, right)[0].clone()
        m.set_options(pipeline=True)
        try:
            assert m.aggregation._pipeline_ok(
                m.cost_volume_construction(left, right), True)
            got = [t.clone() for t in m(left, right)]
            assert np.abs(got[0].cpu().numpy() - g["disp0"]).max() <= DISP_TOL
            assert (got[0] - ref).abs().max().item() <= DISP_TOL
            _prep_runs(m, left, right, got)
        finally:
            m.set_options(pipeline=False)


@pytest.mark.parametrize("chains", [2, 3])
def test_batch_chains_bit_identical_eager_and_graph(chains):
    """The batch-pipelined schedule (set_options(batch_chains=k): chunk c of the batch aggregated
    on its own stream, every edge through the capturing stream) gives the one-chain result bit for
    bit -- each pair's kernels and inputs are the same -- eagerly on the first (cache-filling) and
    a later call, and in HIP graph replays.  B = 4 (the d64 case twice), so chunks are uneven at
    k = 3."""
    g, sd, m, left, right = _model("hotpath_d64")
    left = [torch.cat([t, t.flip(0)]) for t in left]
    right = [torch.cat([t, t.flip(0)]) for t in right]
    with torch.no_grad():
        one = [t.clone() for t in m(left, right)]
        m.set_options(batch_chains=chains)
        try:
            from aanet_amd.nets._fuse import clear_fold_caches
            clear_fold_caches(m)  # the first chained call refills every cache
            for _ in range(2):
                got = m(left, right)
                assert all(torch.equal(a, b) for a, b in zip(one, got))
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                static = m(left, right)
            for _ in range(3):
                graph.replay()
                torch.cuda.synchronize()
                assert all(torch.equal(a, b) for a, b in zip(one, static))
        finally:
            m.set_options(batch_chains=1)


def test_s2_sums_option_matches_separate_csa_sums():
    """The coarse branches' CSA sums in the stride-2 kernels' epilogues (s2_sums=True, default)
    against separate aanet_csa_sum_f32 kernels (s2_sums=False): the same terms in another fp32
    order, so the disparities agree within the near-tie bound, and each matches the reference."""
    g, _, m, left, right = _model("hotpath_d64")
    with torch.no_grad():
        a = m(left, right)[0].cpu().numpy()
        m.set_options(s2_sums=False)
        b = m(left, right)[0].cpu().numpy()
        m.set_options(s2_sums=True)
    for d in (a, b):
        assert np.abs(d - g["disp0"]).max() <= DISP_TOL
    assert np.abs(a - b).max() <= DISP_TOL


def test_offset_conv_and_heads_deterministic_beside_other_work():
    """The LDS-DMA kernels (offset conv conv_g3, stride-2 heads conv_s2) give the same bits on
    every run while another stream keeps the CUs busy.  Their barrier now also waits for the
    wave's own LDS reads (lgkmcnt(0)): without it a wave could reach the barrier with reads of a
    weight slot still queued while another wave's DMA into that slot landed, and the concurrent
    schedule differed from the one-stream schedule in a few runs of 30 (round 5)."""
    g = torch.Generator(device=DEV).manual_seed(0)
    B, C, H, W = 8, 64, 64, 208
    x = torch.randn(B, C, H, W, device=DEV, generator=g).relu_().contiguous(
        memory_format=torch.channels_last)
    wsp = ops.pack_conv3x3_grouped(torch.randn(54, 32, 3, 3, device=DEV, generator=g) * 0.05, 2)
    b = torch.randn(54, device=DEV, generator=g)
    xn = x.contiguous()
    ws2 = ops.pack_conv3x3s2(torch.randn(96, C, 3, 3, device=DEV, generator=g) * 0.04)
    b2 = torch.randn(96, device=DEV, generator=g)
    big = torch.randn(4096, 4096, device=DEV, generator=g)
    side = torch.cuda.Stream()
    fns = [lambda: ops.conv3x3_grouped_nhwc(x, wsp, b, 54, 2, 2),
           lambda: torch.cat([t.flatten() for t in ops.conv3x3_s2(xn, ws2, b2, 96, 32, "leaky", "leaky")])]
    for fn in fns:
        ref = fn().clone()
        torch.cuda.synchronize()
        for _ in range(20):
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                torch.mm(big, big)
                fns[0]()
            out = fn()
            torch.cuda.current_stream().wait_stream(side)
            assert torch.equal(out, ref)


def test_concurrent_schedule_is_run_to_run_deterministic():
    """The eval aggregation's concurrent-scale schedule repeated eagerly, and replayed from a
    HIP graph, gives the one-stream result bit for bit on every run (round 5: before the LDS-DMA
    barrier fix, 2-4 of 5 runs differed by up to 7e-4 px)."""
    g, sd, m, left, right = _model("hotpath_d64")
    with torch.no_grad():
        m.set_options(concurrent_scales=False)
        single = [t.clone() for t in m(left, right)]
        m.set_options(concurrent_scales=True)
        for _ in range(5):
            got = m(left, right)
            for a, c in zip(got, single):
                assert torch.equal(a, c)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            static = m(left, right)
        for _ in range(3):
            graph.replay()
            torch.cuda.synchronize()
            for a, c in zip(static, single):
                assert torch.equal(a, c)
