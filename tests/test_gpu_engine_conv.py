"""GPU tests of the engine convolution backward used in training (aanet_conv2d_wgrad_f32 and
ops.conv2d_dgrad, wrapped by train.EngineConv2dFunction): gradients against torch's fp32
convolution for every conv shape of the ISA/CSA blocks (1x1, 3x3 pad 1, 3x3 dilation 2,
3x3 stride 2 with even and odd sizes, grouped offset conv), and bit-reproducibility of the
deterministic form."""
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import _lib, nets, ops, train

pytestmark = pytest.mark.gpu
DEV = "cuda"

# (N, C, H, W, Co, k, stride, pad, dil, groups, bias)
SHAPES = [
    (2, 16, 24, 40, 16, 1, 1, 0, 1, 1, False),   # conv1x1 (deform.py:6-14)
    (2, 32, 20, 36, 32, 3, 1, 1, 1, 1, True),    # conv3x3 + bias (aggregation.py fuse layers)
    (2, 64, 16, 28, 54, 3, 1, 2, 2, 2, True),    # offset_conv, dilation 2, deformable groups
    (2, 32, 24, 48, 64, 3, 2, 1, 1, 1, False),   # CSA downsample, even sizes
    (1, 16, 25, 39, 32, 3, 2, 1, 1, 1, False),   # stride 2, odd sizes (dropped row/column)
    (3, 48, 12, 20, 1, 1, 1, 0, 1, 1, True),     # final_conv-like, Co = 1
    (2, 70, 9, 13, 40, 3, 1, 1, 1, 1, True),     # ragged channel counts
    # feature-extractor shapes that Trainer(engine_convs) also routes here:
    (1, 3, 48, 96, 32, 7, 3, 3, 1, 1, False),    # AANetFeature conv1: 7x7 stride 3, Cin 3
    (1, 3, 50, 97, 32, 7, 3, 3, 1, 1, False),    # ... stride-3 dgrad zero insertion, ragged
    (2, 64, 24, 40, 128, 1, 2, 0, 1, 1, False),  # ResNet downsample 1x1 stride 2
    (1, 32, 25, 39, 64, 1, 2, 0, 1, 1, False),   # ... odd sizes
]


def _case(shape, seed=0):
    N, C, H, W, Co, k, s, p, d, g, b = shape
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(N, C, H, W, generator=gen).to(DEV)
    w = (torch.randn(Co, C // g, k, k, generator=gen) / (C * k * k) ** 0.5).to(DEV)
    bias = torch.randn(Co, generator=gen).to(DEV) if b else None
    return x, w, bias


@pytest.mark.parametrize("shape", SHAPES, ids=[f"k{s[5]}s{s[6]}d{s[8]}g{s[9]}c{s[1]}" for s in SHAPES])
@pytest.mark.parametrize("det", [False, True])
def test_engine_conv_grads_match_torch(shape, det):
    N, C, H, W, Co, k, s, p, d, g, b = shape
    x, w, bias = _case(shape)
    xs = [x.clone().requires_grad_(True) for _ in range(2)]
    ws = [w.clone().requires_grad_(True) for _ in range(2)]
    bs = [bias.clone().requires_grad_(True) if b else None for _ in range(2)]
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(det)
    try:
        y = train.EngineConv2dFunction.apply(xs[0], ws[0], bs[0], s, p, d, g)
        gy = torch.randn(y.shape, generator=torch.Generator().manual_seed(9)).to(DEV)
        y.backward(gy)
    finally:
        torch.use_deterministic_algorithms(prev)
    with torch.backends.cudnn.flags(enabled=True, allow_tf32=False):
        yr = F.conv2d(xs[1], ws[1], bs[1], s, p, d, g)
        yr.backward(gy)
    assert y.shape == yr.shape

    def close(a, r, what):
        err = (a - r).abs().max().item()
        assert err <= 2e-4 * max(1.0, r.abs().max().item()), (what, err)

    close(y, yr, "forward")
    close(xs[0].grad, xs[1].grad, "grad_x")
    close(ws[0].grad, ws[1].grad, "grad_w")
    if b:
        close(bs[0].grad, bs[1].grad, "grad_b")


@pytest.mark.parametrize("shape", [SHAPES[1], SHAPES[2], SHAPES[3]])
def test_deterministic_wgrad_is_bit_reproducible(shape):
    N, C, H, W, Co, k, s, p, d, g, b = shape
    x, w, _ = _case(shape, 3)
    Ho = (H + 2 * p - d * (k - 1) - 1) // s + 1
    Wo = (W + 2 * p - d * (k - 1) - 1) // s + 1
    gy = torch.randn(N, Co, Ho, Wo, generator=torch.Generator().manual_seed(4)).to(DEV)
    outs = [ops.conv2d_wgrad(x, gy, w.shape, b, s, p, d, g, deterministic=True) for _ in range(3)]
    for gw, gb in outs[1:]:
        assert torch.equal(gw, outs[0][0])
        if b:
            assert torch.equal(gb, outs[0][1])
    # the default is the fixed-order form; the float-atomic form agrees to fp32 summation order
    dflt = ops.conv2d_wgrad(x, gy, w.shape, b, s, p, d, g)
    assert torch.equal(dflt[0], outs[0][0])
    gw_at, _ = ops.conv2d_wgrad(x, gy, w.shape, b, s, p, d, g, deterministic=False)
    assert (gw_at - outs[0][0]).abs().max().item() <= 1e-4 * max(1.0, outs[0][0].abs().max().item())


def test_engine_convs_model_gradients_and_reproducibility():
    """use_engine_convs on the hot-path model: the same gradients as the MIOpen convs (to fp32
    rounding), and bit-identical gradients over two deterministic runs."""
    def run(engine, det, seed=5):
        torch.manual_seed(seed)
        m = nets.AANetHotPath(16, no_intermediate_supervision=False, num_deform_blocks=3).to(DEV)
        m.train()
        if engine:
            assert train.use_engine_convs(m) > 20
        g = torch.Generator().manual_seed(1)
        sizes = [(24, 48), (12, 24), (6, 12)]
        left = [torch.randn(2, 16, h, w_, generator=g).to(DEV) for h, w_ in sizes]
        right = [torch.randn(2, 16, h, w_, generator=g).to(DEV) for h, w_ in sizes]
        prev = torch.are_deterministic_algorithms_enabled()
        torch.use_deterministic_algorithms(det)
        try:
            loss = sum((d * (i + 1)).mean() for i, d in enumerate(m(left, right)))
            loss.backward()
        finally:
            torch.use_deterministic_algorithms(prev)
        return {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}

    a, b, ref = run(True, True), run(True, True), run(False, False)
    assert a.keys() == b.keys() == ref.keys() and len(a) > 100
    assert not [n for n in a if not torch.equal(a[n], b[n])]
    got = torch.cat([a[n].flatten() for n in sorted(a)])
    want = torch.cat([ref[n].flatten() for n in sorted(a)])
    rel = float((got - want).norm() / want.norm())
    assert rel < 1e-3, rel


@pytest.mark.parametrize("hw,out", [((12, 20), (24, 40)), ((6, 10), (24, 40)), ((32, 64), (96, 192)),
                                    ((8, 16), (96, 192)), ((7, 11), (20, 33)), ((20, 33), (7, 11)),
                                    ((1, 5), (4, 9)), ((96, 192), (288, 576))])
def test_resize_bilinear_backward_matches_torch(hw, out):
    """ops.resize_bilinear's HIP forward (bit-identical to torch's kernel: same stencil, same
    order) and gather backward against torch's bilinear backward (2x/4x CSA exchanges, 3x/12x
    loss upsampling, non-integer and downsampling ratios, a 1-pixel axis)."""
    g = torch.Generator().manual_seed(2)
    x = torch.randn(2, 3, *hw, generator=g).to(DEV)
    gy = torch.randn(2, 3, *out, generator=g).to(DEV)
    xa, xb = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    ya = ops.resize_bilinear(xa, out)
    ya.backward(gy)
    yb = F.interpolate(xb, size=out, mode="bilinear", align_corners=False)
    yb.backward(gy)
    assert torch.equal(ya, yb)
    err = (xa.grad - xb.grad).abs().max().item()
    assert err <= 1e-5 * max(1.0, xb.grad.abs().max().item()), err
    again = torch.empty_like(xa.grad)
    xa.grad = None
    ops.resize_bilinear(xa, out).backward(gy)
    again.copy_(xa.grad)
    xa.grad = None
    ops.resize_bilinear(xa, out).backward(gy)
    assert torch.equal(again, xa.grad)


def test_wgrad_modes_accumulate_or_store():
    """aanet_conv2d_wgrad_f32 deterministic = 1 ADDS to grad_weight / grad_bias (the reference's
    accumulate semantics), 2 STORES them (what ops.conv2d_wgrad uses: no zero fill), both with the
    same fixed-order sums."""
    shape = SHAPES[1]
    N, C, H, W, Co, k, s, p, d, g, b = shape
    x, w, _ = _case(shape, 3)
    Ho = (H + 2 * p - d * (k - 1) - 1) // s + 1
    Wo = (W + 2 * p - d * (k - 1) - 1) // s + 1
    gy = torch.randn(N, Co, Ho, Wo, generator=torch.Generator().manual_seed(4)).to(DEV)
    ref_w, ref_b = ops.conv2d_wgrad(x, gy, w.shape, True, s, p, d, g)
    lib = _lib.lib()
    nbytes = lib.aanet_conv2d_wgrad_workspace_size(N, C, H, W, Co, k, k, s, p, d, g)
    ws = torch.empty((nbytes,), device=DEV, dtype=torch.uint8)
    for mode, init in ((1, 0.5), (2, float("nan"))):
        gw = torch.full(tuple(w.shape), init, device=DEV)
        gb = torch.full((Co,), init, device=DEV)
        ops.call("aanet_conv2d_wgrad_f32", ops.ptr(x), ops.ptr(gy), ops.ptr(gw), ops.ptr(gb), N, C, H,
                 W, Co, k, k, s, p, d, g, mode, ops.ptr(ws), nbytes, ops.stream_of(x))
        torch.cuda.synchronize()
        if mode == 1:
            assert torch.equal(gw, ref_w + 0.5) and torch.equal(gb, ref_b + 0.5)
        else:
            assert torch.equal(gw, ref_w) and torch.equal(gb, ref_b)
    with pytest.raises(_lib.AanetError):
        ops.call("aanet_conv2d_wgrad_f32", ops.ptr(x), ops.ptr(gy), ops.ptr(gw), ops.ptr(gb), N, C, H,
                 W, Co, k, k, s, p, d, g, 3, ops.ptr(ws), nbytes, ops.stream_of(x))


@pytest.mark.parametrize("co,cg,k,groups", [(32, 16, 3, 1), (54, 32, 3, 2), (16, 3, 7, 1), (64, 32, 1, 1),
                                            (40, 70, 3, 1)])
def test_dgrad_weight_pack_equals_transposed_flipped_pack(co, cg, k, groups):
    """aanet_conv_weight_pack_dgrad_f32 (one launch) == pack_weight of the per-group transposed,
    spatially flipped weight that ops.conv2d_dgrad used to build with two torch copies."""
    w = torch.randn(co, cg, k, k, generator=torch.Generator().manual_seed(7)).to(DEV)
    wt = (w.view(groups, co // groups, cg, k, k).transpose(1, 2)
          .reshape(groups * cg, co // groups, k, k).flip(-2, -1).contiguous())
    want = ops.pack_weight(wt)
    got = torch.empty_like(want)
    ops.call("aanet_conv_weight_pack_dgrad_f32", ops.ptr(w), ops.ptr(got), co, cg, k, k, groups,
             ops.stream_of(w))
    assert torch.equal(got, want)
