"""The hourglasses' transposed convs (Conv2x(deconv=True): ConvTranspose2d(k=4, s=2, p=1) + BN +
ReLU, then the concat with the skip; nets/feature.py:342-376, nets/refinement.py:109-197) on the
HIP path: ops.deconv2x = one 2x2 pad-1 phase conv on the engine + aanet_deconv2x_assemble_f32.
Checked against torch CPU fp64 at fp32 accuracy, and the fused modules against the reference op
order (MIOpen transposed conv, fp32-pinned) on the GPU."""
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import ops
from aanet_amd.nets.feature import Conv2x

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # N, ci, h, w, co: the hourglass deconvs (4 -> 1 of GANetFeature / HourglassRefinement)
    (2, 128, 8, 26, 96),
    (1, 96, 16, 52, 64),
    (1, 64, 32, 104, 48),
    (1, 48, 48, 156, 32),     # 48 input channels: the plain-f32 engine form (no split pack)
    (1, 64, 7, 9, 48),        # odd sizes: the assembly's partial quads (2w % 4 != 0)
]


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("with_rem", [False, True])
def test_deconv2x_vs_torch_fp64(case, with_rem):
    N, ci, h, w, co = case
    g = torch.Generator().manual_seed(ci + co + h)
    x = torch.randn(N, ci, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(ci, co, 4, 4, generator=g, dtype=torch.float64) / (ci * 4) ** 0.5
    scale = torch.rand(co, generator=g, dtype=torch.float64) + 0.5
    shift = torch.randn(co, generator=g, dtype=torch.float64)
    rem = torch.randn(N, co, 2 * h, 2 * w, generator=g, dtype=torch.float64)
    ref = F.relu(F.conv_transpose2d(x, wt, stride=2, padding=1) * scale.view(1, -1, 1, 1) +
                 shift.view(1, -1, 1, 1))
    if with_rem:
        ref = torch.cat((ref, rem), 1)
    wd = ops.deconv2x_phase_weight(wt.float().to(DEV), scale.float().to(DEV))
    wp = ops.pack_weight_split(wd)
    if wp is None:
        wp = ops.pack_weight(wd)
    got = ops.deconv2x(x.float().to(DEV), wd, shift.float().to(DEV).repeat_interleave(4), "relu",
                       packed_weight=wp, rem=rem.float().to(DEV) if with_rem else None)
    assert got.shape == ref.shape
    err = (got.cpu().double() - ref).abs().max().item()
    assert err <= 2e-5 * (1 + ref.abs().max().item()), err


@pytest.mark.parametrize("ci,co,h,w", [(128, 96, 8, 26), (48, 32, 24, 78)])
def test_conv2x_deconv_fused_matches_reference_order(ci, co, h, w):
    """Conv2x(deconv=True) in eval: the fused path (phase conv + channels-last assembly + concat,
    then the 3x3 conv on the engine's halo tile, NCHW out) against the module's reference op order on the GPU (MIOpen transposed
    conv + BN + ReLU + torch.cat + conv), nonzero BN statistics."""
    torch.manual_seed(3)
    m = Conv2x(ci, co, deconv=True)
    with torch.no_grad():
        for bn in (m.conv1.bn, m.conv2.bn):
            bn.running_mean.normal_(0, 0.1)
            bn.running_var.uniform_(0.5, 1.5)
            bn.weight.uniform_(0.5, 1.5)
            bn.bias.normal_(0, 0.1)
    m = m.to(DEV).eval()
    x = torch.randn(2, ci, h, w, device=DEV)
    rem = torch.randn(2, co, 2 * h, 2 * w, device=DEV)
    with torch.no_grad():
        fused = m(x, rem)
        m.conv1.aanet_fuse = m.conv2.aanet_fuse = m.aanet_fuse = False
        ref = m(x, rem)
    assert (fused - ref).abs().max().item() <= 1e-4 * (1 + ref.abs().max().item())
    assert not fused.is_contiguous(memory_format=torch.channels_last) or fused.shape[1] == 1


@pytest.mark.parametrize("case", CASES + [(1, 32, 5, 7, 6)])  # + 6 / 12 channels: scalar stores
@pytest.mark.parametrize("with_rem", [False, True])
def test_deconv2x_nhwc_assembly_equals_nchw(case, with_rem):
    """aanet_deconv2x_assemble_nhwc_f32 (channels-last out, for Conv2x's conv2 on the halo tile)
    moves the same values as the NCHW assembly: bit-identical after the layout change, including
    rows whose 2w is not a multiple of the 32-column tile."""
    N, ci, h, w, co = case
    g = torch.Generator().manual_seed(7 * ci + co)
    x = torch.randn(N, ci, h, w, generator=g).to(DEV)
    wt = (torch.randn(ci, co, 4, 4, generator=g) / (ci * 4) ** 0.5).to(DEV)
    rem = torch.randn(N, co, 2 * h, 2 * w, generator=g).to(DEV) if with_rem else None
    wd = ops.deconv2x_phase_weight(wt)
    wp = ops.pack_weight_split(wd)
    if wp is None:
        wp = ops.pack_weight(wd)
    a = ops.deconv2x(x, wd, None, "relu", packed_weight=wp, rem=rem)
    b = ops.deconv2x(x, wd, None, "relu", packed_weight=wp, rem=rem, out_nhwc=True)
    assert b.is_contiguous(memory_format=torch.channels_last) and b.shape == a.shape
    assert torch.equal(a, b)


@pytest.mark.parametrize("shape", [(2, 48, 48, 24, 78), (1, 64, 64, 12, 40), (1, 6, 3, 4, 6)])
def test_concat_nhwc_equals_torch_cat(shape):
    """aanet_concat_nhwc_f32: torch.cat((a, b), 1) written channels-last, bit-identical."""
    N, ca, cb, H, W = shape
    a = torch.randn(N, ca, H, W, device=DEV)
    b = torch.randn(N, cb, H, W, device=DEV)
    got = ops.concat_nhwc(a, b)
    assert got.is_contiguous(memory_format=torch.channels_last)
    assert torch.equal(got, torch.cat((a, b), 1))


@pytest.mark.parametrize("ci,co,h,w", [(32, 48, 48, 156), (48, 64, 24, 78)])
def test_conv2x_plain_fused_matches_reference_order(ci, co, h, w):
    """Conv2x (stride-2 conv, concat, 3x3 conv; the hourglasses' conv1b / conv2b) in eval: the
    fused path (concat written channels-last, conv2 on the halo tile) against the reference op
    order on the GPU (MIOpen convs + BN + ReLU + torch.cat)."""
    torch.manual_seed(5)
    m = Conv2x(ci, co)
    with torch.no_grad():
        for bn in (m.conv1.bn, m.conv2.bn):
            bn.running_mean.normal_(0, 0.1)
            bn.running_var.uniform_(0.5, 1.5)
    m = m.to(DEV).eval()
    x = torch.randn(2, ci, h, w, device=DEV)
    rem = torch.randn(2, co, h // 2, w // 2, device=DEV)
    with torch.no_grad():
        fused = m(x, rem)
        m.conv1.aanet_fuse = m.conv2.aanet_fuse = m.aanet_fuse = False
        ref = m(x, rem)
    assert (fused - ref).abs().max().item() <= 1e-4 * (1 + ref.abs().max().item())
