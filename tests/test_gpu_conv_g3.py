"""GPU tests of the grouped direct 3x3 kernel that runs the deformable offset_conv in eval
(aanet_amd/csrc/conv_g3.hip, aanet_conv3x3_grouped_nhwc_f32; nets/deform.py:58-60): channels-
last input, NCHW output + bias, against an fp64 reference and held to the exact-f32 conv
engine's error on the same conv (as tests/test_gpu_conv_s2.py); every border, dilation 1 and 2,
one and two groups, partial co blocks (27 of 32 rows), and the C2 scale-0 shape."""
import pytest
import torch
import torch.nn.functional as F

from aanet_amd import _lib, nets, ops

pytestmark = pytest.mark.gpu
DEV = "cuda"

CASES = [
    # N, C, H, W, co, groups, dil
    (1, 64, 128, 416, 54, 2, 2),  # C2 scale-0 offset_conv, one image
    (2, 64, 17, 23, 54, 2, 2),    # odd H, W: partial tiles, padding at every border
    (2, 64, 9, 30, 54, 2, 1),     # dilation 1
    (1, 64, 10, 20, 18, 2, 2),    # one co block per group
    (1, 32, 12, 20, 27, 1, 2),    # one group of 32
    (1, 64, 9, 17, 32, 1, 2),     # one group, two chunks
    (3, 64, 5, 4, 54, 2, 2),      # image smaller than the dilated stencil
    (1, 32, 11, 19, 32, 1, 1),    # one group of 32, 32 outputs (full co blocks), dilation 1
]


class exact_f32:
    def __enter__(self):
        self.prev = _lib.set_exact_f32(True)

    def __exit__(self, *a):
        _lib.set_exact_f32(self.prev)


@pytest.mark.parametrize("case", CASES, ids=[f"c{c[1]}co{c[4]}g{c[5]}d{c[6]}h{c[2]}w{c[3]}" for c in CASES])
def test_conv3x3_grouped_nhwc_vs_fp64(case):
    N, C, H, W, co, groups, dil = case
    g = torch.Generator().manual_seed(5)
    x = torch.randn(N, C, H, W, generator=g) * 2
    w = torch.randn(co, C // groups, 3, 3, generator=g) / (3 * (C // groups) ** 0.5)
    b = torch.randn(co, generator=g)
    y = F.conv2d(x.double(), w.double(), b.double(), padding=dil, dilation=dil, groups=groups)
    scale = F.conv2d(x.double().abs(), w.double().abs(), padding=dil, dilation=dil, groups=groups) + 1.0
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    wd, bd = w.to(DEV), b.to(DEV)
    ws = ops.pack_conv3x3_grouped(wd, groups)
    assert ws is not None
    got = ops.conv3x3_grouped_nhwc(xd, ws, bd, co, groups, dil)
    assert got.shape == (N, co, H, W) and got.is_contiguous()
    with exact_f32():  # the engine's exact-f32 contraction of the same conv, as the error bar
        ref_e = ops.conv2d_fused(x.to(DEV), wd, bd, 1, dil, dil, groups, None,
                                 packed_weight=ops.pack_weight(wd))
    err_e = ((ref_e.cpu().double() - y).abs() / scale).max().item()
    err = ((got.cpu().double() - y).abs() / scale).max().item()
    assert err <= max(4 * err_e, 2e-7), (err, err_e)
    again = ops.conv3x3_grouped_nhwc(xd, ws, bd, co, groups, dil)
    assert torch.equal(again, got)  # no atomics, fixed order


def test_offset_conv_eval_uses_kernel_and_matches_engine():
    """DeformSimpleBottleneck's eval offset_conv (nets/_fuse.offset_conv_eval) takes the grouped
    halo kernel for the scale-0 shape and agrees with the conv engine's form within the split
    contraction's error."""
    from aanet_amd.nets import _fuse
    torch.manual_seed(0)
    blk = nets.DeformSimpleBottleneck(64, 64, mdconv_dilation=2, deformable_groups=2).to(DEV).eval()
    oc = blk.conv2.offset_conv
    with torch.no_grad():
        oc.weight.normal_(0, 0.05)
        oc.bias.normal_(0, 0.5)
        x = torch.randn(2, 64, 24, 40, device=DEV).contiguous(memory_format=torch.channels_last)
        assert _fuse.offset_conv_pack(oc) is not None
        got = _fuse.offset_conv_eval(x, oc)
        ref = _fuse.conv_bn_act(x, oc)
    assert got.shape == ref.shape
    assert (got - ref).abs().max().item() <= 1e-4


def test_conv3x3_grouped_rejects_unsupported_shapes():
    lib = _lib.lib()
    assert lib.aanet_conv3x3_grouped_pack_bytes(54, 48, 2) == 0   # 24 channels per group
    assert lib.aanet_conv3x3_grouped_pack_bytes(80, 64, 2) == 0   # 40 outputs per group
    assert ops.pack_conv3x3_grouped(torch.zeros(54, 32, 1, 1, device=DEV), 2) is None
    x = torch.zeros(1, 64, 8, 8, device=DEV).contiguous(memory_format=torch.channels_last)
    ws = torch.zeros(64, device=DEV, dtype=torch.int16)
    with pytest.raises(_lib.AanetError):
        ops.conv3x3_grouped_nhwc(x, ws, None, 54, 4, 2)  # 16 channels per group
