"""CPU-side checks of the host layer: C-ABI library exports, drop-in module API / state-dict keys,
and loud failure (no silent CPU fallback)."""
import contextlib
import ctypes
import os
import re

import numpy as np
import pytest
import torch

import aanet_amd
from aanet_amd import _lib, nets, ops
from tests.golden_io import golden, state_dict_of

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    txt = open(os.path.join(REPO, "include", "aanet_mi355x.h")).read()
    return sorted(set(re.findall(r"\b(aanet_[a-z0-9_]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = ctypes.CDLL(_lib.LIB_PATH)
    fns = header_functions()
    assert len(fns) >= 15
    for f in fns:
        assert hasattr(L, f), f"{f} declared in include/aanet_mi355x.h but not exported"
    assert set(fns) == set(_lib.exported_symbols())


def test_library_version_and_status_strings():
    L = _lib.lib()
    assert L.aanet_version() == _lib.ABI_VERSION == 4
    assert b"struct_size" in L.aanet_status_string(_lib.EABI)
    assert L.aanet_status_string(0) == b"ok"
    assert L.aanet_status_string(-1) == b"invalid argument"
    assert L.aanet_status_string(-2) == b"unsupported configuration"


def test_invalid_arguments_are_rejected_without_a_gpu():
    """Argument validation runs on the host before any launch: bad sizes return AANET_EINVAL."""
    L = _lib.lib()
    assert L.aanet_corr_volume_f32(None, None, None, 1, 1, 1, 1, 1, None) == -1
    assert L.aanet_disp_regress_f32(None, None, 0, 1, 1, 1, 0, None) == -1
    # C not divisible by groups
    args = [None] * 6 + [1, 3, 4, 4, 4, 3, 3, 1, 1, 1, 2, 1, None]
    assert L.aanet_mdcn_fwd_f32(*args) == -1
    with pytest.raises(_lib.AanetError):
        _lib.call("aanet_corr_volume_f32", None, None, None, 0, 1, 1, 1, 1, None)


def test_conv_fused_null_arguments_rejected_before_the_direct_kernel():
    """aanet_conv2d_fused_f32 on a few-channel shape (3 -> 32, 7x7 / 3: the direct VALU kernel of
    small_conv.hip) with a null x / weight / out, or post_scale without post_shift, returns
    AANET_EINVAL on the host instead of launching (the direct dispatch ran before the
    engine's checks).  No GPU is touched: the checks come first."""
    import ctypes as C
    L = _lib.lib()
    f = L.aanet_conv2d_fused_f32
    buf = (C.c_float * 4)()
    p = C.cast(buf, C.c_void_p)
    shape = [1, 3, 48, 96, 32, 7, 7, 3, 2, 1, 1, 0, None]  # n c h w co kh kw s pad dil g layout st
    for x, w, out, ps, sh in ((None, p, p, None, None), (p, None, p, None, None),
                              (p, p, None, None, None), (p, p, p, p, None)):
        assert f(x, w, None, ps, sh, None, 1, 0, out, *shape) == -1


def test_descriptor_size_is_checked_without_a_gpu():
    """Descriptor structs carry struct_size (ABI version 4): a caller built against another
    header layout gets AANET_EABI before anything is read past the struct or launched (ADVICE r3:
    a version-1 caller passed the smaller aanet_csa_epilogue_t and the library read `post` past
    its end)."""
    import ctypes as C
    L = _lib.lib()
    d = _lib.CsaEpilogue()
    assert d.struct_size == C.sizeof(_lib.CsaEpilogue)
    assert _lib.PostStage().struct_size == C.sizeof(_lib.PostStage)
    assert _lib.S2Terms(None, 0).struct_size == C.sizeof(_lib.S2Terms)
    dummy = C.c_void_p(16)  # never dereferenced: the descriptor check comes first
    args = lambda desc: ([None] * 5 + [0, dummy, None, None, 0, 64, None, 1, 64, 8, 8, 64, 3, 3, 1, 1, 1]  # noqa: E731
                         + [C.byref(desc), 1, None])
    d.struct_size -= 8  # the version-1 layout had no `post` pointer
    assert L.aanet_conv2d_pw_f32(*args(d)) == _lib.EABI
    d.struct_size += 8
    p = _lib.PostStage()
    p.struct_size = 8
    d.post = C.pointer(p)
    assert L.aanet_conv2d_pw_f32(*args(d)) == _lib.EABI
    t = _lib.S2Terms(None, 0)
    t.struct_size = 0
    assert L.aanet_conv3x3s2_terms_f32(None, None, None, 1, 32, 8, 8, 16, 16, None, 0, None, 0,
                                       C.byref(t), None) == _lib.EABI


def test_import_leaves_global_torch_flags_alone():
    """importing the package no longer turns TF32 off process-wide; the package's module
    forwards switch it off for their own MIOpen convs and restore it."""
    import subprocess
    import sys
    code = ("import torch; a = torch.backends.cudnn.allow_tf32; import aanet_amd; "
            "from aanet_amd._precision import fp32_convs; "
            "seen = []; f = fp32_convs(lambda: seen.append(torch.backends.cudnn.allow_tf32)); f(); "
            "print(a, torch.backends.cudnn.allow_tf32, seen[0])")
    out = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, text=True,
                         timeout=120).stdout.split()
    assert out == ["True", "True", "False"], out


def test_fp32_scope_covers_the_conv_backward():
    """autograd's conv backward reads the global TF32 flag at loss.backward(), outside
    the decorated forward.  fp32_scope (what Trainer runs its step in) keeps it off there too; a
    bare decorated forward alone does not (the documented reason for the scope)."""
    from aanet_amd._precision import fp32_convs, fp32_scope
    conv = torch.nn.Conv2d(2, 2, 3)
    fwd = fp32_convs(lambda x: conv(x))
    prev = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = True
    try:
        for scoped in (True, False):
            seen = []
            h = conv.weight.register_hook(lambda g: seen.append(torch.backends.cudnn.allow_tf32))
            ctx = fp32_scope() if scoped else contextlib.nullcontext()
            with ctx:
                fwd(torch.randn(1, 2, 5, 5)).sum().backward()
            h.remove()
            assert seen == [not scoped], (scoped, seen)
            assert torch.backends.cudnn.allow_tf32 is True
    finally:
        torch.backends.cudnn.allow_tf32 = prev


def test_ops_fail_loudly_on_cpu_tensors():
    x = torch.zeros(1, 4, 3, 5)
    with pytest.raises(NotImplementedError):
        ops.corr_volume(x, x, 2)
    with pytest.raises(NotImplementedError):
        nets.DisparityEstimation(4)(torch.zeros(1, 4, 3, 5))
    with pytest.raises(NotImplementedError):
        nets.ModulatedDeformConv(4, 4, 3, padding=1)(x, torch.zeros(1, 18, 3, 5), torch.ones(1, 9, 3, 5))


@pytest.mark.parametrize("inter", [True, False])
def test_state_dict_keys_match_reference(inter):
    g = golden("aggregation_inter" if inter else "aggregation_final")
    ref = state_dict_of(g)
    m = nets.AdaptiveAggregation(16, num_scales=3, num_fusions=6, num_stage_blocks=1,
                                 num_deform_blocks=3, intermediate_supervision=inter)
    ours = m.state_dict()
    assert set(ours) == set(ref)
    for k, v in ref.items():
        assert tuple(ours[k].shape) == v.shape, k


def test_hot_path_module_api_mirrors_aanet():
    m = nets.AANetHotPath(64, no_intermediate_supervision=True)
    # AANet eval config (max_disp=192 -> 64): final fusion has one output branch, one final conv
    assert len(m.aggregation.final_conv) == 1
    assert len(m.aggregation.fusions[-1].fuse_layers) == 1
    assert isinstance(m.cost_volume, nets.CostVolumePyramid)
    # the DCN-bearing keys the training LR grouping relies on (utils/utils.py:156-169)
    keys = list(m.state_dict())
    assert any(k.endswith("conv2.offset_conv.weight") for k in keys)
    assert any(k.endswith("conv2.deform_conv.weight") for k in keys)
    w = m.state_dict()["aggregation.fusions.5.branches.0.0.conv2.offset_conv.weight"]
    assert tuple(w.shape) == (54, 32, 3, 3)
    # offset_conv is zero-initialised like the reference (deform.py:74-76)
    assert float(w.abs().sum()) == 0.0


def test_package_exposes_native_library_path():
    assert aanet_amd.native_library_path().endswith("libaanet_mi355x.so")
    assert os.path.exists(aanet_amd.native_library_path())


def test_torch_ops_registered_and_refuse_cpu():
    """torch.ops.aanet.* exist (SURVEY §8b op-level API), shape-propagate through fake kernels,
    and have no CPU kernel (the reference DCN is CUDA-only)."""
    import torch
    import aanet_amd  # noqa: F401  (registers the ops)
    from aanet_amd.torch_ops import OPS
    for name in OPS:
        assert hasattr(torch.ops.aanet, name), name
    from torch._subclasses.fake_tensor import FakeTensorMode
    with FakeTensorMode():
        x = torch.empty(2, 8, 10, 12)
        w = torch.empty(6, 8, 3, 3)
        off, msk = torch.empty(2, 18, 10, 12), torch.empty(2, 9, 10, 12)
        y = torch.ops.aanet.mdcn_forward(x, off, msk, w, None, 1, 2, 2, 1, 1)
        assert tuple(y.shape) == (2, 6, 10, 12)
        v = torch.ops.aanet.corr_volume(x, x, 5)
        assert tuple(v.shape) == (2, 5, 10, 12)
        assert tuple(torch.ops.aanet.disp_regress(v, False).shape) == (2, 10, 12)
    with pytest.raises(NotImplementedError):
        torch.ops.aanet.corr_volume(torch.randn(1, 4, 3, 5), torch.randn(1, 4, 3, 5), 2)


def test_mdcn_backward_workspace_sizes():
    """aanet_mdcn_bwd_ws_workspace_size: the NHWC grad_x accumulator + channels-last x + W^T
    (>= 2*n*c*h*w + co*c*k floats); the deterministic layout holds its int64 accumulators too,
    per chunk of images; invalid shapes give 0."""
    L = _lib.lib()
    n, c, h, w, co = 2, 64, 12, 30, 64
    args = (n, c, h, w, co, 3, 3, 1, 2, 2, 1, 2)
    ws = L.aanet_mdcn_bwd_ws_workspace_size(*args)
    det = L.aanet_mdcn_bwd_det_workspace_size(*args)
    assert ws >= 4 * (2 * n * c * h * w + co * c * 9)
    assert det >= 8 * n * c * h * w + 4 * (n * c * h * w + co * c * 9)
    assert L.aanet_mdcn_bwd_ws_workspace_size(n, 63, h, w, co, 3, 3, 1, 2, 2, 1, 2) == 0  # C % dg
    # the window form's int64 weight-gradient accumulator (co*c*9 int64) is present
    assert det >= 8 * n * c * h * w + 4 * n * c * h * w + 8 * co * c * 9
    # the deterministic backward runs in chunks of images (96 MB of int64 grad_x + channels-last
    # x each): the workspace stops growing with the batch -- agg_s0 (64 channels, 128 x 416) at
    # B = 8 and B = 64 takes the same <= 128 MB (round 4: ~0.9 GB at B = 8)
    agg = (64, 128, 416, 64, 3, 3, 1, 2, 2, 1, 2)
    d8 = L.aanet_mdcn_bwd_det_workspace_size(8, *agg)
    d64 = L.aanet_mdcn_bwd_det_workspace_size(64, *agg)
    assert d8 == d64 and d8 <= 128 << 20
    assert d8 >= 12 * 2 * 64 * 128 * 416  # two images per chunk
    assert L.aanet_mdcn_bwd_det_workspace_size(1, *agg) < d8


def test_window_fwd_support_query_without_a_gpu():
    """aanet_mdcn_window_fwd_supported (the op-level DCN forward's window dispatch) takes exactly
    the aggregation's deformable convs: 3x3, stride 1, pad = dil = 2, one conv group, two
    deformable groups, C = Co in {32, 64, 128}, W % 4 == 0 (nets/deform.py:216-226; 128 channels:
    SURVEY C4's feat_s1 shape)."""
    ok = ops.window_fwd_ok
    assert ok(64, 64, 3, 3, 1, 2, 2, 1, 2, 416) and ok(32, 32, 3, 3, 1, 2, 2, 1, 2, 208)
    assert ok(128, 128, 3, 3, 1, 2, 2, 1, 2, 104)
    assert not ok(16, 16, 3, 3, 1, 2, 2, 1, 2, 104)      # scale 2: 8 channels per group
    assert not ok(128, 128, 3, 3, 1, 1, 1, 1, 2, 104)    # feature DCN
    assert not ok(64, 64, 3, 3, 2, 2, 2, 1, 2, 416)      # stride 2
    assert not ok(64, 64, 3, 3, 1, 2, 2, 1, 2, 26)       # W % 4
    assert not ok(64, 32, 3, 3, 1, 2, 2, 1, 2, 416)      # Co != C
    assert not ok(64, 64, 3, 3, 1, 2, 2, 2, 2, 416)      # conv groups
    assert not ok(64, 64, 3, 3, 1, 1, 1, 1, 2, 416)      # dilation 1


@pytest.mark.parametrize("is_3d", [False, True])
def test_pinned_convs_match_torch_autograd(is_3d):
    """on their first forward the drop-in modules pin their convolutions
    (_precision.pin_fp32_convs) -- same parameters and state dict, class Pinned*, whose autograd
    forward/backward are aten's convolution with TF32 off whoever calls backward.  The values and
    every gradient equal torch's own autograd through the plain modules (here on the CPU, where
    both are the same convolution), for the 2-D / 3-D convs and their transposed forms."""
    import copy

    from aanet_amd import _precision
    from aanet_amd.nets.feature import Conv2x
    torch.manual_seed(0)
    m = Conv2x(8, 4, deconv=True, is_3d=is_3d)
    ref = copy.deepcopy(m)
    ref.__dict__["_aanet_pinned"] = True  # the reference copy keeps plain torch modules
    for mod in ref.modules():
        mod.__dict__["_aanet_pinned"] = True
    shape = (2, 8, 3, 4, 5) if is_3d else (2, 8, 5, 6)
    x = torch.randn(shape, requires_grad=True)
    rem_shape = (2, 4, 5, 8, 10) if is_3d else (2, 4, 10, 12)
    rem = torch.randn(rem_shape, requires_grad=True)
    x2, rem2 = x.detach().clone().requires_grad_(), rem.detach().clone().requires_grad_()
    out, out2 = m(x, rem), ref(x2, rem2)
    pinned = {type(mod) for mod in m.modules() if isinstance(mod, (torch.nn.modules.conv._ConvNd))}
    assert pinned == ({_precision.PinnedConvTranspose3d, _precision.PinnedConv3d} if is_3d else
                      {_precision.PinnedConvTranspose2d, _precision.PinnedConv2d}), pinned
    assert all(type(mod).__module__.startswith("torch") for mod in ref.modules()
               if isinstance(mod, torch.nn.modules.conv._ConvNd))
    assert m.state_dict().keys() == ref.state_dict().keys()
    g = torch.randn(out.shape)
    out.backward(g)
    out2.backward(g)
    assert torch.allclose(out, out2, atol=1e-6)
    assert torch.allclose(x.grad, x2.grad, atol=1e-5) and torch.allclose(rem.grad, rem2.grad, atol=1e-5)
    for (n, p), (_, p2) in zip(m.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p.grad, p2.grad, atol=1e-4, rtol=1e-5), n


@pytest.mark.parametrize("ci,co,h,w", [(8, 4, 5, 7), (3, 6, 1, 1), (16, 8, 4, 9)])
def test_deconv2x_phase_weight_is_the_transposed_conv(ci, co, h, w):
    """ops.deconv2x's decomposition on the CPU: the 2x2 pad-1 conv with the phase weight
    (deconv2x_phase_weight), its output [4c+2a+b][y+a][x+b] scattered to [c][2y+a][2x+b] (what
    aanet_deconv2x_assemble_f32 does), equals ConvTranspose2d(k=4, s=2, p=1) in fp64."""
    g = torch.Generator().manual_seed(ci * 100 + co)
    x = torch.randn(2, ci, h, w, generator=g, dtype=torch.float64)
    wt = torch.randn(ci, co, 4, 4, generator=g, dtype=torch.float64)
    scale = torch.rand(co, generator=g, dtype=torch.float64) + 0.5
    ref = torch.nn.functional.conv_transpose2d(x, wt * scale.view(1, -1, 1, 1), stride=2, padding=1)
    ph = torch.nn.functional.conv2d(x, ops.deconv2x_phase_weight(wt, scale), padding=1)
    assert ph.shape == (2, 4 * co, h + 1, w + 1)
    out = torch.empty_like(ref)
    for a in (0, 1):
        for b in (0, 1):
            out[:, :, a::2, b::2] = ph[:, 2 * a + b::4, a:a + h, b:b + w]
    assert torch.allclose(out, ref, rtol=0, atol=1e-12)
