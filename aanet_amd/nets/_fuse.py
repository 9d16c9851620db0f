"""Eval-mode fusion helpers.  In eval mode without autograd every conv of the ISA/CSA blocks runs
on the HIP implicit-GEMM engine (aanet_conv2d_fused_f32) with the following BatchNorm folded
into its weights/bias (cached per parameter version), the activation and the bottleneck's
residual add in its epilogue.  Training mode never uses these: modules then run the reference
op sequence with autograd.
"""
import torch
import torch.nn as nn

from .. import ops
from .. import _lib
from .._lib import is_nhwc
from .._precision import CONV2D_TYPES


def bn_scale_shift(bn):
    """y = x*scale + shift for an eval-mode BatchNorm2d."""
    scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    shift = bn.bias - bn.running_mean * scale
    return scale, shift


def _key(*tensors):
    return tuple((t.data_ptr(), t._version) for t in tensors if t is not None)


def _bn_tensors(bn):
    """The tensors an eval BN's affine depends on.  A train-mode BN forward updates
    running_mean / running_var inside the kernel WITHOUT bumping their _version, but it always
    bumps num_batches_tracked (an in-place add_ at Python level), so that counter's version is
    part of every cache key; clear_fold_caches() covers writes through `.data`."""
    return (bn.weight, bn.bias, bn.running_mean, bn.running_var,
            getattr(bn, "num_batches_tracked", None))


def clear_fold_caches(module):
    """Drop every folded-weight / BN-affine cache in `module`'s subtree (called on each
    train()/eval() switch of the drop-in modules, see FoldCacheMixin, and by Trainer.graph_step),
    including the split-bf16 packs that ops._split_weight keeps on the weight tensors themselves:
    writes through `.data` and HIP graph replays update a weight without bumping its _version."""
    for m in module.modules():
        for attr in ("_aanet_fold", "_aanet_fold_dense", "_aanet_affine", "_aanet_s2pack",
                     "_aanet_s2pack_k", "_aanet_g3pack"):
            if attr in m.__dict__:
                del m.__dict__[attr]
        for p in m.parameters(recurse=False):
            if "_aanet_split_pack" in p.__dict__:
                del p.__dict__["_aanet_split_pack"]


class FoldCacheMixin:
    """nn.Module.train()/eval() that also invalidates the eval-path caches of the subtree, so an
    eval -> train-mode forward (BN statistics updated in place) -> eval sequence never reuses a
    stale folded BatchNorm."""

    def train(self, mode=True):
        clear_fold_caches(self)
        return super().train(mode)


def folded(conv, bn):
    """(weight, bias, packed weight) of conv followed by eval BN (bn may be None), cached on the
    conv module; the packed copy is the [kh][kw][co][cg] layout the HIP engine streams, carrying
    the split-bf16 fragments too when cg % 32 == 0 (ops.pack_weight_split)."""
    tensors = (conv.weight, conv.bias) + (_bn_tensors(bn) if bn is not None else ())
    key = _key(*tensors)
    cache = getattr(conv, "_aanet_fold", None)
    if cache is not None and cache[0] == key:
        return cache[1], cache[2], cache[3]
    with torch.no_grad():
        if bn is None:
            w = conv.weight.contiguous()
            b = None if conv.bias is None else conv.bias.contiguous()
        else:
            scale, shift = bn_scale_shift(bn)
            w = (conv.weight * scale.view(-1, 1, 1, 1)).contiguous()
            b = shift if conv.bias is None else conv.bias * scale + shift
            b = b.contiguous()
    wp = None
    if w.is_cuda:  # split-bf16 engine buffer where the shape has one, else plain packed f32
        wp = ops.pack_weight_split(w, getattr(conv, "groups", 1))
        if wp is None:
            wp = ops.pack_weight(w)
    conv._aanet_fold = (key, w, b, wp)
    _lib.note_cache_fill()
    return w, b, wp


def deconv2x_ok(conv):
    """A transposed conv the phase form takes (ops.deconv2x): 2-D, 4x4, stride 2, padding 1, no
    output padding / groups / dilation (the hourglasses' Conv2x deconvs)."""
    return isinstance(conv, nn.ConvTranspose2d) and conv.kernel_size == (4, 4) and \
        conv.stride == (2, 2) and conv.padding == (1, 1) and conv.output_padding == (0, 0) and \
        conv.groups == 1 and conv.dilation == (1, 1) and conv.padding_mode == "zeros"


def folded_deconv(conv, bn):
    """(phase weight [4co][ci][2][2], bias [4co], packed weight) of a deconv2x_ok transposed conv
    followed by eval BN (bn may be None), cached on the conv like folded()."""
    tensors = (conv.weight, conv.bias) + (_bn_tensors(bn) if bn is not None else ())
    key = _key(*tensors)
    cache = getattr(conv, "_aanet_fold", None)
    if cache is not None and cache[0] == key:
        return cache[1], cache[2], cache[3]
    with torch.no_grad():
        co = conv.out_channels
        if bn is None:
            scale, shift = None, conv.bias if conv.bias is not None else conv.weight.new_zeros(co)
        else:
            scale, shift = bn_scale_shift(bn)
            if conv.bias is not None:
                shift = conv.bias * scale + shift
        w = ops.deconv2x_phase_weight(conv.weight, scale)
        b = shift.repeat_interleave(4).contiguous()
    wp = ops.pack_weight_split(w)
    if wp is None:
        wp = ops.pack_weight(w)
    conv._aanet_fold = (key, w, b, wp)
    _lib.note_cache_fill()
    return w, b, wp


def deconv_bn_act(x, conv, bn=None, act=None, rem=None, out_nhwc=False):
    """act(BN(conv_transpose(x))) [+ the concat with rem] as the engine phase conv + one assembly
    pass (ops.deconv2x); out_nhwc: channels_last result."""
    w, b, wp = folded_deconv(conv, bn)
    return ops.deconv2x(x, w, b, act, packed_weight=wp, rem=rem, out_nhwc=out_nhwc)


def conv_bn_act_s2(x, conv, bn=None, act=None, owner=None):
    """act(BN(conv(x))) of a 3x3 stride-2 pad-1 conv on the dedicated stride-2 kernel
    (ops.conv3x3_s2: whole-Co tiles, im2col straight into MFMA fragments), or None when the
    shape is outside it (s2_conv_ok, co <= 96); the pack is cached on `owner` (default: conv)."""
    if not s2_conv_ok(conv) or act not in (None, "relu", "leaky"):
        return None
    pk = s2_pack(owner if owner is not None else conv, [(conv, bn)])
    if pk is None:
        return None
    co = conv.out_channels
    return ops.conv3x3_s2(x.contiguous(), pk[0], pk[1], co, co, act_a=act)[0]


def halo_input_ok(conv, c_in):
    """Whether a plain conv gains from channels-last input: a 3x3 stride-1 pad-1 conv, one group,
    split-packed weights, 32-channel K chunks -- the engine's halo tile (mdcn.hip HALO), which
    stages an NHWC input once per chunk instead of an im2col per tap."""
    return engine_conv(conv) and conv.kernel_size == (3, 3) and \
        conv.stride == (1, 1) and conv.padding == (1, 1) and conv.dilation == (1, 1) and \
        conv.groups == 1 and c_in % 32 == 0 and c_in <= 496 and conv.out_channels >= 32


def dense_grouped_ok(conv, x):
    """A 2-group conv whose groups are narrower than the split-bf16 engine's 32-channel K chunk
    (the scale-1 offset_conv: 32 -> 54, two 16-channel groups) but whose full input is a multiple
    of 32 channels: run as ONE ungrouped conv with a block-diagonal weight.  Twice the MACs, but
    on the split-bf16 contraction instead of the exact-f32 16-channel form (C2 scale 1, B=8:
    37 -> 29 us, tools/dense_grouped_bench.py); the
    zero blocks add exact zeros, so only the fp32 summation order differs.  The conv's
    `dense_grouped` option (nets/options.py set_options) False keeps the grouped engine."""
    return conv.groups == 2 and (conv.in_channels // 2) % 32 != 0 and conv.in_channels % 32 == 0 \
        and x.is_cuda and getattr(conv, "aanet_dense_grouped", True)


def folded_dense(conv, bn):
    """folded() of a grouped conv as its block-diagonal ungrouped equivalent, cached on the conv
    under the same parameter-version key."""
    w, b, _ = folded(conv, bn)
    key = conv._aanet_fold[0]
    cache = conv.__dict__.get("_aanet_fold_dense")
    if cache is not None and cache[0] == key:
        return cache[1], cache[2], cache[3]
    with torch.no_grad():
        g, co, cg = conv.groups, w.shape[0], w.shape[1]
        wd = torch.zeros((co, cg * g) + tuple(w.shape[2:]), device=w.device, dtype=w.dtype)
        cog = co // g
        for i in range(g):
            wd[i * cog:(i + 1) * cog, i * cg:(i + 1) * cg] = w[i * cog:(i + 1) * cog]
        wd = wd.contiguous()
        wp = ops.pack_weight_split(wd, 1)
    conv.__dict__["_aanet_fold_dense"] = (key, wd, b, wp)
    _lib.note_cache_fill()
    return wd, b, wp


def s2_pack(owner, pairs):
    """(pre-split fragments, bias) of the 3x3 stride-2 convs `pairs` = [(conv, bn), ...] (BN
    folded) concatenated along the output channels, for ops.conv3x3_s2; cached on `owner`, keyed
    by the folded weights' cache keys.  None when the shape is outside the kernel."""
    fs = [folded(c, b) for c, b in pairs]
    key = tuple(c._aanet_fold[0] for c, _ in pairs)
    cache = owner.__dict__.get("_aanet_s2pack")
    if cache is not None and cache[0] == key:
        return cache[1]
    with torch.no_grad():
        w = torch.cat([f[0] for f in fs])
        b = torch.cat([f[1] if f[1] is not None else torch.zeros(f[0].shape[0], device=w.device)
                       for f in fs]).contiguous()
        wsplit = ops.pack_conv3x3s2(w)
    val = None if wsplit is None else (wsplit, b)
    owner.__dict__["_aanet_s2pack"] = (key, val)
    _lib.note_cache_fill()
    return val


def s2_pack_k(owner, pairs):
    """(pre-split fragments, bias) of the 3x3 stride-2 convs `pairs` = [(conv, bn), ...] (BN
    folded) concatenated along the INPUT channels, biases summed: one conv over the channel-
    concatenated inputs whose output is the sum of theirs (ops.conv3x3_s2 with x2).  Cached on
    `owner` like s2_pack; None outside the kernel."""
    fs = [folded(c, b) for c, b in pairs]
    key = tuple(c._aanet_fold[0] for c, _ in pairs)
    cache = owner.__dict__.get("_aanet_s2pack_k")
    if cache is not None and cache[0] == key:
        return cache[1]
    with torch.no_grad():
        w = torch.cat([f[0] for f in fs], 1)
        b = None
        for f in fs:
            if f[1] is not None:
                b = f[1].clone() if b is None else b + f[1]
        if b is None:
            b = torch.zeros(w.shape[0], device=w.device)
        wsplit = ops.pack_conv3x3s2(w)
    val = None if wsplit is None else (wsplit, b.contiguous())
    owner.__dict__["_aanet_s2pack_k"] = (key, val)
    _lib.note_cache_fill()
    return val


def offset_conv_pack(conv):
    """(pre-split fragments, bias) of a deformable offset_conv for ops.conv3x3_grouped_nhwc,
    cached on the conv and keyed by its folded weights; None when the conv is outside the kernel
    (3x3, stride 1, padding = dilation, 32k channels per group, <= 32 outputs per group).
    Round 4: the kernel is the halo form owning every group of its tile (conv_g3.hip): 94-95 vs
    102-103 us for the engine's halo form at C2 scale 0, step 3.636 vs 3.662 ms (same call,
    DESIGN.md 3), so it is the default; the round-3 direct form was slower than the engine."""
    if not engine_conv(conv) or _int(conv.kernel_size) != 3 or _int(conv.stride) != 1 or \
            _int(conv.padding) != _int(conv.dilation) or \
            (conv.in_channels // conv.groups) % 32 or (conv.out_channels // conv.groups) > 32:
        return None
    w, b, _ = folded(conv, None)
    key = conv._aanet_fold[0]
    cache = conv.__dict__.get("_aanet_g3pack")
    if cache is not None and cache[0] == key:
        return cache[1]
    with torch.no_grad():
        wsplit = ops.pack_conv3x3_grouped(w, conv.groups)
        bias = b.contiguous() if b is not None else None
    val = None if wsplit is None else (wsplit, bias)
    conv.__dict__["_aanet_g3pack"] = (key, val)
    _lib.note_cache_fill()
    return val


def offset_conv_eval(x, conv):
    """Eval offset_conv: the grouped direct kernel when x is channels-last and the conv fits
    (offset_conv_pack), else the conv engine (conv_bn_act)."""
    pk = offset_conv_pack(conv) if is_nhwc(x) else None
    if pk is None:
        return conv_bn_act(x, conv)
    try:
        return ops.conv3x3_grouped_nhwc(x, pk[0], pk[1], conv.out_channels, conv.groups,
                                        _int(conv.dilation))
    except _lib.AanetError as e:
        if e.status != _lib.EUNSUPPORTED:
            raise
        return conv_bn_act(x, conv)


def s2_conv_ok(conv):
    """A conv of the CSA down chains that ops.conv3x3_s2 takes (3x3, stride 2, pad 1, plain)."""
    return engine_conv(conv) and _int(conv.kernel_size) == 3 and \
        _int(conv.stride) == 2 and _int(conv.padding) == 1 and _int(conv.dilation) == 1 and \
        conv.groups == 1 and conv.in_channels % 32 == 0 and conv.out_channels % 16 == 0 and \
        conv.out_channels <= 96


def bn_affine(bn):
    """(scale, shift) of an eval BN, cached on the BN module (for kernel epilogues)."""
    key = _key(*_bn_tensors(bn))
    cache = getattr(bn, "_aanet_affine", None)
    if cache is not None and cache[0] == key:
        return cache[1], cache[2]
    with torch.no_grad():
        scale, shift = bn_scale_shift(bn)
        scale, shift = scale.contiguous(), shift.contiguous()
    bn._aanet_affine = (key, scale, shift)
    _lib.note_cache_fill()
    return scale, shift


def _int(v):
    return v[0] if isinstance(v, (tuple, list)) else v


def conv_bn_act(x, conv, bn=None, act=None, residual=None, out_nhwc=False):
    """act(BN(conv(x)) [+ residual]) as ONE HIP kernel (BN folded into the conv).  A channels_last
    x is read as NHWC in place; out_nhwc=True returns a channels_last (NHWC) tensor."""
    groups = conv.groups
    if dense_grouped_ok(conv, x):
        w, b, wp = folded_dense(conv, bn)
        groups = 1
    else:
        w, b, wp = folded(conv, bn)
    for v in (conv.stride, conv.padding, conv.dilation):
        if isinstance(v, (tuple, list)) and v[0] != v[1]:
            raise NotImplementedError("asymmetric conv parameters")
    xin = x if is_nhwc(x) else x.contiguous()
    return ops.conv2d_fused(xin, w, b, _int(conv.stride), _int(conv.padding),
                            _int(conv.dilation), groups, act, residual, packed_weight=wp,
                            out_nhwc=out_nhwc)


def use_fused(module, x):
    """Fast path only in eval mode, without autograd, on the HIP device."""
    return (not module.training) and x.is_cuda and not torch.is_grad_enabled() and \
        getattr(module, "aanet_fuse", True)


def act_name(m):
    """Engine epilogue name of an activation module (None: identity; False: not expressible)."""
    if m is None:
        return None
    if isinstance(m, nn.ReLU):
        return "relu"
    if isinstance(m, nn.LeakyReLU) and m.negative_slope == 0.2:
        return "leaky"
    return False


def engine_conv(conv):
    """A conv the HIP implicit-GEMM engine runs (plain 2-D, zero padding, square parameters)."""
    if type(conv) not in CONV2D_TYPES or conv.padding_mode != "zeros" or isinstance(conv.padding, str):
        return False
    return all(v[0] == v[1] for v in (conv.stride, conv.padding, conv.dilation, conv.kernel_size))


def _leaves(seq):
    for m in seq:
        if isinstance(m, nn.Sequential):
            yield from _leaves(m)
        else:
            yield m


def run_fused_chain(mods, x):
    """Run a flat module list in eval: each conv [+ BatchNorm2d] [+ ReLU | LeakyReLU(0.2)] run of
    it is ONE HIP engine kernel; anything else (pooling, transposed convs, ...) runs as is."""
    i, n = 0, len(mods)
    while i < n:
        m = mods[i]
        if engine_conv(m):
            bn = act = None
            j = i + 1
            if j < n and isinstance(mods[j], nn.BatchNorm2d):
                bn, j = mods[j], j + 1
            if j < n and act_name(mods[j]) not in (None, False):
                act, j = act_name(mods[j]), j + 1
            x = conv_bn_act(x, m, bn, act)
            i = j
        else:
            x = m(x)
            i += 1
    return x


class FusedSequential(FoldCacheMixin, nn.Sequential):
    """nn.Sequential with the reference's children (same state-dict keys, nesting allowed) that
    in eval mode without autograd runs its conv/BN/activation runs as HIP engine kernels
    (run_fused_chain); training / autograd runs the children in order."""

    def forward(self, x):
        if use_fused(self, x):
            return run_fused_chain(list(_leaves(self)), x)
        return super().forward(x)


ConvBNAct = FusedSequential
