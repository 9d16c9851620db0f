"""Torch-facing ops over the C ABI (autograd Functions + functional forms).

Each op allocates its outputs with torch (caching allocator, device memory) and launches on
torch's current HIP stream through ``_lib.call`` -- capturable into a HIP graph.
"""
import ctypes

import torch
from torch.autograd import Function
from torch.autograd.function import once_differentiable

from . import _lib
from ._lib import call, ptr, require_gpu, stream_of


def _out_size(n, k, s, p, d):
    return (n + 2 * p - (d * (k - 1) + 1)) // s + 1


# ------------------------------------------------------------------ cost volumes --------
def corr_volume(left, right, max_disp, out=None):
    """nets/cost.py:40-48 -> [B, D, H, W]."""
    require_gpu(left, right, names=("left", "right"))
    B, C, H, W = left.shape
    if right.shape != left.shape:
        raise ValueError("left/right feature shapes differ")
    if out is None:
        out = torch.empty((B, max_disp, H, W), device=left.device, dtype=left.dtype)
    call("aanet_corr_volume_f32", ptr(left), ptr(right), ptr(out), B, C, H, W, max_disp,
         stream_of(left))
    return out


def corr_pyramid(lefts, rights, max_disp):
    """nets/cost.py:58-76 (correlation): scale s -> [B, max_disp >> s, H_s, W_s], every scale in
    ONE launch (aanet_corr_pyramid_f32)."""
    ns = len(lefts)
    if ns == 0 or len(rights) != ns:
        raise ValueError("left/right pyramids must have the same, non-zero number of scales")
    require_gpu(*lefts, *rights)
    B = lefts[0].shape[0]
    outs = []
    for s, (l, r) in enumerate(zip(lefts, rights)):
        if l.shape != r.shape or l.shape[0] != B:
            raise ValueError("left/right feature shapes differ")
        outs.append(torch.empty((B, max_disp >> s) + tuple(l.shape[2:]), device=l.device, dtype=l.dtype))
    arr = lambda ts: (_lib.ctypes.c_void_p * ns)(*[t.data_ptr() for t in ts])  # noqa: E731
    ints = lambda vals: (_lib.ctypes.c_int * ns)(*vals)  # noqa: E731
    call("aanet_corr_pyramid_f32", ns, arr(lefts), arr(rights), arr(outs),
         ints([l.shape[1] for l in lefts]), ints([l.shape[2] for l in lefts]),
         ints([l.shape[3] for l in lefts]), B, max_disp, stream_of(lefts[0]))
    return outs


def shift_volume(left, right, max_disp, concat):
    """nets/cost.py:22-38 (difference / concat) -> [B, C', D, H, W]."""
    require_gpu(left, right, names=("left", "right"))
    B, C, H, W = left.shape
    oc = 2 * C if concat else C
    out = torch.empty((B, oc, max_disp, H, W), device=left.device, dtype=left.dtype)
    name = "aanet_concat_volume_f32" if concat else "aanet_diff_volume_f32"
    call(name, ptr(left), ptr(right), ptr(out), B, C, H, W, max_disp, stream_of(left))
    return out


class CorrelationVolumeFunction(Function):
    @staticmethod
    def forward(ctx, left, right, max_disp):
        left, right = left.contiguous(), right.contiguous()
        ctx.save_for_backward(left, right)
        ctx.max_disp = max_disp
        return corr_volume(left, right, max_disp)

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_out):
        left, right = ctx.saved_tensors
        grad_out = grad_out.contiguous()
        require_gpu(grad_out, names=("grad_out",))
        gl, gr = torch.empty_like(left), torch.empty_like(right)
        B, C, H, W = left.shape
        call("aanet_corr_volume_bwd_f32", ptr(left), ptr(right), ptr(grad_out), ptr(gl), ptr(gr),
             B, C, H, W, ctx.max_disp, stream_of(left))
        return gl, gr, None


class CorrelationPyramidFunction(Function):
    """CostVolumePyramid (correlation) forward in one launch; backward per scale
    (aanet_corr_volume_bwd_f32).  apply(max_disp, ns, *lefts, *rights) -> ns volumes."""

    @staticmethod
    def forward(ctx, max_disp, ns, *feats):
        lefts = [t.contiguous() for t in feats[:ns]]
        rights = [t.contiguous() for t in feats[ns:]]
        ctx.save_for_backward(*lefts, *rights)
        ctx.max_disp, ctx.ns = max_disp, ns
        return tuple(corr_pyramid(lefts, rights, max_disp))

    @staticmethod
    @once_differentiable
    def backward(ctx, *grads):
        saved = ctx.saved_tensors
        ns = ctx.ns
        gls, grs = [], []
        for s in range(ns):
            left, right = saved[s], saved[ns + s]
            if grads[s] is None:
                gls.append(None)
                grs.append(None)
                continue
            g = grads[s].contiguous()
            gl, gr = torch.empty_like(left), torch.empty_like(right)
            B, C, H, W = left.shape
            call("aanet_corr_volume_bwd_f32", ptr(left), ptr(right), ptr(g), ptr(gl), ptr(gr),
                 B, C, H, W, ctx.max_disp >> s, stream_of(left))
            gls.append(gl)
            grs.append(gr)
        return (None, None, *gls, *grs)


class ShiftVolumeFunction(Function):
    @staticmethod
    def forward(ctx, left, right, max_disp, concat):
        left, right = left.contiguous(), right.contiguous()
        ctx.shape, ctx.max_disp, ctx.concat = left.shape, max_disp, concat
        return shift_volume(left, right, max_disp, concat)

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_out):
        grad_out = grad_out.contiguous()
        require_gpu(grad_out, names=("grad_out",))
        B, C, H, W = ctx.shape
        gl = grad_out.new_empty((B, C, H, W))
        gr = grad_out.new_empty((B, C, H, W))
        name = "aanet_concat_volume_bwd_f32" if ctx.concat else "aanet_diff_volume_bwd_f32"
        call(name, ptr(grad_out), ptr(gl), ptr(gr), B, C, H, W, ctx.max_disp, stream_of(grad_out))
        return gl, gr, None, None


# ------------------------------------------------------------ disparity regression ------
def disp_regress(cost, negate=False, out=None):
    """nets/estimation.py:13-30 -> [B, H, W]."""
    require_gpu(cost, names=("cost",))
    B, D, H, W = cost.shape
    if out is None:
        out = torch.empty((B, H, W), device=cost.device, dtype=cost.dtype)
    call("aanet_disp_regress_f32", ptr(cost), ptr(out), B, D, H, W, int(bool(negate)),
         stream_of(cost))
    return out


class DisparityRegressionFunction(Function):
    @staticmethod
    def forward(ctx, cost, negate):
        cost = cost.contiguous()
        ctx.save_for_backward(cost)
        ctx.negate = negate
        return disp_regress(cost, negate)

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_disp):
        (cost,) = ctx.saved_tensors
        grad_disp = grad_disp.contiguous()
        require_gpu(grad_disp, names=("grad_disp",))
        gc = torch.empty_like(cost)
        B, D, H, W = cost.shape
        call("aanet_disp_regress_bwd_f32", ptr(cost), ptr(grad_disp), ptr(gc), B, D, H, W,
             int(bool(ctx.negate)), stream_of(cost))
        return gc, None


# ------------------------------------------------------------------ disparity warp ------
def disp_warp(img, disp, with_mask=True):
    """nets/warp.py:41-64 (padding 'border') -> (warped [B,C,H,W], valid mask or None)."""
    require_gpu(img, disp, names=("img", "disp"))
    B, C, H, W = img.shape
    if tuple(disp.shape) != (B, 1, H, W):
        raise ValueError(f"disp must be [B, 1, H, W] = {(B, 1, H, W)}, got {tuple(disp.shape)}")
    warped = torch.empty_like(img)
    valid = torch.empty_like(img) if with_mask else None
    call("aanet_disp_warp_f32", ptr(img), ptr(disp), ptr(warped), ptr(valid), B, C, H, W,
         stream_of(img))
    return warped, valid


class DispWarpFunction(Function):
    """Warped image with autograd to the disparity (and to the image when it requires grad)."""

    @staticmethod
    def forward(ctx, img, disp):
        img, disp = img.contiguous(), disp.contiguous()
        ctx.save_for_backward(img, disp)
        return disp_warp(img, disp, with_mask=False)[0]

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_warped):
        img, disp = ctx.saved_tensors
        grad_warped = grad_warped.contiguous()
        require_gpu(grad_warped, names=("grad_warped",))
        gd = torch.empty_like(disp)
        gi = torch.zeros_like(img) if ctx.needs_input_grad[0] else None
        B, C, H, W = img.shape
        call("aanet_disp_warp_bwd_f32", ptr(img), ptr(disp), ptr(grad_warped), ptr(gd), ptr(gi),
             B, C, H, W, stream_of(img))
        return gi, gd


# ------------------------------------------------------- modulated deformable conv ------
def window_fwd_ok(C, Co, kh, kw, stride, padding, dilation, groups, deformable_groups, W):
    """Whether the LDS-window DCN kernel takes an op-level forward shape
    (aanet_mdcn_window_fwd_supported): the aggregation's deformable convs -- 3x3, stride 1,
    padding = dilation = 2, one conv group, two deformable groups of 64, 32 or 16 channels
    (C = Co = 128, 64 or 32), W % 4 == 0."""
    return bool(_lib.lib().aanet_mdcn_window_fwd_supported(C, Co, kh, kw, stride, padding, dilation,
                                                           groups, deformable_groups, W))


def _split_weight(weight):
    """pack_weight_split(weight), kept on the weight tensor itself with the (storage, version,
    shape) it was packed from: an optimizer step bumps the version, so training re-packs once per
    step; eval packs once.  (A module-level dict keyed by data_ptr returned a freed weight's packing
    to a new tensor that reused its address at version 0.)  During HIP graph capture it always
    packs, so every replay re-packs from the weights' current values."""
    key = (weight.data_ptr(), weight._version, tuple(weight.shape))
    capturing = torch.cuda.is_current_stream_capturing()
    hit = getattr(weight, "_aanet_split_pack", None)
    if hit is not None and hit[0] == key and not capturing:
        return hit[1]
    wp = pack_weight_split(weight)
    if not capturing:
        try:
            weight._aanet_split_pack = (key, wp)
            _lib.note_cache_fill()
        except (AttributeError, RuntimeError):
            pass
    return wp


def direct_fwd_ok(C, Co, kh, kw, stride, padding, dilation, groups, deformable_groups):
    """Whether the DCN forward entry points take the direct few-channel kernel (dcn_small.hip
    dcn_small_supported: 16 channels in two 8-channel groups, Co = 16, 3x3, stride 1, pad = dil)."""
    return (C, Co, kh, kw, stride, groups, deformable_groups) == (16, 16, 3, 3, 1, 1, 2) and \
        padding == dilation >= 1


def mdcn_forward(x, offset, mask, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
                 deformable_groups=1, out=None, algo="auto"):
    """deform_conv_cuda.cpp:490-569 -> [N, Co, Ho, Wo].

    algo "auto": the aggregation's DCN shapes (window_fwd_ok) run the LDS-window kernel on the
    split-bf16 contraction (weights packed by pack_weight_split, cached per weight version),
    the rest aanet_mdcn_fwd_f32 (16 channels in two groups: the direct kernel, dcn_small.hip;
    else the generic engine); "generic" forces the generic engine (AANET_CONV_GENERIC_DCN)."""
    require_gpu(x, offset, mask, weight, bias, names=("input", "offset", "mask", "weight", "bias"))
    N, C, H, W = x.shape
    Co, _, kh, kw = weight.shape
    Ho, Wo = _out_size(H, kh, stride, padding, dilation), _out_size(W, kw, stride, padding, dilation)
    if out is None:
        out = torch.empty((N, Co, Ho, Wo), device=x.device, dtype=x.dtype)
    if algo == "auto" and not _lib.exact_f32_enabled() and \
            window_fwd_ok(C, Co, kh, kw, stride, padding, dilation, groups, deformable_groups, W):
        wp = _split_weight(weight)
        K = kh * kw
        call("aanet_mdcn_fwd_fused_f32", ptr(x), ptr(offset), 2 * deformable_groups * K * Ho * Wo,
             ptr(mask), deformable_groups * K * Ho * Wo, 0, 1.0, ptr(wp), 1, ptr(bias), None, None,
             0, ptr(out), N, C, H, W, Co, kh, kw, stride, padding, dilation, groups,
             deformable_groups, _lib.CONV_WEIGHTS_SPLIT, stream_of(x))
        return out
    if algo == "generic":
        K = kh * kw
        call("aanet_mdcn_fwd_fused_f32", ptr(x), ptr(offset), 2 * deformable_groups * K * Ho * Wo,
             ptr(mask), deformable_groups * K * Ho * Wo, 0, 1.0, ptr(weight), 0, ptr(bias), None,
             None, 0, ptr(out), N, C, H, W, Co, kh, kw, stride, padding, dilation, groups,
             deformable_groups, _lib.CONV_GENERIC_DCN, stream_of(x))
        return out
    call("aanet_mdcn_fwd_f32", ptr(x), ptr(offset), ptr(mask), ptr(weight), ptr(bias), ptr(out),
         N, C, H, W, Co, kh, kw, stride, padding, dilation, groups, deformable_groups, stream_of(x))
    return out


def mdcn_forward_fused(x, offset_mask, weight, bias=None, post_scale=None, post_shift=None, act=None,
                       stride=1, padding=0, dilation=1, deformable_groups=1, mask_scale=2.0,
                       packed_weight=None, groups=1):
    """Eval fast path of DeformConv2d (nets/deform.py:78-97) + BN + activation.

    offset_mask is the raw offset_conv output [N, dg*3*K, Ho, Wo]: channels [0, 2*dg*K) are
    offsets, the rest mask logits (m = mask_scale * sigmoid), read in place (no slicing copies).
    """
    require_gpu(x, offset_mask, weight, bias, post_scale, post_shift, packed_weight,
                names=("input", "offset_mask", "weight", "bias", "post_scale", "post_shift", "packed"),
                nhwc_ok=(0,))
    N, C, H, W = x.shape
    Co, Cg, kh, kw = weight.shape
    if groups < 1 or C % groups or Co % groups or Cg * groups != C:
        raise ValueError(f"weight {tuple(weight.shape)} does not match input channels {C} / groups {groups}")
    K = kh * kw
    layout = (_lib.LAYOUT_IN_NHWC if _lib.is_nhwc(x) else 0) | _lib.conv_flags(packed_weight)
    Ho, Wo = _out_size(H, kh, stride, padding, dilation), _out_size(W, kw, stride, padding, dilation)
    if offset_mask.shape != (N, deformable_groups * 3 * K, Ho, Wo):
        raise ValueError(f"offset_mask shape {tuple(offset_mask.shape)} unexpected")
    out = torch.empty((N, Co, Ho, Wo), device=x.device, dtype=x.dtype)
    bs = offset_mask.stride(0)
    mask_ptr = offset_mask.data_ptr() + 4 * deformable_groups * 2 * K * Ho * Wo
    wsrc = packed_weight if packed_weight is not None else weight
    call("aanet_mdcn_fwd_fused_f32", ptr(x), ptr(offset_mask), bs, _lib.ctypes.c_void_p(mask_ptr),
         bs, 1, float(mask_scale), ptr(wsrc), int(packed_weight is not None), ptr(bias),
         ptr(post_scale), ptr(post_shift),
         ACT[act] if not isinstance(act, int) else act, ptr(out), N, C, H, W, Co, kh, kw, stride,
         padding, dilation, groups, deformable_groups, layout, stream_of(x))
    return out


ACT = {None: 0, "relu": 1, "leaky": 2}


def pack_weight(weight):
    """[co][cg][kh][kw] -> [kh][kw][co][cg] (aanet_conv_weight_pack_f32)."""
    require_gpu(weight, names=("weight",))
    Co, Cg, kh, kw = weight.shape
    out = torch.empty((kh, kw, Co, Cg), device=weight.device, dtype=weight.dtype)
    call("aanet_conv_weight_pack_f32", ptr(weight), ptr(out), Co, Cg, kh, kw, stream_of(weight))
    return out


def pack_weight_split(weight, groups=1):
    """Weight buffer of the split-bf16 contraction (aanet_conv_weight_pack_split_f32): the
    pack_weight layout, followed in the same allocation by the bf16 piece fragments.  Returned as
    the [kh][kw][co][cg] float view of its head (so it is also a valid pack_weight result) and
    tagged ``_aanet_split``; None when the shape has no split form (cg % 32 != 0)."""
    require_gpu(weight, names=("weight",))
    Co, Cg, kh, kw = weight.shape
    nbytes = _lib.lib().aanet_conv_weight_pack_split_bytes(Co, Cg, kh, kw, groups)
    if nbytes <= 0:
        return None
    buf = torch.empty(nbytes // 4, device=weight.device, dtype=torch.float32)
    call("aanet_conv_weight_pack_split_f32", ptr(weight.contiguous()), ptr(buf), Co, Cg, kh, kw,
         groups, stream_of(weight))
    wp = buf[: Co * Cg * kh * kw].view(kh, kw, Co, Cg)
    wp._aanet_split = True
    wp._aanet_buf = buf
    return wp


def conv2d_fused(x, weight, bias=None, stride=1, padding=0, dilation=1, groups=1, act=None,
                 residual=None, post_scale=None, post_shift=None, packed_weight=None,
                 out_nhwc=False):
    """Plain conv on the HIP implicit-GEMM engine: act(post_scale*(conv+bias)+post_shift+residual).
    weight gives the shape ([co][cg][kh][kw]); packed_weight (pack_weight(weight)) if given is
    what the kernel reads, and then `weight` may be just that shape (a tuple).  x may be
    channels_last (NHWC staging); out_nhwc=True returns a channels_last tensor (residual then
    channels_last too).  NHWC needs packed_weight and 32-channel groups (AANET_LAYOUT_*)."""
    if not torch.is_tensor(weight):
        if packed_weight is None:
            raise ValueError("a weight shape alone needs packed_weight")
        weight_shape, weight = tuple(weight), None
    else:
        weight_shape = tuple(weight.shape)
    require_gpu(x, weight, bias, residual, post_scale, post_shift, packed_weight,
                names=("input", "weight", "bias", "residual", "post_scale", "post_shift", "packed"),
                nhwc_ok=(0, 3) if out_nhwc else (0,))
    N, C, H, W = x.shape
    Co, _, kh, kw = weight_shape
    Ho, Wo = _out_size(H, kh, stride, padding, dilation), _out_size(W, kw, stride, padding, dilation)
    if residual is not None and tuple(residual.shape) != (N, Co, Ho, Wo):
        raise ValueError("residual shape must match the output")
    layout = ((_lib.LAYOUT_IN_NHWC if _lib.is_nhwc(x) else 0) | (_lib.LAYOUT_OUT_NHWC if out_nhwc else 0)
              | _lib.conv_flags(packed_weight))
    if residual is not None and out_nhwc and not (_lib.is_nhwc(residual) or Co == 1):
        raise ValueError("residual must be channels_last when out_nhwc=True")
    out = torch.empty((N, Co, Ho, Wo), device=x.device, dtype=x.dtype,
                      memory_format=torch.channels_last if out_nhwc else torch.contiguous_format)
    wsrc = packed_weight if packed_weight is not None else weight
    call("aanet_conv2d_fused_f32", ptr(x), ptr(wsrc), ptr(bias), ptr(post_scale), ptr(post_shift),
         ptr(residual), ACT[act], int(packed_weight is not None), ptr(out), N, C, H, W, Co, kh, kw,
         stride, padding, dilation, groups, layout, stream_of(x))
    return out


def _post_stage(out, post):
    """(aanet_post_stage_t, {"out": NHWC tensor or None, "disp": tensor or None}) for a tail
    kernel's post stage; post = dict(packed=<pack_weight_split buffer of a [64][64][1][1]
    weight, BN folded>, bias=<[64] or None>, act="relu"/None, nhwc=bool, disp=bool,
    skip_outputs=bool: the tail's own outputs are left unwritten)."""
    if post is None:
        return None, None
    require_gpu(post["packed"], post.get("bias"))
    N, _, H, W = out.shape
    res = {"out": None, "disp": None}
    ps = _lib.PostStage()
    ps.weight = post["packed"].data_ptr()
    ps.bias = 0 if post.get("bias") is None else post["bias"].data_ptr()
    ps.act = ACT[post.get("act")]
    ps.skip_outputs = int(bool(post.get("skip_outputs")))
    if post.get("nhwc"):
        res["out"] = torch.empty((N, 64, H, W), device=out.device, dtype=out.dtype,
                                 memory_format=torch.channels_last)
        ps.out_nhwc = res["out"].data_ptr()
    if post.get("disp"):
        res["disp"] = torch.empty((N, H, W), device=out.device, dtype=out.dtype)
        ps.disp = res["disp"].data_ptr()
    return ps, res


def _call_tail(name, desc, ps, args_before, args_after):
    """Call a tail kernel with its CSA descriptor; a post stage the kernel cannot take
    (AANET_EUNSUPPORTED, returned before any launch) is dropped and the call repeated without
    it.  -> whether the post stage ran."""
    if desc is not None and ps is not None:
        desc.post = _lib.ctypes.pointer(ps)
        try:
            call(name, *args_before, _lib.ctypes.byref(desc), *args_after)
            return True
        except _lib.AanetError as e:
            if e.status != _lib.EUNSUPPORTED:
                raise
        desc.post = None
    call(name, *args_before, None if desc is None else _lib.ctypes.byref(desc), *args_after)
    return False


def _csa_epilogue(out, csa_up, csa_act):
    """(aanet_csa_epilogue_t, its output) for the tail kernels; csa_up: the coarser exchange
    terms [n][co2][h/r][w/r] (r = 2 or 4) summed into this output branch."""
    if csa_up is None:
        return None, None
    if len(csa_up) > 3:
        raise ValueError("at most 3 upsampled CSA terms")
    require_gpu(*csa_up)
    csa_out = torch.empty_like(out)
    d = _lib.CsaEpilogue()
    d.out = csa_out.data_ptr()
    d.num_up = len(csa_up)
    for j, t in enumerate(csa_up):
        if t.shape[:2] != out.shape[:2]:
            raise ValueError("CSA term batch/channels must match the output")
        d.up[j] = t.data_ptr()
        d.up_h[j], d.up_w[j] = t.shape[2], t.shape[3]
    d.act = ACT[csa_act]
    return d, csa_out


def conv2d_pw(x, weight, packed_weight, bias, post_scale, post_shift, act, pw_packed, pw_bias,
              residual=None, pw_act=None, stride=1, padding=0, dilation=1, csa_up=None,
              csa_act="leaky", post=None):
    """Plain conv + fused pointwise tail (bottleneck conv2 -> conv3, aanet_conv2d_pw_f32).
    x may be channels_last (NHWC staging); the output is NCHW.  csa_up (list of coarser
    exchange terms): also return the CSA sum act(out + up(csa_up...)) -> (out, csa_out).
    post (with csa_up; see _post_stage): -> (out, csa_out, post results or None when the kernel
    did not take the stage)."""
    require_gpu(x, packed_weight, bias, post_scale, post_shift, pw_packed, pw_bias, residual,
                nhwc_ok=(0,))
    N, C, H, W = x.shape
    Co, _, kh, kw = weight.shape
    Co2 = pw_packed.shape[-2]
    Ho, Wo = _out_size(H, kh, stride, padding, dilation), _out_size(W, kw, stride, padding, dilation)
    out = torch.empty((N, Co2, Ho, Wo), device=x.device, dtype=x.dtype)
    desc, csa_out = _csa_epilogue(out, csa_up, csa_act)
    ps, pres = _post_stage(out, post if desc is not None else None)
    ran = _call_tail("aanet_conv2d_pw_f32",
                     desc, ps,
                     (ptr(x), ptr(packed_weight), ptr(bias), ptr(post_scale), ptr(post_shift),
                      ACT[act], ptr(pw_packed), ptr(pw_bias), ptr(residual), ACT[pw_act], Co2,
                      ptr(out), N, C, H, W, Co, kh, kw, stride, padding, dilation),
                     ((_lib.LAYOUT_IN_NHWC if _lib.is_nhwc(x) else 0)
                      | _lib.conv_flags(packed_weight, pw_packed), stream_of(x)))
    if desc is None:
        return out
    return (out, csa_out) if post is None else (out, csa_out, pres if ran else None)


def mdcn_pw(x, offset_mask, weight, packed_weight, bias, post_scale, post_shift, act, pw_packed,
            pw_bias, residual=None, pw_act=None, stride=1, padding=0, dilation=1,
            deformable_groups=1, mask_scale=2.0, csa_up=None, csa_act="leaky", generic_dcn=False,
            post=None):
    """DCN (offset/mask read in place from offset_conv's output) + fused pointwise tail.
    x may be channels_last (NHWC corner loads); the output is NCHW.  csa_up, post: as conv2d_pw.
    generic_dcn: keep the generic engine where the LDS-window tail would run (A/B, tests)."""
    require_gpu(x, offset_mask, packed_weight, bias, post_scale, post_shift, pw_packed, pw_bias,
                residual, nhwc_ok=(0,))
    N, C, H, W = x.shape
    Co, _, kh, kw = weight.shape
    K = kh * kw
    Co2 = pw_packed.shape[-2]
    Ho, Wo = _out_size(H, kh, stride, padding, dilation), _out_size(W, kw, stride, padding, dilation)
    if offset_mask.shape != (N, deformable_groups * 3 * K, Ho, Wo):
        raise ValueError(f"offset_mask shape {tuple(offset_mask.shape)} unexpected")
    out = torch.empty((N, Co2, Ho, Wo), device=x.device, dtype=x.dtype)
    desc, csa_out = _csa_epilogue(out, csa_up, csa_act)
    ps, pres = _post_stage(out, post if desc is not None else None)
    bs = offset_mask.stride(0)
    mask_ptr = offset_mask.data_ptr() + 4 * deformable_groups * 2 * K * Ho * Wo
    ran = _call_tail("aanet_mdcn_pw_f32", desc, ps,
                     (ptr(x), ptr(offset_mask), bs, _lib.ctypes.c_void_p(mask_ptr), bs, 1,
                      float(mask_scale), ptr(packed_weight), ptr(bias), ptr(post_scale),
                      ptr(post_shift), ACT[act], ptr(pw_packed), ptr(pw_bias), ptr(residual),
                      ACT[pw_act], Co2, ptr(out), N, C, H, W, Co, kh, kw, stride, padding,
                      dilation, deformable_groups),
                     ((_lib.LAYOUT_IN_NHWC if _lib.is_nhwc(x) else 0)
                      | _lib.conv_flags(packed_weight, pw_packed)
                      | (_lib.CONV_GENERIC_DCN if generic_dcn else 0), stream_of(x)))
    if desc is None:
        return out
    return (out, csa_out) if post is None else (out, csa_out, pres if ran else None)


_DECONV_TAP = ((3, 1), (2, 0))  # [phase][2x2 tap] -> 4x4 transposed-conv tap (deconv.hip)


def deconv2x_phase_weight(weight, scale=None):
    """ConvTranspose2d(k=4, s=2, p=1) weight [ci][co][4][4] (times a per-output-channel scale,
    e.g. a folded BN) -> the [4co][ci][2][2] weight of the equivalent 2x2 pad-1 conv whose output
    channel 4c + 2a + b is the phase (a, b) of output channel c (deconv.hip)."""
    ci, co = weight.shape[:2]
    if tuple(weight.shape[2:]) != (4, 4):
        raise ValueError("deconv2x: 4x4 kernels only")
    w = weight if scale is None else weight * scale.view(1, -1, 1, 1)
    idx = torch.tensor(_DECONV_TAP, device=weight.device)
    g = w.permute(1, 0, 2, 3)[:, :, idx]          # [co][ci][a][ty][kx]
    g = g[:, :, :, :, idx]                         # [co][ci][a][ty][b][tx]
    return g.permute(0, 2, 4, 1, 3, 5).reshape(4 * co, ci, 2, 2).contiguous()


def deconv2x(x, phase_weight, bias=None, act=None, packed_weight=None, rem=None, out_nhwc=False):
    """act(ConvTranspose2d(k=4, stride 2, padding 1)(x) + bias) [, rem concatenated after its
    channels] -> [N, co (+ cr), 2H, 2W]: the 2x2 pad-1 phase conv on the HIP engine (weights from
    deconv2x_phase_weight, bias repeated per phase), then aanet_deconv2x_assemble_f32 (phase
    scatter + the concat).  nets/feature.py:342-376 (Conv2x with deconv=True).  out_nhwc=True:
    a channels_last result (aanet_deconv2x_assemble_nhwc_f32) for an NHWC-staging consumer."""
    require_gpu(x, phase_weight, bias, packed_weight, rem,
                names=("input", "weight", "bias", "packed", "rem"))
    N, C, H, W = x.shape
    co = phase_weight.shape[0] // 4
    ph = conv2d_fused(x.contiguous(), phase_weight, bias, 1, 1, 1, 1, act,
                      packed_weight=packed_weight)
    cr = 0
    if rem is not None:
        rem = rem.contiguous()
        if tuple(rem.shape[0:1]) + tuple(rem.shape[2:]) != (N, 2 * H, 2 * W):
            raise ValueError(f"deconv2x: rem {tuple(rem.shape)} does not match the output "
                             f"{(N, co, 2 * H, 2 * W)}")
        cr = rem.shape[1]
    out = torch.empty((N, co + cr, 2 * H, 2 * W), device=x.device, dtype=x.dtype,
                      memory_format=torch.channels_last if out_nhwc else torch.contiguous_format)
    call("aanet_deconv2x_assemble_nhwc_f32" if out_nhwc else "aanet_deconv2x_assemble_f32",
         ptr(ph), ptr(rem), ptr(out), N, co, cr, H, W, stream_of(x))
    return out


def concat_nhwc(a, b):
    """torch.cat((a, b), 1) of two NCHW tensors as a channels_last tensor (aanet_concat_nhwc_f32;
    even H and W, at most 496 channels)."""
    require_gpu(a, b, names=("a", "b"))
    N, ca, H, W = a.shape
    if b.shape[0] != N or tuple(b.shape[2:]) != (H, W):
        raise ValueError(f"concat_nhwc: {tuple(a.shape)} and {tuple(b.shape)} do not concatenate")
    cb = b.shape[1]
    out = torch.empty((N, ca + cb, H, W), device=a.device, dtype=a.dtype,
                      memory_format=torch.channels_last)
    call("aanet_concat_nhwc_f32", ptr(a.contiguous()), ptr(b.contiguous()), ptr(out), N, ca, cb,
         H, W, stream_of(a))
    return out


def refine_stem(warped, left, disp, w1, b1, w2, b2, act="leaky"):
    """torch.cat((act(conv1(cat(warped - left, left))), act(conv2(disp))), 1) as one channels-last
    [N, 32, H, W] tensor (aanet_refine_stem_f32; nets/refinement.py:92-99 with BN folded into
    w1/b1, w2/b2)."""
    require_gpu(warped, left, disp, w1, b1, w2, b2)
    N, _, H, W = left.shape
    if tuple(warped.shape) != (N, 3, H, W) or tuple(disp.shape) != (N, 1, H, W) or \
            tuple(w1.shape) != (16, 6, 3, 3) or tuple(w2.shape) != (16, 1, 3, 3):
        raise ValueError("refine_stem: unexpected shapes")
    out = torch.empty((N, 32, H, W), device=left.device, dtype=left.dtype,
                      memory_format=torch.channels_last)
    call("aanet_refine_stem_f32", ptr(warped.contiguous()), ptr(left.contiguous()),
         ptr(disp.contiguous()), ptr(w1.contiguous()), ptr(b1), ptr(w2.contiguous()), ptr(b2),
         ACT[act], ptr(out), N, H, W, stream_of(left))
    return out


def pack_conv3x3s2(weight):
    """Pre-split A fragments of a [co][c][3][3] weight for conv3x3_s2 (aanet_conv3x3s2_pack_f32;
    co % 16 == 0, co <= 96, c % 32 == 0), or None when the shape is outside the kernel."""
    co, c, kh, kw = weight.shape
    if (kh, kw) != (3, 3) or co % 16 or co > 96 or c % 32 or not weight.is_cuda:
        return None
    nbytes = _lib.lib().aanet_conv3x3s2_pack_bytes(co, c)
    out = torch.empty(nbytes // 2, device=weight.device, dtype=torch.int16)
    w = weight.contiguous().float()
    call("aanet_conv3x3s2_pack_f32", ptr(w), co, c, ptr(out), stream_of(w))
    return out


def conv3x3_s2(x, wsplit, bias, co, co_a, act_a=None, act_b=None, x2=None, identity=None,
               up=None):
    """3x3 stride-2 pad-1 conv (BN folded) with its output channels split over two outputs:
    [0, co_a) -> out_a (act_a), [co_a, co) -> out_b (act_b); returns (out_a, out_b), either None
    when empty.  The CSA down exchange convs that share an input run as one launch
    (aanet_conv3x3s2_f32, nets/aggregation.py:362-371).  With the CSA terms
    (aanet_conv3x3s2_terms_f32): x2 is a second input whose channels follow x's in the
    contraction (wsplit packs the [co][C + C2][3][3] weight: two down terms of one branch as one
    conv); out_a = act_a(conv + bias [+ identity] [+ bilinear resize of up to out_a's size])."""
    require_gpu(x, bias, x2, identity, up)
    N, C, H, W = x.shape
    Ho, Wo = (H + 1) // 2, (W + 1) // 2
    out_a = torch.empty((N, co_a, Ho, Wo), device=x.device, dtype=x.dtype) if co_a > 0 else None
    out_b = torch.empty((N, co - co_a, Ho, Wo), device=x.device, dtype=x.dtype) if co_a < co else None
    if x2 is None and identity is None and up is None:
        call("aanet_conv3x3s2_f32", ptr(x), ptr(wsplit), ptr(bias), N, C, H, W, co, co_a,
             ptr(out_a), ACT[act_a], ptr(out_b), ACT[act_b], stream_of(x))
        return out_a, out_b
    if x2 is not None and (x2.shape[0] != N or tuple(x2.shape[2:]) != (H, W)):
        raise ValueError("conv3x3_s2: x2 must match x's batch and spatial size")
    if identity is not None and tuple(identity.shape) != (N, co_a, Ho, Wo):
        raise ValueError("conv3x3_s2: identity must have out_a's shape")
    if up is not None and tuple(up.shape[:2]) != (N, co_a):
        raise ValueError("conv3x3_s2: up must have out_a's batch and channels")
    x2c = None if x2 is None else x2.contiguous()
    idc = None if identity is None else identity.contiguous()
    upc = None if up is None else up.contiguous()
    t = _lib.S2Terms(ptr(x2c), 0 if x2c is None else x2c.shape[1], ptr(idc), ptr(upc),
                     1 if upc is None else upc.shape[2], 1 if upc is None else upc.shape[3])
    call("aanet_conv3x3s2_terms_f32", ptr(x), ptr(wsplit), ptr(bias), N, C, H, W, co, co_a,
         ptr(out_a), ACT[act_a], ptr(out_b), ACT[act_b], ctypes.byref(t), stream_of(x))
    return out_a, out_b


def pack_conv3x3_grouped(weight, groups):
    """Pre-split A fragments of a grouped [co][c/groups][3][3] weight for conv3x3_grouped_nhwc
    (aanet_conv3x3_grouped_pack_f32), or None when the shape is outside the kernel."""
    co, cg, kh, kw = weight.shape
    if (kh, kw) != (3, 3) or not weight.is_cuda:
        return None
    nbytes = _lib.lib().aanet_conv3x3_grouped_pack_bytes(co, cg * groups, groups)
    if not nbytes:
        return None
    out = torch.empty(nbytes // 2, device=weight.device, dtype=torch.int16)
    w = weight.contiguous().float()
    call("aanet_conv3x3_grouped_pack_f32", ptr(w), co, cg * groups, groups, ptr(out), stream_of(w))
    return out


def conv3x3_grouped_nhwc(x, wsplit, bias, co, groups, dilation):
    """The offset_conv of a deformable bottleneck in eval (deform.py:58-60): 3x3 stride-1 conv
    with padding = dilation, `groups` groups and bias, from a channels-last x to an NCHW output
    (aanet_conv3x3_grouped_nhwc_f32)."""
    require_gpu(x, bias, nhwc_ok=(0,))
    if not _lib.is_nhwc(x):
        raise ValueError("conv3x3_grouped_nhwc: x must be channels-last")
    N, C, H, W = x.shape
    out = torch.empty((N, co, H, W), device=x.device, dtype=x.dtype)
    call("aanet_conv3x3_grouped_nhwc_f32", ptr(x), ptr(wsplit), ptr(bias), N, C, H, W, co, groups,
         dilation, ptr(out), stream_of(x))
    return out


def csa_sum(inputs, act="leaky"):
    """act(inputs[0] + resize(inputs[1]) + ...) at inputs[0]'s size (aggregation.py:387-400)."""
    require_gpu(*inputs)
    N, C, H, W = inputs[0].shape
    for t in inputs:
        if t.shape[:2] != (N, C):
            raise ValueError("csa_sum inputs must share batch and channels")
    out = torch.empty_like(inputs[0])
    k = len(inputs)
    ptrs = (_lib.ctypes.c_void_p * k)(*[t.data_ptr() for t in inputs])
    hs = (_lib.ctypes.c_int * k)(*[t.shape[2] for t in inputs])
    ws = (_lib.ctypes.c_int * k)(*[t.shape[3] for t in inputs])
    call("aanet_csa_sum_f32", ptr(out), N, C, H, W, k, ptrs, hs, ws, ACT[act], stream_of(out))
    return out


class ResizeBilinearFunction(Function):
    """F.interpolate(x, size, mode='bilinear', align_corners=False) on the HIP kernels: the
    forward one thread per output element (aanet_resize_bilinear_f32; torch's NCHW kernel loops
    over the planes inside a thread), the backward a gather (aanet_resize_bilinear_bwd_f32):
    atomic-free and bit-reproducible, where torch's CUDA backward scatters with atomics (or, under
    deterministic algorithms, sorts for index_put)."""

    @staticmethod
    def forward(ctx, x, size):
        x = x.contiguous()
        require_gpu(x, names=("input",))
        ctx.in_hw = tuple(x.shape[2:])
        N, C, ih, iw = x.shape
        y = x.new_empty((N, C) + tuple(size))
        if y.numel() == 0:
            return y
        call("aanet_resize_bilinear_f32", ptr(x), ptr(y), N * C, ih, iw, size[0], size[1], stream_of(x))
        return y

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_out):
        grad_out = grad_out.contiguous()
        require_gpu(grad_out, names=("grad_output",))
        N, C, oh, ow = grad_out.shape
        ih, iw = ctx.in_hw
        gx = grad_out.new_empty((N, C, ih, iw))
        call("aanet_resize_bilinear_bwd_f32", ptr(grad_out), ptr(gx), N * C, ih, iw, oh, ow,
             stream_of(grad_out))
        return gx, None


def resize_bilinear(x, size):
    """Bilinear resize (align_corners=False) of [N, C, h, w] to `size`; on the GPU its backward
    is ResizeBilinearFunction's HIP gather."""
    size = tuple(int(v) for v in size)
    if not x.is_cuda:
        return torch.nn.functional.interpolate(x, size=size, mode="bilinear", align_corners=False)
    return ResizeBilinearFunction.apply(x, size)


DCN_BWD_ALGOS = {"auto": 0, "global": 1, "window": 2}  # AANET_DCN_BWD_* (include/aanet_mi355x.h)


def window_bwd_ok(C, Co, kh, kw, stride, dilation, deformable_groups):
    """Whether AANET_DCN_BWD_WINDOW takes a DCN backward shape (mdcn.hip win_shape_ok; the full
    list of include/aanet_mi355x.h).  The LDS term: gOut tile, W^T slice, sampling / partial
    buffers, sampled columns and the int64 window of (7 s + 1 + (k-1) dil + 4)^2 positions x 16
    channels, within the CU's 160 KiB."""
    cpg = C // deformable_groups
    if stride not in (1, 2) or cpg > 128 or C % 4 or cpg % 4 or kh * kw > 9 or Co > 128 or Co % 16:
        return False
    pitch = lambda v: v + (2 - v % 32) % 32  # noqa: E731  (mdcn.hip round_pitch(v, 2))
    # mdcn.hip win_rows: 7 * stride + 1 rows under an 8-pixel tile + the taps' reach + 2 x 2
    wr, wc = 7 * stride + 1 + (kh - 1) * dilation + 4, 7 * stride + 1 + (kw - 1) * dilation + 4
    smem = 4 * (Co * pitch(64) + 16 * pitch(Co) + 16 * 66 + 64 * 16 + 3 * 9 * 64 + 16 * 66) \
        + wr * wc * 16 * 8
    return smem <= 160 * 1024


def mdcn_backward(x, offset, mask, weight, grad_out, with_bias, stride, padding, dilation, groups,
                  deformable_groups, deterministic=None, nchw_scatter=False, algo="auto"):
    """deform_conv_cuda.cpp:571-685 -> (gX, gOffset, gMask, gW, gB or None).

    Default: aanet_mdcn_bwd_algo_f32 with the caller-owned workspace; algo "auto" takes the
    LDS-window form of grad_x where it measured faster (stride 1, <= 32 channels per deformable
    group, Co <= 64: the aggregation's DCNs; int64 fixed-point window in both modes) and the
    global-atomic form otherwise; "window" / "global" force one form ("window" also takes the
    feature extractor's stride-2, 64-channel-group, Co = 128 shapes -- window_bwd_ok --
    AANET_EUNSUPPORTED where it does not apply).  nchw_scatter=True: the workspace-free aanet_mdcn_bwd_f32 (global atomics in NCHW).

    deterministic (default: torch.are_deterministic_algorithms_enabled()): the bit-reproducible
    form (fixed-point grad_x accumulation, ordered grad_W reduction) instead of float atomics."""
    require_gpu(x, offset, mask, weight, grad_out,
                names=("input", "offset", "mask", "weight", "grad_output"))
    N, C, H, W = x.shape
    Co, _, kh, kw = weight.shape
    gx, goff, gm = torch.empty_like(x), torch.empty_like(offset), torch.empty_like(mask)
    gw = torch.zeros_like(weight)
    gb = x.new_zeros((Co,)) if with_bias else None
    if deterministic is None:
        deterministic = torch.are_deterministic_algorithms_enabled()
    if algo not in DCN_BWD_ALGOS:
        raise ValueError(f"mdcn_backward: algo must be one of {sorted(DCN_BWD_ALGOS)}")
    if nchw_scatter and not deterministic:  # the workspace-free entry point (grad_x atomics in NCHW)
        call("aanet_mdcn_bwd_f32", ptr(x), ptr(offset), ptr(mask), ptr(weight), ptr(grad_out),
             ptr(gx), ptr(goff), ptr(gm), ptr(gw), ptr(gb), N, C, H, W, Co, kh, kw, stride, padding,
             dilation, groups, deformable_groups, stream_of(x))
        return gx, goff, gm, gw, gb
    size_fn = "aanet_mdcn_bwd_det_workspace_size" if deterministic else "aanet_mdcn_bwd_ws_workspace_size"
    nbytes = getattr(_lib.lib(), size_fn)(N, C, H, W, Co, kh, kw, stride, padding, dilation, groups,
                                          deformable_groups)
    if nbytes == 0:
        raise ValueError(f"{size_fn}: invalid shape")
    ws = torch.empty((nbytes,), device=x.device, dtype=torch.uint8)
    call("aanet_mdcn_bwd_algo_f32", ptr(x), ptr(offset), ptr(mask), ptr(weight), ptr(grad_out),
         ptr(gx), ptr(goff), ptr(gm), ptr(gw), ptr(gb), N, C, H, W, Co, kh, kw, stride, padding,
         dilation, groups, deformable_groups, int(bool(deterministic)), DCN_BWD_ALGOS[algo],
         ptr(ws), nbytes, stream_of(x))
    return gx, goff, gm, gw, gb


def conv2d_wgrad(x, grad_out, weight_shape, with_bias, stride=1, padding=0, dilation=1, groups=1,
                 deterministic=None):
    """(grad_weight, grad_bias or None) of an ordinary convolution (aanet_conv2d_wgrad_f32):
    the DCN weight-gradient kernel with the tap's shifted window as its column.
    deterministic (default True): per-split partials reduced in a fixed order; False: one float
    atomic per (workgroup, element).  The fixed-order form is also the faster one: in the
    training step (bench.py --train, profiles/r05d_train_breakdown*.txt) the atomic form's
    launches averaged 35.7 us, the partials 18.0 us + 6.3 us for the reduction -- every pixel
    split of a chunk adds into the same weight elements, so the atomics contend."""
    require_gpu(x, grad_out, names=("input", "grad_output"))
    N, C, H, W = x.shape
    Co, _, kh, kw = weight_shape
    if kh != kw:
        raise ValueError("square kernels only")
    if deterministic is None:
        deterministic = True
    # the fixed-order form stores its results (mode 2): no zero fill; the atomic form adds
    alloc = x.new_empty if deterministic else x.new_zeros
    gw = alloc(tuple(weight_shape))
    gb = alloc((Co,)) if with_bias else None
    ws, nbytes = None, 0
    if deterministic:
        nbytes = _lib.lib().aanet_conv2d_wgrad_workspace_size(N, C, H, W, Co, kh, kw, stride, padding,
                                                               dilation, groups)
        if nbytes == 0:
            raise ValueError("aanet_conv2d_wgrad_workspace_size: invalid shape")
        ws = torch.empty((nbytes,), device=x.device, dtype=torch.uint8)
    call("aanet_conv2d_wgrad_f32", ptr(x), ptr(grad_out), ptr(gw), ptr(gb), N, C, H, W, Co, kh, kw,
         stride, padding, dilation, groups, 2 if deterministic else 0, ptr(ws), nbytes, stream_of(x))
    return gw, gb


def conv2d_dgrad(grad_out, weight, input_hw, stride=1, padding=0, dilation=1, groups=1):
    """Data gradient of an ordinary convolution as a forward conv on the engine
    (aanet_conv2d_fused_f32): the weight transposed per group and flipped, padding
    dil*(k-1) - pad; stride s > 1 first spreads grad_out onto every s-th pixel of a zero plane
    (plus the rows/columns the forward's floor division dropped)."""
    require_gpu(grad_out, weight, names=("grad_output", "weight"))
    Co, Cg, kh, kw = weight.shape
    if kh != kw:
        raise ValueError("square kernels only")
    pad_t = dilation * (kh - 1) - padding
    if pad_t < 0:
        raise ValueError("padding > dilation*(k-1) has no engine data gradient")
    N, _, Ho, Wo = grad_out.shape
    H, W = input_hw
    # the per-group transposed, flipped weight, packed for the engine in one launch
    wp = torch.empty((kh, kw, groups * Cg, Co // groups), device=weight.device, dtype=weight.dtype)
    call("aanet_conv_weight_pack_dgrad_f32", ptr(weight.contiguous()), ptr(wp), Co, Cg, kh, kw, groups,
         stream_of(weight))
    if stride > 1:
        rh = H + 2 * padding - dilation * (kh - 1) - 1 - (Ho - 1) * stride
        rw = W + 2 * padding - dilation * (kw - 1) - 1 - (Wo - 1) * stride
        dz = grad_out.new_zeros((N, Co, (Ho - 1) * stride + 1 + rh, (Wo - 1) * stride + 1 + rw))
        dz[:, :, : (Ho - 1) * stride + 1 : stride, : (Wo - 1) * stride + 1 : stride] = grad_out
        grad_out = dz
    gx = conv2d_fused(grad_out.contiguous(), (groups * Cg, Co // groups, kh, kw), padding=pad_t,
                      dilation=dilation, groups=groups, packed_weight=wp)
    if tuple(gx.shape[2:]) != (H, W):
        raise RuntimeError(f"dgrad shape {tuple(gx.shape)} != input {(H, W)}")
    return gx


def mdcn_im2col(x, offset, mask, kh, kw, stride, padding, dilation, deformable_groups):
    """Debug export (one image): col [C*K, Ho*Wo], kernel.cu:570-633."""
    require_gpu(x, offset, mask, names=("input", "offset", "mask"))
    C, H, W = x.shape
    Ho, Wo = _out_size(H, kh, stride, padding, dilation), _out_size(W, kw, stride, padding, dilation)
    col = torch.empty((C * kh * kw, Ho * Wo), device=x.device, dtype=x.dtype)
    call("aanet_mdcn_im2col_f32", ptr(x), ptr(offset), ptr(mask), ptr(col), C, H, W, kh, kw,
         stride, padding, dilation, deformable_groups, stream_of(x))
    return col


def mdcn_sample_index(offset, H, W, kh, kw, stride, padding, dilation, deformable_groups):
    """Debug export: (h_low, w_low, valid) int32 [N, dg, K, Ho*Wo]."""
    require_gpu(offset, names=("offset",))
    N = offset.shape[0]
    Ho, Wo = _out_size(H, kh, stride, padding, dilation), _out_size(W, kw, stride, padding, dilation)
    shp = (N, deformable_groups, kh * kw, Ho * Wo)
    hl, wl, vd = (torch.empty(shp, device=offset.device, dtype=torch.int32) for _ in range(3))
    call("aanet_mdcn_sample_index", ptr(offset), ptr(hl), ptr(wl), ptr(vd), N, H, W, kh, kw, stride,
         padding, dilation, deformable_groups, stream_of(offset))
    return hl, wl, vd


class ModulatedDeformConvFunction(Function):
    """Same argument order / returns as nets/deform_conv/deform_conv.py:113-171."""

    @staticmethod
    def forward(ctx, input, offset, mask, weight, bias=None, stride=1, padding=0, dilation=1,
                groups=1, deformable_groups=1):
        if input is not None and input.dim() != 4:
            raise ValueError(f"Expected 4D tensor as input, got {input.dim()}D tensor instead.")
        if not input.is_cuda:
            raise NotImplementedError  # as the reference (deform_conv.py:135-136)
        ctx.stride, ctx.padding, ctx.dilation = stride, padding, dilation
        ctx.groups, ctx.deformable_groups = groups, deformable_groups
        ctx.with_bias = bias is not None
        input, offset, mask = input.contiguous(), offset.contiguous(), mask.contiguous()
        weight = weight.contiguous()
        if weight.requires_grad or mask.requires_grad or offset.requires_grad or input.requires_grad:
            ctx.save_for_backward(input, offset, mask, weight)
        return mdcn_forward(input, offset, mask, weight, bias, stride, padding, dilation, groups,
                            deformable_groups)

    @staticmethod
    @once_differentiable
    def backward(ctx, grad_output):
        if not grad_output.is_cuda:
            raise NotImplementedError
        input, offset, mask, weight = ctx.saved_tensors
        gx, goff, gm, gw, gb = mdcn_backward(input, offset, mask, weight, grad_output.contiguous(),
                                             ctx.with_bias, ctx.stride, ctx.padding, ctx.dilation,
                                             ctx.groups, ctx.deformable_groups)
        return gx, goff, gm, gw, gb, None, None, None, None, None


modulated_deform_conv = ModulatedDeformConvFunction.apply
