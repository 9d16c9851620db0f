"""CPU oracle for the AANet cost-volume hot path -- TEST INFRASTRUCTURE ONLY.

numpy front-end over ``oracle/liboracle.so`` (plain C restatement in oracle_impl.h).
Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker -- never as the thing measured or shipped.

Reference citations (wuzhongwulidong/aanet):
  corr_volume / concat_volume / diff_volume  -> nets/cost.py:19-55
  cost_volume_pyramid                        -> nets/cost.py:58-76
  disp_regress (+ _bwd)                      -> nets/estimation.py:13-30
  mdcn_im2col / mdcn_forward / mdcn_backward -> nets/deform_conv/src/deform_conv_cuda_kernel.cu:467-767,
                                                deform_conv_cuda.cpp:490-685
Parity pinning: cost volumes and regression are pinned by golden vectors generated from the
reference's own Python (tests/golden/make_golden.py); the DCN restatement is pinned by
known-answer tests (tests/test_oracle.py) because the reference DCN is CUDA-only.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def _sfx(dtype):
    return "_f64" if np.dtype(dtype) == np.float64 else "_f32"


def _c(a, dtype):
    return np.ascontiguousarray(a, dtype=dtype)


def _fn(name, dtype):
    f = getattr(lib(), name + _sfx(dtype))
    f.restype = None
    return f


def out_size(n, k, s, p, d):
    """deform_conv.py:174-183."""
    return (n + 2 * p - (d * (k - 1) + 1)) // s + 1


# ------------------------------------------------------------------ cost volumes ---------
def corr_volume(left, right, max_disp, dtype=np.float32):
    """nets/cost.py:40-48 -> [B, D, H, W]."""
    L, R = _c(left, dtype), _c(right, dtype)
    B, C, H, W = L.shape
    out = np.empty((B, max_disp, H, W), dtype)
    _fn("orc_corr_volume", dtype)(_ptr(L), _ptr(R), _ptr(out), B, C, H, W, max_disp)
    return out


def concat_volume(left, right, max_disp, dtype=np.float32):
    """nets/cost.py:31-38 -> [B, 2C, D, H, W]."""
    L, R = _c(left, dtype), _c(right, dtype)
    B, C, H, W = L.shape
    out = np.empty((B, 2 * C, max_disp, H, W), dtype)
    _fn("orc_concat_volume", dtype)(_ptr(L), _ptr(R), _ptr(out), B, C, H, W, max_disp)
    return out


def diff_volume(left, right, max_disp, dtype=np.float32):
    """nets/cost.py:22-29 -> [B, C, D, H, W]."""
    L, R = _c(left, dtype), _c(right, dtype)
    B, C, H, W = L.shape
    out = np.empty((B, C, max_disp, H, W), dtype)
    _fn("orc_diff_volume", dtype)(_ptr(L), _ptr(R), _ptr(out), B, C, H, W, max_disp)
    return out


def cost_volume(left, right, max_disp, feature_similarity="correlation", dtype=np.float32):
    if feature_similarity == "correlation":
        return corr_volume(left, right, max_disp, dtype)
    if feature_similarity == "concat":
        return concat_volume(left, right, max_disp, dtype)
    if feature_similarity == "difference":
        return diff_volume(left, right, max_disp, dtype)
    raise NotImplementedError(feature_similarity)


def cost_volume_pyramid(left_pyr, right_pyr, max_disp, feature_similarity="correlation",
                        dtype=np.float32):
    """nets/cost.py:64-76: scale s uses max_disp // 2**s."""
    return [cost_volume(l, r, max_disp // (2 ** s), feature_similarity, dtype)
            for s, (l, r) in enumerate(zip(left_pyr, right_pyr))]


def corr_volume_bwd(left, right, grad_out, dtype=np.float32):
    """Autograd of nets/cost.py:40-48 -> (grad_left, grad_right)."""
    L, R, g = _c(left, dtype), _c(right, dtype), _c(grad_out, dtype)
    B, C, H, W = L.shape
    gl, gr = np.empty_like(L), np.empty_like(R)
    _fn("orc_corr_volume_bwd", dtype)(_ptr(L), _ptr(R), _ptr(g), _ptr(gl), _ptr(gr), B, C, H, W,
                                      g.shape[1])
    return gl, gr


def shift_volume_bwd(grad_out, C, concat, dtype=np.float32):
    """Autograd of nets/cost.py:22-38 -> (grad_left, grad_right)."""
    g = _c(grad_out, dtype)
    B, _, D, H, W = g.shape
    gl, gr = np.empty((B, C, H, W), dtype), np.empty((B, C, H, W), dtype)
    _fn("orc_shift_volume_bwd", dtype)(_ptr(g), _ptr(gl), _ptr(gr), B, C, H, W, D, int(concat))
    return gl, gr


# ------------------------------------------------------------ disparity regression -------
def disp_regress(cost, match_similarity=True, dtype=np.float32):
    """nets/estimation.py:13-30 -> [B, H, W]."""
    c = _c(cost, dtype)
    B, D, H, W = c.shape
    out = np.empty((B, H, W), dtype)
    _fn("orc_disp_regress", dtype)(_ptr(c), _ptr(out), B, D, H, W, 0 if match_similarity else 1)
    return out


def disp_regress_bwd(cost, grad_disp, match_similarity=True, dtype=np.float32):
    c = _c(cost, dtype)
    g = _c(grad_disp, dtype)
    B, D, H, W = c.shape
    out = np.empty_like(c)
    _fn("orc_disp_regress_bwd", dtype)(_ptr(c), _ptr(g), _ptr(out), B, D, H, W,
                                       0 if match_similarity else 1)
    return out


# ------------------------------------------------------- modulated deformable conv -------
def mdcn_im2col(x, offset, mask, kh, kw, stride, pad, dil, dg, dtype=np.float32):
    """kernel.cu:570-633 for one image x[C,H,W] -> col[C*K, Ho*Wo]."""
    x, offset, mask = _c(x, dtype), _c(offset, dtype), _c(mask, dtype)
    C, H, W = x.shape
    Ho, Wo = out_size(H, kh, stride, pad, dil), out_size(W, kw, stride, pad, dil)
    col = np.empty((C * kh * kw, Ho * Wo), dtype)
    _fn("orc_mdcn_im2col", dtype)(_ptr(x), _ptr(offset), _ptr(mask), _ptr(col),
                                  C, H, W, kh, kw, stride, pad, dil, dg)
    return col


def mdcn_sample_index(offset, H, W, kh, kw, stride, pad, dil, dg, dtype=np.float32):
    """(h_low, w_low, valid) per [N, dg, K, Ho*Wo] -- the bit-exact index pin."""
    off = _c(offset, dtype)
    N = off.shape[0]
    Ho, Wo = out_size(H, kh, stride, pad, dil), out_size(W, kw, stride, pad, dil)
    shp = (N, dg, kh * kw, Ho * Wo)
    hl, wl, vd = (np.empty(shp, np.int32) for _ in range(3))
    _fn("orc_mdcn_sample_index", dtype)(_ptr(off), _ptr(hl), _ptr(wl), _ptr(vd),
                                        N, H, W, kh, kw, stride, pad, dil, dg)
    return hl, wl, vd


def mdcn_forward(x, offset, mask, weight, bias=None, stride=1, padding=0, dilation=1, groups=1,
                 deformable_groups=1, dtype=np.float32):
    """deform_conv_cuda.cpp:490-569 -> [N, Co, Ho, Wo]."""
    x, offset, mask, weight = (_c(a, dtype) for a in (x, offset, mask, weight))
    b = _c(bias, dtype) if bias is not None else None
    N, C, H, W = x.shape
    Co, _, kh, kw = weight.shape
    Ho, Wo = out_size(H, kh, stride, padding, dilation), out_size(W, kw, stride, padding, dilation)
    out = np.empty((N, Co, Ho, Wo), dtype)
    _fn("orc_mdcn_forward", dtype)(_ptr(x), _ptr(offset), _ptr(mask), _ptr(weight), _ptr(b),
                                   _ptr(out), N, C, H, W, Co, kh, kw, stride, padding, dilation,
                                   groups, deformable_groups)
    return out


def mdcn_backward(x, offset, mask, weight, grad_out, with_bias=False, stride=1, padding=0,
                  dilation=1, groups=1, deformable_groups=1, dtype=np.float32):
    """deform_conv_cuda.cpp:571-685 -> (gX, gOffset, gMask, gW, gB or None)."""
    x, offset, mask, weight, go = (_c(a, dtype) for a in (x, offset, mask, weight, grad_out))
    N, C, H, W = x.shape
    Co, _, kh, kw = weight.shape
    gx, goff, gm = np.empty_like(x), np.empty_like(offset), np.empty_like(mask)
    gw = np.zeros_like(weight)
    gb = np.zeros((Co,), dtype) if with_bias else None
    _fn("orc_mdcn_backward", dtype)(_ptr(x), _ptr(offset), _ptr(mask), _ptr(weight), _ptr(go),
                                    _ptr(gx), _ptr(goff), _ptr(gm), _ptr(gw), _ptr(gb),
                                    N, C, H, W, Co, kh, kw, stride, padding, dilation, groups,
                                    deformable_groups)
    return gx, goff, gm, gw, gb


# ------------------------------------------------------------------ disparity warp --------
def _warp_coords(disp, H, W):
    """nets/warp.py:5-16 + grid_sample(align_corners=True) unnormalisation, in float32 steps."""
    f = np.float32
    x = np.arange(W, dtype=f)[None, None, :]
    y = np.arange(H, dtype=f)[None, :, None]
    nx = f(2) * ((x - disp[:, 0]) / f(W - 1)) - f(1)
    ny = f(2) * (y / f(H - 1)) - f(1)
    ix = ((nx + f(1)) / f(2)) * f(W - 1)
    iy = np.broadcast_to(((ny + f(1)) / f(2)) * f(H - 1), ix.shape)
    return ix.astype(f), iy.astype(f)


def _corners(ix, iy):
    x0, y0 = np.floor(ix), np.floor(iy)
    w = ((x0 + 1 - ix) * (y0 + 1 - iy), (ix - x0) * (y0 + 1 - iy),
         (x0 + 1 - ix) * (iy - y0), (ix - x0) * (iy - y0))
    pos = ((y0, x0), (y0, x0 + 1), (y0 + 1, x0), (y0 + 1, x0 + 1))
    return [(yy.astype(np.int64), xx.astype(np.int64), ww) for (yy, xx), ww in zip(pos, w)]


def disp_warp(img, disp):
    """nets/warp.py:41-64 (padding 'border'): (warped [B,C,H,W], valid mask [B,C,H,W]).
    grid_sample's border clip is min(size-1, max(v, 0)); corners outside the image add 0."""
    img = np.ascontiguousarray(img, np.float32)
    disp = np.ascontiguousarray(disp, np.float32)
    B, C, H, W = img.shape
    ix, iy = _warp_coords(disp, H, W)
    ixc = np.minimum(np.float32(W - 1), np.maximum(ix, np.float32(0)))
    iyc = np.minimum(np.float32(H - 1), np.maximum(iy, np.float32(0)))
    b = np.arange(B)[:, None, None]
    out = np.zeros_like(img)
    for yy, xx, ww in _corners(ixc, iyc):
        ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
        v = img[b, :, np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)]  # [B,H,W,C]
        out += np.moveaxis(v * (ww * ok)[..., None], -1, 1)
    m = np.zeros(ix.shape, np.float32)
    for yy, xx, ww in _corners(ix, iy):  # grid_sample(ones, zeros padding): unclipped
        m += ww * ((yy >= 0) & (yy < H) & (xx >= 0) & (xx < W))
    valid = np.where(m < np.float32(0.9999), np.float32(0), np.float32(1))
    return out, np.repeat(valid[:, None], C, axis=1)


def disp_warp_bwd(img, disp, grad_warped):
    """d(sum grad_warped * warped)/d disp of disp_warp (float64): the x-derivative of the
    bilinear sample times the border clip's pass-through (0 where clipped) times -1."""
    img = np.asarray(img, np.float64)
    g = np.asarray(grad_warped, np.float64)
    B, C, H, W = img.shape
    ix, iy = (a.astype(np.float64) for a in _warp_coords(np.asarray(disp, np.float32), H, W))
    pas = ((ix > 0) & (ix < W - 1)).astype(np.float64)
    ixc, iyc = np.clip(ix, 0, W - 1), np.clip(iy, 0, H - 1)
    x0, y0 = np.floor(ixc), np.floor(iyc)
    b = np.arange(B)[:, None, None]
    gix = np.zeros(ix.shape)
    for dy, dx, sgn_x, wy in ((0, 0, -1, y0 + 1 - iyc), (0, 1, 1, y0 + 1 - iyc),
                              (1, 0, -1, iyc - y0), (1, 1, 1, iyc - y0)):
        yy, xx = (y0 + dy).astype(np.int64), (x0 + dx).astype(np.int64)
        ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
        v = img[b, :, np.clip(yy, 0, H - 1), np.clip(xx, 0, W - 1)]  # [B,H,W,C]
        gv = np.moveaxis(g, 1, -1)
        gix += sgn_x * wy * ok * (v * gv).sum(-1)
    return (-gix * pas)[:, None]
