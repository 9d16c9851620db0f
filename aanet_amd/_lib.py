"""ctypes binding of the gfx950 C-ABI library ``libaanet_mi355x.so`` (include/aanet_mi355x.h).

This is the only way the Python package reaches the GPU: every op passes raw device pointers
and torch's current HIP stream to an ``extern "C"`` entry point.  There is NO CPU fallback:
if the library is missing or a tensor is not on a ROCm device, the call raises.
"""
import contextlib
import contextvars
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AANET_MI355X_LIB", os.path.join(_HERE, "libaanet_mi355x.so"))

_P = ctypes.c_void_p
_I = ctypes.c_int
_L = ctypes.c_long
_F = ctypes.c_float

# name -> argtypes (every function returns int status)
_SIGNATURES = {
    "aanet_corr_volume_f32": [_P, _P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_corr_volume_bwd_f32": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_concat_volume_f32": [_P, _P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_diff_volume_f32": [_P, _P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_concat_volume_bwd_f32": [_P, _P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_diff_volume_bwd_f32": [_P, _P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_corr_pyramid_f32": [_I, _P, _P, _P, _P, _P, _P, _I, _I, _P],
    "aanet_disp_regress_f32": [_P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_disp_regress_bwd_f32": [_P, _P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_disp_warp_f32": [_P, _P, _P, _P, _I, _I, _I, _I, _P],
    "aanet_disp_warp_bwd_f32": [_P, _P, _P, _P, _P, _I, _I, _I, _I, _P],
    "aanet_mdcn_fwd_f32": [_P, _P, _P, _P, _P, _P] + [_I] * 12 + [_P],
    "aanet_mdcn_fwd_fused_f32": [_P, _P, _L, _P, _L, _I, _F, _P, _I, _P, _P, _P, _I, _P] + [_I] * 13 + [_P],
    "aanet_mdcn_bwd_f32": [_P] * 10 + [_I] * 12 + [_P],
    "aanet_mdcn_bwd_det_f32": [_P] * 10 + [_I] * 12 + [_P, ctypes.c_size_t, _P],
    "aanet_mdcn_bwd_ws_f32": [_P] * 10 + [_I] * 12 + [_P, ctypes.c_size_t, _P],
    "aanet_mdcn_bwd_algo_f32": [_P] * 10 + [_I] * 14 + [_P, ctypes.c_size_t, _P],
    "aanet_conv2d_wgrad_f32": [_P] * 4 + [_I] * 12 + [_P, ctypes.c_size_t, _P],
    "aanet_resize_bilinear_bwd_f32": [_P, _P, _L] + [_I] * 4 + [_P],
    "aanet_resize_bilinear_f32": [_P, _P, _L] + [_I] * 4 + [_P],
    "aanet_deconv2x_assemble_f32": [_P, _P, _P] + [_I] * 5 + [_P],
    "aanet_deconv2x_assemble_nhwc_f32": [_P, _P, _P] + [_I] * 5 + [_P],
    "aanet_concat_nhwc_f32": [_P, _P, _P] + [_I] * 5 + [_P],
    "aanet_refine_stem_f32": [_P] * 7 + [_I, _P, _I, _I, _I, _P],
    "aanet_conv2d_fused_f32": [_P] * 6 + [_I, _I, _P] + [_I] * 12 + [_P],
    "aanet_conv_weight_pack_f32": [_P, _P, _I, _I, _I, _I, _P],
    "aanet_conv_weight_pack_dgrad_f32": [_P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_conv_weight_pack_split_f32": [_P, _P, _I, _I, _I, _I, _I, _P],
    "aanet_conv2d_pw_f32": [_P] * 5 + [_I] + [_P] * 3 + [_I, _I, _P] + [_I] * 10 + [_P, _I, _P],
    "aanet_mdcn_pw_f32": [_P, _P, _L, _P, _L, _I, _F, _P, _P, _P, _P, _I, _P, _P, _P, _I, _I, _P]
    + [_I] * 11 + [_P, _I, _P],
    "aanet_csa_sum_f32": [_P, _I, _I, _I, _I, _I, _P, _P, _P, _I, _P],
    "aanet_conv3x3s2_pack_f32": [_P, _I, _I, _P, _P],
    "aanet_conv3x3s2_f32": [_P, _P, _P] + [_I] * 6 + [_P, _I, _P, _I, _P],
    "aanet_conv3x3s2_terms_f32": [_P, _P, _P] + [_I] * 6 + [_P, _I, _P, _I, _P, _P],
    "aanet_conv3x3_grouped_pack_f32": [_P, _I, _I, _I, _P, _P],
    "aanet_conv3x3_grouped_nhwc_f32": [_P, _P, _P] + [_I] * 7 + [_P, _P],
    "aanet_mdcn_im2col_f32": [_P, _P, _P, _P] + [_I] * 9 + [_P],
    "aanet_mdcn_sample_index": [_P, _P, _P, _P] + [_I] * 9 + [_P],
}

# size / query functions (not int-status): name, argtypes, restype
_SIZE_FUNCTIONS = [
    ("aanet_version", [], _I),
    ("aanet_mdcn_bwd_det_workspace_size", [_I] * 12, ctypes.c_size_t),
    ("aanet_mdcn_bwd_ws_workspace_size", [_I] * 12, ctypes.c_size_t),
    ("aanet_conv2d_wgrad_workspace_size", [_I] * 11, ctypes.c_size_t),
    ("aanet_conv_weight_pack_split_bytes", [_I] * 5, _L),
    ("aanet_conv3x3s2_pack_bytes", [_I, _I], ctypes.c_size_t),
    ("aanet_conv3x3_grouped_pack_bytes", [_I, _I, _I], ctypes.c_size_t),
    ("aanet_mdcn_window_fwd_supported", [_I] * 10, _I),
]

_lib = None


class AanetError(RuntimeError):
    def __init__(self, msg, status=None):
        super().__init__(msg)
        self.status = status


EUNSUPPORTED = -2  # AANET_EUNSUPPORTED (include/aanet_mi355x.h)


def lib():
    """Load the HIP library (raises loudly when it is absent -- never falls back)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"aanet_amd: HIP library not found at {LIB_PATH}; build it with "
                "`python -c 'import __graft_entry__ as g; g.build()'` (make -C aanet_amd/csrc)")
        L = ctypes.CDLL(LIB_PATH)
        ab_build = "AANET_MI355X_LIB" in os.environ  # an older build under A/B timing
        for name, argtypes in _SIGNATURES.items():
            if ab_build and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.argtypes = argtypes
            f.restype = _I
        if not ab_build and L.aanet_version() != ABI_VERSION:
            raise ImportError(f"aanet_amd: {LIB_PATH} has ABI version {L.aanet_version()}, "
                              f"this package needs {ABI_VERSION}; rebuild it (make -C aanet_amd/csrc)")
        L.aanet_status_string.argtypes = [_I]
        L.aanet_status_string.restype = ctypes.c_char_p
        for name, argtypes, restype in _SIZE_FUNCTIONS:
            if ab_build and not hasattr(L, name):  # an older build under A/B timing
                continue
            f = getattr(L, name)
            f.argtypes, f.restype = argtypes, restype
        _lib = L
    return _lib


def exported_symbols():
    return ["aanet_status_string"] + [n for n, _, _ in _SIZE_FUNCTIONS] + list(_SIGNATURES)


def call(name, *args):
    rc = getattr(lib(), name)(*args)
    if rc != 0:
        msg = lib().aanet_status_string(rc).decode()
        ints = [a for a in args if isinstance(a, int)]
        raise AanetError(f"{name} failed: {msg} (status {rc}); integer args {ints}", rc)


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def is_nhwc(t):
    """channels_last 4-D tensor that is not also NCHW-contiguous (physical layout NHWC)."""
    return (t is not None and t.dim() == 4 and not t.is_contiguous()
            and t.is_contiguous(memory_format=torch.channels_last))


LAYOUT_IN_NHWC, LAYOUT_OUT_NHWC = 1, 2  # AANET_LAYOUT_* (include/aanet_mi355x.h)
CONV_EXACT_F32 = 8  # AANET_CONV_EXACT_F32: exact f32 MFMA instead of the split-bf16 contraction
CONV_WEIGHTS_SPLIT = 16  # AANET_CONV_WEIGHTS_SPLIT: weight buffers carry bf16 piece fragments
CONV_GENERIC_DCN = 32  # AANET_CONV_GENERIC_DCN: generic engine instead of the LDS-window DCN tail

# The contraction arithmetic of the fused eval paths, per execution context (a ContextVar: each
# thread / asyncio task has its own, and nothing is read from the process environment).
_EXACT_F32 = contextvars.ContextVar("aanet_exact_f32", default=False)


_CACHE_FILLS = [0]


def note_cache_fill():
    """Counted by every eval-path cache (re)fill -- folded / packed weights, BN affines (nets/
    _fuse.py, ops._split_weight): AdaptiveAggregation._run_chains must order the other chains
    after the current stream when one happened (the fill's kernels run there)."""
    _CACHE_FILLS[0] += 1


def cache_fills():
    return _CACHE_FILLS[0]


def exact_f32_enabled():
    return _EXACT_F32.get()


def set_exact_f32(on):
    """Select the conv engine's contraction arithmetic for the fused eval paths of the current
    context: False (default) = split-bf16 pieces with fp32 accumulation where the engine has the
    configuration (fp32-accurate, include/aanet_mi355x.h AANET_CONV_EXACT_F32); True = exact f32
    MFMA everywhere.  Returns the previous setting (bench.py --exact-f32; `exact_f32` below is the
    scoped form)."""
    prev = _EXACT_F32.get()
    _EXACT_F32.set(bool(on))
    return prev


@contextlib.contextmanager
def exact_f32(on=True):
    """Scope: the enclosed fused eval calls run the exact f32 engine (on=True) or the split-bf16
    contraction (on=False); the previous setting comes back on exit."""
    token = _EXACT_F32.set(bool(on))
    try:
        yield
    finally:
        _EXACT_F32.reset(token)


def conv_flags(*packed):
    """Contraction flags for a fused conv call whose packed weight buffers are `packed`: the split
    contraction when every buffer carries its pieces (ops.pack_weight_split) and exact mode is
    off, else the exact f32 engine."""
    if _EXACT_F32.get():
        return CONV_EXACT_F32
    if packed and all(getattr(w, "_aanet_split", False) for w in packed):
        return CONV_WEIGHTS_SPLIT
    return 0


class _Descriptor(ctypes.Structure):
    """A descriptor struct of the C ABI: `struct_size` (the first member) is filled in with the
    struct's size, which the library checks against its own (AANET_EABI on a mismatch)."""

    def __init__(self, *args, **kwargs):
        super().__init__(ctypes.sizeof(self), *args, **kwargs)


class PostStage(_Descriptor):
    """aanet_post_stage_t (include/aanet_mi355x.h)."""
    _fields_ = [("struct_size", ctypes.c_size_t), ("weight", ctypes.c_void_p),
                ("bias", ctypes.c_void_p), ("act", ctypes.c_int), ("out_nhwc", ctypes.c_void_p),
                ("disp", ctypes.c_void_p), ("skip_outputs", ctypes.c_int)]


class CsaEpilogue(_Descriptor):
    """aanet_csa_epilogue_t (include/aanet_mi355x.h)."""
    _fields_ = [("struct_size", ctypes.c_size_t), ("out", ctypes.c_void_p),
                ("num_up", ctypes.c_int), ("up", ctypes.c_void_p * 3),
                ("up_h", ctypes.c_int * 3), ("up_w", ctypes.c_int * 3), ("act", ctypes.c_int),
                ("post", ctypes.POINTER(PostStage))]


class S2Terms(_Descriptor):
    """aanet_s2_terms_t (include/aanet_mi355x.h)."""
    _fields_ = [("struct_size", ctypes.c_size_t), ("x2", ctypes.c_void_p), ("c2", ctypes.c_int),
                ("identity", ctypes.c_void_p), ("up", ctypes.c_void_p), ("up_h", ctypes.c_int),
                ("up_w", ctypes.c_int)]


ABI_VERSION = 4  # AANET_ABI_VERSION (include/aanet_mi355x.h)
EABI = -3  # AANET_EABI


def stream_of(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_gpu(*tensors, names=None, nhwc_ok=()):
    """fp32, contiguous, on the same ROCm device: the C ABI takes raw NCHW pointers.  Tensors at
    the positions in nhwc_ok may instead be channels_last (physically NHWC, AANET_LAYOUT_*)."""
    dev = None
    for i, t in enumerate(tensors):
        if t is None:
            continue
        nm = names[i] if names else f"arg{i}"
        if not t.is_cuda:
            raise NotImplementedError(
                f"aanet_amd ops run only on the MI355X (HIP) device; {nm} is on {t.device}")
        if t.dtype != torch.float32:
            raise TypeError(f"aanet_amd ops compute in fp32; {nm} is {t.dtype}")
        if not (t.is_contiguous() or (i in nhwc_ok and is_nhwc(t))):
            raise ValueError(f"{nm} must be contiguous")
        if dev is None:
            dev = t.device
        elif t.device != dev:
            raise ValueError(f"{nm} is on {t.device}, expected {dev}")
    return dev
