"""aanet_amd -- MI355X-native (gfx950) AANet cost-volume hot path.

Layers: include/aanet_mi355x.h (C ABI, HIP kernels in aanet_amd/csrc) -> aanet_amd._lib (ctypes)
-> aanet_amd.ops (autograd ops; also registered as torch.ops.aanet.*, aanet_amd.torch_ops)
-> aanet_amd.nets (drop-in modules mirroring the reference's
nets/ API).  No CPU fallback: ops raise on non-HIP tensors or a missing library.
"""
import torch

from . import _lib, ops  # noqa: F401
from . import torch_ops  # noqa: F401  (registers torch.ops.aanet.*)

# fp32 semantics for the convolutions left to MIOpen (transposed convs; every conv of the
# reference-order / training path): torch allows TF32 for cudnn (= MIOpen) convolutions by
# default, and on gfx950 MIOpen then computes them below fp32 precision -- the PSMNet-AA
# reference-order path had 2.8x the reference's own near-tie flips at full resolution with it,
# 1.05x without (tools/flip_report.py).  The reference is fp32 (cuDNN 7.6, no TF32).
# A caller may switch it back on after importing this package.
torch.backends.cudnn.allow_tf32 = False

__version__ = "0.1.0"


def native_library_path():
    return _lib.LIB_PATH
