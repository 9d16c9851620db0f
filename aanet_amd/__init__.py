"""aanet_amd -- MI355X-native (gfx950) AANet cost-volume hot path.

Layers: include/aanet_mi355x.h (C ABI, HIP kernels in aanet_amd/csrc) -> aanet_amd._lib (ctypes)
-> aanet_amd.ops (autograd ops; also registered as torch.ops.aanet.*, aanet_amd.torch_ops)
-> aanet_amd.nets (drop-in modules mirroring the reference's
nets/ API).  No CPU fallback: ops raise on non-HIP tensors or a missing library.
"""
import torch

from . import _lib, ops  # noqa: F401
from . import torch_ops  # noqa: F401  (registers torch.ops.aanet.*)

# fp32 convolutions on MIOpen: scoped to this package's module forwards (_precision.fp32_convs)
# and, for the backward, to a training step (fp32_scope; Trainer uses it); importing the package
# changes no global torch setting.
from ._precision import fp32_scope  # noqa: F401,E402

__version__ = "0.1.0"


def native_library_path():
    return _lib.LIB_PATH
