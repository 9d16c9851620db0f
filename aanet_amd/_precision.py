"""fp32 semantics for the convolutions this package leaves to MIOpen (transposed convs, and every
conv of the training / reference-order path).  torch allows TF32 for cudnn (= MIOpen)
convolutions by default, and on gfx950 MIOpen then computes them below fp32 precision (the
PSMNet-AA reference-order path had 2.8x the reference's own near-tie flips with it, 1.05x
without).  The reference is fp32 (cuDNN 7.6, no TF32).

The switch is scoped to this package's module forwards (the flag is an argument of each conv op,
so their backward follows it too); the process-wide torch setting is restored on exit and is
never changed at import."""
import functools

import torch


def fp32_convs(forward):
    """Decorator: run `forward` with torch.backends.cudnn.allow_tf32 off, restoring it after."""

    @functools.wraps(forward)
    def wrapped(*args, **kwargs):
        prev = torch.backends.cudnn.allow_tf32
        if not prev:
            return forward(*args, **kwargs)
        torch.backends.cudnn.allow_tf32 = False
        try:
            return forward(*args, **kwargs)
        finally:
            torch.backends.cudnn.allow_tf32 = prev

    return wrapped
