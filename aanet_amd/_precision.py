"""fp32 semantics for the convolutions this package leaves to MIOpen (transposed convs, and every
conv of the training / reference-order path).  torch allows TF32 for cudnn (= MIOpen)
convolutions by default, and on gfx950 MIOpen then computes them below fp32 precision (the
PSMNet-AA reference-order path had 2.8x the reference's own near-tie flips with it, 1.05x
without).  The reference is fp32 (cuDNN 7.6, no TF32).

Two scopes, both restoring the process-wide torch setting on exit (it is never changed at import):
  * `fp32_convs` decorates the package's module forwards: the FORWARD convs run in fp32.
  * `fp32_scope()` is a context manager for a whole training step.  Autograd's conv backward
    reads the global flag when it runs, i.e. at loss.backward(), outside any decorated forward
    (torch 2.10's miopen_convolution takes no allow_tf32 argument), so the backward convs are in
    fp32 only inside this scope.  aanet_amd.train.Trainer runs forward, loss and backward in it;
    a caller with its own training loop wraps its step the same way:
        with aanet_amd.fp32_scope():
            loss = criterion(model(left, right), gt); loss.backward()

The flag is process-global torch state, so neither scope is thread-safe: modules running their
forwards in several threads at once (nn.DataParallel replicas) may interleave the save/restore.
Such callers set torch.backends.cudnn.allow_tf32 = False once themselves."""
import contextlib
import functools

import torch


@contextlib.contextmanager
def fp32_scope():
    """Run the enclosed forward AND backward convolutions with allow_tf32 off."""
    prev = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = False
    try:
        yield
    finally:
        torch.backends.cudnn.allow_tf32 = prev


def fp32_convs(forward):
    """Decorator: run `forward` with torch.backends.cudnn.allow_tf32 off, restoring it after (the
    backward of those convs needs fp32_scope, see the module docstring)."""

    @functools.wraps(forward)
    def wrapped(*args, **kwargs):
        if not torch.backends.cudnn.allow_tf32:
            return forward(*args, **kwargs)
        with fp32_scope():
            return forward(*args, **kwargs)

    return wrapped
