"""fp32 semantics for the convolutions this package leaves to MIOpen (transposed convs, 3-D convs,
and every conv of the training / reference-order path).  torch allows TF32 for cudnn (= MIOpen)
convolutions by default, and on gfx950 MIOpen then computes them below fp32 precision (the
PSMNet-AA reference-order path had 2.8x the reference's own near-tie flips with it, 1.05x
without).  The reference is fp32 (cuDNN 7.6, no TF32).

Three mechanisms, none of which changes the process-wide torch setting outside its own call:
  * `fp32_convs` decorates the package's module forwards: the FORWARD convs run in fp32.  On its
    first call it also pins the module's convolutions (`pin_fp32_convs`, below).
  * Pinned convolutions (round 6): every nn.Conv2d / ConvTranspose2d / Conv3d /
    ConvTranspose3d of a drop-in module becomes the same-named subclass `Pinned*` (parameters,
    buffers and state-dict keys unchanged).  With autograd recording, its forward is one
    autograd Function whose forward AND backward call aten's convolution with TF32 off, so the
    backward is fp32 whoever calls loss.backward() -- the reference's own loop (model.py:137)
    included.  (Autograd's own conv backward reads the global flag when it runs, and torch
    2.10's miopen_convolution takes no allow_tf32 argument.)  Without autograd it is the plain
    module forward (inside the fp32_convs scope).
  * `fp32_scope()`: a context manager for a whole training step, for convs that are not the
    package's (aanet_amd.train.Trainer runs forward, loss and backward in it).

The flag is process-global torch state, so the scopes are not thread-safe: modules running their
forwards in several threads at once (nn.DataParallel replicas) may interleave the save/restore.
Such callers set torch.backends.cudnn.allow_tf32 = False once themselves."""
import contextlib
import functools

import torch
import torch.nn as nn


@contextlib.contextmanager
def fp32_scope():
    """Run the enclosed forward AND backward convolutions with allow_tf32 off."""
    prev = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = False
    try:
        yield
    finally:
        torch.backends.cudnn.allow_tf32 = prev


class _PinnedConvFn(torch.autograd.Function):
    """aten.convolution forward and aten.convolution_backward, both with TF32 off."""

    @staticmethod
    def forward(ctx, x, weight, bias, conf):
        stride, padding, dilation, transposed, output_padding, groups = conf
        ctx.save_for_backward(x, weight)
        ctx.conf = conf
        ctx.bias_sizes = None if bias is None else list(bias.shape)
        with fp32_scope():
            return torch.ops.aten.convolution(x, weight, bias, stride, padding, dilation,
                                              transposed, output_padding, groups)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad_out):
        x, weight = ctx.saved_tensors
        stride, padding, dilation, transposed, output_padding, groups = ctx.conf
        need = [ctx.needs_input_grad[0], ctx.needs_input_grad[1],
                ctx.bias_sizes is not None and ctx.needs_input_grad[2]]
        with fp32_scope():
            gx, gw, gb = torch.ops.aten.convolution_backward(
                grad_out.contiguous(), x, weight, ctx.bias_sizes, stride, padding, dilation,
                transposed, output_padding, groups, need)
        return gx, gw, gb, None


def _recording(m, x):
    return torch.is_grad_enabled() and (x.requires_grad or m.weight.requires_grad or
                                        (m.bias is not None and m.bias.requires_grad))


def _pinned(m, x, transposed, output_padding):
    if m.padding_mode != "zeros" or isinstance(m.padding, str) or not _recording(m, x):
        return None
    conf = (list(m.stride), list(m.padding), list(m.dilation), transposed, list(output_padding),
            m.groups)
    return _PinnedConvFn.apply(x, m.weight, m.bias, conf)


class PinnedConv2d(nn.Conv2d):
    """nn.Conv2d whose autograd forward/backward run with TF32 off (see the module docstring)."""

    def forward(self, x):
        y = _pinned(self, x, False, (0, 0))
        return nn.Conv2d.forward(self, x) if y is None else y


class PinnedConv3d(nn.Conv3d):
    def forward(self, x):
        y = _pinned(self, x, False, (0, 0, 0))
        return nn.Conv3d.forward(self, x) if y is None else y


class _PinnedTransposed:
    _dims = 2

    def forward(self, x, output_size=None):
        base = self.__class__.__mro__[2]
        op = self._output_padding(x, output_size, self.stride, self.padding, self.kernel_size,
                                  self._dims, self.dilation)
        y = _pinned(self, x, True, op)
        return base.forward(self, x, output_size) if y is None else y


class PinnedConvTranspose2d(_PinnedTransposed, nn.ConvTranspose2d):
    _dims = 2


class PinnedConvTranspose3d(_PinnedTransposed, nn.ConvTranspose3d):
    _dims = 3


_PINNED = {nn.Conv2d: PinnedConv2d, nn.Conv3d: PinnedConv3d,
           nn.ConvTranspose2d: PinnedConvTranspose2d, nn.ConvTranspose3d: PinnedConvTranspose3d}
# the plain 2-D conv classes the HIP engine may take (train.EngineConv2d registers itself)
CONV2D_TYPES = {nn.Conv2d, PinnedConv2d}


def pin_fp32_convs(module):
    """Swap the class of every plain torch convolution in `module`'s subtree to its Pinned*
    subclass in place (an already-pinned, or engine, conv is left alone); returns how many."""
    n = 0
    for m in module.modules():
        cls = _PINNED.get(type(m))
        if cls is not None:
            m.__class__ = cls
            n += 1
    return n


def fp32_convs(forward):
    """Decorator: run `forward` with torch.backends.cudnn.allow_tf32 off, restoring it after; on the
    first call, pin the module's convolutions (pin_fp32_convs) so their backward is fp32 too."""

    @functools.wraps(forward)
    def wrapped(*args, **kwargs):
        self = args[0] if args else None
        if isinstance(self, nn.Module) and not self.__dict__.get("_aanet_pinned", False):
            pin_fp32_convs(self)
            self.__dict__["_aanet_pinned"] = True
        if not torch.backends.cudnn.allow_tf32:
            return forward(*args, **kwargs)
        with fp32_scope():
            return forward(*args, **kwargs)

    return wrapped
