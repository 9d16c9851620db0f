"""Training step of the hot path with data-parallel gradient all-reduce.

What the reference's training loop does around the path, restated on the drop-in modules:

* loss -- model.py:97-134: every disparity in the pyramid is bilinearly upsampled to the
  ground-truth size (align_corners=False) and scaled by W_gt / W_pred, then
  smooth-L1 over the valid mask (mean), weighted by the pyramid weights of model.py:98-107;
  the optional pseudo-ground-truth term (model.py:126-134) is added the same way;
* parameter groups -- train.py:199-215 with utils/utils.py:156-169: `offset_conv.weight` /
  `offset_conv.bias` train at 0.1x the base learning rate (Adam);
* data parallelism -- train.py:184-190: SyncBatchNorm conversion, then DistributedDataParallel;
  micro-steps that are not on an accumulation boundary run under `no_sync()` (model.py:82-85),
  the loss is divided by the accumulation count (model.py:136) and the optimizer steps on
  boundaries (model.py:151-153).

MI355X specifics: one process per GPU over RCCL (torch.distributed backend "nccl").  The
gradient of the path is ~16 MB (AANet) -- one or two buckets: the bucket cap is raised to 32 MB
so the all-reduce is a single large ring over xGMI instead of the default 25 MB split, and
gradients are bucket views (no extra copy).  The DCN backward is the HIP one; with
torch.use_deterministic_algorithms(True) it is the bit-reproducible form
(aanet_mdcn_bwd_det_f32) -- the HIP cost-volume and regression backwards are gathers and are
reproducible either way; the loss's bilinear upsampling backward is torch's and follows torch's
own deterministic-algorithms rules.
"""
import contextlib

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from ._precision import CONV2D_TYPES, PinnedConv2d, fp32_scope
from .nets._fuse import clear_fold_caches

# model.py:98-107: pyramid weights by pyramid length
PYRAMID_WEIGHTS = {5: [1 / 3, 2 / 3, 1.0, 1.0, 1.0],  # AANet and AANet+
                   4: [1 / 3, 2 / 3, 1.0, 1.0],
                   3: [1.0, 1.0, 1.0],
                   1: [1.0]}

SPECIFIC_PARAMS = ("offset_conv.weight", "offset_conv.bias")  # utils/utils.py:156-169


def pyramid_weights(n, highest_loss_only=False):
    if highest_loss_only:
        return [1.0]
    if n not in PYRAMID_WEIGHTS:
        raise NotImplementedError(f"no pyramid weights for {n} predictions")
    return PYRAMID_WEIGHTS[n]


def disparity_loss(pred_pyramid, gt_disp, mask, weights=None, pseudo_gt=None, pseudo_mask=None):
    """model.py:109-134 -> (weighted total, per-scale losses).  pred_pyramid: coarse-to-fine
    list of [B, h, w]; gt_disp, mask: [B, H, W] (mask bool); pseudo_gt / pseudo_mask the
    optional pseudo ground truth (args.load_pseudo_gt)."""
    if weights is None:
        weights = pyramid_weights(len(pred_pyramid))
    if len(weights) != len(pred_pyramid):
        raise ValueError("one weight per prediction")
    # mean over the mask as a masked sum / count: the same value as smooth_l1(pred[mask], ...)
    # (model.py:121) without the boolean gather, whose nonzero() syncs the host every scale
    # (masked-out ground truth may be inf/nan in real data: zero it so 0 * term stays 0)
    maskf = mask.to(gt_disp.dtype)
    count = maskf.sum()
    gt_disp = torch.where(mask, gt_disp, torch.zeros_like(gt_disp))
    pmaskf = pcount = None
    if pseudo_gt is not None:
        pmaskf = pseudo_mask.to(gt_disp.dtype)
        pcount = pmaskf.sum()
        pseudo_gt = torch.where(pseudo_mask, pseudo_gt, torch.zeros_like(pseudo_gt))
    total, per_scale = 0.0, []
    for pred, w in zip(pred_pyramid, weights):
        if pred.size(-1) != gt_disp.size(-1):
            pred = ops.resize_bilinear(pred.unsqueeze(1), gt_disp.shape[-2:]) * \
                (gt_disp.size(-1) / pred.size(-1))
            pred = pred.squeeze(1)
        loss = (F.smooth_l1_loss(pred, gt_disp, reduction="none") * maskf).sum() / count
        total = total + w * loss
        per_scale.append(loss)
        if pseudo_gt is not None:
            ploss = (F.smooth_l1_loss(pred, pseudo_gt, reduction="none") * pmaskf).sum() / pcount
            total = total + w * ploss
    return total, per_scale


def param_groups(model, lr):
    """Base parameters at lr, offset_conv at 0.1 * lr (train.py:199-215)."""
    base, specific = [], []
    for name, p in model.named_parameters():
        (specific if any(s in name for s in SPECIFIC_PARAMS) else base).append(p)
    return [{"params": base, "lr": lr}, {"params": specific, "lr": lr * 0.1}]


def wrap_data_parallel(model, device, sync_bn=True, bucket_cap_mb=32):
    """SyncBN + DDP (train.py:184-190) when torch.distributed is initialised with >1 rank;
    otherwise the module itself."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1):
        return model
    if sync_bn:
        model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
    dev_ids = [device.index] if device.type == "cuda" and dist.get_backend() == "nccl" else None
    return nn.parallel.DistributedDataParallel(model, device_ids=dev_ids,
                                               bucket_cap_mb=bucket_cap_mb,
                                               gradient_as_bucket_view=True)


class EngineConv2dFunction(torch.autograd.Function):
    """An nn.Conv2d on the HIP engine end to end: forward aanet_conv2d_fused_f32, data gradient
    as the engine's forward conv of grad_out (ops.conv2d_dgrad), weight/bias gradient
    aanet_conv2d_wgrad_f32 with fixed-order partial sums (deterministic in every mode, and faster
    than its float-atomic form; under torch.use_deterministic_algorithms(True) MIOpen would fall
    back to its naive kernels)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, padding, dilation, groups):
        from . import ops
        x = x.contiguous()
        ctx.save_for_backward(x, weight)
        ctx.conf = (bias is not None, stride, padding, dilation, groups)
        return ops.conv2d_fused(x, weight.contiguous(), bias, stride, padding, dilation, groups)

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, grad_out):
        from . import ops
        x, weight = ctx.saved_tensors
        with_bias, stride, padding, dilation, groups = ctx.conf
        grad_out = grad_out.contiguous()
        gx = gw = gb = None
        if ctx.needs_input_grad[0]:
            gx = ops.conv2d_dgrad(grad_out, weight.contiguous(), x.shape[2:], stride, padding,
                                  dilation, groups)
        if ctx.needs_input_grad[1] or (with_bias and ctx.needs_input_grad[2]):
            gw, gb = ops.conv2d_wgrad(x, grad_out, weight.shape, with_bias, stride, padding,
                                      dilation, groups)
        return gx, gw, gb, None, None, None, None


def _engine_conv_ok(m):
    if type(m) not in (nn.Conv2d, PinnedConv2d):
        return False
    k, s, p, d = m.kernel_size, m.stride, m.padding, m.dilation
    return (m.padding_mode == "zeros" and not isinstance(p, str)
            and k[0] == k[1] and s[0] == s[1] and p[0] == p[1] and d[0] == d[1]
            and p[0] <= d[0] * (k[0] - 1))


class EngineConv2d(PinnedConv2d):
    """nn.Conv2d whose training forward runs EngineConv2dFunction (use_engine_convs swaps a
    module's class to this one in place).  Same parameters, buffers and state-dict keys; being a
    module-level subclass, a whole-model torch.save / torch.load round-trips (a bound method
    stored in the instance __dict__ did not unpickle)."""

    def forward(self, x):
        if x.dtype != torch.float32 or not x.is_cuda:  # the HIP engine takes fp32 device tensors
            return PinnedConv2d.forward(self, x)
        return EngineConv2dFunction.apply(x, self.weight, self.bias, self.stride[0],
                                          self.padding[0], self.dilation[0], self.groups)


CONV2D_TYPES.add(EngineConv2d)


def use_engine_convs(model):
    """Route every nn.Conv2d of `model` that the engine takes (square kernel, symmetric
    stride/padding/dilation, zero padding) through EngineConv2dFunction; returns how many.
    Only the class changes (nn.Conv2d -> EngineConv2d, a subclass): parameters, state_dict,
    DDP and the eval-mode folding of nets/_fuse.py see the same module."""
    n = 0
    for m in model.modules():
        if _engine_conv_ok(m):
            m.__class__ = EngineConv2d
            m._aanet_engine = True
            n += 1
    return n


class Trainer:
    """One optimizer step per `accumulation_steps` micro-batches (model.py:64-153)."""

    def __init__(self, model, lr=1e-3, weight_decay=1e-4, accumulation_steps=1,
                 highest_loss_only=False, max_disp=192, engine_convs=None, capturable=False):
        """max_disp: the image-resolution disparity range of the valid mask (train.py --max_disp,
        default 192), NOT the cost-volume D.  engine_convs: run the plain convs on the HIP engine
        (use_engine_convs); default: when the model is on the GPU (measured round 5: the training
        step 17.3 -> 15.7 ms against MIOpen, whose NHWC kernels transpose around every NCHW conv;
        under torch.use_deterministic_algorithms(True) MIOpen has only its naive kernels).  capturable: Adam keeps its step count on
        the device, so that the step can be captured into a HIP graph (graph_step)."""
        if engine_convs is None:
            params = list(model.parameters())
            engine_convs = bool(params) and all(p.is_cuda for p in params)
        if engine_convs:
            use_engine_convs(model)
        self.model = model
        self.accumulation_steps = accumulation_steps
        self.highest_loss_only = highest_loss_only
        self.max_disp = max_disp
        # fused Adam (one multi-tensor kernel per step) when every parameter is on the GPU: the
        # foreach form's capturable branch divides by 0-dim step tensors, which this torch build
        # runs as two broadcast kernels PER PARAMETER (~360 launches, ~2 ms of a 20 ms step);
        # same update rule (torch.optim.Adam), different rounding order only
        fused = all(p.is_cuda and p.dtype == torch.float32 for p in model.parameters())
        self.optimizer = torch.optim.Adam(param_groups(model, lr), weight_decay=weight_decay,
                                          capturable=capturable, fused=fused or None)
        self.micro = 0
        self._graph = None

    def graph_step(self, left_feature, right_feature, gt_disp, mask, warmup=3):
        """The whole step (forward, loss, backward, Adam) as ONE HIP graph replay, for a single
        process with static inputs (the tensors passed on the first call are captured by address
        and must be refilled in place for new data) and one micro-batch per optimizer step.  The
        eager step issues ~2.9k kernel launches; replayed, the host cost is one launch.  The first
        call runs `warmup` eager steps on a side stream (allocator and MIOpen algorithm state),
        then captures; it needs Trainer(capturable=True).  Returns the loss tensor (overwritten by
        every replay).  The empty-mask skip of step() is a host synchronisation and is not taken
        here: the caller guarantees valid pixels."""
        if self._graph is None:
            if self.accumulation_steps != 1 or isinstance(self.model, nn.parallel.DistributedDataParallel):
                raise RuntimeError("graph_step: one process, no gradient accumulation")
            if not self.optimizer.param_groups[0].get("capturable", False):
                raise RuntimeError("graph_step needs Trainer(capturable=True)")
            self.model.train()

            def body():
                with fp32_scope():  # forward AND backward convs in fp32 (_precision.py)
                    pyramid = self.model(left_feature, right_feature)
                    if self.highest_loss_only:
                        pyramid = [pyramid[-1]]
                    total, _ = disparity_loss(pyramid, gt_disp, mask,
                                              pyramid_weights(len(pyramid), self.highest_loss_only))
                    total.backward()
                self.optimizer.step()
                return total.detach()
            # the warm-up steps must not count: parameters, BN buffers and the optimizer state are
            # restored in place afterwards (the graph holds their addresses).  Optimizer state
            # that exists already (eager step() calls before the first graph_step) is restored to
            # its values; state the warm-up creates is zeroed (Adam's initial state).
            snap = [(t, t.detach().clone()) for t in
                    list(self.model.parameters()) + list(self.model.buffers())]
            opt_snap = {id(v): (v, v.detach().clone()) for st in self.optimizer.state.values()
                        for v in st.values() if torch.is_tensor(v)}
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                for _ in range(warmup):
                    self.optimizer.zero_grad(set_to_none=True)
                    body()
            torch.cuda.current_stream().wait_stream(side)
            self.optimizer.zero_grad(set_to_none=True)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph):
                self._graph_loss = body()
            self._graph = graph
            with torch.no_grad():
                for t, v in snap:
                    t.copy_(v)
                for st in self.optimizer.state.values():
                    for v in st.values():
                        if not torch.is_tensor(v):
                            continue
                        prev = opt_snap.get(id(v))
                        if prev is not None and prev[0] is v:
                            v.copy_(prev[1])
                        else:  # created by the warm-up: Adam's step, exp_avg, exp_avg_sq start at 0
                            v.zero_()
        # a replay updates parameters and BN running statistics in place without bumping their
        # _version, which the eval path's folded-weight caches key on: drop the caches (and put
        # the model in train mode, as step() does) so a later eval forward refolds
        self.model.train()
        clear_fold_caches(self.model)
        self._graph.replay()
        return self._graph_loss

    def valid_mask(self, disp):
        """model.py:71,75: 0 < d < max_disp."""
        return (disp > 0) & (disp < self.max_disp)

    def step(self, left_feature, right_feature, gt_disp, mask=None, pseudo_gt=None,
             pseudo_mask=None):
        """Forward + backward of one micro-batch; returns the (unscaled) total loss, or None when
        the batch has no valid pixel (model.py:78-79: skipped -- no forward, no backward, no
        optimizer step -- but it still counts towards the accumulation index, as the reference's
        enumerate() index does).  The optimizer steps (and DDP all-reduces) on accumulation
        boundaries only (model.py:151-153)."""
        self.model.train()
        if mask is None:
            mask = self.valid_mask(gt_disp)
        if pseudo_gt is not None and pseudo_mask is None:
            pseudo_mask = self.valid_mask(pseudo_gt) & ~mask  # model.py:75-76
        self.micro += 1
        if not bool(mask.any()):
            return None
        boundary = self.micro % self.accumulation_steps == 0
        sync_ctx = contextlib.nullcontext()
        if not boundary and isinstance(self.model, nn.parallel.DistributedDataParallel):
            sync_ctx = self.model.no_sync()
        with sync_ctx, fp32_scope():  # forward AND backward convs in fp32 (_precision.py)
            pyramid = self.model(left_feature, right_feature)
            if self.highest_loss_only:
                pyramid = [pyramid[-1]]
            total, _ = disparity_loss(pyramid, gt_disp, mask,
                                      pyramid_weights(len(pyramid), self.highest_loss_only),
                                      pseudo_gt, pseudo_mask)
            (total / self.accumulation_steps).backward()
        if boundary:
            self.optimizer.step()
            self.optimizer.zero_grad(set_to_none=True)
        return total.detach()
