"""Functional CPU restatement of AdaptiveAggregation (eval mode) -- TEST INFRASTRUCTURE ONLY.

Restates, from a state dict with the reference's keys:
  AdaptiveAggregation.forward        nets/aggregation.py:452-464
  AdaptiveAggregationModule.forward  nets/aggregation.py:375-402 (ISA branches + CSA fuse)
  SimpleBottleneck.forward           nets/deform.py:164-184
  DeformSimpleBottleneck.forward     nets/deform.py:216-236
  DeformConv2d.forward               nets/deform.py:78-97 (offset/mask split, 2*sigmoid)
  DisparityEstimation / disparity_computation  nets/estimation.py:13-30, nets/aanet.py:156-167
Stock convolutions / batch norm / bilinear interpolation use torch CPU functional ops (the
reference itself uses torch for these); the modulated DCN and the regression use the C oracle.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import oracle

BN_EPS = 1e-5
TRAINING = False  # batch statistics in BN (module-level switch used by training-mode tests)


def _t(a):
    return a if isinstance(a, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(a))


def _bn(x, sd, p):
    if TRAINING:
        return F.batch_norm(x, None, None, _t(sd[p + ".weight"]), _t(sd[p + ".bias"]), True, 0.0,
                            BN_EPS)
    return F.batch_norm(x, _t(sd[p + ".running_mean"]), _t(sd[p + ".running_var"]),
                        _t(sd[p + ".weight"]), _t(sd[p + ".bias"]), False, 0.0, BN_EPS)


class OracleMDCN(torch.autograd.Function):
    """CPU autograd wrapper of the C oracle (forward cpp:490-569, backward cpp:571-685)."""

    @staticmethod
    def forward(ctx, x, offset, mask, weight, bias, dilation, dg):
        ctx.save_for_backward(x, offset, mask, weight)
        ctx.dilation, ctx.dg, ctx.with_bias = dilation, dg, bias is not None
        out = oracle.mdcn_forward(x.detach().numpy(), offset.detach().numpy(),
                                  mask.detach().numpy(), weight.detach().numpy(),
                                  None if bias is None else bias.detach().numpy(), 1, dilation,
                                  dilation, 1, dg)
        return torch.from_numpy(out)

    @staticmethod
    def backward(ctx, g):
        x, offset, mask, weight = ctx.saved_tensors
        gx, go, gm, gw, gb = oracle.mdcn_backward(x.numpy(), offset.numpy(), mask.numpy(),
                                                  weight.numpy(), g.contiguous().numpy(),
                                                  ctx.with_bias, 1, ctx.dilation, ctx.dilation,
                                                  1, ctx.dg)
        t = torch.from_numpy
        return t(gx), t(go), t(gm), t(gw), (t(gb) if gb is not None else None), None, None


def _conv(x, sd, p, stride=1, padding=0, dilation=1, groups=1):
    b = sd.get(p + ".bias")
    return F.conv2d(x, _t(sd[p + ".weight"]), None if b is None else _t(b), stride, padding,
                    dilation, groups)


def deform_conv2d(x, sd, p, dilation, dg):
    """nets/deform.py:78-97 with the oracle DCN."""
    om = _conv(x, sd, p + ".offset_conv", padding=dilation, dilation=dilation, groups=dg)
    k2 = 9
    offset = om[:, :dg * 2 * k2]
    mask = torch.sigmoid(om[:, dg * 2 * k2:]) * 2
    b = sd.get(p + ".deform_conv.bias")
    return OracleMDCN.apply(x.contiguous(), offset.contiguous(), mask.contiguous(),
                            _t(sd[p + ".deform_conv.weight"]), None if b is None else _t(b),
                            dilation, dg)


def bottleneck(x, sd, p, deform, dilation=2, dg=2):
    """nets/deform.py:164-184 (plain) / 216-236 (deformable)."""
    out = F.relu(_bn(_conv(x, sd, p + ".conv1"), sd, p + ".bn1"))
    if deform:
        out = deform_conv2d(out, sd, p + ".conv2", dilation, dg)
    else:
        out = _conv(out, sd, p + ".conv2", padding=1)
    out = F.relu(_bn(out, sd, p + ".bn2"))
    out = _bn(_conv(out, sd, p + ".conv3"), sd, p + ".bn3")
    return F.relu(out + x)


def aa_module(x, sd, p, num_scales, num_out, deform, dilation=2, dg=2):
    """nets/aggregation.py:375-402."""
    x = [bottleneck(x[i], sd, f"{p}.branches.{i}.0", deform, dilation, dg) for i in range(num_scales)]
    if num_scales == 1:
        return x
    fused = []
    for i in range(num_out):
        acc = None
        for j in range(num_scales):
            q = f"{p}.fuse_layers.{i}.{j}"
            if i == j:
                y = x[j]
            elif i < j:
                y = _bn(_conv(x[j], sd, q + ".0"), sd, q + ".1")
            else:
                y = x[j]
                for k in range(i - j - 1):
                    y = F.leaky_relu(_bn(_conv(y, sd, f"{q}.{k}.0", stride=2, padding=1), sd,
                                         f"{q}.{k}.1"), 0.2)
                y = _bn(_conv(y, sd, f"{q}.{i - j - 1}.0", stride=2, padding=1), sd,
                        f"{q}.{i - j - 1}.1")
            if acc is None:
                acc = y
            else:
                if y.shape[2:] != acc.shape[2:]:
                    y = F.interpolate(y, size=acc.shape[2:], mode="bilinear", align_corners=False)
                acc = acc + y
        fused.append(acc)
    return [F.leaky_relu(f, 0.2) for f in fused]


def adaptive_aggregation(volumes, sd, num_scales=3, num_fusions=6, num_deform_blocks=3,
                         intermediate_supervision=True, dilation=2, dg=2):
    """nets/aggregation.py:406-464 (eval mode), sd keys without the 'aggregation.' prefix."""
    x = [_t(v) for v in volumes]
    for f in range(num_fusions):
        num_out = num_scales if intermediate_supervision else (1 if f == num_fusions - 1 else num_scales)
        deform = f >= num_fusions - num_deform_blocks
        x = aa_module(x, sd, f"fusions.{f}", num_scales, num_out, deform, dilation, dg)
    n_final = num_scales if intermediate_supervision else 1
    return [_conv(x[i], sd, f"final_conv.{i}") for i in range(n_final)]


def hot_path(left_pyr, right_pyr, sd, max_disp, **kw):
    """cost volume pyramid -> AdaptiveAggregation -> regression in reverse order (aanet.py:146-167)."""
    vols = oracle.cost_volume_pyramid(left_pyr, right_pyr, max_disp)
    aggs = [a.detach().numpy() for a in adaptive_aggregation(vols, sd, **kw)]
    return [oracle.disp_regress(aggs[len(aggs) - 1 - i]) for i in range(len(aggs))]
