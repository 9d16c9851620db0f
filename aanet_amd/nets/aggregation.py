"""Drop-in for the adaptive aggregation of nets/aggregation.py (ISA + CSA).

AdaptiveAggregationModule (aggregation.py:313-402) and AdaptiveAggregation (406-464) with the
reference's constructor signatures, module tree (state-dict keys `fusions.{f}.branches.{s}.0.*`,
`fusions.{f}.fuse_layers.{i}.{j}.*`, `final_conv.{i}.*`) and forward semantics, including the
in-place mutation of the caller's list (`x[i] = dconv(x[i])`, aggregation.py:382).
ISA bottlenecks run the HIP DCN.  In eval mode without autograd every conv is a HIP
implicit-GEMM kernel (BN folded) and each CSA output branch is one fused resize+sum+LeakyReLU
kernel; training mode runs the reference op sequence with autograd.
The 3D-conv aggregators (StereoNet/PSMNet/GCNet) are out of scope.
"""
import contextlib

import torch
import torch.nn as nn

from .. import _lib, ops
from ._fuse import FoldCacheMixin, conv_bn_act, folded, s2_conv_ok, s2_pack, s2_pack_k, use_fused
from .deform import DeformSimpleBottleneck, SimpleBottleneck
from .._precision import fp32_convs
from .options import get_option, set_options


_SIDE_STREAMS = {}


def side_streams(device, n):
    """The side HIP streams of the concurrent-scale schedule: one per coarse scale (created once
    per device, outside any graph capture: the first eval forward is a warm-up)."""
    ss = _SIDE_STREAMS.setdefault(device, [])
    while len(ss) < n:
        ss.append(torch.cuda.Stream(device=device))
    return ss[:n]


_PREP_STREAMS = {}


def prep_stream(device):
    """The side stream of the deformable scale-0 conv1 + offset conv (option prep_stream)."""
    if device not in _PREP_STREAMS:
        _PREP_STREAMS[device] = torch.cuda.Stream(device=device)
    return _PREP_STREAMS[device]


def _record(stream):
    ev = torch.cuda.Event()
    ev.record(stream)
    return ev


def csa_epilogue_ok(x0, up):
    """Whether the tail kernels' CSA epilogue (aanet_csa_epilogue_t) takes output branch 0: at
    most two coarser terms, each exactly 2x or 4x smaller than the (same-size) block output, and
    quad-aligned rows (mdcn.hip launch_fwd).  Otherwise branch 0 is summed by aanet_csa_sum_f32,
    which implements the general bilinear resize of aggregation.py:396-398."""
    H, W = x0.shape[2], x0.shape[3]
    if W % 4 or len(up) > 2:
        return False
    for t in up:
        h, w = t.shape[2], t.shape[3]
        r = H // h if h > 0 else 0
        if r not in (2, 4) or h * r != H or w * r != W:
            return False
    return True


class AdaptiveAggregationModule(FoldCacheMixin, nn.Module):
    def __init__(self, num_scales, num_output_branches, max_disp, num_blocks=1,
                 simple_bottleneck=False, deformable_groups=2, mdconv_dilation=2):
        super(AdaptiveAggregationModule, self).__init__()
        self.num_scales = num_scales
        self.num_output_branches = num_output_branches
        self.max_disp = max_disp
        self.num_blocks = num_blocks

        self.branches = nn.ModuleList()
        # Adaptive intra-scale aggregation (aggregation.py:328-340)
        for i in range(self.num_scales):
            num_candidates = max_disp // (2 ** i)
            branch = nn.ModuleList()
            for j in range(num_blocks):
                if simple_bottleneck:
                    branch.append(SimpleBottleneck(num_candidates, num_candidates))
                else:
                    branch.append(DeformSimpleBottleneck(num_candidates, num_candidates,
                                                         modulation=True,
                                                         mdconv_dilation=mdconv_dilation,
                                                         deformable_groups=deformable_groups))
            self.branches.append(nn.Sequential(*branch))

        # Adaptive cross-scale aggregation (aggregation.py:342-371)
        self.fuse_layers = nn.ModuleList()
        for i in range(self.num_output_branches):
            self.fuse_layers.append(nn.ModuleList())
            for j in range(self.num_scales):
                if i == j:
                    self.fuse_layers[-1].append(nn.Identity())
                elif i < j:
                    self.fuse_layers[-1].append(
                        nn.Sequential(nn.Conv2d(max_disp // (2 ** j), max_disp // (2 ** i),
                                                kernel_size=1, bias=False),
                                      nn.BatchNorm2d(max_disp // (2 ** i))))
                else:
                    layers = nn.ModuleList()
                    for k in range(i - j - 1):
                        layers.append(nn.Sequential(
                            nn.Conv2d(max_disp // (2 ** j), max_disp // (2 ** j), kernel_size=3,
                                      stride=2, padding=1, bias=False),
                            nn.BatchNorm2d(max_disp // (2 ** j)),
                            nn.LeakyReLU(0.2, inplace=True)))
                    layers.append(nn.Sequential(
                        nn.Conv2d(max_disp // (2 ** j), max_disp // (2 ** i), kernel_size=3,
                                  stride=2, padding=1, bias=False),
                        nn.BatchNorm2d(max_disp // (2 ** i))))
                    self.fuse_layers[-1].append(nn.Sequential(*layers))

        self.relu = nn.LeakyReLU(0.2, inplace=True)

    def _exchange_up(self, x, i, j):
        """Exchange term fuse_layers[i][j] for i < j: 1x1 conv + BN at scale j's resolution."""
        layer = self.fuse_layers[i][j]
        return conv_bn_act(x[j], layer[0], layer[1], None)

    def _down(self, y, i, j, start=0):
        """Exchange term fuse_layers[i][j] for i > j from y = x[j] (or, start > 0, from the output
        of its first `start` convs): the chain of 3x3 stride-2 convs (+BN, LeakyReLU between
        them), each on the stride-2 kernel (ops.conv3x3_s2) where it takes the shape."""
        layer = self.fuse_layers[i][j]
        for k in range(start, len(layer)):
            conv, bn = layer[k][0], layer[k][1]
            act = None if k == len(layer) - 1 else "leaky"
            pk = s2_pack(conv, [(conv, bn)]) if s2_conv_ok(conv) else None
            if pk is None:
                y = conv_bn_act(y, conv, bn, act)
            else:
                y = ops.conv3x3_s2(y.contiguous(), pk[0], pk[1], conv.out_channels,
                                   conv.out_channels, act)[0]
        return y

    def _down0_heads(self, x0):
        """The first convs of the down chains that start at scale 0 (branches 1 and 2 at S = 3),
        as ONE stride-2 launch that reads x0 once: {branch i: that conv's output}, or {} when
        the convs do not fit the kernel (then every chain runs conv by conv, _down)."""
        nout = len(self.fuse_layers)
        heads = list(range(1, nout))
        if not heads or len(heads) > 2:
            return {}
        pairs = [(self.fuse_layers[i][0][0][0], self.fuse_layers[i][0][0][1]) for i in heads]
        if not all(s2_conv_ok(c) for c, _ in pairs) or \
                sum(c.out_channels for c, _ in pairs) > 96:
            return {}
        pk = s2_pack(self.fuse_layers[heads[0]][0], pairs)
        if pk is None:
            return {}
        acts = [None if len(self.fuse_layers[i][0]) == 1 else "leaky" for i in heads]
        co_a = pairs[0][0].out_channels
        co = co_a + (pairs[1][0].out_channels if len(pairs) > 1 else 0)
        ya, yb = ops.conv3x3_s2(x0.contiguous(), pk[0], pk[1], co, co_a, acts[0],
                                acts[1] if len(acts) > 1 else None)
        return {heads[0]: ya, **({heads[1]: yb} if len(heads) > 1 else {})}

    def _s2_sums_ok(self, x):
        """Whether output branches 1 and 2 (S = 3) are summed inside the stride-2 kernels:
          branch 1 = LeakyReLU(down(x0) + x1 + resize(up(x2))): the scale-0 heads launch, with x1
            and the up term as CSA terms of its first output (ops.conv3x3_s2 identity / up);
          branch 2 = LeakyReLU(down(down(x0)) + down(x1) + x2): ONE conv over the channel-
            concatenated inputs [head output, x1] (weights concatenated along the input
            channels, biases summed: the two down terms' sum), x2 as its identity term.
        Needs the reference's S = 3 structure (one conv from scale 0 to 1, two from 0 to 2, one
        from 1 to 2), every conv on the stride-2 kernel, and sizes that need no resize of the
        same-resolution terms (aggregation.py:395: x1 / x2 already have the down terms' size)."""
        if len(self.branches) != 3 or len(self.fuse_layers) != 3 or \
                not get_option(self, "s2_sums"):
            return False
        l10, l20, l21 = self.fuse_layers[1][0], self.fuse_layers[2][0], self.fuse_layers[2][1]
        if len(l10) != 1 or len(l20) != 2 or len(l21) != 1:
            return False
        convs = [l10[0][0], l20[0][0], l20[1][0], l21[0][0]]
        if not all(s2_conv_ok(c) for c in convs) or \
                l10[0][0].out_channels + l20[0][0].out_channels > 96 or \
                l20[1][0].out_channels != l21[0][0].out_channels:
            return False
        h1, w1 = (x[0].shape[2] + 1) // 2, (x[0].shape[3] + 1) // 2
        h2, w2 = (h1 + 1) // 2, (w1 + 1) // 2
        return tuple(x[1].shape[2:]) == (h1, w1) and tuple(x[2].shape[2:]) == (h2, w2) and \
            x[1].shape[1] == l10[0][0].out_channels and x[2].shape[1] == l21[0][0].out_channels

    def _heads_sum1(self, x0, x1, t12):
        """The scale-0 heads launch (see _down0_heads) that also completes output branch 1:
        -> (branch 1 output, first conv of the branch-2 chain)."""
        l10, l20 = self.fuse_layers[1][0], self.fuse_layers[2][0]
        pairs = [(l10[0][0], l10[0][1]), (l20[0][0], l20[0][1])]
        pk = s2_pack(l10, pairs)
        co_a = pairs[0][0].out_channels
        return ops.conv3x3_s2(x0.contiguous(), pk[0], pk[1], co_a + pairs[1][0].out_channels,
                              co_a, "leaky", "leaky", identity=x1.contiguous(),
                              up=t12.contiguous())

    def _branch2_sum(self, hb, x1, x2):
        """Output branch 2 as one stride-2 conv over [hb, x1] + x2 (see _s2_sums_ok)."""
        l20, l21 = self.fuse_layers[2][0], self.fuse_layers[2][1]
        pk = s2_pack_k(l21, [(l20[1][0], l20[1][1]), (l21[0][0], l21[0][1])])
        co = l21[0][0].out_channels
        return ops.conv3x3_s2(hb, pk[0], pk[1], co, co, "leaky", None, x2=x1.contiguous(),
                              identity=x2.contiguous())[0]

    def _term_down0(self, x, i, heads):
        """Exchange term (i, 0) given the head outputs of _down0_heads."""
        if i in heads:
            return self._down(heads[i], i, 0, start=1)
        return self._down(x[0], i, 0)

    def _forward_eval(self, x, streams=None, keep=None, conv1_pre=None, post=None, sched=None):
        """Eval ISA + CSA.  The coarser scales run first, so that their exchange terms for output
        branch 0 exist when the scale-0 bottleneck runs: its tail kernel then writes both the
        block output and the cross-scale sum of branch 0 (aanet_csa_epilogue_t), which removes
        the scale-0 resize-sum kernel.  The in-place list mutation of aggregation.py:382 and the
        term order of aggregation.py:388-400 are unchanged (the branches are independent).

        streams (AdaptiveAggregation's concurrent-scale schedule): [current stream, side stream
        of scale 1, ..., of scale S-1] (side streams may repeat).  Every piece of work runs on
        the stream of the scale it produces, as soon as its inputs exist (HIP events):
          scale j >= 1: block j -> the up terms (i < j, 1x1 at scale j) -> [every coarse
                        block done] the down terms from the coarse scales j' < j (stride-2
                        chains) -> [block 0 done] the down term from scale 0 -> branch j's sum;
          scale 0:      conv1 -> offset conv -> [coarse up terms done] the tail kernel (block
                        output + branch 0's CSA sum).
        After the scale-0 tail, the down chains of the coarse branches run concurrently on their
        own streams, and with them the next module's coarse blocks and exchange terms: that is
        the dependency chain between two scale-0 tail kernels.  Tensors read
        across streams are appended to `keep` (alive until the caller joins the streams, so the
        caching allocator cannot hand their memory to another stream).

        conv1_pre: the scale-0 bottleneck's conv1 output, already computed by the previous
        module's tail kernel (its post stage); post: this module's scale-0 tail post stage (the
        next module's conv1, or final_conv + regression), result in post["result"].
        sched: state shared by the modules of one AdaptiveAggregation run.  With the prep_stream
        option a deformable scale-0 block's conv1 + offset conv run on their own side stream as
        soon as the previous module's scale-0 tail has written x[0] (sched["tail_ev"]), beside
        that module's stride-2 heads, instead of after them on the current stream."""
        S = len(self.branches)
        nout = len(self.fuse_layers)
        if streams is None:
            for i in range(1, S):
                for j in range(self.num_blocks):
                    x[i] = self.branches[i][j](x[i])
            up0 = [self._exchange_up(x, 0, j) for j in range(1, S)]
            terms = {(0, j): t for j, t in zip(range(1, S), up0)}
            for j in range(self.num_blocks - 1):
                x[0] = self.branches[0][j](x[0])
            ok = csa_epilogue_ok(x[0], up0)
            x[0], csa0 = self.branches[0][self.num_blocks - 1].forward_csa(
                x[0], up0 if ok else None, conv1_out=conv1_pre if self.num_blocks == 1 else None,
                post=post if ok else None)
            if post is not None and not ok:
                post["result"] = None
            return self._fuse_eval(x, {0: csa0} if csa0 is not None else {}, terms)

        main = streams[0]
        terms, up_ev = {}, {}
        # coarse blocks and their up terms (i < j: 1x1 at scale j), each on its scale's stream
        for j in range(1, S):
            with torch.cuda.stream(streams[j]):
                for b in range(self.num_blocks):
                    x[j] = self.branches[j][b](x[j])
                for i in range(min(j, nout)):
                    terms[(i, j)] = self._exchange_up(x, i, j)
                up_ev[j] = _record(streams[j])
        keep.extend(x[1:])
        keep.extend(terms.values())
        # scale 0: joins the coarse streams just before its tail kernel.  Every cross-stream edge
        # goes through the current stream: HIP graph capture crashes (host segfault in
        # hipStreamEndCapture) when two side streams wait on each other's events.
        up0 = [terms[(0, j)] for j in range(1, S)]
        mark = {}

        def join():
            for j in range(1, S):
                main.wait_event(up_ev[j])
            mark["coarse"] = _record(main)  # every coarse block and up term is done

        for b in range(self.num_blocks - 1):
            x[0] = self.branches[0][b](x[0])
        ok = csa_epilogue_ok(x[0], up0)
        prep = None
        if sched is not None and self.num_blocks == 1 and sched.get("tail_ev") is not None and \
                get_option(self, "prep_stream"):
            prep = (prep_stream(x[0].device), sched["tail_ev"], keep)
        x[0], csa0 = self.branches[0][self.num_blocks - 1].forward_csa(
            x[0], up0 if ok else None, before_tail=join,
            conv1_out=conv1_pre if self.num_blocks == 1 else None, post=post if ok else None,
            prep=prep)
        if post is not None and not ok:
            post["result"] = None
        if sched is not None:
            sched["tail_ev"] = _record(main)  # x[0] / out[0] written: the next module's prep
        if post is not None and post.get("result") is not None:
            keep.extend(v for v in post["result"].values() if v is not None)
        keep.append(x[0])
        if "coarse" not in mark:  # the tail kernel did not take the block
            join()
        sums = self._s2_sums_ok(x)
        if sums:  # heads + branch 1's sum (x[1] and the up term exist: the join above)
            out1, hb = self._heads_sum1(x[0], x[1], terms[(1, 2)])
            keep.extend((out1, hb))
            heads = {}
        else:
            heads = self._down0_heads(x[0])  # on the current stream: both branches need them
            keep.extend(heads.values())
        b0_ev = _record(main)
        out = [None] * nout
        if csa0 is None:  # no tail epilogue: branch 0's sum on the current stream
            out[0] = ops.csa_sum([x[0]] + [t.contiguous() for t in up0], act="leaky")
        else:
            out[0] = csa0
        # coarse branches: the down terms from the coarse scales (concurrent with the scale-0
        # tail), then the one from scale 0, then the sum, on the branch's stream (with the
        # stride-2 sums: branch 1 comes from the heads launch, branch 2 is one launch)
        for i in range(1, nout):
            st = streams[i]
            with torch.cuda.stream(st):
                st.wait_event(mark["coarse"])
                if sums:
                    st.wait_event(b0_ev)
                    out[i] = out1 if i == 1 else self._branch2_sum(hb, x[1], x[2])
                    keep.append(out[i])
                    continue
                for j in range(1, i):
                    terms[(i, j)] = self._down(x[j], i, j)
                st.wait_event(b0_ev)
                terms[(i, 0)] = self._term_down0(x, i, heads)
                out[i] = ops.csa_sum([(x[i] if i == j else terms[(i, j)]).contiguous()
                                      for j in range(S)], act="leaky")
            keep.append(out[i])
        return out

    def _fuse_eval(self, x, done=None, terms_cache=None):
        """Eval CSA: each exchange conv (+BN folded, +LeakyReLU inside strided chains) is one HIP
        conv kernel at its own resolution (the first convs of the down chains from scale 0 as one
        stride-2 launch, _down0_heads); the resize + sum + LeakyReLU of every output branch is
        one aanet_csa_sum_f32 kernel (same term order as aggregation.py:388-400).  done: output
        branches already summed (by a tail-kernel epilogue); terms_cache: exchange terms already
        computed, keyed (i, j)."""
        done = dict(done or {})
        terms_cache = terms_cache or {}
        if 1 not in done and 2 not in done and self._s2_sums_ok(x):
            t12 = terms_cache.get((1, 2))
            if t12 is None:
                t12 = self._exchange_up(x, 1, 2)
            done[1], hb = self._heads_sum1(x[0], x[1], t12)
            done[2] = self._branch2_sum(hb, x[1], x[2])
        heads = self._down0_heads(x[0]) if any(i not in done for i in range(1, len(self.fuse_layers))) else {}
        x_fused = []
        for i in range(len(self.fuse_layers)):
            if i in done:
                x_fused.append(done[i])
                continue
            terms = []
            for j in range(len(self.branches)):
                layer = self.fuse_layers[i][j]
                if i == j:
                    terms.append(x[j])
                elif (i, j) in terms_cache:
                    terms.append(terms_cache[(i, j)])
                elif i < j:
                    terms.append(conv_bn_act(x[j], layer[0], layer[1], None))
                elif j == 0:
                    terms.append(self._term_down0(x, i, heads))
                else:
                    terms.append(self._down(x[j], i, j))
            x_fused.append(ops.csa_sum([t.contiguous() for t in terms], act="leaky"))
        return x_fused

    @fp32_convs
    def forward(self, x, streams=None, keep=None, conv1_pre=None, post=None, sched=None):
        """aggregation.py:375-402.  streams / keep / sched: the concurrent-scale schedule of
        AdaptiveAggregation (eval only, see _forward_eval); conv1_pre / post: the cross-module
        pointwise fusions of AdaptiveAggregation (eval only)."""
        assert len(self.branches) == len(x)
        if self.num_scales > 1 and use_fused(self, x[0]) and getattr(self, "aanet_fuse_csa", True):
            return self._forward_eval(x, streams, keep, conv1_pre, post, sched)
        if post is not None:
            post["result"] = None
        if streams is not None:  # reference op sequence: one stream
            for st in streams[1:]:
                streams[0].wait_stream(st)
        for i in range(len(self.branches)):
            branch = self.branches[i]
            for j in range(self.num_blocks):
                dconv = branch[j]
                x[i] = dconv(x[i])

        if self.num_scales == 1:  # without fusions
            return x

        if use_fused(self, x[0]):
            return self._fuse_eval(x)
        x_fused = []
        for i in range(len(self.fuse_layers)):
            for j in range(len(self.branches)):
                if j == 0:
                    x_fused.append(self.fuse_layers[i][0](x[0]))
                else:
                    exchange = self.fuse_layers[i][j](x[j])
                    if exchange.size()[2:] != x_fused[i].size()[2:]:
                        exchange = ops.resize_bilinear(exchange, x_fused[i].size()[2:])
                    x_fused[i] = x_fused[i] + exchange

        for i in range(len(x_fused)):
            x_fused[i] = self.relu(x_fused[i])
        return x_fused


class AdaptiveAggregation(FoldCacheMixin, nn.Module):
    """Stacked AAModules (aggregation.py:406-464)."""

    def __init__(self, max_disp, num_scales=3, num_fusions=6, num_stage_blocks=1,
                 num_deform_blocks=2, intermediate_supervision=True, deformable_groups=2,
                 mdconv_dilation=2):
        super(AdaptiveAggregation, self).__init__()
        self.max_disp = max_disp
        self.num_scales = num_scales
        self.num_fusions = num_fusions
        self.intermediate_supervision = intermediate_supervision

        fusions = nn.ModuleList()
        for i in range(num_fusions):
            if self.intermediate_supervision:
                num_out_branches = self.num_scales
            else:
                num_out_branches = 1 if i == num_fusions - 1 else self.num_scales
            simple_bottleneck_module = not (i >= num_fusions - num_deform_blocks)
            fusions.append(AdaptiveAggregationModule(num_scales=self.num_scales,
                                                     num_output_branches=num_out_branches,
                                                     max_disp=max_disp,
                                                     num_blocks=num_stage_blocks,
                                                     mdconv_dilation=mdconv_dilation,
                                                     deformable_groups=deformable_groups,
                                                     simple_bottleneck=simple_bottleneck_module))
        self.fusions = nn.Sequential(*fusions)

        self.final_conv = nn.ModuleList()
        for i in range(self.num_scales):
            in_channels = max_disp // (2 ** i)
            self.final_conv.append(nn.Conv2d(in_channels, max_disp // (2 ** i), kernel_size=1))
            if not self.intermediate_supervision:
                break

    def set_options(self, **options):
        """Eval schedule options of this aggregation (nets/options.py: concurrent_scales,
        post_fusion, s2_sums, dense_grouped); returns self."""
        return set_options(self, **options)

    def _post_for(self, i, regress):
        """The post stage of fusion i's scale-0 tail kernel (eval, fused): the next module's
        bottleneck conv1 + BN1 + ReLU (NHWC), or for the last fusion, with `regress`, final_conv +
        the soft-argmin.  None when the shapes do not fit (64 channels at scale 0, 1x1, one
        stage block)."""
        if i + 1 < self.num_fusions:
            if get_option(self, "post_fusion") != "all":
                return None
            # the window DCN tail (dcn_tile.hip) pays more for the conv1 stage (spills of its POST
            # instantiation: +60-65 us per launch) than the separate 1x1 launch costs (46-56 us);
            # the plain 3x3 tail takes it for +25-30 us
            if isinstance(self.fusions[i].branches[0][-1], DeformSimpleBottleneck):
                return None
            nxt = self.fusions[i + 1]
            if nxt.num_blocks != 1 or len(nxt.branches) == 0:
                return None
            blk = nxt.branches[0][0]
            c1 = blk.conv1
            if tuple(c1.weight.shape) != (64, 64, 1, 1):
                return None
            _, b1, p1 = folded(c1, blk.bn1)
            if not getattr(p1, "_aanet_split", False):
                return None
            return {"packed": p1, "bias": b1, "act": "relu", "nhwc": True}
        if not regress:
            return None
        fc = self.final_conv[0]
        if tuple(fc.weight.shape) != (64, 64, 1, 1):
            return None
        _, bf, pf = folded(fc, None)
        if not getattr(pf, "_aanet_split", False):
            return None
        # the last module's block output and CSA sum feed nothing but final_conv: not stored
        return {"packed": pf, "bias": bf, "act": None, "disp": True, "skip_outputs": True}

    @fp32_convs
    def forward(self, cost_volume):
        """aggregation.py:452-464 (final 1x1 conv with bias on the HIP conv engine in eval)."""
        return self._run(cost_volume)[0]

    def _run(self, cost_volume, regress=False, chains=1):
        """-> (aggregated cost volumes, disparity or None).  In eval on the fused path each
        fusion's scale-0 tail kernel also computes the next fusion's conv1 (post stage); with
        `regress` (the caller's DisparityEstimation is the plain similarity soft-argmin and there
        is one output scale) the last tail computes final_conv + the regression too, and the
        cost-volume list is then None.  chains > 1 (the whole-model callers, option
        batch_chains): the batch is split into that many chunks, each aggregated on its own
        stream (_run_chains); the caller's list is then not mutated."""
        assert isinstance(cost_volume, list)
        fused = use_fused(self, cost_volume[0])
        if self._pipeline_ok(cost_volume, fused):
            return self._run_pipelined(cost_volume)
        if chains > 1 and fused and cost_volume[0].is_cuda and cost_volume[0].shape[0] >= 2:
            return self._run_chains(cost_volume, regress, min(chains, cost_volume[0].shape[0]))
        return self._run_one(cost_volume, regress, fused)

    def _run_chains(self, cost_volume, regress, k):
        """Batch pipelining: the pairs are independent, so chunk c of the batch runs the whole
        aggregation on its own stream -- chunk 0 on the current stream (with the concurrent-scale
        side streams), chunk c >= 1 on side stream S - 1 + c with the one-stream schedule.  The
        small, serially dependent kernels of one chunk (stride-2 heads, the coarse scales) then
        run beside the large scale-0 tail kernels of another.  Every stream waits only for the
        current stream and the current stream joins every stream (the only cross-stream edges
        HIP graph capture takes).  Each pair's arithmetic is unchanged: bit-identical results."""
        dev = cost_volume[0].device
        main = torch.cuda.current_stream(dev)
        B = cost_volume[0].shape[0]
        bounds = [B * c // k for c in range(k + 1)]
        chunks = [[t[bounds[c]:bounds[c + 1]] for t in cost_volume] for c in range(k)]
        extra = side_streams(dev, max(self.num_scales - 1, 0) + k - 1)[max(self.num_scales - 1, 0):]
        ready = _record(main)  # the cost volumes exist
        strm = [main] + extra[:k - 1]
        gens = [self._run_steps(chunks[0], regress, True)]
        for c in range(1, k):
            strm[c].wait_event(ready)
            with torch.cuda.stream(strm[c]):
                gens.append(self._run_steps(chunks[c], regress, True, concurrent=False))
        # Issue the chunks fusion by fusion, round robin: the HIP graph executor launches the
        # captured nodes in capture order, and chunk-by-chunk issue ran the chunks one after the
        # other (profiles/r06_chains_timeline.txt, tools/step_big_kernels.py).  A step that (re)fills a weight cache (first
        # call, new weights) ran those kernels on its own stream: the other streams catch up with
        # it, through the current stream, before their next step.
        results, live, behind = [None] * k, list(range(k)), set()
        while live:
            for c in list(live):
                if c in behind:
                    strm[c].wait_stream(main)
                    behind.discard(c)
                fills = _lib.cache_fills()
                try:
                    with torch.cuda.stream(strm[c]):
                        next(gens[c])
                except StopIteration as done:
                    results[c] = done.value
                    live.remove(c)
                if _lib.cache_fills() != fills:
                    if c:
                        main.wait_stream(strm[c])
                    behind = set(range(1, k)) - {c}
        for c in range(1, k):
            r = results[c]
            for t in ([r[1]] if r[1] is not None else r[0]):
                t.record_stream(main)  # allocated on a side stream, read on main below
        for st in extra[:k - 1]:
            main.wait_stream(st)
        if results[0][1] is not None:
            return None, torch.cat([r[1] for r in results])
        return [torch.cat([r[0][i] for r in results]) for i in range(len(results[0][0]))], None

    def _pipeline_ok(self, cost_volume, fused):
        """Whether the cross-module pipelined schedule (option `pipeline`, _run_pipelined) takes
        this aggregation: eval fast path on the GPU, three scales, one block per branch, and the
        stride-2 sums (heads kernel + branch-2 conv) for every module with three outputs."""
        if not (fused and cost_volume[0].is_cuda and self.num_scales == 3 and
                get_option(self, "pipeline") and len(cost_volume) == 3 and
                csa_epilogue_ok(cost_volume[0], cost_volume[1:])):
            return False
        for f in self.fusions:
            if f.num_blocks != 1 or (len(f.fuse_layers) == 3 and not f._s2_sums_ok(cost_volume)):
                return False
            if len(f.fuse_layers) not in (1, 3):
                return False
        return True

    def _run_pipelined(self, cost_volume):
        """Cross-module pipelined eval schedule (option `pipeline`).  Module m's scale-0 block
        T(m) needs only the previous module's scale-0 CSA sum, so it runs on side stream F while
        the current stream runs the previous module's stride-2 heads H(m-1) and this module's
        coarse blocks (scale 1 here, scale 2 on side stream B); the scale-0 CSA sum S(m) (one
        aanet_csa_sum_f32) follows on F once both are done:
            F:    S(m-1) -> T(m) ---------------------(wait chains(m))-> S(m) -> T(m+1) ...
            main: (wait T(m-1)) H(m-1) -> scale-1 block + up terms (m) -> (wait T(m)) H(m) ...
            B:    (wait H(m-1)) scale-2 block + up terms (m)
        so the heads and the small, serially dependent coarse kernels overlap the large scale-0
        tails instead of running between them.  Every cross-stream edge goes through the current
        stream (side streams wait only for it; it waits for them), which HIP graph capture needs.
        Same arithmetic per term as the default schedule except that branch 0's sum is the
        separate aanet_csa_sum_f32 kernel instead of the tail kernel's CSA epilogue, and conv1
        of each scale-0 block is its own launch.  (A fused sum + conv1 kernel measured 192 us
        alone against 45 + 55 us for the two.)"""
        dev = cost_volume[0].device
        main = torch.cuda.current_stream(dev)
        F, B = side_streams(dev, 2)
        ready = _record(main)
        F.wait_event(ready)
        B.wait_event(ready)
        keep = list(cost_volume)
        x0, x1, x2 = cost_volume
        y0 = None          # the scale-0 block's conv1 output, from the previous S
        nf = self.num_fusions

        def block0(fu):
            with torch.cuda.stream(F):
                out = fu.branches[0][0].forward_csa(x0, None, conv1_out=y0)[0] if y0 is not None \
                    else fu.branches[0](x0)
            return out, _record(F)

        out0, ev_t = block0(self.fusions[0])       # T(0)
        for m, fu in enumerate(self.fusions):
            nout = len(fu.fuse_layers)
            with torch.cuda.stream(B):      # scale 2: block + its up terms
                y2 = fu.branches[2](x2)
                t02 = fu._exchange_up([None, None, y2], 0, 2)
                t12 = fu._exchange_up([None, None, y2], 1, 2) if nout > 1 else None
            ev_b = _record(B)
            y1 = fu.branches[1](x1)         # scale 1 on the current stream
            t01 = fu._exchange_up([None, y1], 0, 1)
            main.wait_event(ev_b)
            main.wait_event(ev_t)
            keep.extend(t for t in (out0, y1, y2, t01, t02, t12) if t is not None)
            # S(m): branch 0's sum, then the next block's conv1 (both alone on the GPU)
            x0 = ops.csa_sum([out0, t01.contiguous(), t02.contiguous()], act="leaky")
            keep.append(x0)
            nxt = self._pipeline_conv(m + 1) if m + 1 < nf else None
            y0 = conv_bn_act(x0, nxt.conv1, nxt.bn1, "relu", out_nhwc=True) if nxt is not None \
                else None
            if y0 is not None:
                keep.append(y0)
            h_in = out0
            if m + 1 < nf:
                # T(m + 1) is captured BEFORE H(m): the HIP graph executor launches nodes in
                # capture order, and T(m + 1) captured after H(m) and the coarse blocks ran after
                # them (no overlap)
                F.wait_event(_record(main))
                out0, ev_t = block0(self.fusions[m + 1])
            if nout == 3:                   # H(m): branches 1 and 2, beside T(m + 1)
                x1, hb = fu._heads_sum1(h_in, y1, t12)
                x2 = fu._branch2_sum(hb, y1, y2)
                keep.extend((x1, hb, x2))
                B.wait_event(_record(main))
            else:
                x1 = x2 = None
        out = [conv_bn_act(x0, self.final_conv[0])]
        if len(self.final_conv) > 1:
            out += [conv_bn_act(t, c) for t, c in zip((x1, x2), self.final_conv[1:])]
        main.wait_stream(F)
        main.wait_stream(B)
        del keep
        return out, None

    def _pipeline_conv(self, i):
        """Fusion i's scale-0 block when its conv1 can run ahead of the block (the pipelined
        schedule computes it right after the previous module's branch-0 sum, on the current
        stream, channels-last as the tail kernels read it), or None."""
        blk = self.fusions[i].branches[0][0]
        if self.fusions[i].num_blocks != 1 or blk.conv1.weight.shape[0] % 32:
            return None
        return blk

    def _run_one(self, cost_volume, regress, fused, concurrent=True):
        gen = self._run_steps(cost_volume, regress, fused, concurrent)
        while True:
            try:
                next(gen)
            except StopIteration as done:
                return done.value

    def _run_steps(self, cost_volume, regress, fused, concurrent=True):
        """_run_one as a generator: one fusion per step (yields after each), the result as its
        return value; the caller keeps the stream it started on current across steps."""
        streams = None
        if fused and cost_volume[0].is_cuda and self.num_scales > 1 and concurrent and \
                get_option(self, "concurrent_scales"):
            dev = cost_volume[0].device
            main = torch.cuda.current_stream(dev)
            ss = side_streams(dev, self.num_scales - 1)
            streams = [main] + ss  # scale i >= 1 on side stream i - 1
            for st in ss:
                st.wait_stream(main)  # the cost volumes are written on the current stream
            keep = list(cost_volume)
            sched = {}
        pre, disp = None, None
        post_ok = fused and cost_volume[0].is_cuda and get_option(self, "post_fusion") != "none"
        for i in range(self.num_fusions):
            fusion = self.fusions[i]
            post = self._post_for(i, regress) if post_ok else None
            if streams is not None:
                cost_volume = fusion(cost_volume, streams, keep, conv1_pre=pre, post=post,
                                     sched=sched)
            elif post_ok:
                cost_volume = fusion(cost_volume, conv1_pre=pre, post=post)
            else:
                cost_volume = fusion(cost_volume)
            res = post.get("result") if post is not None else None
            pre = res["out"] if res is not None else None
            if res is not None and res.get("disp") is not None:
                disp = res["disp"]
            yield
        if streams is not None:
            for st in ss:
                main.wait_stream(st)
            if dev in _PREP_STREAMS:
                main.wait_stream(_PREP_STREAMS[dev])
            del keep
        if disp is not None:
            return None, disp
        out = []  # 1/3, 1/6, 1/12
        for i in range(len(self.final_conv)):
            if fused:
                out = out + [conv_bn_act(cost_volume[i], self.final_conv[i])]
            else:
                out = out + [self.final_conv[i](cost_volume[i])]
        return out, None
