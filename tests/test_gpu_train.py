"""GPU tests of the training step on the drop-in path: the Trainer over
AANetHotPath (HIP forward + backward kernels, Adam with the offset_conv 0.1x group), and
data parallelism with SyncBatchNorm -- two ranks sharing cuda:0 over gloo (one GPU on the test
box; the production backend is nccl=RCCL, one process per GPU) against one process on the full
batch with plain BatchNorm."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aanet_amd import nets, train

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _inputs(B, seed):
    g = torch.Generator().manual_seed(seed)
    sizes = [(24, 48), (12, 24), (6, 12)]
    left = [torch.randn(B, 16, h, w, generator=g).to(DEV) for h, w in sizes]
    right = [torch.randn(B, 16, h, w, generator=g).to(DEV) for h, w in sizes]
    gt = (torch.rand(B, 48, 96, generator=g) * 12 + 1).to(DEV)   # 2x the scale-0 resolution
    return left, right, gt


def _model(seed=0):
    torch.manual_seed(seed)
    return nets.AANetHotPath(16, no_intermediate_supervision=False, num_deform_blocks=3).to(DEV)


def test_trainer_steps_hot_path():
    m = _model()
    t = train.Trainer(m, lr=1e-3)
    off0 = {n: p.detach().clone() for n, p in m.named_parameters() if "offset_conv" in n}
    base0 = {n: p.detach().clone() for n, p in m.named_parameters() if "offset_conv" not in n}
    assert off0 and base0
    l, r, gt = _inputs(2, 0)
    losses = [float(t.step(l, r, gt)) for _ in range(4)]
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < losses[0], losses
    # both groups moved; Adam's first step moves each weight by ~lr, so the offset group (0.1 lr)
    # moves about a tenth as far
    named = {n: p.detach() for n, p in m.named_parameters()}
    d_off = max(float((named[n] - p).abs().max()) for n, p in off0.items())
    d_base = max(float((named[n] - p).abs().max()) for n, p in base0.items())
    assert 0 < d_off < 0.5 * d_base, (d_off, d_base)


def _conv_grad_vs_fp64(conv, run_step):
    """Run `run_step()` with torch's global allow_tf32=True; return (the flags seen by conv's weight
    hook, its weight gradient's max error against an fp64 recomputation / the gradient scale)."""
    seen, captured = [], {}

    def hook(g):
        seen.append(torch.backends.cudnn.allow_tf32)
        captured["g"] = g.detach().clone()
    conv.weight.register_hook(hook)
    xin, gout = {}, {}

    def fwd_hook(mod, inp, out):
        xin["x"] = inp[0].detach().clone()
        out.register_hook(lambda g: gout.setdefault("g", g.detach().clone()))
    conv.register_forward_hook(fwd_hook)
    prev = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = True
    try:
        run_step()
        assert torch.backends.cudnn.allow_tf32 is True
    finally:
        torch.backends.cudnn.allow_tf32 = prev
    x64, g64 = xin["x"].double(), gout["g"].double()
    ref = torch.nn.grad.conv2d_weight(x64, conv.weight.shape, g64, conv.stride, conv.padding,
                                      conv.dilation, conv.groups)
    scale = torch.nn.grad.conv2d_weight(x64.abs(), conv.weight.shape, g64.abs(), conv.stride,
                                        conv.padding, conv.dilation, conv.groups).max()
    return seen, float((captured["g"].double() - ref).abs().max() / scale)


def test_drop_in_backward_convs_fp32_without_trainer():
    """the reference's own loop calls total_loss.backward() (model.py:137) with no
    Trainer and no fp32_scope, under torch's default global allow_tf32=True.  The drop-in's MIOpen
    convs are pinned (_precision.PinnedConv2d: aten convolution forward/backward with TF32 off), so
    a conv weight gradient still matches fp64 at fp32 tolerance; and a transposed conv (AANet+'s
    hourglass deconvolutions, Conv2x) against a float64 copy of the module."""
    from aanet_amd import _precision
    m = _model(3).train()
    conv = m.aggregation.fusions[0].branches[0][0].conv1

    def step():
        l, r, gt = _inputs(2, 4)
        total, _ = train.disparity_loss(m(l, r), gt, gt > 0)
        total.backward()
    seen, err = _conv_grad_vs_fp64(conv, step)
    assert type(conv) is _precision.PinnedConv2d
    assert err <= 1e-5, err

    from aanet_amd.nets.feature import Conv2x
    torch.manual_seed(1)
    c = Conv2x(48, 32, deconv=True).to(DEV).train()
    c64 = copy.deepcopy(c).cpu().double()
    x = torch.randn(2, 48, 12, 16, device=DEV, requires_grad=True)
    rem = torch.randn(2, 32, 24, 32, device=DEV)
    g = torch.randn(2, 32, 24, 32, device=DEV)
    prev = torch.backends.cudnn.allow_tf32
    torch.backends.cudnn.allow_tf32 = True
    try:
        (c(x, rem) * g).sum().backward()
    finally:
        torch.backends.cudnn.allow_tf32 = prev
    x64 = x.detach().cpu().double().requires_grad_()
    (c64(x64, rem.cpu().double()) * g.cpu().double()).sum().backward()
    assert type(c.conv1.conv) is _precision.PinnedConvTranspose2d
    for (n, p), (_, p64) in zip(c.named_parameters(), c64.named_parameters()):
        e = float((p.grad.cpu().double() - p64.grad).abs().max() / p64.grad.abs().max())
        assert e <= 1e-5, (n, e)
    e = float((x.grad.cpu().double() - x64.grad).abs().max() / x64.grad.abs().max())
    assert e <= 1e-5, ("input", e)


def test_trainer_backward_convs_run_fp32_under_global_tf32():
    """with torch's global allow_tf32=True, the MIOpen conv backward of a Trainer step
    runs with TF32 off, and the weight gradient of such a conv matches an fp64 recomputation at
    fp32 tolerance.  engine_convs=False keeps the conv on MIOpen (with the engine
    convs, the default on the GPU, this conv is an EngineConv2d -- the next test)."""
    from aanet_amd import _precision
    m = _model(3)
    conv = m.aggregation.fusions[0].branches[0][0].conv1    # a MIOpen conv in training
    t = train.Trainer(m, lr=1e-3, accumulation_steps=2, engine_convs=False)  # no optimizer step

    def step():
        l, r, gt = _inputs(2, 4)
        t.step(l, r, gt)
    seen, err = _conv_grad_vs_fp64(conv, step)
    assert type(conv) is _precision.PinnedConv2d, type(conv)
    assert seen == [False], seen
    assert err <= 1e-5, err


def test_trainer_engine_convs_wgrad_fp32():
    """The Trainer's default on the GPU: the plain convs on the HIP engine (EngineConv2d, fp32
    forward / dgrad / wgrad kernels whatever the TF32 flag) -- the same fp64 check."""
    m = _model(3)
    conv = m.aggregation.fusions[0].branches[0][0].conv1
    t = train.Trainer(m, lr=1e-3, accumulation_steps=2)

    def step():
        l, r, gt = _inputs(2, 4)
        t.step(l, r, gt)
    _, err = _conv_grad_vs_fp64(conv, step)
    assert type(conv) is train.EngineConv2d, type(conv)
    assert err <= 1e-5, err


def test_deterministic_training_step_is_bit_reproducible():
    """Same seed and data, deterministic algorithms on: every gradient of the path is
    bit-identical across two runs (the DCN weight/input gradients come from the fixed-point
    aanet_mdcn_bwd_det_f32).  The loss is taken on the pyramid directly -- torch's bilinear
    upsample backward (the loss's resizing) has no deterministic CUDA kernel."""
    grads = []
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True)
    try:
        for _ in range(2):
            m = _model(5).train()
            l, r, _ = _inputs(2, 1)
            loss = sum((d * (i + 1)).mean() for i, d in enumerate(m(l, r)))
            loss.backward()
            grads.append({n: p.grad.clone() for n, p in m.named_parameters()
                          if p.grad is not None})
    finally:
        torch.use_deterministic_algorithms(prev)
    a, b = grads
    assert a.keys() == b.keys() and len(a) > 100
    diff = [n for n in a if not torch.equal(a[n], b[n])]
    assert not diff, diff[:20]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_worker(rank, world, port, q):
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        torch.cuda.set_device(0)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        m = _model(11)
        ref = copy.deepcopy(m)
        ddp = train.wrap_data_parallel(m, torch.device(DEV), sync_bn=True)
        assert isinstance(ddp, torch.nn.parallel.DistributedDataParallel)
        assert any(isinstance(x, torch.nn.SyncBatchNorm) for x in ddp.modules())
        l, r, gt = _inputs(2 * world, 3)
        sl = slice(2 * rank, 2 * rank + 2)
        ddp.train()
        tot, _ = train.disparity_loss(ddp([x[sl] for x in l], [x[sl] for x in r]), gt[sl],
                                      gt[sl] > 0)
        tot.backward()
        # reference: one process, full batch, plain BatchNorm (batch statistics over all ranks)
        ref.train()
        rtot, _ = train.disparity_loss(ref(l, r), gt, gt > 0)
        rtot.backward()
        got = torch.cat([p.grad.flatten() for p in m.parameters() if p.grad is not None])
        want = torch.cat([p.grad.flatten() for p in ref.parameters() if p.grad is not None])
        cos = float(got @ want / (got.norm() * want.norm()))
        rel = float((got - want).norm() / want.norm())
        sums = [torch.zeros(1) for _ in range(world)]
        dist.all_gather(sums, torch.tensor([float(got.double().sum())]))
        if rank == 0:
            q.put(("ok", cos, rel, [float(s) for s in sums]))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on q.get
        q.put(("error", repr(e), 0.0, []))
        raise


def test_ddp_syncbn_two_ranks_match_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        status, cos, rel, sums = q.get(timeout=300)
    finally:
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert status == "ok", cos
    for p in procs:
        assert p.exitcode == 0
    assert sums[0] == sums[1]                 # all-reduced gradients identical on both ranks
    assert cos > 0.9999 and rel < 1e-2, (cos, rel)


@pytest.mark.parametrize("det", [False, True])
def test_graph_step_matches_eager_steps(det):
    """Trainer.graph_step (the whole step as one HIP graph replay, warm-up steps undone) gives the
    parameters of the same number of eager steps (same capturable Adam), and the loss falls."""
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(det, warn_only=True)
    try:
        l, r, gt = _inputs(2, 7)
        mask = (gt > 0) & (gt < 192)
        runs = []
        for graph in (False, True):
            m = _model(13).train()
            t = train.Trainer(m, lr=1e-3, capturable=True)
            losses = []
            for _ in range(3):
                loss = t.graph_step(l, r, gt, mask) if graph else t.step(l, r, gt, mask)
                losses.append(float(loss))
            runs.append(([p.detach().clone() for p in m.parameters()], losses))
    finally:
        torch.use_deterministic_algorithms(prev)
    (pe, le), (pg, lg) = runs
    assert abs(le[0] - lg[0]) <= 1e-5 * abs(le[0]), (le, lg)
    assert lg[-1] < lg[0]
    num = sum(float((a - b).double().norm() ** 2) for a, b in zip(pe, pg)) ** 0.5
    den = sum(float(a.double().norm() ** 2) for a in pe) ** 0.5
    # Non-deterministic mode sums gradients with float atomics, so two eager runs already differ in
    # the last bits; Adam's m / sqrt(v) turns that into lr-sized moves of near-zero-gradient
    # elements (measured 1.5e-5 relative after 3 steps).  Deterministic mode must agree tightly.
    assert num <= (1e-5 if det else 1e-4) * den, (num, den)


def test_graph_step_keeps_prior_eager_optimizer_state():
    """eager step()s before the first graph_step -- the capture's warm-up is undone
    back to THAT state (Adam moments and step count kept), so 2 eager + 2 graph steps give the
    parameters of 4 eager steps."""
    prev = torch.are_deterministic_algorithms_enabled()
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        l, r, gt = _inputs(2, 9)
        mask = (gt > 0) & (gt < 192)
        runs = []
        for graph in (False, True):
            m = _model(17).train()
            t = train.Trainer(m, lr=1e-3, capturable=True)
            for i in range(4):
                if graph and i >= 2:
                    t.graph_step(l, r, gt, mask)
                else:
                    t.step(l, r, gt, mask)
            torch.cuda.synchronize()
            runs.append([p.detach().clone() for p in m.parameters()])
    finally:
        torch.use_deterministic_algorithms(prev)
    num = sum(float((a - b).double().norm() ** 2) for a, b in zip(*runs)) ** 0.5
    den = sum(float(a.double().norm() ** 2) for a in runs[0]) ** 0.5
    assert num <= 1e-5 * den, (num, den)


def test_graph_step_then_eval_refolds():
    """graph replays update parameters and BN statistics without bumping _version;
    graph_step, eval forward, graph_step, eval forward must match a freshly folded model."""
    l, r, gt = _inputs(2, 11)
    mask = (gt > 0) & (gt < 192)
    m = _model(19).train()
    t = train.Trainer(m, lr=1e-2, capturable=True)
    t.graph_step(l, r, gt, mask)
    m.eval()
    with torch.no_grad():
        first = m(l, r)[0].clone()
    t.graph_step(l, r, gt, mask)
    for mod in m.modules():  # eval mode WITHOUT Module.eval(), whose override clears the caches:
        mod.training = False  # only graph_step's own clearing can make the forward refold
    with torch.no_grad():
        second = m(l, r)[0].clone()
    fresh = _model(19)
    fresh.load_state_dict(m.state_dict())
    fresh.eval()
    with torch.no_grad():
        ref = fresh(l, r)[0]
    assert not torch.equal(first, second)  # the second replay moved the weights
    assert (second - ref).abs().max().item() <= 1e-4, (second - ref).abs().max().item()
