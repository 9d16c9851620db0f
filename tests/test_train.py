"""CPU tests of the training-side host logic (aanet_amd/train.py): pyramid loss (model.py:97-134),
offset_conv parameter groups (train.py:199-215), accumulation with no_sync (model.py:82-153) and
the DDP wrapping over gloo with world size 2.  The path's modules are GPU-only, so the CPU tests
drive the Trainer with a small stand-in module that has the same call signature (left, right
feature lists -> coarse-to-fine disparity pyramid) and an `offset_conv` child."""
import copy
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn as nn
import torch.nn.functional as F

from aanet_amd import nets, train


class TinyPath(nn.Module):
    def __init__(self):
        super().__init__()
        self.offset_conv = nn.Conv2d(4, 4, 3, padding=1)
        self.head = nn.Conv2d(4, 1, 1)

    def forward(self, left, right):
        out = []
        for lf, rf in zip(reversed(left), reversed(right)):   # coarse to fine
            out.append(F.softplus(self.head(torch.relu(self.offset_conv(lf - rf)))).squeeze(1))
        return out


def _features(B, seed=0):
    g = torch.Generator().manual_seed(seed)
    sizes = [(16, 32), (8, 16), (4, 8)]
    left = [torch.randn(B, 4, h, w, generator=g) for h, w in sizes]
    right = [torch.randn(B, 4, h, w, generator=g) for h, w in sizes]
    gt = torch.rand(B, 32, 64, generator=g) * 8 + 0.5
    return left, right, gt


def test_pyramid_weights_follow_reference():
    assert train.pyramid_weights(5) == [1 / 3, 2 / 3, 1.0, 1.0, 1.0]
    assert train.pyramid_weights(4) == [1 / 3, 2 / 3, 1.0, 1.0]
    assert train.pyramid_weights(3) == [1.0, 1.0, 1.0]
    assert train.pyramid_weights(1) == [1.0]
    assert train.pyramid_weights(3, highest_loss_only=True) == [1.0]
    with pytest.raises(NotImplementedError):
        train.pyramid_weights(2)


def test_disparity_loss_upsamples_and_scales():
    torch.manual_seed(0)
    gt = torch.rand(2, 8, 16) * 10
    mask = gt > 1
    # a half-resolution prediction that is exactly gt/2 on a constant field upsamples to gt
    const = torch.full((2, 4, 8), 3.0)
    total, per = train.disparity_loss([const], torch.full((2, 8, 16), 6.0),
                                      torch.ones(2, 8, 16, dtype=torch.bool), [1.0])
    assert float(total) == 0.0 and len(per) == 1
    # hand restatement of model.py:109-124 for a two-level pyramid
    p0, p1 = torch.rand(2, 4, 8) * 5, torch.rand(2, 8, 16) * 10
    up = F.interpolate(p0.unsqueeze(1), size=(8, 16), mode="bilinear",
                       align_corners=False).squeeze(1) * 2
    want = 0.5 * F.smooth_l1_loss(up[mask], gt[mask]) + 1.0 * F.smooth_l1_loss(p1[mask], gt[mask])
    got, per = train.disparity_loss([p0, p1], gt, mask, [0.5, 1.0])
    assert torch.allclose(got, want)
    assert len(per) == 2
    with pytest.raises(ValueError):
        train.disparity_loss([p0, p1], gt, mask, [1.0])
    # non-finite ground truth outside the mask does not leak into the loss or its gradient
    gt_bad = torch.where(mask, gt, torch.full_like(gt, float("inf")))
    gt_bad[0, 0, 0] = float("nan") if not mask[0, 0, 0] else gt_bad[0, 0, 0]
    p1g = p1.clone().requires_grad_()
    bad, _ = train.disparity_loss([p1g], gt_bad, mask, [1.0])
    bad.backward()
    assert torch.allclose(bad, F.smooth_l1_loss(p1[mask], gt[mask]))
    assert torch.isfinite(p1g.grad).all()
    # pseudo ground truth adds a second weighted term over its own mask
    got2, _ = train.disparity_loss([p1], gt, mask, [1.0], pseudo_gt=gt * 0, pseudo_mask=mask)
    assert torch.allclose(got2, F.smooth_l1_loss(p1[mask], gt[mask])
                          + F.smooth_l1_loss(p1[mask], gt[mask] * 0))


def test_param_groups_offset_conv_at_tenth_lr():
    m = TinyPath()
    groups = train.param_groups(m, 1e-3)
    assert groups[0]["lr"] == 1e-3 and groups[1]["lr"] == pytest.approx(1e-4)
    spec = {id(p) for p in groups[1]["params"]}
    assert spec == {id(m.offset_conv.weight), id(m.offset_conv.bias)}
    assert len(groups[0]["params"]) + len(groups[1]["params"]) == len(list(m.parameters()))


def test_accumulation_steps_match_one_big_batch():
    """Two micro-batches with accumulation_steps=2 take one optimizer step on the mean of the two
    micro-batch losses (model.py:136, 151)."""
    torch.manual_seed(1)
    m = TinyPath()
    ref = copy.deepcopy(m)
    t = train.Trainer(m, lr=1e-2, accumulation_steps=2)
    l, r, gt = _features(4)
    halves = [([x[:2] for x in l], [x[:2] for x in r], gt[:2]),
              ([x[2:] for x in l], [x[2:] for x in r], gt[2:])]
    before = [p.detach().clone() for p in m.parameters()]
    t.step(*halves[0])
    assert all(torch.equal(a, b) for a, b in zip(before, m.parameters()))  # no step yet
    t.step(*halves[1])
    assert not all(torch.equal(a, b) for a, b in zip(before, m.parameters()))

    opt = torch.optim.Adam(train.param_groups(ref, 1e-2), weight_decay=1e-4)
    loss = 0
    for lh, rh, gh in halves:
        tot, _ = train.disparity_loss(ref(lh, rh), gh, gh > 0)
        loss = loss + tot / 2
    loss.backward()
    opt.step()
    for a, b in zip(m.parameters(), ref.parameters()):
        assert torch.allclose(a, b, atol=1e-6)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _ddp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(3)
    m = TinyPath()
    ref = copy.deepcopy(m)
    ddp = train.wrap_data_parallel(m, torch.device("cpu"), sync_bn=False)
    assert isinstance(ddp, nn.parallel.DistributedDataParallel)
    t = train.Trainer(ddp, lr=1e-2, accumulation_steps=2)
    # 2 micro-batches per rank, 2 samples each; rank r owns samples [4r, 4r+4)
    l, r, gt = _features(4 * world, seed=7)
    mine = lambda x, k: x[4 * rank + 2 * k: 4 * rank + 2 * k + 2]
    for k in range(2):
        t.step([mine(x, k) for x in l], [mine(x, k) for x in r], mine(gt, k))
    # reference: one process, mean over ranks of each rank's accumulated gradient
    opt = torch.optim.Adam(train.param_groups(ref, 1e-2), weight_decay=1e-4)
    loss = 0
    for rr in range(world):
        for k in range(2):
            sl = slice(4 * rr + 2 * k, 4 * rr + 2 * k + 2)
            tot, _ = train.disparity_loss(ref([x[sl] for x in l], [x[sl] for x in r]), gt[sl],
                                          gt[sl] > 0)
            loss = loss + tot / 2 / world
    loss.backward()
    opt.step()
    err = max(float((a - b).abs().max()) for a, b in zip(m.parameters(), ref.parameters()))
    gathered = [torch.zeros(1) for _ in range(world)]
    dist.all_gather(gathered, torch.tensor([float(sum(p.sum() for p in m.parameters()))]))
    if rank == 0:
        q.put((err, [float(g) for g in gathered]))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_accumulation_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    err, sums = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert err <= 1e-6, err
    assert sums[0] == sums[1]          # replicas stay identical after the synced step


def test_wrap_is_identity_without_process_group():
    m = TinyPath()
    assert train.wrap_data_parallel(m, torch.device("cpu")) is m


def test_default_mask_is_bounded_by_max_disp():
    """model.py:71: mask = (gt > 0) & (gt < max_disp) -- disparities at or past max_disp are
    excluded from the loss."""
    t = train.Trainer(TinyPath(), max_disp=8)
    gt = torch.tensor([[[0.0, 0.5, 7.9, 8.0, 9.0, -1.0]]])
    assert t.valid_mask(gt).tolist() == [[[False, True, True, False, False, False]]]


def test_all_invalid_batch_is_skipped_like_the_reference():
    """model.py:78-79: a batch without one valid pixel is skipped -- no backward, no optimizer
    step, no NaN written into the weights (a masked mean over zero pixels would be 0/0) -- but it
    still counts towards the accumulation index (enumerate's i)."""
    torch.manual_seed(3)
    m = TinyPath()
    t = train.Trainer(m, lr=1e-2, max_disp=8, accumulation_steps=2)
    l, r, _ = _features(2)
    before = [p.detach().clone() for p in m.parameters()]
    bad_gt = torch.full((2, 32, 64), 50.0)   # every pixel >= max_disp
    assert t.step(l, r, bad_gt) is None
    assert all(torch.equal(a, b) for a, b in zip(before, m.parameters()))
    assert all(p.grad is None for p in m.parameters())
    # the skipped batch was micro-step 1, so this one is the boundary and steps the optimizer
    good_gt = torch.rand(2, 32, 64) * 6 + 0.5
    loss = t.step(l, r, good_gt)
    assert loss is not None and torch.isfinite(loss)
    assert not all(torch.equal(a, b) for a, b in zip(before, m.parameters()))
    assert all(torch.isfinite(p).all() for p in m.parameters())


def test_use_engine_convs_marks_convs_and_keeps_cpu_path():
    """use_engine_convs patches every engine-eligible nn.Conv2d (the grouped dilated offset conv
    too) without changing the module tree; CPU tensors still take the reference convolution."""
    torch.manual_seed(0)
    m = nets.AANetHotPath(16, no_intermediate_supervision=False, num_deform_blocks=3)
    keys = set(m.state_dict())
    n = train.use_engine_convs(m)
    convs = [c for c in m.modules() if isinstance(c, torch.nn.Conv2d)]
    assert n == len(convs) > 20 and all(getattr(c, "_aanet_engine", False) for c in convs)
    assert set(m.state_dict()) == keys
    assert train.use_engine_convs(m) == 0  # idempotent
    conv = convs[0]
    x = torch.randn(1, conv.in_channels, 9, 11)
    ref = torch.nn.functional.conv2d(x, conv.weight, conv.bias, conv.stride, conv.padding,
                                     conv.dilation, conv.groups)
    assert torch.equal(conv(x), ref)


def test_engine_convs_model_pickles(tmp_path):
    """a whole-model torch.save of a model with engine convs loads back (the engine
    conv is a module-level nn.Conv2d subclass, not a bound method in the instance dict)."""
    torch.manual_seed(0)
    m = nets.AANetHotPath(16, no_intermediate_supervision=False, num_deform_blocks=3)
    assert train.use_engine_convs(m) > 20
    path = tmp_path / "whole.pt"
    torch.save(m, path)
    m2 = torch.load(path, weights_only=False)  # a file this test wrote itself
    convs = [c for c in m2.modules() if isinstance(c, torch.nn.Conv2d)]
    assert all(isinstance(c, train.EngineConv2d) for c in convs)
    for (k, a), (k2, b) in zip(m.state_dict().items(), m2.state_dict().items()):
        assert k == k2 and torch.equal(a, b)
    x = torch.randn(1, convs[0].in_channels, 9, 11)
    assert torch.equal(convs[0](x), torch.nn.functional.conv2d(
        x, convs[0].weight, convs[0].bias, convs[0].stride, convs[0].padding, convs[0].dilation,
        convs[0].groups))
