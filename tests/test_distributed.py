"""World-size-2 gloo test (CPU) of the data-parallel plumbing bench.py uses on RCCL."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from aanet_amd import dist as adist


def test_shard_covers_batch_exactly():
    for B in (1, 7, 8, 64, 65):
        for world in (1, 2, 3, 8):
            parts = [adist.shard(B, world, r) for r in range(world)]
            assert sum(c for _, c in parts) == B
            assert [s for s, _ in parts] == sorted(s for s, _ in parts)
            for (s0, c0), (s1, _) in zip(parts, parts[1:]):
                assert s0 + c0 == s1


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    start, count = adist.shard(16, world, rank)
    # each rank "processes" its own pairs; elapsed differs per rank
    rec = adist.make_record("cpu", pairs=count, elapsed_s=1.0 + rank, sum_abs_err=0.5 * count,
                            max_abs_err=0.01 * (rank + 1), n_px=10.0 * count, disp_min=rank,
                            disp_max=10 + rank)
    recs = adist.gather_records(rec)
    summ = adist.summarize(recs)
    if rank == 0:
        q.put((start, count, recs.tolist(), summ))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_and_summarize_gloo(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    start, count, recs, summ = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert (start, count) == (0, 8)
    assert len(recs) == world
    assert summ["pairs"] == 16
    assert summ["elapsed_max_s"] == 2.0          # max over ranks, not the mean
    assert summ["pairs_per_s"] == 8.0
    assert summ["epe"] == pytest.approx(0.05)
    assert summ["max_abs_err"] == pytest.approx(0.02)
    assert summ["disp_min"] == 0 and summ["disp_max"] == 11


def test_single_process_gather_is_identity():
    rec = adist.make_record("cpu", pairs=8, elapsed_s=0.5)
    recs = adist.gather_records(rec)
    assert recs.shape == (1, len(adist.RECORD_FIELDS))
    assert adist.summarize(recs)["pairs_per_s"] == 16.0
