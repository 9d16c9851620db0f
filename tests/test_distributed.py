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


def test_bench_self_launch_two_ranks_gloo():
    """`bench.py --gpus 2` with no external launcher starts its own 2 rank processes (the path the
    GPU run takes when WORLD_SIZE is unset), gathers one record per rank and reports whole-job
    pairs over the MAX elapsed over ranks -- exercised with the --plumbing stand-in step on CPU."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    res = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2",
                          "--plumbing", "--steps", "3", "--warmup", "1", "--batch", "4"],
                         env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 0, res.stderr[-2000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout  # rank 0 prints ONE line
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2
    assert len(line["per_rank"]) == 2
    assert line["pairs"] == 2 * 4 * 3 == sum(r["pairs"] for r in line["per_rank"])
    assert line["elapsed_max_s"] == max(r["elapsed_s"] for r in line["per_rank"])
    assert line["value"] == pytest.approx(line["pairs"] / line["elapsed_max_s"])
    assert line["max_abs_disp_err_vs_ref"] == pytest.approx(2e-6)  # max over ranks


def test_bench_self_launch_propagates_rank_failure():
    """A failing rank makes the launcher exit non-zero (and the other rank is not left hanging)."""
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    env["AANET_PLUMBING_FAIL_RANK"] = "1"  # rank 1 exits; rank 0 would wait in all_gather
    res = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--gpus", "2",
                          "--plumbing", "--steps", "2", "--warmup", "0"],
                         env=env, capture_output=True, text=True, timeout=240)
    assert res.returncode == 3
    assert not [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
