"""Data-parallel plumbing for the hot path: stereo pairs are independent, so
ranks share nothing on the data path; one all_gather of a small per-rank metrics record runs
at the end (RCCL over xGMI on the MI355X node, gloo in CPU tests)."""
import torch
import torch.distributed as dist

# metrics record layout (float64): pairs, elapsed_s, sum|dd|, max|dd|, n_px, disp_min, disp_max
RECORD_FIELDS = ("pairs", "elapsed_s", "sum_abs_err", "max_abs_err", "n_px", "disp_min", "disp_max")


def shard(global_batch, world, rank):
    """Contiguous B/world slice of a global batch: (start, count); the first B % world ranks get
    one extra pair."""
    base, extra = divmod(global_batch, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def make_record(device, **kw):
    vals = [float(kw.get(f, 0.0)) for f in RECORD_FIELDS]
    return torch.tensor(vals, dtype=torch.float64, device=device)


def gather_records(record):
    """all_gather of one record per rank -> [world, len(RECORD_FIELDS)] on CPU."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return record.detach().cpu().view(1, -1)
    out = [torch.empty_like(record) for _ in range(dist.get_world_size())]
    dist.all_gather(out, record)
    return torch.stack(out).cpu()


def summarize(records):
    """Whole-job numbers: total pairs / max elapsed over ranks (the bench's clock)."""
    r = records.double()
    pairs, t_max = float(r[:, 0].sum()), float(r[:, 1].max())
    n_px = float(r[:, 4].sum())
    return {"pairs": pairs, "elapsed_max_s": t_max, "pairs_per_s": pairs / t_max if t_max > 0 else 0.0,
            "epe": float(r[:, 2].sum()) / n_px if n_px > 0 else None,
            "max_abs_err": float(r[:, 3].max()), "disp_min": float(r[:, 5].min()),
            "disp_max": float(r[:, 6].max())}
