"""Per-forward kernel breakdown of a rocprofv3 kernel-trace database (the rocpd SQLite file
rocprofv3 writes by default) of `tools/full_model_stages.py`.

The profiled run holds the reference-order FLOP-count pass (MIOpen find, fp64 naive convs) and
then the fused forwards.  Dispatches are split into segments at host gaps > --gap ms; the LAST
segment is the timed fused forwards.  Per-forward figures divide by --forwards (default: the
count of the first kernel name given by --marker, divided by --per-forward).

Usage: python tools/prof_db_breakdown.py DB [--forwards N] [--top K] [--gap MS]
"""
import argparse
import collections
import sqlite3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--forwards", type=float, default=5.0)
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--gap", type=float, default=2.0)
    args = ap.parse_args()
    c = sqlite3.connect(args.db)
    rows = c.execute("select start, end, name, grid_x, grid_y from kernels order by start").fetchall()
    segs = [[rows[0]]]
    for r in rows[1:]:
        if r[0] - segs[-1][-1][1] > args.gap * 1e6:
            segs.append([])
        segs[-1].append(r)
    s = segs[-1]
    cnt, tm = collections.Counter(), collections.Counter()
    for a, b, n, _, _ in s:
        cnt[n] += 1
        tm[n] += b - a
    nf = args.forwards
    print(f"# last segment: {len(s)} dispatches, {sum(tm.values()) / 1e6 / nf:.3f} ms kernel time "
          f"per forward ({nf:g} forwards)")
    for n, t in tm.most_common(args.top):
        print(f"{t / 1e3 / nf:9.1f} us/fwd {cnt[n] / nf:6.1f}x {t / 1e3 / cnt[n]:8.1f} us  {n[:110]}")


if __name__ == "__main__":
    main()
