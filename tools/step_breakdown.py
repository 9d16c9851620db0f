"""Per-step kernel breakdown of the bench step from a rocprofv3 kernel trace (tools/gpu_r05t.sh).
Steps are delimited by the marker kernel (one launch per step: the first of the scale-0 tail
post-stage launches); over the last N complete steps: wall time per step, busy time (sum of kernel
durations; > wall where side streams overlap), and per-kernel launches / time per step.
Usage: python tools/step_breakdown.py TRACE.csv [N]"""
import collections
import csv
import sys

path = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
mark = "dcn_tile_kernel<2, 32, true"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
per = 1  # one post-stage tail launch per step (the last fusion's scale-0 tail: final_conv + regression)
starts = idx[::per]
sel_steps = starts[-(N + 1):]  # N complete steps between N+1 markers
t0, t1 = int(rows[sel_steps[0]]["Start_Timestamp"]), int(rows[sel_steps[-1]]["Start_Timestamp"])
sel = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in sel:
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
print(f"# {N} steps: {(t1 - t0) / 1e6 / N:.3f} ms/step wall in the trace, {busy / N / 1e3:.3f} ms/step of "
      f"kernel time, {len(sel) / N:.0f} launches/step")
print(f"{'per step':>8s} {'avg_us':>8s} {'us/step':>8s} {'share':>6s}  kernel")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{v[0] / N:8.1f} {v[1] / v[0]:8.1f} {v[1] / N:8.1f} {v[1] / busy:6.1%}  {k[:100]}")
