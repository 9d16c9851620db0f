"""Per-step kernel breakdown of the timed training steps from a rocprofv3 kernel trace
(tools/gpu_r05l.sh): kernels that start in the last `steps` x `ms` milliseconds of the trace,
grouped by name; launches and time per step.  Usage:
python tools/train_breakdown.py gpurun_out/train_prof/tr_kernel_trace.csv [steps] [ms_per_step]"""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ms = float(sys.argv[3]) if len(sys.argv) > 3 else 20.5
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
end = int(rows[-1]["End_Timestamp"])
sel = [r for r in rows if int(r["Start_Timestamp"]) >= end - steps * ms * 1e6]
agg = collections.defaultdict(lambda: [0, 0.0])
for r in sel:
    a = agg[r["Kernel_Name"]]
    a[0] += 1
    a[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
print(f"# last {steps} steps ({(end - int(sel[0]['Start_Timestamp'])) / 1e6 / steps:.2f} ms/step wall in the trace): "
      f"{len(sel) / steps:.0f} kernels/step, {busy / steps / 1e3:.2f} ms/step busy")
print(f"{'per step':>8s} {'avg_us':>8s} {'ms/step':>8s} {'share':>6s}  kernel")
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])[:30]:
    print(f"{v[0] / steps:8.1f} {v[1] / v[0]:8.1f} {v[1] / steps / 1e3:8.3f} {v[1] / busy:6.1%}  {k[:110]}")
