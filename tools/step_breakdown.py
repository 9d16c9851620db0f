"""Summarise one steady-state step of a rocprofv3 kernel trace (per-launch durations)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_step/run_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# a step starts with the scale-0 correlation launch followed by the scale-1 one
idx = [i for i, r in enumerate(rows[:-1]) if 'corr_volume_kernel<5' in r['Kernel_Name']
       and 'corr_volume_kernel<3' in rows[i + 1]['Kernel_Name']]
a, b = idx[-2], idx[-1]
seg = rows[a:b]
t0 = int(seg[0]['Start_Timestamp'])
t1 = int(rows[b]['Start_Timestamp'])
print(f"step wall {(t1 - t0) / 1e6:.3f} ms, {len(seg)} kernels")
agg = defaultdict(lambda: [0, 0.0])
for r in seg:
    d = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    name = r['Kernel_Name'].replace('void ', '').replace('(anonymous namespace)::', '').split('(')[0]
    key = f"{name[:48]} g{r['Grid_Size_X']}x{r['Grid_Size_Y']}"
    agg[key][0] += 1
    agg[key][1] += d
    if '-v' in sys.argv:
        print(f"  {d:8.1f} us  {key}  vgpr {r['VGPR_Count']} lds {r['LDS_Block_Size']}")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t / 1e3:8.3f} ms {c:4d}  {k}")
