"""Summarise one steady-state step of a rocprofv3 kernel trace (per-launch durations)."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_step/run_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
# a step starts with the one-launch correlation pyramid
idx = [i for i, r in enumerate(rows) if 'corr_pyramid' in r['Kernel_Name']]
# the bench's roofline loops repeat single kernels after the timed steps: take the last pair of
# pyramid launches with a whole step between them
pairs = [(i, j) for i, j in zip(idx[:-1], idx[1:]) if 50 < j - i < 400]
a, b = pairs[len(pairs) // 2]  # a step from the middle of the timed run
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
        q = r.get('Stream_Id', r.get('Queue_Id', '?'))
        st = (int(r['Start_Timestamp']) - t0) / 1e3
        print(f"  {st:8.1f} {d:8.1f} us  q{q}  {key}  vgpr {r['VGPR_Count']} lds {r['LDS_Block_Size']}")
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{t / 1e3:8.3f} ms {c:4d}  {k}")
