"""One bench step as a timeline, from a rocprofv3 kernel trace (tools/profile_step.sh; HIP graph or
eager).  Steps are delimited like tools/step_breakdown.py (the last fusion's scale-0 tail, one
launch per step).  For the median-length step of the last N it prints every kernel: start offset,
duration, queue, workgroups, a short name; then the intervals in which exactly ONE kernel runs
(the serial stretches of the schedule) grouped by kernel, and the idle gaps.

Usage: python tools/step_timeline.py TRACE_kernel_trace.csv [N] [MARK]
(MARK: the kernel-name substring that delimits steps; default the last tail's post-stage form,
"corr_pyramid" for schedules without it)"""
import collections
import csv
import re
import sys

path = sys.argv[1]
N = int(sys.argv[2]) if len(sys.argv) > 2 else 10
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
mark = sys.argv[3] if len(sys.argv) > 3 else "dcn_tile_kernel<2, 32, true"
idx = [i for i, r in enumerate(rows) if mark in r["Kernel_Name"]]
# consecutive marks at least 1 ms apart delimit whole steps (not a kernel-only timing loop)
gaps = [(idx[k], idx[k + 1]) for k in range(len(idx) - 1)
        if int(rows[idx[k + 1]]["Start_Timestamp"]) - int(rows[idx[k]]["Start_Timestamp"]) > 1_000_000]
steps = gaps[-N:]
lens = [int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"]) for a, b in steps]
order = sorted(range(len(steps)), key=lambda k: lens[k])
a, b = steps[order[len(order) // 2]]
t0 = int(rows[a]["Start_Timestamp"])
t1 = int(rows[b]["Start_Timestamp"])


def short(name):
    n = re.sub(r"\(anonymous namespace\)::", "", name)
    n = re.sub(r"^void ", "", n)
    return n.split("(")[0][:58]


def wgs(r):
    try:
        g = [int(r.get(k, 0) or 0) for k in ("Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z")]
        w = [max(1, int(r.get(k, 1) or 1)) for k in ("Workgroup_Size_X", "Workgroup_Size_Y",
                                                     "Workgroup_Size_Z")]
        n = 1
        for gi, wi in zip(g, w):
            n *= max(1, gi // wi)
        return n
    except ValueError:
        return -1


sel = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
print(f"# median of {len(steps)} steps: {(t1 - t0) / 1e3:.1f} us, {len(sel)} launches")
print(f"{'start':>7s} {'dur':>6s} {'q':>3s} {'wgs':>6s}  kernel")
ev = []
for r in sel:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    ev.append((s, e, short(r["Kernel_Name"])))
    q = r.get("Queue_Id", r.get("Stream_Id", "?"))
    print(f"{s / 1e3:7.1f} {(e - s) / 1e3:6.1f} {q:>3s} {wgs(r):6d}  {short(r['Kernel_Name'])}")

# sweep: intervals with exactly one kernel running, and idle gaps
pts = sorted([(s, 1, n) for s, e, n in ev] + [(e, -1, n) for s, e, n in ev])
run = collections.Counter()
alone = collections.defaultdict(float)
idle = 0.0
prev = 0
for t, d, n in pts:
    t = min(max(t, 0), t1 - t0)
    active = [k for k, v in run.items() if v > 0]
    dt = (t - prev) / 1e3
    if len(active) == 1:
        alone[active[0]] += dt
    elif not active:
        idle += dt
    run[n] += d
    prev = t
print(f"\n# serial stretches (exactly one kernel on the GPU) per step: "
      f"{sum(alone.values()):.1f} us; idle {idle:.1f} us")
for k, v in sorted(alone.items(), key=lambda kv: -kv[1]):
    print(f"{v:8.1f} us  {k}")
