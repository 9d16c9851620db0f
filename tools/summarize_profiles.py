"""Summarise a collect_profiles.sh run into profiles/ (tracked): kernel stats of the bench
command, per-launch HBM traffic of the roofline kernels from the PMC passes (gfx950
correction: FETCH_SIZE counts half the bytes of wide coalesced reads -> doubled, per
MI355X_MICROARCH.md §HBM), and SQ counter ratios."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

src = sys.argv[1]
tag = sys.argv[2]
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles")
os.makedirs(dst, exist_ok=True)

# bench.py kernel_rooflines keys -> kernel names
KMAP = {"corr_volume_s0": r"corr_reg_kernel<5, 8, 2>", "disp_regress_s0": r"disp_regress_fixed_kernel<64>",
        "corr_pyramid": r"corr_pyramid_reg_kernel",
        # the streaming 1x1 conv (pointwise.hip, input split once), NCHW input, 4 output-channel blocks, NHWC out
        "conv1x1_s0": r"pw_conv_nchw_s_kernel<64, 4, 1>",
        # the LDS-window deformable tail (dcn_tile.hip), common form (no post stage)
        "mdcn_pw_s0": r"dcn_tile_kernel<2, 32, false, false, false>",
        # MODE, CO_T, PTT, PACKED, TAIL, SCHED, FULL, LAYOUT, CFG, PREC (1: split-bf16), HALO (= dil),
        # POST (0: no post stage)
        "conv3x3_pw_s0": r"conv_fwd_kernel<0, 64, 128, 1, 1, 1, 1, 1, 0, 1, 1, 0>",
        # the scale-0 offset_conv (conv_g3.hip halo kernel: G=2 groups in one WG, NCC=1, NCB=2, dil 2)
        "offset_conv_s0": r"conv3x3_g3_kernel<2, 1, 2, 2>",
        # the scale-0 heads launch of the CSA exchange (conv_s2.hip row form, 6 co blocks, 2 chunks)
        "s2_heads_s0": r"conv3x3s2_rows_kernel<6, 2>",
        # the C5 concat volume (shift_volume_band_kernel, concat form)
        "concat_volume_c5": r"shift_volume_band_kernel<true>"}

# 1. kernel stats of the bench command
stats = list(csv.DictReader(open(os.path.join(src, "trace", "bench_kernel_stats.csv"))))
tot = sum(float(r["TotalDurationNs"]) for r in stats)
lines = [f"# rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline ({tag})",
         f"# total GPU kernel time {tot / 1e6:.3f} ms over the whole run (warmup, graph capture, timed steps, roofline loops)",
         f"{'total_ms':>10} {'calls':>6} {'avg_us':>9} {'pct':>6}  kernel"]
for r in sorted(stats, key=lambda r: -float(r["TotalDurationNs"])):
    name = re.sub(r"\(anonymous namespace\)::", "", r["Name"])[:110]
    lines.append(f"{float(r['TotalDurationNs']) / 1e6:10.3f} {int(r['Calls']):6d} "
                 f"{float(r['AverageNs']) / 1e3:9.1f} {100 * float(r['TotalDurationNs']) / tot:6.2f}  {name}")
open(os.path.join(dst, f"{tag}_bench_kernel_stats.txt"), "w").write("\n".join(lines) + "\n")

# 2. PMC passes
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        for key, pat in KMAP.items():
            if re.search(re.escape(pat), r["Kernel_Name"]):
                vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
traffic, report = {}, {}
for key, d in vals.items():
    avg = {c: sum(v) / len(v) for c, v in d.items()}
    fetch = avg.get("FETCH_SIZE", 0.0) * 1024 * 2   # KB -> B, x2 gfx950 read correction
    write = avg.get("WRITE_SIZE", 0.0) * 1024
    traffic[key] = fetch + write
    rep = {"fetch_bytes_corrected": fetch, "write_bytes": write, "fetch_size_raw_kb": avg.get("FETCH_SIZE"),
           "write_size_raw_kb": avg.get("WRITE_SIZE"), "launches_sampled": len(d.get("FETCH_SIZE", []))}
    wc = avg.get("SQ_WAVE_CYCLES")
    if wc:
        for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if c in avg:
                rep[c + "_frac"] = avg[c] / wc
    waves = avg.get("SQ_WAVES")
    if waves:
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_LDS_BANK_CONFLICT"):
            if c in avg:
                rep[c + "_per_wave"] = avg[c] / waves
    if "TCC_HIT_sum" in avg:
        rep["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    report[key] = rep
json.dump(traffic, open(os.path.join(dst, "pmc_traffic.json"), "w"), indent=1)
json.dump(report, open(os.path.join(dst, f"{tag}_pmc_report.json"), "w"), indent=1)
print(json.dumps(report, indent=1))
