"""Summarise tools/c4_sweep.sh into profiles/<tag>_c4_dcn_sweep.txt: the sweep's JSON lines plus,
per DCN kernel (forward / backward data / backward weight / deterministic helpers), the rocprof
average duration, MFMA and VALU instructions per wave, MFMA-busy fraction and HBM bytes per
launch (FETCH_SIZE x2, gfx950 correction, + WRITE_SIZE).  Usage: python tools/c4_summary.py
gpurun_out/c4 r02"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

src, tag = sys.argv[1], sys.argv[2]
dst = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                   f"{tag}_c4_dcn_sweep.txt")
lines = [f"# SURVEY C4 sweep ({tag}): bench.py --dcn-sweep (B=8, dg=2, 3x3, dil 2, offsets N(0,0.5^2))", ""]
for l in open(os.path.join(src, "sweep.jsonl")):
    l = l.strip()
    if l.startswith("{"):
        d = json.loads(l)
        if "shape" in d:
            lines.append(f"{d['shape']:8s} in {d['input']} s{d['stride']}: fwd {d['fwd_us']:8.1f} us "
                         f"({d['fwd_tflops']:5.1f} TF/s, {d['fwd_frac_f32_mfma']:.2f} of f32 MFMA"
                         f"{', window' if d.get('fwd_window') else ''}; generic {d.get('fwd_generic_us', 0):.1f} us)  "
                         f"bwd {d['bwd_us']:8.1f} us  bwd det {d['bwd_det_us']:8.1f} us")
        else:
            lines.append(f"num_scales {d['num_scales']}: fwd {d['fwd_us']:.1f} us, fwd+bwd {d['fwd_bwd_us']:.1f} us")
stats = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
lines += ["", "# rocprofv3 --kernel-trace --stats (whole sweep, every shape and entry point)",
          f"{'calls':>6} {'avg_us':>9} {'total_ms':>9}  kernel"]
for r in sorted(csv.DictReader(open(stats[0])), key=lambda r: -float(r["TotalDurationNs"]))[:25]:
    nm = re.sub(r"\(anonymous namespace\)::", "", r["Name"])[:100]
    lines.append(f"{int(r['Calls']):6d} {float(r['AverageNs']) / 1e3:9.1f} {float(r['TotalDurationNs']) / 1e6:9.3f}  {nm}")
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(src, "pmc*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        nm = re.sub(r"\(anonymous namespace\)::", "", r["Kernel_Name"]).split("(")[0][:60]
        if "mdcn" not in nm and "conv_fwd" not in nm and "det_" not in nm and "nhwc" not in nm and "weight" not in nm:
            continue
        key = f"{nm} grid {r.get('Grid_Size', '?')}"
        vals[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
lines += ["", "# PMC per kernel launch shape (averages): MFMA/VALU instructions per wave, MFMA busy / "
          "busy cycles, HBM bytes per launch (FETCH x2 + WRITE)"]
for k, d in sorted(vals.items()):
    a = {c: sum(v) / len(v) for c, v in d.items()}
    w = a.get("SQ_WAVES") or 1.0
    busy = a.get("SQ_BUSY_CYCLES") or 0.0
    hbm = a.get("FETCH_SIZE", 0.0) * 2048 + a.get("WRITE_SIZE", 0.0) * 1024
    mf = a.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    lines.append(f"{k:70s} mfma/wave {a.get('SQ_INSTS_MFMA', 0) / w:7.1f}  valu/wave {a.get('SQ_INSTS_VALU', 0) / w:8.1f}  "
                 f"mfma_busy_cycles {mf:12.0f}  hbm {hbm / 1e6:8.1f} MB")
open(dst, "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
