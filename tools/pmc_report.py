"""Aggregate rocprofv3 --pmc passes (tools/pmc.sh output) per kernel: mean counter value per
dispatch, for kernels whose name contains one of the given substrings.
Usage: python tools/pmc_report.py gpurun_out/<PMC_NAME> [substr ...]"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict

root = sys.argv[1]
subs = sys.argv[2:] or [""]
vals = defaultdict(lambda: defaultdict(list))
files = sorted(glob.glob(os.path.join(root, "pass*", "**", "*counter_collection.csv"), recursive=True)) or \
    sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True))
for f in files:
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        key = next((s for s in subs if s in name), None)
        if key is None:
            continue
        m = re.search(r"(\w+<[^>]*>|\w+)\(", name.replace("(anonymous namespace)::", ""))
        kname = (m.group(1) if m else name[:60]) + f" g{r.get('Grid_Size', '')}"
        vals[kname][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in vals.items():
    print(k)
    for c, v in sorted(d.items()):
        print(f"   {c:34s} {sum(v) / len(v):16.1f}  (n={len(v)})")
