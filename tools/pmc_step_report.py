"""Per-kernel summary of two rocprofv3 --pmc passes over the step (tools/pmc.sh, serial schedule):
MFMA-pipe busy fraction of the kernel's wall time, wave-time split (parked on s_waitcnt/barrier,
issue-stalled, issuing), VALU and MFMA instructions per wave, LDS bank-conflict fraction.
usage: python tools/pmc_step_report.py gpurun_out/pmc_step"""
import collections
import csv
import sys

d = sys.argv[1]


def load(p):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in csv.DictReader(open(f"{d}/{p}/run_counter_collection.csv")):
        n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")
        n = n[:n.find("(")] if "(" in n else n
        key = (n[:60], r["Grid_Size"])
        per[key][r["Counter_Name"]] += float(r["Counter_Value"])
        per[key]["_wg"] = float(r["Workgroup_Size"])
        cnt[(key, r["Counter_Name"])] += 1
    out = {}
    for k, v in per.items():
        out[k] = {c: (x / cnt[(k, c)] if c[0] != "_" else x) for c, x in v.items()}
    return out


a, b = load("pass1"), load("pass2")
rows = []
for k in a:
    if k not in b:
        continue
    v = {**a[k], **b[k]}
    grbm = v.get("GRBM_GUI_ACTIVE", 0) / 8  # 8 XCDs
    if grbm <= 0:
        continue
    waves = float(k[1]) / 64
    wc = v["SQ_WAVE_CYCLES"]
    rows.append((grbm, k, v["SQ_VALU_MFMA_BUSY_CYCLES"] / (grbm * 1024),
                 v["SQ_WAIT_ANY"] / wc, v["SQ_WAIT_INST_ANY"] / wc, v["SQ_ACTIVE_INST_ANY"] / wc,
                 v["SQ_INSTS_VALU"] / waves, v["SQ_INSTS_MFMA"] / waves,
                 v["SQ_LDS_BANK_CONFLICT"] / max(v["SQ_LDS_IDX_ACTIVE"], 1)))
rows.sort(reverse=True)
print(f"{'kernel':62s} {'kcyc':>7s} {'mfma%':>6s} {'park%':>6s} {'stall%':>6s} {'issue%':>6s} {'valu/w':>7s} {'mfma/w':>7s} {'ldsconf':>7s}")
for grbm, k, mf, wa, wi, ac, va, mm, lc in rows[:25]:
    print(f"{k[0]:62s} {grbm/1e3:7.1f} {100*mf:6.1f} {100*wa:6.1f} {100*wi:6.1f} {100*ac:6.1f} {va:7.0f} {mm:7.0f} {lc:7.3f}")
