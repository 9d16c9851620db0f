"""Per-basic-block instruction census of one kernel in a hipcc --save-temps .s file: VALU / MFMA /
SALU / DS / VMEM / branch counts per block, loop depth and the scratch (spill) accesses, so a
kernel's main loop and epilogue can be compared build to build without a GPU.
Usage: python tools/isa_blocks.py <file.s> <kernel-name-substring> [--min N]"""
import re
import sys


def main():
    path, key = sys.argv[1], sys.argv[2]
    minn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 8
    text = open(path).read().split("\n")
    start = None
    for i, l in enumerate(text):
        if re.match(r"^_Z\S*:", l) and key in l.split(":")[0]:
            start = i
            break
    if start is None:
        raise SystemExit("kernel not found")
    end = len(text)
    for i in range(start + 1, len(text)):
        if re.match(r"^_Z\S*:", text[i]) or text[i].startswith("\t.size"):
            end = i
            break
    blocks, cur, depth = [], ["entry", {}, 0, start], 0
    tot = {}
    for i in range(start + 1, end):
        l = text[i]
        m = re.match(r"^(\.LBB\S+):(.*)", l)
        if m:
            blocks.append(cur)
            dm = re.search(r"Depth=(\d+)", m.group(2))
            cur = [m.group(1), {}, int(dm.group(1)) if dm else 0, i]
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        if "mfma" in op:
            cat = "mfma"
        elif op.startswith("scratch_"):
            cat = "scratch"
        elif op.startswith("v_"):
            cat = "valu"
        elif op.startswith(("s_cbranch", "s_branch")):
            cat = "br"
        elif op.startswith("s_waitcnt"):
            cat = "wait"
        elif op.startswith("s_"):
            cat = "salu"
        elif op.startswith("ds_"):
            cat = "ds"
        elif op.startswith(("buffer_", "global_", "flat_")):
            cat = "vmem"
        else:
            cat = "other"
        cur[1][cat] = cur[1].get(cat, 0) + 1
        tot[cat] = tot.get(cat, 0) + 1
    blocks.append(cur)
    cats = ["valu", "mfma", "salu", "ds", "vmem", "wait", "br", "scratch"]
    print(f"{'block':<12} {'line':>6} {'dep':>3} " + " ".join(f"{c:>6}" for c in cats))
    for name, c, d, ln in blocks:
        if sum(c.values()) >= minn or c.get("scratch"):
            print(f"{name:<12} {ln:>6} {d:>3} " + " ".join(f"{c.get(k, 0):>6}" for k in cats))
    print(f"{'TOTAL':<12} {'':>6} {'':>3} " + " ".join(f"{tot.get(k, 0):>6}" for k in cats))


if __name__ == "__main__":
    main()
