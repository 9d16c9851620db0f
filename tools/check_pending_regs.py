"""Audit of the hand-waited kernels (conv_s2.hip): in the device assembly, no instruction may read
the destination VGPR of an inline-asm buffer load before the next s_waitcnt vmcnt (the compiler
does not know those loads are pending).  usage: python tools/check_pending_regs.py file.s"""
import re
import sys

src = open(sys.argv[1]).read()
bad = 0
for m in re.finditer(r'^(_Z\S*conv3x3s2_kernel\S*):\n', src, re.M):
    body = src[m.end():src.index('.Lfunc_end', m.end())].split('\n')
    pending = set()
    inasm = False
    for ln in body:
        l = ln.strip()
        if l.startswith(';;#ASMSTART'):
            inasm = True
            continue
        if l.startswith(';;#ASMEND'):
            inasm = False
            continue
        if l.startswith('s_waitcnt') and 'vmcnt' in l:
            pending.clear()
            continue
        d = re.match(r'buffer_load_dword (v\d+), ', l)
        if d and inasm:
            pending.add(d.group(1))
            continue
        if not pending or l.startswith(';') or not l:
            continue
        regs = set(re.findall(r'\bv(\d+)\b', l))
        ranges = re.findall(r'v\[(\d+):(\d+)\]', l)
        for a, b in ranges:
            regs.update(str(r) for r in range(int(a), int(b) + 1))
        hit = {'v' + r for r in regs} & pending
        if hit:
            bad += 1
            print(m.group(1)[:60], 'reads pending', sorted(hit), ':', l)
print('violations:', bad)
sys.exit(1 if bad else 0)
