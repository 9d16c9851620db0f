"""Audit of the hand-waited kernels (conv_s2.hip): in the device assembly, no instruction may read
the destination VGPRs of an inline-asm buffer load before an s_waitcnt vmcnt(N) has retired that
load (vmcnt counts vector-memory ops in issue order: vmcnt(N) retires all but the N youngest; the
compiler does not know the inline-asm loads are pending).  usage: python tools/check_pending_regs.py file.s"""
import re
import sys

src = open(sys.argv[1]).read()
bad = 0
VMEM = re.compile(r'^(buffer_load|buffer_store|global_load|global_store|scratch_load|scratch_store|'
                  r'buffer_atomic|global_atomic)')
for m in re.finditer(r'^(_Z\S*conv3x3(?:s2_(?:rows_)?|_g3_)kernel\S*):\n', src, re.M):
    body = src[m.end():src.index('.Lfunc_end', m.end())].split('\n')
    ops = []  # in issue order: set of pending destination registers (empty for untracked ops)
    inasm = False
    for ln in body:
        l = ln.strip()
        if l.startswith(';;#ASMSTART'):
            inasm = True
            continue
        if l.startswith(';;#ASMEND'):
            inasm = False
            continue
        w = re.match(r's_waitcnt.*vmcnt\((\d+)\)', l)
        if w:
            n = int(w.group(1))
            ops = ops[len(ops) - n:] if n else []
            continue
        if VMEM.match(l):
            dst = set()
            d = re.match(r'buffer_load_dword\w* (v\d+|v\[(\d+):(\d+)\]), ', l)
            if d and inasm:
                if d.group(2):
                    dst = {'v%d' % r for r in range(int(d.group(2)), int(d.group(3)) + 1)}
                else:
                    dst = {d.group(1)}
            ops.append(dst)
            if dst:
                continue
        pending = set().union(*ops) if ops else set()
        if not pending or l.startswith(';') or not l:
            continue
        regs = set(re.findall(r'\bv(\d+)\b', l))
        for a, b in re.findall(r'v\[(\d+):(\d+)\]', l):
            regs.update(str(r) for r in range(int(a), int(b) + 1))
        hit = {'v' + r for r in regs} & pending
        if hit:
            bad += 1
            print(m.group(1)[:70], 'reads pending', sorted(hit), ':', l)
print('violations:', bad)
sys.exit(1 if bad else 0)
