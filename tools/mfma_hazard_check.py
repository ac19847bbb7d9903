"""Static check on a -save-temps .s: wait states (instructions + s_nop counts) between every MFMA
and the first instruction reading one of its destination registers, within a straight window.
Usage: python tools/mfma_hazard_check.py file.s kernel_symbol"""
import re
import sys

L = open(sys.argv[1]).read().split('\n')
start = next(i for i, l in enumerate(L) if l.startswith(sys.argv[2] + ':'))
end = next(i for i in range(start, len(L)) if 's_endpgm' in L[i])
L = L[start:end]
worst = None
for i, l in enumerate(L):
    m = re.search(r'v_mfma\S* ([av])\[(\d+):(\d+)\]', l)
    if not m:
        continue
    regs = {f'{m.group(1)}{r}' for r in range(int(m.group(2)), int(m.group(3)) + 1)}
    cnt = 0
    for l2 in L[i + 1:i + 80]:
        t = l2.strip()
        if not t or t.startswith(';') or t.endswith(':'):
            continue
        if t.startswith('s_nop'):
            cnt += int(t.split()[1]) + 1
            continue
        ops = re.findall(r'([av])\[(\d+):(\d+)\]|\b([av])(\d+)\b', t)
        used = set()
        for a, lo, hi, b, n in ops:
            if a:
                used |= {f'{a}{r}' for r in range(int(lo), int(hi) + 1)}
            else:
                used.add(f'{b}{n}')
        if used & regs and not t.startswith('v_mfma'):
            worst = cnt if worst is None else min(worst, cnt)
            break
        cnt += 1
print('min wait states before an MFMA result is read:', worst)
