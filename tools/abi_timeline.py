"""Per-token timeline of the ABI decode from rocprofv3 kernel + memory-copy traces (tools/abi_trace.py).
Usage: python tools/abi_timeline.py DIR...   For each trace: copies by direction and engine (kind),
their durations, and for the last complete tokens the gaps in the kernel stream that copies cover."""
import csv
import glob
import sys


def load(d, pat):
    f = glob.glob(f'{d}/**/*{pat}.csv', recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


for d in sys.argv[1:]:
    ks = load(d, 'kernel_trace')
    cs = load(d, 'memory_copy_trace')
    print(f'== {d}: {len(ks)} kernels, {len(cs)} copies')
    if cs:
        print('   copy columns:', list(cs[0].keys()))
    by = {}
    for c in cs:
        key = (c.get('Direction', c.get('Operation', '?')), c.get('Agent_Id', '') or c.get('Src_Agent_Id', ''))
        dur = (int(c['End_Timestamp']) - int(c['Start_Timestamp'])) / 1e3
        size = int(c.get('Bytes', c.get('Size', 0)) or 0)
        b = by.setdefault(key, [0, 0.0, 0])
        b[0] += 1
        b[1] += dur
        b[2] += size
    for k, (n, us, sz) in sorted(by.items()):
        print(f'   copies {k}: {n} x, avg {us / n:.1f} us, avg {sz / n / 1e6:.2f} MB, {sz / max(us, 1e-9) / 1e3:.1f} GB/s')
    blit = [k for k in ks if 'rocclr' in k['Kernel_Name']]
    names = {}
    for k in blit:
        n = k['Kernel_Name'][:40]
        dur = (int(k['End_Timestamp']) - int(k['Start_Timestamp'])) / 1e3
        names.setdefault(n, [0, 0.0])
        names[n][0] += 1
        names[n][1] += dur
    for n, (c, us) in names.items():
        print(f'   runtime kernel {n}: {c} x avg {us / c:.1f} us')
    # per-token span: k_embed_ln starts a token
    ks.sort(key=lambda k: int(k['Start_Timestamp']))
    starts = [int(k['Start_Timestamp']) for k in ks if 'k_embed_ln' in k['Kernel_Name']]
    if len(starts) > 4:
        per = [(b - a) / 1e3 for a, b in zip(starts[-5:-1], starts[-4:])]
        print('   token periods (us, last 4):', [round(p, 1) for p in per])
        t0, t1 = starts[-3], starts[-2]
        busy = sum(min(int(k['End_Timestamp']), t1) - max(int(k['Start_Timestamp']), t0)
                   for k in ks if int(k['End_Timestamp']) > t0 and int(k['Start_Timestamp']) < t1
                   and 'rocclr' not in k['Kernel_Name']) / 1e3
        print(f'   one token: period {(t1 - t0) / 1e3:.1f} us, model kernels busy {busy:.1f} us')
        for c in cs:
            a, b = int(c['Start_Timestamp']), int(c['End_Timestamp'])
            if b > t0 and a < t1:
                print(f"      copy {c.get('Direction', c.get('Operation', '?'))} +{(a - t0) / 1e3:.1f} .. +{(b - t0) / 1e3:.1f} us "
                      f"{int(c.get('Bytes', c.get('Size', 0)) or 0) / 1e6:.2f} MB")
        for k in ks:
            a, b = int(k['Start_Timestamp']), int(k['End_Timestamp'])
            if b > t0 and a < t1 and 'rocclr' in k['Kernel_Name']:
                print(f"      runtime kernel +{(a - t0) / 1e3:.1f} .. +{(b - t0) / 1e3:.1f} us {k['Kernel_Name'][:40]}")
