"""Summarize a rocprofv3 kernel trace: per-kernel stats and one decode token's kernel sequence."""
import csv
import sys

d = sys.argv[1]
rows = list(csv.DictReader(open(f'{d}/run_kernel_stats.csv')))
tot = sum(float(r['TotalDurationNs']) for r in rows)
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:20]:
    print(f"{r['Name'][:58]:58s} {int(r['Calls']):6d} avg {float(r['AverageNs'])/1e3:9.2f}us {float(r['TotalDurationNs'])/tot*100:6.2f}%")
tr = [r for r in csv.DictReader(open(f'{d}/run_kernel_trace.csv')) if 'rwkvmi' in r['Kernel_Name']]
tr.sort(key=lambda r: int(r['Start_Timestamp']))
idx = [i for i, r in enumerate(tr) if 'k_embed_ln' in r['Kernel_Name']]
if len(idx) > 40:
    a, b = idx[30], idx[31]
    span = (int(tr[b]['Start_Timestamp']) - int(tr[a]['Start_Timestamp'])) / 1e3
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in tr[a:b]) / 1e3
    print(f'one decode token: {b - a} kernels, span {span:.1f} us, kernel-busy {busy:.1f} us')
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    for r in tr[a:a + n] + [None] + tr[b - 3:b]:
        if r is None:
            print('  ...')
            continue
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        print(f"  {r['Kernel_Name'][:56]:56s} {(e - s) / 1e3:8.2f}us grid {r['Grid_Size_X']:>7} vgpr {r['VGPR_Count']}")
