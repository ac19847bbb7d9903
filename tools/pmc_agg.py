"""Per-kernel averages of rocprofv3 --pmc counter CSVs: python tools/pmc_agg.py DIR [kernel-substring]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ''
for f in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(lambda: collections.Counter())
    for r in csv.DictReader(open(f)):
        k = r.get('Kernel_Name', '')
        if sub not in k:
            continue
        key = k.split('(')[0][:60]
        agg[key][r['Counter_Name']] += float(r['Counter_Value'])
        cnt[key][r['Counter_Name']] += 1
    for k, m in sorted(agg.items()):
        print(k)
        for c, v in sorted(m.items()):
            print(f'    {c:28s} {v / cnt[k][c]:.4g}  (n={cnt[k][c]})')
