"""Summarize rocprofv3 PMC passes (tools/pmc_traffic.sh) into per-launch HBM traffic.

FETCH_SIZE is doubled (gfx950 tallies 128-B requests of wide streaming reads at 64 B,
MI355X_MICROARCH.md HBM section); WRITE_SIZE is taken as is.  Both are in KiB per dispatch.
All decode matvec instantiations (k_mv<...>, k_mva<...>) are pooled under the name bench.py reports, "k_mv".
Usage: python tools/pmc_summary.py TAG CONFIG  ->  updates profiles/pmc_traffic.json
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get('Counter_Name') != counter:
                continue
            name = r['Kernel_Name']
            key = 'k_mv' if ('k_mv<' in name or 'k_mva<' in name) else name.split('(')[0]
            tot[key] += float(r['Counter_Value']) * 1024.0
            cnt[key] += 1
    return tot, cnt


def main():
    tag, config = sys.argv[1], sys.argv[2]
    out = os.path.join(REPO, 'profiles', 'pmc_traffic.json')
    fetch, fc = per_kernel(os.path.join(REPO, 'gpurun_out', f'pmc_{tag}_fetch'), 'FETCH_SIZE')
    write, wc = per_kernel(os.path.join(REPO, 'gpurun_out', f'pmc_{tag}_write'), 'WRITE_SIZE')
    res = {}
    for k in fetch:
        if not fc[k] or not wc.get(k):
            continue
        f = 2.0 * fetch[k] / fc[k]
        w = write[k] / wc[k]
        res[k] = {'launches': fc[k], 'fetch_bytes_per_launch_x2': round(f), 'write_bytes_per_launch': round(w),
                  'traffic_bytes_per_launch': round(f + w),
                  'source': f'rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, tag {tag}'}
    data = json.load(open(out)) if os.path.isfile(out) else {}
    data[config] = res
    json.dump(data, open(out, 'w'), indent=1, sort_keys=True)
    for k, v in sorted(res.items(), key=lambda kv: -kv[1]['traffic_bytes_per_launch'] * kv[1]['launches'])[:12]:
        print(f"{k[:60]:60s} {v['launches']:6d} {v['traffic_bytes_per_launch'] / 1e6:10.3f} MB/launch")


if __name__ == '__main__':
    main()
