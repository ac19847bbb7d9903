"""Recompute the bench line's decode roofline from a rocprofv3 kernel_stats.csv of `bench.py --decode-only`.

Usage: python tools/roofline_from_csv.py KERNEL_STATS_CSV BENCH_JSON_LINE_FILE

The pooled kernel class is bench.py's STREAM_KERNELS (every decode launch that streams layer or head
weights).  avg duration = sum(TotalDurationNs) / sum(Calls) over those kernels; achieved = the bench
line's algorithmic bytes per launch / that average; frac = achieved / 8000 GB/s.  Prints both the
recomputed and the line's own (per-dispatch HIP event) numbers and their ratio.
"""
import csv
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import HBM_PEAK_GBS, STREAM_KERNELS  # noqa: E402


def kernel_base(name):
    m = re.search(r'rwkvmi::(\w+)', name)
    return m.group(1) if m else name


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    line = None
    for ln in open(sys.argv[2]):
        if ln.startswith('{'):
            line = json.loads(ln)
    rl = line['roofline']
    calls = ns = 0
    per = {}
    for r in rows:
        b = kernel_base(r['Name'])
        if b in STREAM_KERNELS:
            calls += int(r['Calls'])
            ns += int(r['TotalDurationNs'])
            p = per.setdefault(b, [0, 0])
            p[0] += int(r['Calls'])
            p[1] += int(r['TotalDurationNs'])
    avg_us = ns / calls / 1e3
    achieved = rl['algorithmic_bytes_per_launch'] / (avg_us * 1e-6) / 1e9
    out = {
        'csv': sys.argv[1], 'kernels': {k: {'calls': v[0], 'avg_us': round(v[1] / v[0] / 1e3, 3)} for k, v in per.items()},
        'pooled_calls': calls, 'pooled_avg_us': round(avg_us, 3),
        'algorithmic_bytes_per_launch (bench line)': rl['algorithmic_bytes_per_launch'],
        'achieved_GBps': round(achieved, 1), 'frac': round(achieved / HBM_PEAK_GBS, 4),
        'bench_line_frac': rl['frac'], 'bench_line_avg_us': rl['avg_launch_us'],
        'ratio_line_over_csv': round(rl['frac'] / (achieved / HBM_PEAK_GBS), 4),
    }
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
