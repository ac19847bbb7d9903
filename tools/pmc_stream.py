"""Pooled HBM traffic per launch of the decode weight-streaming kernels (bench.py STREAM_KERNELS) from
two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE: separate runs, MI355X_MICROARCH.md HBM section).

Usage: python tools/pmc_stream.py FETCH_DIR WRITE_DIR  -> JSON on stdout

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced streaming read, so fetch bytes = 2 x 1024 x FETCH_SIZE (the guide's correction); WRITE_SIZE
reads 16-B streaming stores exactly.  traffic per launch = (fetch + write) / launches, pooled over the
same kernel class as the bench line's roofline, and per kernel.
"""
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import STREAM_KERNELS  # noqa: E402


def base(name):
    m = re.search(r'rwkvmi::(\w+)', name)
    return m.group(1) if m else name.split('(')[0]


def collect(d, counter):
    per = {}
    for f in glob.glob(f'{d}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(f)):
            if r['Counter_Name'] != counter:
                continue
            b = base(r.get('Kernel_Name', ''))
            p = per.setdefault(b, [0, 0.0])
            p[0] += 1
            p[1] += float(r['Counter_Value']) * 1024.0
    return per


def main():
    fe, wr = collect(sys.argv[1], 'FETCH_SIZE'), collect(sys.argv[2], 'WRITE_SIZE')
    out = {'source': 'rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes) of bench.py --decode-only; '
                     'fetch x2 (gfx950 FETCH_SIZE correction)', 'kernels': {}}
    pool_n, pool_b = 0, 0.0
    for k in sorted(set(fe) | set(wr)):
        n = fe.get(k, [0, 0.0])[0] or wr.get(k, [0, 0.0])[0]
        if not n:
            continue
        fb = 2.0 * fe.get(k, [0, 0.0])[1] / max(1, fe.get(k, [1, 0])[0])
        wb = wr.get(k, [0, 0.0])[1] / max(1, wr.get(k, [1, 0])[0])
        out['kernels'][k] = {'launches': n, 'fetch_bytes_per_launch_x2': round(fb), 'write_bytes_per_launch': round(wb),
                             'traffic_bytes_per_launch': round(fb + wb)}
        if k in STREAM_KERNELS:
            pool_n += n
            pool_b += (fb + wb) * n
    out['decode_stream'] = {'kernels': sorted(k for k in out['kernels'] if k in STREAM_KERNELS), 'launches': pool_n,
                            'traffic_bytes_per_launch': round(pool_b / pool_n) if pool_n else None}
    print(json.dumps(out, indent=1))


if __name__ == '__main__':
    main()
