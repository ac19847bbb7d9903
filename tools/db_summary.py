"""Per-kernel totals from a rocprofv3 kernel_stats.csv (or the rocpd .db of a run without csv)."""
import csv
import glob
import sqlite3
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
csvs = glob.glob(f'{d}/**/*kernel_stats.csv', recursive=True)
if csvs:
    rows = [(r['Name'], int(r['Calls']), float(r['TotalDurationNs'])) for r in csv.DictReader(open(csvs[0]))]
else:
    db = sqlite3.connect(glob.glob(f'{d}/**/*.db', recursive=True)[0])
    rows = db.execute('select name, count(*), sum(end-start) from kernels group by name').fetchall()
rows.sort(key=lambda r: -r[2])
for name, calls, tot in rows[:n]:
    print(f'{tot / 1e6:9.3f} ms {calls:6d} {tot / calls / 1e3:8.2f} us  {name[:110]}')
