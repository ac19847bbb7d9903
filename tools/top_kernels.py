"""Print the top kernels of a rocprofv3 kernel_stats.csv (name, calls, total us, average us, %)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 22]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {int(r['TotalDurationNs']) // 1000:8d} us "
          f"{float(r['AverageNs']) / 1000:8.2f} us {float(r['Percentage']):6.2f}%")
