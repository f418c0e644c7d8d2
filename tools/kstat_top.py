"""Top kernels of a rocprofv3 --stats kernel_stats.csv: name, calls, total ms, avg us.
  python tools/kstat_top.py <run_kernel_stats.csv> [n]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f'{r["Name"][:90]:90s} {r["Calls"]:>6s} {float(r["TotalDurationNs"]) / 1e6:9.2f} '
          f'{float(r["AverageNs"]) / 1e3:9.1f}')
