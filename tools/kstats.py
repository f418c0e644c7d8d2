"""Per-step kernel time table from a rocprofv3 *_kernel_stats.csv.
Usage: python tools/kstats.py <stats.csv> <steps timed+warmup>"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:int(sys.argv[3]) if len(sys.argv) > 3 else 40]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.2f} ms/step {int(r['Calls']):5d} "
          f"{float(r['AverageNs']) / 1e3:9.1f}us {r['Name'][:120]}")
print(f"total {tot / 1e6 / steps:.2f} ms/step")
