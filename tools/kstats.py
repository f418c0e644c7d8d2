"""Compare two rocprofv3 kernel_stats.csv files: average µs per kernel and total ms."""
import csv
import sys


def load(p):
    d = {}
    for r in csv.DictReader(open(p)):
        d[r['Name'][:64]] = (int(r['Calls']), float(r['AverageNs']) / 1e3, float(r['TotalDurationNs']) / 1e6)
    return d


def main(a, b, n=30):
    A, B = load(a), load(b)
    z = (0, 0.0, 0.0)
    keys = sorted(set(A) | set(B), key=lambda k: -B.get(k, z)[2])
    print(f"{'kernel':64s} {'avg_a':>9s} {'avg_b':>9s} {'tot_b ms':>9s}")
    for k in keys[:n]:
        print(f"{k:64s} {A.get(k, z)[1]:9.1f} {B.get(k, z)[1]:9.1f} {B.get(k, z)[2]:9.2f}")
    print(f"{'TOTAL':64s} {'':9s} {'':9s} {sum(v[2] for v in B.values()):9.2f}  (a: {sum(v[2] for v in A.values()):.2f})")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 30)
