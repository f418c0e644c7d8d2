"""Splits a decode kernel trace into step replays (a step = the kernels between
two launches of the step's first kernel) and prints, for the median step, each
kernel's duration and the gap before it.  python tools/decode_gaps.py <trace dir>"""
import collections
import csv
import glob
import sys


def main(d):
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    ev = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    # the step's kernels: those launched at least 100 times
    cnt = collections.Counter(n for n, _, _ in ev)
    step = [e for e in ev if cnt[e[0]] >= 100]
    first = step[0][0]
    steps, cur = [], []
    for e in step:
        if e[0] == first and cur:
            steps.append(cur)
            cur = []
        cur.append(e)
    steps.append(cur)
    n = collections.Counter(len(s) for s in steps).most_common(1)[0][0]
    steps = [s for s in steps if len(s) == n]
    span = sorted((s[-1][2] - s[0][1], i) for i, s in enumerate(steps))
    print(f"{len(steps)} steps of {n} kernels; span us min {span[0][0] / 1e3:.1f} median {span[len(span) // 2][0] / 1e3:.1f}")
    s = steps[span[0][1]]  # the fastest replay (graph)
    busy = sum(e[2] - e[1] for e in s)
    print(f"fastest step: span {(s[-1][2] - s[0][1]) / 1e3:.1f} us, kernel time {busy / 1e3:.1f} us")
    agg = collections.OrderedDict()
    prev = None
    for name, a, b in s:
        k = name[:70]
        g = (a - prev) / 1e3 if prev else 0.0
        t = agg.setdefault(k, [0, 0.0, 0.0])
        t[0] += 1
        t[1] += (b - a) / 1e3
        t[2] += g
        prev = b
    for k, (c, dur, gap) in agg.items():
        print(f"{c:3d} x  dur {dur:7.1f} us  gaps {gap:6.1f} us  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
