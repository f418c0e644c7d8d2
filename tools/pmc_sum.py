"""Averages per-dispatch PMC values from tools/pmc.sh output directories.
Usage: python tools/pmc_sum.py gpurun_out/pmc_<tag>"""
import csv
import glob
import sys
from collections import defaultdict

tot = defaultdict(float)
cnt = defaultdict(set)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"][:60], r["Counter_Name"])
        tot[k] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
for k in sorted(tot):
    print(f"{k[0]:60s} {k[1]:28s} {tot[k] / len(cnt[k]):16.1f}")
