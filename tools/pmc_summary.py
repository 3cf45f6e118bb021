"""Summarise rocprofv3 --pmc csv output per kernel (sum over dispatches)."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(root + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"][:60]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in tot.items():
    if "run_kernel" not in k and "build_kernel" not in k:
        continue
    print("==", k)
    for n in sorted(c):
        print("  %-22s %.4g" % (n, c[n]))
