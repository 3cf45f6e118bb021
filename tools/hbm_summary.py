"""Summarise tools/profile_round.sh output: per-kernel stats and HBM bytes per run-kernel launch.

FETCH_SIZE / WRITE_SIZE are in KiB summed over the dispatch (rocprofv3).  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE on gfx950 reports half the bytes of coalesced
reads, so reads are doubled; writes are taken as reported.  Our access widths (8-16 B per
lane, scattered per env) are not the calibrated streaming case: the absolute figure is
indicative, ratios between builds are exact."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

out = sys.argv[1]


def pmc(sub, name):
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != name:
                continue
            k = r["Kernel_Name"]
            tot[k] += float(r["Counter_Value"])
            cnt[(k, r.get("Dispatch_Id", ""))] += 1
    return tot, cnt


fetch, fc = pmc("fetch", "FETCH_SIZE")
write, _ = pmc("write", "WRITE_SIZE")
run = [k for k in fetch if "mxa_run_kernel" in k]
res = {}
for k in run:
    n = len({d for (kk, d) in fc if kk == k}) or 1
    rd = 2 * fetch[k] * 1024 / n
    wr = write.get(k, 0.0) * 1024 / n
    res[k] = {"launches": n, "fetch_size_kib": fetch[k] / n, "write_size_kib": write.get(k, 0.0) / n,
              "read_bytes_corrected": rd, "write_bytes": wr, "bytes_per_launch": rd + wr}
stats = glob.glob(os.path.join(out, "trace", "**", "*kernel_stats.csv"), recursive=True)
print(json.dumps(res, indent=1))
for f in stats:
    print(open(f).read())
json.dump(res, open(os.path.join(out, "hbm_summary.json"), "w"), indent=1)
