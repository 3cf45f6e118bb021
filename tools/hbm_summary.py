"""Summarise tools/profile_round.sh output: per-kernel stats and HBM bytes per run-kernel launch.

FETCH_SIZE / WRITE_SIZE are in KiB summed over the dispatch (rocprofv3).  Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE on gfx950 reports half the bytes of coalesced
reads, so reads are doubled; writes are taken as reported.  Our access widths (8-16 B per
lane, scattered per env) are not the calibrated streaming case: the absolute figure is
indicative, ratios between builds are exact.

    python tools/hbm_summary.py OUTDIR [--record CONFIG ENVS PARITY_HASH(0|1) SOURCE...]

With --record, also writes profiles/hbm_traffic_<CONFIG>.json: the run kernel's bytes per
launch stamped with the build id of the library that was profiled (mxa_build_id()), which is
what bench.py matches before it reports the figure as roofline.traffic."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
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
# the dominant kernel: the run kernel (Kernel.runner configs) or the step kernel (GymKernel ones)
run = [k for k in fetch if "mxa_run_kernel" in k or "mxa_step_kernel" in k]
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

if "--record" in sys.argv:
    i = sys.argv.index("--record")
    cfg, envs, ph = sys.argv[i + 1], int(sys.argv[i + 2]), sys.argv[i + 3] == "1"
    source = " ".join(sys.argv[i + 4:])
    sys.path.insert(0, os.path.join(ROOT, "marl-optimal-execution_amd"))
    import mxabides
    assert len(res) == 1, "expected exactly one run- or step-kernel instantiation, got %s" % list(res)
    (k, r), = res.items()
    rec = {"config": cfg, "envs": envs, "kernel": k, "build_id": mxabides.build_id(), "parity_hash": ph}
    tape = os.environ.get("MXA_PROF_TAPE")  # marketreplay on another tape than IBM_2003-01-14
    if tape:
        rec["tape"] = tape
    rec.update({x: r[x] for x in ("bytes_per_launch", "read_bytes_corrected", "write_bytes", "fetch_size_kib",
                                  "write_size_kib", "launches")})
    rec["source"] = source
    with open(os.path.join(out, "hbm_traffic_%s.json" % (cfg + ("_" + tape if tape else ""))), "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec, indent=1))
