"""Issue-rate record of the dominant kernel from tools/sq_counters.sh's PMC passes:
python tools/issue_summary.py OUT_DIR CONFIG ENVS [TAPE] -> OUT_DIR/issue_<config>.json.

Per launch-summed counters of the run / step kernel: SQ instruction counts by type and
GRBM_GUI_ACTIVE.  GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs (one GRBM each), so the
kernel's elapsed shader cycles are GRBM_GUI_ACTIVE / 8.  A CU issues at most one instruction per
type per cycle (one SIMD's turn per cycle, one wave per type; MI355X_MICROARCH.md: 4 SIMDs and
ONE scalar unit per CU), so <type> instructions / (256 CUs x elapsed cycles) is that type's issue
rate against its 1.0 ceiling: SALU near 1.0 means the scalar unit bounds the kernel."""
import csv
import glob
import json
import os
import subprocess
import sys
from collections import defaultdict

out, cfg, envs = sys.argv[1], sys.argv[2], int(sys.argv[3])
tape = sys.argv[4] if len(sys.argv) > 4 else None
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
cands = [k for k in tot if "mxa_run_kernel" in k or "mxa_step_kernel" in k]
k = max(cands, key=lambda x: tot[x].get("GRBM_GUI_ACTIVE", 0))
c = tot[k]
events = None
for line in open(os.path.join(out, "p1.log")):
    if line.startswith("{") and '"events_per_step"' in line:
        events = json.loads(line)["config"]["events_per_step"]
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
bid = subprocess.check_output([sys.executable, "-c", "import sys; sys.path.insert(0, %r); import mxabides; print(mxabides.build_id())"
                               % os.path.join(root, "marl-optimal-execution_amd")]).decode().strip()
XCDS, CUS = 8, 256
cyc = c["GRBM_GUI_ACTIVE"] / XCDS
rec = {"config": cfg, "envs": envs, "kernel": k, "build_id": bid, "parity_hash": False,
       "elapsed_cycles": cyc, "cus": CUS, "events": events,
       "per_cu_cycle": {t: c["SQ_INSTS_" + t] / (CUS * cyc) for t in ("SALU", "VALU", "LDS", "SMEM", "BRANCH", "VMEM_RD", "VMEM_WR")},
       "per_event": {t: c["SQ_INSTS_" + t] / events for t in ("SALU", "VALU", "LDS", "SMEM", "BRANCH", "VMEM_RD", "VMEM_WR")} if events else None,
       "counters": dict(c),
       "source": "tools/sq_counters.sh: rocprofv3 --pmc passes of 'bench.py --config %s --envs %d --steps 1 --warmup 0 "
                 "--no-cpu --no-count --no-latency'; per-CU-cycle rates = instructions / (256 CUs x GRBM_GUI_ACTIVE / 8)" % (cfg, envs)}
if tape:
    rec["tape"] = tape
name = cfg if tape in (None, "IBM_2003-01-14") else "%s_%s" % (cfg, tape)
with open(os.path.join(out, "issue_%s.json" % name), "w") as f:
    json.dump(rec, f, indent=1)
print(json.dumps({"kernel": k[:60], "per_cu_cycle": rec["per_cu_cycle"], "per_event": rec["per_event"]}))
