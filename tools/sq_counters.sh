#!/bin/bash
# SQ instruction-mix and wait counters of one bench command, in PMC passes of their own (at most
# 8 SQ_ counters per pass; no tracing options with --pmc).  usage: tools/sq_counters.sh TAG CONFIG ENVS
#   -> gpurun_out/sq_TAG/{p1,p2}/ and a per-kernel summary in gpurun_out/sq_TAG/summary.txt
set -o pipefail
export TMPDIR=/tmp
R=$PWD
TAG=$1; CFG=$2; ENVS=$3
OUT=$R/gpurun_out/sq_$TAG
mkdir -p $OUT
cd /tmp
B="$R/bench.py --config $CFG --envs $ENVS --steps 1 --warmup 0 --no-cpu --no-count --no-latency"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_INSTS_FLAT"
P3="SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_FLAT SQ_ACTIVE_INST_MISC SQ_INSTS_SALU"
# the clock: GPU-busy cycles (GRBM) and SQ busy cycles, to turn instruction counts into issue rates
P4="GRBM_GUI_ACTIVE GRBM_COUNT SQ_BUSY_CYCLES SQ_CYCLES"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $OUT/p$i -o pmc -- python3 $B > $OUT/p$i.log 2>&1 \
    || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
cd $R
python3 - "$OUT" > $OUT/summary.txt <<'PY'
import csv, glob, os, sys
from collections import defaultdict
out = sys.argv[1]
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        tot[r["Kernel_Name"][:60]][r["Counter_Name"]] += float(r["Counter_Value"])
for k, d in tot.items():
    print("==", k)
    for c in sorted(d):
        print("  %-24s %.4g" % (c, d[c]))
PY
cat $OUT/summary.txt
python3 tools/issue_summary.py $OUT $CFG $ENVS
