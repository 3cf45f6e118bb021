#!/bin/bash
# HBM bytes per event of one configuration's run kernel across library variants (A/B of a
# traffic change): rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes of
# tools/ab_config.py, first run-kernel dispatch (parity hash off), reads doubled as
# tools/hbm_summary.py does.  usage: tools/ab_traffic.sh TAG VARIANT:CONFIG:ENVS ...
#   -> gpurun_out/TAG/traffic.txt
set -o pipefail
export TMPDIR=/tmp
R=$PWD
TAG=$1; shift
mkdir -p $R/gpurun_out/$TAG
for spec in "$@"; do
  IFS=: read v cfg n <<< "$spec"
  O=$R/gpurun_out/$TAG/${v}_$cfg
  mkdir -p $O
  cd /tmp
  for c in FETCH_SIZE WRITE_SIZE; do
    MXA_LIB=$R/marl-optimal-execution_amd/lib/libmxa_$v.so timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv \
      -d $O/$c -o pmc -- python3 $R/tools/ab_config.py $cfg $n 1 > $O/$c.log 2>&1 \
      || { echo "pass $c of $spec failed"; tail -5 $O/$c.log; exit 1; }
  done
  cd $R
  python3 - "$O" "$spec" >> $R/gpurun_out/$TAG/traffic.txt <<'PY' || exit 1
import csv, glob, os, re, sys
o, spec = sys.argv[1], sys.argv[2]
def first(c):
    rows = {}
    for f in glob.glob(os.path.join(o, c, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == c and "mxa_run_kernel" in r["Kernel_Name"]:
                d = int(r["Dispatch_Id"])
                rows[d] = rows.get(d, 0.0) + float(r["Counter_Value"])
    return rows[min(rows)]
line = open(os.path.join(o, "FETCH_SIZE.log")).read()
m = re.search(r"best ([0-9.]+)\), ([0-9.]+) M env-steps/s", line)
ev = float(m.group(2)) * 1e6 * float(m.group(1)) * 1e-3
rd, wr = 2 * first("FETCH_SIZE") * 1024 / ev, first("WRITE_SIZE") * 1024 / ev
print("%s: %.4g events, read %.1f B/event, write %.1f B/event, total %.1f" % (spec, ev, rd, wr, rd + wr))
PY
  tail -1 $R/gpurun_out/$TAG/traffic.txt
done
