#!/bin/bash
# copy one evidence call's records from gpurun_out/ into profiles/ (run here, after the call):
# PMC records -> profiles/hbm_traffic_*.json, summaries and kernel stats -> profiles/r06/final/,
# the GPU suite and smoke logs, SQ records -> profiles/issue_*.json and profiles/r06/final/sq/.
# usage: tools/collect_evidence.sh TAG
set -e
T=${1:?tag}
F=profiles/r06/final
mkdir -p $F/sq
for d in gpurun_out/prof_${T}_*; do
  [ -d "$d" ] || continue
  c=${d#gpurun_out/prof_${T}_}
  cp $d/hbm_traffic_*.json profiles/
  cp $d/hbm_summary.json $F/hbm_summary_$c.json
  cp $d/trace/run_kernel_stats.csv $F/kernel_stats_$c.csv
  echo "prof $c"
done
[ -f gpurun_out/final_$T/pytest_gpu.log ] && cp gpurun_out/final_$T/pytest_gpu.log $F/pytest_gpu.log
[ -f gpurun_out/final_$T/smoke.log ] && cp gpurun_out/final_$T/smoke.log $F/smoke.log
for d in gpurun_out/sq_${T}_*/; do
  [ -d "$d" ] || continue
  c=${d#gpurun_out/sq_${T}_}
  c=${c%/}
  for f in $d/issue_*.json; do [ -f "$f" ] && cp $f profiles/; done
  [ -f $d/summary.txt ] && cp $d/summary.txt $F/sq/summary_$c.txt
  echo "sq $c"
done
true
