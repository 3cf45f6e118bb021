#!/bin/bash
# SQ counters of the current build (tools/pmc_sq.sh) plus the instruction-cache hit/miss pair of
# the rmsc03 bench step, in its own pass
set -o pipefail
R=$PWD
bash tools/pmc_sq.sh s5 || exit 1
OUT=$R/gpurun_out/pmc_icache_s5; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $OUT/p1 -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/p1.log 2>&1 || { echo "icache pass failed"; tail -5 $OUT/p1.log; exit 1; }
cd $R
python3 tools/pmc_summary.py $OUT
