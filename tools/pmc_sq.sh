#!/bin/bash
# SQ issue/stall counters for the bench workload (one bench step, no CPU leg).
# usage: tools/pmc_sq.sh TAG [extra bench args]
set -o pipefail
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out/pmc_sq_$1
shift
mkdir -p $OUT
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS \
  --output-format csv -d $OUT/p1 -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu "$@" > $OUT/p1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_BRANCH SQ_INSTS_FLAT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT \
  --output-format csv -d $OUT/p2 -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu "$@" > $OUT/p2.log 2>&1
rc=$?
cd $R
python3 tools/pmc_summary.py $OUT
exit $rc
