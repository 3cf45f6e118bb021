#!/bin/bash
# GPU parity suite + phase profile (MXA_PROF build) + SQ counters of the default build.
# usage: tools/gpu_check.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp
R=$PWD
TAG=$1
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -1 $OUT/pytest_gpu.log
fi
MXA_LIB=$R/marl-optimal-execution_amd/lib/libmxa_prof.so timeout -k 10 300 python tools/prof_phases.py > $OUT/phases.txt 2>&1 || { echo "phases failed"; tail $OUT/phases.txt; exit 1; }
cat $OUT/phases.txt
bash tools/pmc_sq.sh $TAG > $OUT/sq.txt 2>&1 || { echo "pmc failed"; tail $OUT/sq.txt; exit 1; }
cat $OUT/sq.txt
