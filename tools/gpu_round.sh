#!/bin/bash
# One GPU session: parity tests, bench, rocprofv3 kernel trace + HBM counters.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
OUT=$R/gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
timeout -k 10 600 python -m pytest tests -x -q -m gpu > $OUT/pytest_gpu_$TAG.log 2>&1; echo "pytest rc=$?" ; tail -3 $OUT/pytest_gpu_$TAG.log
timeout -k 10 400 python bench.py > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err || { echo bench failed; tail $OUT/bench_$TAG.err; exit 1; }
cat $OUT/bench_$TAG.json | cut -c1-400
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$TAG -o trace -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/prof_$TAG.log 2>&1 || { echo prof failed; tail $OUT/prof_$TAG.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$TAG -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/pmc_fetch_$TAG.log 2>&1 || { echo pmc fetch failed; tail $OUT/pmc_fetch_$TAG.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$TAG -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/pmc_write_$TAG.log 2>&1 || { echo pmc write failed; tail $OUT/pmc_write_$TAG.log; exit 1; }
find $OUT/prof_$TAG $OUT/pmc_fetch_$TAG $OUT/pmc_write_$TAG -name "*.csv" | head -20
