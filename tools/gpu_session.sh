#!/bin/bash
# One GPU session: parity tests, the default bench, the GymKernel (rmsc03_rl) bench, then
# rocprofv3 kernel-trace stats of each bench and HBM counters (FETCH_SIZE, WRITE_SIZE) of the
# default bench in passes of their own.  usage: tools/gpu_session.sh TAG [skip-tests]
set -o pipefail
export TMPDIR=/tmp
R=$PWD
TAG=${1:-r01}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
    || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
  tail -2 $OUT/pytest_gpu.log
fi
timeout -k 10 300 python bench.py > $OUT/bench_rmsc03.json 2> $OUT/bench_rmsc03.err || { echo bench failed; tail $OUT/bench_rmsc03.err; exit 1; }
cut -c1-600 $OUT/bench_rmsc03.json
timeout -k 10 300 python bench.py --config rmsc03_rl > $OUT/bench_rmsc03_rl.json 2> $OUT/bench_rmsc03_rl.err || { echo rl bench failed; tail $OUT/bench_rmsc03_rl.err; exit 1; }
cut -c1-600 $OUT/bench_rmsc03_rl.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/bench.py --no-cpu > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_rl -o run -- \
  python3 $R/bench.py --config rmsc03_rl --no-cpu > $OUT/trace_rl.log 2>&1 || { echo "rl trace pass failed"; tail $OUT/trace_rl.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/write.log 2>&1 || { echo "write pass failed"; tail $OUT/write.log; exit 1; }
cd $R
python3 tools/hbm_summary.py $OUT > $OUT/hbm_summary.txt && head -20 $OUT/hbm_summary.txt
find $OUT -name "*kernel_stats.csv" | while read f; do echo "== $f"; cut -d, -f1-6 "$f" | head -8; done
