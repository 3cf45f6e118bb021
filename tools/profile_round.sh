#!/bin/bash
# rocprofv3 evidence for one round: kernel trace + stats of the default bench command, then
# HBM traffic counters in their own passes (FETCH_SIZE, WRITE_SIZE; never mixed with traces).
# usage: tools/profile_round.sh TAG      -> gpurun_out/prof_TAG/...  (copy summaries to profiles/)
set -o pipefail
export TMPDIR=/tmp
R=$PWD
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/bench.py --no-cpu > $OUT/trace.log 2>&1 || { echo "trace pass failed"; tail $OUT/trace.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/fetch.log 2>&1 || { echo "fetch pass failed"; tail $OUT/fetch.log; exit 1; }
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- \
  python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/write.log 2>&1 || { echo "write pass failed"; tail $OUT/write.log; exit 1; }
cd $R
python3 tools/hbm_summary.py $OUT
