#!/bin/bash
# session-5 evidence: every bench config, rocprofv3 stats + HBM passes of the default bench and of
# sparse_zi_1000 x1024 (configs[2])
set -o pipefail
R=$PWD
bash tools/bench_all2.sh s5 || exit 1
bash tools/profile_round.sh s5 || exit 1
OUT=$R/gpurun_out/prof_s5_z1k; mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
A="--config sparse_zi_1000 --envs 1024 --no-cpu"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/bench.py $A --steps 2 --warmup 1 > $OUT/trace.log 2>&1 || { echo "z1k trace failed"; tail $OUT/trace.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o pmc -- \
  python3 $R/bench.py $A --steps 1 --warmup 0 > $OUT/fetch.log 2>&1 || { echo "z1k fetch failed"; tail $OUT/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o pmc -- \
  python3 $R/bench.py $A --steps 1 --warmup 0 > $OUT/write.log 2>&1 || { echo "z1k write failed"; tail $OUT/write.log; exit 1; }
cd $R
python3 tools/hbm_summary.py $OUT
