#!/bin/bash
# A/B of record write-back variants (rmsc03-only builds): bench + WRITE_SIZE/FETCH_SIZE per
# variant, and an envs sweep of the default variant (per-wave event latency vs occupancy).
# usage: tools/exp_store.sh TAG VARIANT...
set -o pipefail
export TMPDIR=/tmp
R=$PWD
TAG=$1; shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
for w in "$@"; do
  L=$R/marl-optimal-execution_amd/lib/libmxa_$w.so
  MXA_LIB=$L timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$w.log 2>&1 || { echo "smoke $w failed"; tail $OUT/smoke_$w.log; exit 1; }
  MXA_LIB=$L timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench_$w.json 2>$OUT/bench_$w.err || { echo "bench $w failed"; tail $OUT/bench_$w.err; exit 1; }
  echo "$w $(python3 -c "import json;d=json.load(open('$OUT/bench_$w.json'));print(round(d['value']/1e6,1),'M ev/s', round(d['roofline']['avg_launch_ms'],1),'ms')")"
  cd /tmp
  MXA_LIB=$L timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/$w/write -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/$w.write.log 2>&1 || { echo "write pass $w failed"; tail $OUT/$w.write.log; exit 1; }
  MXA_LIB=$L timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/$w/fetch -o pmc -- python3 $R/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/$w.fetch.log 2>&1 || { echo "fetch pass $w failed"; tail $OUT/$w.fetch.log; exit 1; }
  cd $R
  python3 tools/hbm_summary.py $OUT/$w > $OUT/$w/hbm_summary.json && grep -E "write_bytes|read_bytes" $OUT/$w/hbm_summary.json
done
W=$1
for n in 256 1024 2048; do
  MXA_LIB=$R/marl-optimal-execution_amd/lib/libmxa_$W.so timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --envs $n > $OUT/sweep_$n.json 2>$OUT/sweep_$n.err || { echo "sweep $n failed"; tail $OUT/sweep_$n.err; exit 1; }
  echo "envs $n $(python3 -c "import json;d=json.load(open('$OUT/sweep_$n.json'));print(round(d['value']/1e6,1),'M ev/s', round(d['roofline']['avg_launch_ms'],1),'ms', d['config']['events_per_step'])")"
done
