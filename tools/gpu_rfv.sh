#!/bin/bash
# random_fund_value on the GPU: the whole parity suite (the event key layout is shared by every
# configuration), then bench lines at 512 and 1024 envs.  usage: tools/gpu_rfv.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-rfv}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error|error" $OUT/pytest_gpu.log | head -20; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for n in ${RFV_ENVS:-512 1024}; do
  timeout -k 10 300 python bench.py --config random_fund_value --envs $n --steps 2 --warmup 1 > $OUT/bench_rfv_$n.json 2> $OUT/bench_rfv_$n.err || { echo "bench $n failed"; tail $OUT/bench_rfv_$n.err; exit 1; }
  cut -c1-400 $OUT/bench_rfv_$n.json
done
timeout -k 10 200 python bench.py > $OUT/bench_rmsc03.json 2> $OUT/bench_rmsc03.err || { echo "bench rmsc03 failed"; tail $OUT/bench_rmsc03.err; exit 1; }
cut -c1-300 $OUT/bench_rmsc03.json
# optional extra configurations (A/B of shared-code changes): EXTRA="sparse_zi_1000:1024 rmsc01:4096"
for ce in $EXTRA; do
  c=${ce%%:*}; n=${ce##*:}
  timeout -k 10 300 python bench.py --config $c --envs $n --steps 2 --warmup 1 --no-cpu > $OUT/bench_${c}_$n.json 2> $OUT/bench_${c}_$n.err || { echo "bench $c failed"; tail $OUT/bench_${c}_$n.err; exit 1; }
  cut -c1-250 $OUT/bench_${c}_$n.json
done
