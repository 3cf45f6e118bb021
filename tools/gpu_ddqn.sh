#!/bin/bash
# DDQN learner on the GPU: its parity test, then the rmsc03_ddqn and rmsc03_rl benches.
# usage: tools/gpu_ddqn.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-ddqn}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddqn.py -x -v --timeout 240 --timeout-method thread -m gpu > $OUT/pytest_ddqn.log 2>&1 \
  || { echo "pytest failed"; tail -40 $OUT/pytest_ddqn.log; exit 1; }
tail -3 $OUT/pytest_ddqn.log
timeout -k 10 300 python bench.py --config rmsc03_ddqn --steps 2 --warmup 1 > $OUT/bench_ddqn.json 2> $OUT/bench_ddqn.err \
  || { echo "ddqn bench failed"; tail $OUT/bench_ddqn.err; exit 1; }
cut -c1-1500 $OUT/bench_ddqn.json
timeout -k 10 300 python bench.py --config rmsc03_rl --steps 2 --warmup 1 --no-cpu > $OUT/bench_rl.json 2> $OUT/bench_rl.err \
  || { echo "rl bench failed"; tail $OUT/bench_rl.err; exit 1; }
cut -c1-300 $OUT/bench_rl.json
