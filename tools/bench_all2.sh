#!/bin/bash
# every bench configuration once (one JSON line each) into gpurun_out/TAG/
set -o pipefail
OUT=gpurun_out/${1:-benches}
mkdir -p $OUT
run() {
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > $OUT/bench_$name.json 2> $OUT/bench_$name.err || { echo "$name failed"; tail $OUT/bench_$name.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_$name.json'));print('$name', round(d['value']/1e6,1),'M', d['unit'], round(d['ms_per_step'],1),'ms/step', round(d['roofline']['avg_launch_ms'],2), d['config'].get('gym_steps_per_s'), d.get('cpu_baseline',{}).get('value'))"
}
run rmsc03_rl_4096 --config rmsc03_rl --steps 2 --warmup 1
run rmsc03_ddqn_4096 --config rmsc03_ddqn --steps 2 --warmup 1
run replay_IBM_512 --config marketreplay --envs 512 --steps 2 --warmup 1
run replay_GOOG_512 --config marketreplay --envs 512 --steps 2 --warmup 1 --tape GOOG_2012-06-21 --no-cpu
run sparse_zi_1000_1024 --config sparse_zi_1000 --envs 1024 --steps 2 --warmup 1
run sparse_zi_100_4096 --config sparse_zi_100 --envs 4096 --steps 2 --warmup 1
run value_noise_4096 --config value_noise --envs 4096 --steps 3 --warmup 1
run rmsc01_4096 --config rmsc01 --envs 4096 --steps 2 --warmup 1
run rmsc02_4096 --config rmsc02 --envs 4096 --steps 2 --warmup 1
run obi_rmsc02_4096 --config obi_rmsc02 --envs 4096 --steps 2 --warmup 1
run random_fund_value_2048 --config random_fund_value --envs 2048 --steps 2 --warmup 1
run random_fund_diverse_2048 --config random_fund_diverse --envs 2048 --steps 2 --warmup 1
