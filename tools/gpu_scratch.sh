set -o pipefail
O=gpurun_out/dq1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ddqn.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --config rmsc03_ddqn --steps 3 --warmup 1 > $O/bench_ddqn.json 2> $O/bench_ddqn.err || { tail $O/bench_ddqn.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_ddqn.json'));print(round(d['value']/1e9,3),'G', round(d['ms_per_step'],1), d['config']['gym_steps_per_s'], d['config']['learn_steps'], d['config']['step_kernel_ms_total'])"
