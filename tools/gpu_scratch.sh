set -o pipefail
O=gpurun_out/phr3
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_rl.py tests/test_gpu_hash_switch.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_replay.log 2>&1 || { tail -30 $O/pytest_replay.log; exit 1; }
tail -1 $O/pytest_replay.log
for tp in IBM_2003-01-14 GOOG_2012-06-21; do
timeout -k 10 300 python bench.py --config marketreplay --envs 512 --steps 2 --warmup 1 --tape $tp --no-cpu > $O/bench_$tp.json 2> $O/bench_$tp.err || { tail $O/bench_$tp.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_$tp.json'));print('$tp', round(d['value']/1e6,1),'M', round(d['ms_per_step'],1),'ms/step', round(d['roofline']['avg_launch_ms'],3))"
done
