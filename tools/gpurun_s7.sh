set -o pipefail
O=gpurun_out/s7; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_replay_runner.py tests/test_gpu_episodes.py tests/test_gpu_rl.py tests/test_gpu_booklog.py tests/test_gpu_bench_sizes.py -k "replay or rl or episode or booklog or book_log" -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof3.so timeout -k 10 300 python tools/prof_replay.py IBM_2003-01-14 512 > $O/prof_replay_ibm.txt 2>&1 || { tail $O/prof_replay_ibm.txt; exit 1; }
cat $O/prof_replay_ibm.txt
timeout -k 10 300 python bench.py --config marketreplay --no-latency --no-cpu > $O/bench_replay.json 2> $O/bench_replay.err || { tail $O/bench_replay.err; exit 1; }
cut -c1-300 $O/bench_replay.json
timeout -k 10 900 bash tools/ab_cfg.sh s7 random_fund_value 2048 v9new v9sg v9grp v9old && timeout -k 10 600 bash tools/ab_cfg.sh s7 sparse_zi_1000 1024 v2new v2sg
