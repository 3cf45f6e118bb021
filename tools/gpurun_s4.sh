set -o pipefail
O=gpurun_out/s4; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_replay_runner.py tests/test_gpu_episodes.py tests/test_gpu_rl.py tests/test_gpu_ddqn.py tests/test_gpu_booklog.py tests/test_gpu_bench_sizes.py -k "replay or rl or episode or ddqn or booklog or book_log" -x -v --timeout 600 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof3.so timeout -k 10 300 python tools/prof_replay.py IBM_2003-01-14 512 > $O/prof_replay_ibm.txt 2>&1 || { tail $O/prof_replay_ibm.txt; exit 1; }
cat $O/prof_replay_ibm.txt
timeout -k 10 300 python bench.py --config marketreplay --no-latency > $O/bench_replay.json 2> $O/bench_replay.err || { tail $O/bench_replay.err; exit 1; }
cut -c1-300 $O/bench_replay.json
timeout -k 10 300 python bench.py --config rmsc03_rl --no-cpu > $O/bench_rl.json 2> $O/bench_rl.err || { tail $O/bench_rl.err; exit 1; }
cut -c1-300 $O/bench_rl.json
timeout -k 10 600 bash tools/profile_round.sh r04s4 rmsc03 4096 > $O/prof_round.log 2>&1 || { tail $O/prof_round.log; exit 1; }
tail -5 $O/prof_round.log
