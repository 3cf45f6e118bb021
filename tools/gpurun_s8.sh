set -o pipefail
O=gpurun_out/s8; mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_replay_runner.py tests/test_gpu_episodes.py tests/test_gpu_rl.py tests/test_gpu_booklog.py tests/test_gpu_bench_sizes.py tests/test_gpu_random_fund.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof3.so timeout -k 10 300 python tools/prof_replay.py IBM_2003-01-14 512 > $O/prof_replay_ibm.txt 2>&1 || { tail $O/prof_replay_ibm.txt; exit 1; }
head -30 $O/prof_replay_ibm.txt
timeout -k 10 300 python bench.py --config marketreplay --no-latency --no-cpu > $O/bench_replay.json 2> $O/bench_replay.err || { tail $O/bench_replay.err; exit 1; }
cut -c1-250 $O/bench_replay.json
timeout -k 10 300 python bench.py --config random_fund_value --no-cpu --no-latency > $O/bench_rfv.json 2> $O/bench_rfv.err || { tail $O/bench_rfv.err; exit 1; }
cut -c1-250 $O/bench_rfv.json
timeout -k 10 300 python bench.py --no-cpu --no-latency > $O/bench_rmsc03.json 2> $O/bench_rmsc03.err || { tail $O/bench_rmsc03.err; exit 1; }
cut -c1-250 $O/bench_rmsc03.json
timeout -k 10 600 bash tools/profile_round.sh r04s8 random_fund_value 2048 > $O/prof_rfv.log 2>&1 || { tail $O/prof_rfv.log; exit 1; }
grep -E "bytes_per_launch|AverageNs|mxa_run" $O/prof_rfv.log | head -5
