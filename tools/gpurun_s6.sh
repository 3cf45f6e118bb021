set -o pipefail
O=gpurun_out/s6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "rng or gauss or kat or math" -x -v --timeout 200 --timeout-method thread -m gpu > $O/pytest_rng.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_rng.log | head; tail -30 $O/pytest_rng.log; exit 1; }
tail -2 $O/pytest_rng.log
timeout -k 10 700 python -u -m pytest tests/test_gpu_replay.py tests/test_gpu_replay_runner.py tests/test_gpu_episodes.py tests/test_gpu_rl.py tests/test_gpu_booklog.py tests/test_gpu_bench_sizes.py tests/test_gpu_random_fund.py -k "replay or rl or episode or booklog or book_log or random_fund or hist_fund or zi_1000" -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof3.so timeout -k 10 300 python tools/prof_replay.py IBM_2003-01-14 512 > $O/prof_replay_ibm.txt 2>&1 || { tail $O/prof_replay_ibm.txt; exit 1; }
cat $O/prof_replay_ibm.txt
timeout -k 10 300 python bench.py --config marketreplay --no-latency > $O/bench_replay.json 2> $O/bench_replay.err || { tail $O/bench_replay.err; exit 1; }
cut -c1-300 $O/bench_replay.json
timeout -k 10 300 python bench.py --config random_fund_value --no-cpu --no-latency > $O/bench_rfv.json 2> $O/bench_rfv.err || { tail $O/bench_rfv.err; exit 1; }
cut -c1-300 $O/bench_rfv.json
timeout -k 10 300 python bench.py --config sparse_zi_1000 --no-cpu --no-latency > $O/bench_z1k.json 2> $O/bench_z1k.err || { tail $O/bench_z1k.err; exit 1; }
cut -c1-300 $O/bench_z1k.json
timeout -k 10 300 python bench.py --no-cpu --no-latency > $O/bench_rmsc03.json 2> $O/bench_rmsc03.err || { tail $O/bench_rmsc03.err; exit 1; }
cut -c1-300 $O/bench_rmsc03.json
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof2.so timeout -k 10 300 python tools/prof_phases.py sparse_zi_1000 1024 > $O/phases_z1k.txt 2>&1 || { tail $O/phases_z1k.txt; exit 1; }
timeout -k 10 600 bash tools/profile_round.sh r04s6 random_fund_value 2048 > $O/prof_rfv.log 2>&1 || { tail $O/prof_rfv.log; exit 1; }
tail -5 $O/prof_rfv.log
