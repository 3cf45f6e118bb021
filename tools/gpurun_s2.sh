set -o pipefail
O=gpurun_out/s2; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_ddqn.py tests/test_gpu_records.py tests/test_gpu_bench_sizes.py -k "ddqn or records or sparse_zi_1000" -x -v --timeout 600 --timeout-method thread -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench_rmsc03.json 2> $O/bench_rmsc03.err || { tail $O/bench_rmsc03.err; exit 1; }
cut -c1-400 $O/bench_rmsc03.json
timeout -k 10 300 python bench.py --config rmsc03_ddqn > $O/bench_ddqn.json 2> $O/bench_ddqn.err || { tail $O/bench_ddqn.err; exit 1; }
cut -c1-300 $O/bench_ddqn.json
timeout -k 10 300 python bench.py --config rmsc03_sweep > $O/bench_sweep.json 2> $O/bench_sweep.err || { tail $O/bench_sweep.err; exit 1; }
cut -c1-300 $O/bench_sweep.json
