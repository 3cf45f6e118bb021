set -o pipefail
O=gpurun_out/s3; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench_rmsc03.json 2> $O/bench_rmsc03.err || { tail $O/bench_rmsc03.err; exit 1; }
cut -c1-300 $O/bench_rmsc03.json
timeout -k 10 300 python bench.py --config rmsc03_sweep > $O/bench_sweep.json 2> $O/bench_sweep.err || { tail $O/bench_sweep.err; exit 1; }
cut -c1-300 $O/bench_sweep.json
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof3.so timeout -k 10 300 python tools/prof_replay.py IBM_2003-01-14 512 > $O/prof_replay_ibm.txt 2>&1 || { tail $O/prof_replay_ibm.txt; exit 1; }
cat $O/prof_replay_ibm.txt
