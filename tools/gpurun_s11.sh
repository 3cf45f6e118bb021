set -o pipefail
O=gpurun_out/s11; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAILED|Error" $O/pytest.log | head; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
MXA_LIB=marl-optimal-execution_amd/lib/libmxa_prof3.so timeout -k 10 300 python tools/prof_replay.py IBM_2003-01-14 512 > $O/prof_replay_ibm.txt 2>&1 || { tail $O/prof_replay_ibm.txt; exit 1; }
head -16 $O/prof_replay_ibm.txt
timeout -k 10 300 python bench.py --config marketreplay --no-latency --no-cpu > $O/bench_replay.json 2> $O/bench_replay.err || { tail $O/bench_replay.err; exit 1; }
python -c "import json;b=json.load(open('$O/bench_replay.json'));print(b['value'], b['roofline']['avg_launch_ms'])"
