# sparse_zi_1000 x1024: default vs MXA_QREG library, QREG parity, phase profile
set -o pipefail
O=gpurun_out/z1k; mkdir -p $O
L=marl-optimal-execution_amd/lib
timeout -k 10 120 python bench.py --config sparse_zi_1000 --envs 1024 --steps 2 --warmup 1 > $O/bench_base.json 2> $O/bench_base.err || exit 1
MXA_LIB=$L/libmxa_qreg.so timeout -k 10 120 python bench.py --config sparse_zi_1000 --envs 1024 --steps 2 --warmup 1 > $O/bench_qreg.json 2> $O/bench_qreg.err || exit 1
MXA_LIB=$L/libmxa_qreg.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "sparse_zi_1000 or rmsc03" > $O/pytest_qreg.log 2>&1 || { tail -20 $O/pytest_qreg.log; exit 1; }
MXA_LIB=$L/libmxa_prof.so timeout -k 10 120 python tools/prof_phases2.py sparse_zi_1000 1024 > $O/phases.txt 2>&1 || exit 1
for f in $O/bench_*.json; do python -c "import json;d=json.loads(open('$f').read().splitlines()[-1]);print('$f',d['value'],d['roofline']['avg_launch_ms'])"; done
tail -2 $O/pytest_qreg.log; cat $O/phases.txt
