# queue group-size sweep: sparse_zi_1000 x1024 per MXA_QG variant; sparse_zi_100 x4096 grouped vs flat
set -o pipefail
O=gpurun_out/qg; mkdir -p $O
L=marl-optimal-execution_amd/lib
b() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['avg_launch_ms'])"; }
for v in qg4 qg6 qg12; do
  MXA_LIB=$L/libmxa_$v.so timeout -k 10 120 python bench.py --config sparse_zi_1000 --envs 1024 --steps 2 --warmup 1 > $O/z1k_$v.json 2> $O/z1k_$v.err || exit 1
  b $O/z1k_$v.json
done
timeout -k 10 120 python bench.py --config sparse_zi_100 --envs 4096 --steps 3 --warmup 1 > $O/z100_base.json 2> $O/z100_base.err || exit 1
b $O/z100_base.json
MXA_LIB=$L/libmxa_z100.so timeout -k 10 120 python bench.py --config sparse_zi_100 --envs 4096 --steps 3 --warmup 1 > $O/z100_hier.json 2> $O/z100_hier.err || exit 1
b $O/z100_hier.json
MXA_LIB=$L/libmxa_z100.so timeout -k 10 300 python -u -m pytest tests -x -v --timeout 200 --timeout-method thread -m gpu -k "sparse_zi_100" > $O/pytest_z100.log 2>&1 || { tail -20 $O/pytest_z100.log; exit 1; }
tail -1 $O/pytest_z100.log
