# queue groups: full GPU parity with the new defaults; sparse_zi_1000 QG 12/16/24; value_noise grouped vs flat
set -o pipefail
O=gpurun_out/qg2; mkdir -p $O
L=marl-optimal-execution_amd/lib
b() { python -c "import json;d=json.loads(open('$1').read().splitlines()[-1]);print('$1',d['value'],d['roofline']['avg_launch_ms'])"; }
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python bench.py --config sparse_zi_1000 --envs 1024 --steps 2 --warmup 1 > $O/z1k_qg12.json 2> $O/z1k_qg12.err || exit 1
b $O/z1k_qg12.json
for v in qg16 qg24; do
  MXA_LIB=$L/libmxa_$v.so timeout -k 10 120 python bench.py --config sparse_zi_1000 --envs 1024 --steps 2 --warmup 1 > $O/z1k_$v.json 2> $O/z1k_$v.err || exit 1
  b $O/z1k_$v.json
done
timeout -k 10 120 python bench.py --config value_noise --envs 4096 --steps 3 --warmup 1 > $O/vn_hier.json 2> $O/vn_hier.err || exit 1
b $O/vn_hier.json
MXA_LIB=$L/libmxa_vnflat.so timeout -k 10 120 python bench.py --config value_noise --envs 4096 --steps 3 --warmup 1 > $O/vn_flat.json 2> $O/vn_flat.err || exit 1
b $O/vn_flat.json
timeout -k 10 120 python bench.py --config sparse_zi_100 --envs 4096 --steps 3 --warmup 1 > $O/z100.json 2> $O/z100.err || exit 1
b $O/z100.json
