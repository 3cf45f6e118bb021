# GPU parity suite + sparse_zi_1000 x1024 bench
set -o pipefail
O=gpurun_out/z1k2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python bench.py --config sparse_zi_1000 --envs 1024 --steps 2 --warmup 1 > $O/bench_sparse_zi_1000_1024.json 2> $O/bench.err || { tail $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_sparse_zi_1000_1024.json').read().splitlines()[-1]);print(d['value'],d['roofline']['avg_launch_ms'])"
