set -o pipefail
O=gpurun_out/s2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_rmsc03_4096.json 2> $O/bench_rmsc03_4096.err || { tail $O/bench_rmsc03_4096.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench_rmsc03_4096.json'));print('rmsc03', round(d['value']/1e9,3),'G', round(d['ms_per_step'],1), round(d['roofline']['avg_launch_ms'],2), d['cpu_baseline']['value'])"
bash tools/bench_all2.sh s2
