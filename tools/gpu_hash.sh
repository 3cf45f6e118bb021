#!/bin/bash
# parity suite (incl. the hash-switch tests), then the default bench (parity hash off) and the
# same with --parity-hash.  usage: tools/gpu_hash.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-hash}
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo bench failed; tail $OUT/bench.err; exit 1; }
timeout -k 10 400 python bench.py --parity-hash --no-cpu > $OUT/bench_hash.json 2> $OUT/bench_hash.err || { echo bench failed; tail $OUT/bench_hash.err; exit 1; }
for f in bench bench_hash; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', round(d['value']/1e6,1),'M ev/s', round(d['roofline']['avg_launch_ms'],1),'ms', d['config']['parity_hash'])"; done
