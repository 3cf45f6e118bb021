#!/bin/bash
# A/B: GPU parity suite on the default libmxa, then smoke + bench of rmsc03-only variants
# (tools/build_variants.sh), twice each in alternating order.  usage: tools/gpu_ab.sh TAG V1 V2 ...
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 300 --timeout-method thread -m gpu > $OUT/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
for rep in 1 2; do
  for w in "$@"; do
    L=marl-optimal-execution_amd/lib/libmxa_$w.so
    if [ $rep = 1 ]; then
      MXA_LIB=$L timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke_$w.log 2>&1 || { echo "smoke $w failed"; tail $OUT/smoke_$w.log; exit 1; }
    fi
    MXA_LIB=$L timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu > $OUT/bench_${w}_$rep.json 2>$OUT/bench_${w}_$rep.err || { echo "bench $w failed"; tail $OUT/bench_${w}_$rep.err; exit 1; }
    echo "$w $(python3 -c "import json;d=json.load(open('$OUT/bench_${w}_$rep.json'));print(round(d['value']/1e6,1),'M ev/s', round(d['roofline']['avg_launch_ms'],1),'ms')")"
  done
done
