#!/bin/bash
# r06 s9: the GPU suite on the build with k-step launches, then the GymKernel bench lines both ways
set -o pipefail
O=gpurun_out/s9; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -30; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for spec in "marketreplay:IBM_2003-01-14" "marketreplay:GOOG_2012-06-21" "rmsc03_rl:"; do
  IFS=: read cfg tp <<< "$spec"
  a="--config $cfg --no-cpu --no-latency --steps 3"; [ -n "$tp" ] && a="$a --tape $tp"
  for v in many per; do
    x=""; [ $v = per ] && x="--per-step"
    timeout -k 10 400 python bench.py $a $x > $O/bench_${cfg}_${tp}_$v.json 2> $O/bench_${cfg}_${tp}_$v.err || { tail $O/bench_${cfg}_${tp}_$v.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/bench_${cfg}_${tp}_$v.json').read().strip().splitlines()[-1]); print('$cfg $tp $v', '%.4g'%d['value'], '%.2f ms/step'%d['ms_per_step'], d['roofline']['avg_launch_ms'], d['roofline']['launches'])"
  done
done
