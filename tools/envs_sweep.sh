#!/bin/bash
# per-wave event latency vs waves per SIMD: the rmsc03 bench at 256/1024/2048/4096 envs
set -o pipefail
OUT=gpurun_out/${1:-sweep}
mkdir -p $OUT
for n in 256 1024 2048 4096; do
  timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu --envs $n > $OUT/sweep_$n.json 2>$OUT/sweep_$n.err || { echo "sweep $n failed"; tail $OUT/sweep_$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/sweep_$n.json'));print($n, 'envs', round(d['value']/1e6,1),'M ev/s', round(d['roofline']['avg_launch_ms'],1),'ms', int(d['config']['events_per_step']), 'events')"
done
