#!/bin/bash
# r06: rocprofv3 kernel stats of the rmsc03_ddqn bench with the fused learner kernels and with the
# PyTorch ops (the small kernels between step launches)
set -o pipefail
export TMPDIR=/tmp
R=$PWD; O=$R/gpurun_out/r06ddqnprof; mkdir -p $O
cd /tmp
for v in fused torch; do
  X=""; [ $v = torch ] && X="--ddqn-torch"
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o run -- \
    python3 $R/bench.py --config rmsc03_ddqn --no-cpu --no-count --no-latency $X > $O/$v.log 2>&1 || { echo "$v failed"; tail $O/$v.log; exit 1; }
done
echo done
