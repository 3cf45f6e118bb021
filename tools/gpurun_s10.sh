#!/bin/bash
# r06 s10: the GPU suite on the build with the per-configuration transacted-volume scan and the
# builder's book initialisation, then run kernels of the configurations the scan choice touches
set -o pipefail
O=gpurun_out/s10; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -x -v --timeout 600 --timeout-method thread -m gpu > $O/pytest_gpu.log 2>&1 \
  || { echo "pytest failed"; grep -E "FAILED|Error|assert" $O/pytest_gpu.log | head -30; tail -5 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for c in "rmsc03 4096 3" "rmsc01 4096 1" "rmsc02 4096 1" "value_noise 4096 3" "sparse_zi_100 4096 2"; do
  timeout -k 10 300 python tools/ab_config.py $c >> $O/run_kernels.txt 2>&1 || { tail $O/run_kernels.txt; exit 1; }
done
cat $O/run_kernels.txt
