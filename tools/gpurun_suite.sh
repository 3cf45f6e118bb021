#!/bin/bash
# the GPU suite and smoke() on the current tree.  usage: tools/gpurun_suite.sh TAG
set -o pipefail
O=gpurun_out/suite_${1:?tag}; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
