#!/bin/bash
# final evidence A (round 6): the GPU suite and smoke on the frozen build, then PMC records part 1
set -o pipefail
T=${1:?tag}
O=gpurun_out/final_$T; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { grep -E "FAILED|Error" $O/pytest_gpu.log | head; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 700 bash tools/final_evidence.sh $T rmsc03:4096 rmsc03_rl:4096 rmsc03_ddqn:4096 sparse_zi_1000:1024 marketreplay:512 marketreplay:512:GOOG_2012-06-21 > $O/pmc1.log 2>&1 || { tail $O/pmc1.log; exit 1; }
grep profiled $O/pmc1.log
