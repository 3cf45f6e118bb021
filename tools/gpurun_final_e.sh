#!/bin/bash
# final evidence E (on the GPU box): the headline bench line and its rocprofv3 kernel stats on the
# same box, then bench lines part 2.  usage: tools/gpurun_final_e.sh TAG
set -o pipefail
T=${1:?tag}
timeout -k 10 300 bash tools/bench_sweep.sh ${T}_e rmsc03 || exit 1
timeout -k 10 400 bash tools/final_evidence.sh ${T}e rmsc03:4096 > gpurun_out/${T}_e/pmc.log 2>&1 || { tail gpurun_out/${T}_e/pmc.log; exit 1; }
bash tools/gpurun_final_bench2.sh $T
