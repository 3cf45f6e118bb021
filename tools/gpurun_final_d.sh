#!/bin/bash
# final evidence D (on the GPU box): the SQ issue records (copied into profiles/ on the box so the
# bench lines that follow attach them), then bench lines part 1.  usage: tools/gpurun_final_d.sh TAG
set -o pipefail
T=${1:?tag}
bash tools/gpurun_final_sq.sh $T rmsc03:4096 rmsc03_rl:4096 rmsc01:4096 rmsc02:4096 random_fund_value:2048 sparse_zi_1000:1024 marketreplay:512 || exit 1
for d in gpurun_out/sq_${T}_*/; do cp $d/issue_*.json profiles/ || exit 1; done
bash tools/gpurun_final_bench1.sh $T
