#!/bin/bash
# final evidence C (on the GPU box): the PMC records of the remaining configurations, then the SQ
# issue records.  usage: tools/gpurun_final_c.sh TAG
set -o pipefail
T=${1:?tag}
bash tools/gpurun_final_pmc.sh $T 3 rmsc02:4096 obi_rmsc02:4096 random_fund_diverse:2048 hist_fund_value:2048 hist_fund_diverse:2048 || exit 1
bash tools/gpurun_final_sq.sh $T rmsc03:4096 rmsc03_rl:4096 rmsc01:4096 rmsc02:4096 random_fund_value:2048 sparse_zi_1000:1024 marketreplay:512
