#!/bin/bash
# final evidence F (on the GPU box): the PMC records of the remaining configurations, then bench
# lines part 3 (north_star's per-shard sizes and the runtime compositions).  usage: TAG
set -o pipefail
T=${1:?tag}
bash tools/gpurun_final_pmc.sh $T 3 rmsc02:4096 obi_rmsc02:4096 random_fund_diverse:2048 hist_fund_value:2048 hist_fund_diverse:2048 || exit 1
bash tools/gpurun_final_bench3.sh $T
