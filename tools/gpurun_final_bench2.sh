# final bench lines, part 2 (on the GPU box).  usage: tools/gpurun_final_bench2.sh TAG
set -o pipefail
T=${1:?tag}
timeout -k 10 1100 bash tools/bench_sweep.sh ${T}_b2 rmsc01 rmsc02 obi_rmsc02 random_fund_diverse hist_fund_value hist_fund_diverse sparse_zi_100 rmsc03_sbmm rmsc03_sbmm_poll
