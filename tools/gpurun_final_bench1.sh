# final bench lines, part 1 (on the GPU box).  usage: tools/gpurun_final_bench1.sh TAG
set -o pipefail
T=${1:?tag}
timeout -k 10 900 bash tools/bench_sweep.sh ${T}_b1 rmsc03 sparse_zi_1000 marketreplay random_fund_value rmsc03_rl rmsc03_ddqn rmsc03_sweep value_noise || exit 1
timeout -k 10 200 bash tools/bench_sweep.sh ${T}_goog marketreplay -- --tape GOOG_2012-06-21
