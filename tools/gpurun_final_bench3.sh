# final bench lines, part 3 (on the GPU box): north_star's per-shard sizes (configs[3] x4096 on 8
# GPUs = 512 per GPU, configs[4] x512 on 8 GPUs = 64 per GPU) and the runtime compositions.
# usage: tools/gpurun_final_bench3.sh TAG
set -o pipefail
T=${1:?tag}
timeout -k 10 300 bash tools/bench_sweep.sh ${T}_shard rmsc03_ddqn:512 marketreplay:64 || exit 1
timeout -k 10 200 bash tools/bench_sweep.sh ${T}_shard_goog marketreplay:64 -- --tape GOOG_2012-06-21 || exit 1
timeout -k 10 600 bash tools/bench_sweep.sh ${T}_cfg cfg.rmsc03_n100_v20 cfg.rmsc03_alt cfg.sparse_zi_alt cfg.sparse_zi_matrix_200 cfg.value_noise_alt
