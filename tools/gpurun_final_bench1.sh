set -o pipefail
timeout -k 10 900 bash tools/bench_sweep.sh r04fb rmsc03 sparse_zi_1000 marketreplay random_fund_value rmsc03_rl rmsc03_ddqn rmsc03_sweep value_noise || exit 1
timeout -k 10 200 bash tools/bench_sweep.sh r04fb_goog marketreplay -- --tape GOOG_2012-06-21
