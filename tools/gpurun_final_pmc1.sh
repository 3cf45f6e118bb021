set -o pipefail
timeout -k 10 1100 bash tools/final_evidence.sh r04f rmsc03:4096 rmsc03_rl:4096 rmsc03_ddqn:4096 sparse_zi_1000:1024 marketreplay:512 marketreplay:512:GOOG_2012-06-21 random_fund_value:2048 sparse_zi_100:4096 value_noise:4096 rmsc03_sbmm:4096 rmsc03_sbmm_poll:4096 rmsc03_sweep:4096
