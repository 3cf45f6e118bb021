set -o pipefail
timeout -k 10 1100 bash tools/bench_sweep.sh r04fb2 rmsc01 rmsc02 obi_rmsc02 random_fund_diverse hist_fund_value hist_fund_diverse sparse_zi_100 rmsc03_sbmm rmsc03_sbmm_poll
