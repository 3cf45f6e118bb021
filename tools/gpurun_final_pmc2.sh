set -o pipefail
timeout -k 10 1100 bash tools/final_evidence.sh r04f rmsc01:4096 rmsc02:4096 obi_rmsc02:4096 random_fund_diverse:2048 hist_fund_value:2048 hist_fund_diverse:2048
