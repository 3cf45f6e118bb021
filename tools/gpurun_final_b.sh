set -o pipefail
timeout -k 10 300 bash tools/ab_cfg.sh s14 rmsc02 4096 v7ser v7wave v7r03 || exit 1
bash tools/gpurun_final_a.sh
