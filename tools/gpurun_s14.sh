set -o pipefail
timeout -k 10 600 bash tools/ab_cfg.sh s14 rmsc02 4096 v7ser v7wave v7r03
